"""Cluster route delta feed on the host engine (no device):
tm_route_apply through emqx_router_helper.RouteFeed / cleanup_routes and the
emqx_shared_sub route rules, checked against oracle.RouteTable
(src/emqx_router.erl:113-124, 163-169, 229-247; src/emqx_router_helper.erl:173-177;
src/emqx_shared_sub.erl:297-315, 358-367)."""

import random

import numpy as np
import pytest

from emqx_amd import _native as N
from emqx_amd import emqx_router as R
from emqx_amd import emqx_router_helper as H
from emqx_amd import emqx_shared_sub as S
from emqx_amd.emqx_router import Route
from emqx_amd.engine import Engine
from oracle.oracle import RouteTable

NODES = ["n0@h", "n1@h", "n2@h"]
GROUPS = ["gA", "gB"]
TOPICS = [b"a/+/c", b"a/b/c", b"a/#", b"#", b"+/b/+", b"$SYS/#", b"x/y", b"x/+", b"s/1/t/#", b"s/+/t/+"]


@pytest.fixture
def host_router():
    R.use(Engine(device=-1))
    R._routes.clear()
    S.clear()
    yield R.engine()
    R._routes.clear()
    S.clear()
    R._engine = None


def _dest(rng):
    return rng.choice(NODES) if rng.random() < 0.6 else (rng.choice(GROUPS), rng.choice(NODES))


def _check_same(orc: RouteTable, eng: Engine):
    assert {t: list(d) for t, d in R._routes.items()} == orc.routes
    assert eng.stats()["filters"] == len(orc.routes)
    for t in orc.routes:
        assert eng.filter_id(t) >= 0
    assert eng.empty() == (not orc.routes)


def test_feed_random_events_match_oracle(host_router):
    rng = random.Random(11)
    orc = RouteTable()
    feed = H.RouteFeed(max_pending=97)
    changed = 0
    for _ in range(3000):
        t, d = rng.choice(TOPICS), _dest(rng)
        if rng.random() < 0.55:
            changed += orc.write(t, d)
            feed.push((H.WRITE, Route(t, d)))
        else:
            changed += orc.delete_object(t, d)
            feed.push((H.DELETE_OBJECT, Route(t, d)))
        if rng.random() < 0.01:
            feed.flush()
    feed.flush()
    assert feed.applied == changed
    _check_same(orc, host_router)


def test_nodedown_cleanup_matches_oracle(host_router):
    rng = random.Random(5)
    orc = RouteTable()
    feed = H.RouteFeed()
    for _ in range(800):
        t, d = rng.choice(TOPICS), _dest(rng)
        orc.write(t, d)
        feed.push((H.WRITE, Route(t, d)))
    feed.flush()
    for node in NODES[:2]:
        gone = orc.cleanup_routes(node)
        assert H.nodedown(node) == len(gone)
        _check_same(orc, host_router)
    assert H.cleanup_routes(NODES[0]) == 0          # nothing left of a dead node
    gone = orc.cleanup_routes(NODES[2])
    assert H.cleanup_routes(NODES[2]) == len(gone)
    assert host_router.empty() and not R._routes


def test_feed_rejects_bad_events(host_router):
    feed = H.RouteFeed()
    with pytest.raises(ValueError):
        feed.push(("delete", Route(b"a", NODES[0])))
    with pytest.raises(TypeError):
        feed.push((H.WRITE, Route("a/b", NODES[0])))


def test_route_apply_abi_semantics(host_router):
    e = host_router
    assert e.route_apply([]) == 0
    ev = [(N.TM_ROUTE_WRITE, b"a/+", 1), (N.TM_ROUTE_WRITE, b"a/+", 1), (N.TM_ROUTE_DELETE, b"zz/#", 4),
          (N.TM_ROUTE_DELETE, b"a/+", 2), (N.TM_ROUTE_DELETE, b"a/+", 1)]
    assert e.route_apply(ev) == 3                   # absent (topic, dest) deletes are no-ops
    assert e.filter_id(b"a/+") >= 0                 # one of the two (a/+, 1) refs left
    assert e.route_apply([(N.TM_ROUTE_DELETE, b"a/+", 1)]) == 1
    assert e.empty()
    with pytest.raises(N.TmError):                  # unknown op
        e.route_apply([(7, b"a", 1)])


def test_shared_sub_routes_follow_members(host_router):
    orc = RouteTable()
    S.subscribe("g1", b"t/+", "p1")
    S.subscribe("g1", b"t/+", "p2")
    S.subscribe("g1", b"t/+", "p2")                 # idempotent
    S.subscribe("g2", b"t/+", "p3")
    orc.write(b"t/+", ("g1", R.NODE))
    orc.write(b"t/+", ("g2", R.NODE))
    _check_same(orc, host_router)
    assert S.subscribers("g1", b"t/+") == ["p1", "p2"]
    S.unsubscribe("g1", b"t/+", "p1")
    _check_same(orc, host_router)                   # p2 still holds the g1 route
    assert S.member_down("p2") == 1
    orc.delete_object(b"t/+", ("g1", R.NODE))
    _check_same(orc, host_router)
    S.unsubscribe("g2", b"t/+", "nobody")
    _check_same(orc, host_router)
    S.member_down("p3")
    assert host_router.empty() and not R._routes
