"""Route table semantics on the host engine (no device): emqx_router:do_add_route/2
and do_delete_route/2 (src/emqx_router.erl:113-124, 163-169, 229-247) with the
aggre/1 destination refcount (src/emqx_broker.erl:250-261)."""

import pytest

from emqx_amd import _native as N
from emqx_amd import emqx_router as R
from emqx_amd.engine import Engine


def test_first_route_inserts_last_route_deletes():
    e = Engine(device=-1)
    assert e.empty()
    e.route_add(b"a/+/c", 7)
    assert not e.empty() and e.filter_id(b"a/+/c") >= 0
    e.route_add(b"a/+/c", 7)            # same aggregated dest: counted, not duplicated
    e.route_add(b"a/+/c", 9)
    assert e.route_delete(b"a/+/c", 7)
    assert e.route_delete(b"a/+/c", 9)
    assert e.filter_id(b"a/+/c") >= 0   # one (a/+/c, 7) route left
    assert e.route_delete(b"a/+/c", 7)
    with pytest.raises(KeyError):
        e.filter_id(b"a/+/c")
    assert e.empty()
    assert not e.route_delete(b"a/+/c", 7)   # ENOENT
    assert not e.route_delete(b"never", 1)


def test_exact_topics_go_into_the_trie():
    e = Engine(device=-1)
    e.route_add(b"a/b/c", 1)
    assert e.lookup(b"a/b/c") == (0, b"a/b/c")
    e.route_delete(b"a/b/c", 1)
    assert e.lookup(b"a/b/c") is None


def test_router_mirror_kat_host_side():
    # t_add_delete (test/emqx_router_SUITE.erl:66-73) through the device route table
    R.use(Engine(device=-1))
    R._routes.clear()
    R.add_route(b"a/b/c")
    R.add_route(b"a/b/c", R.NODE)
    R.add_route(b"a/+/b", R.NODE)
    assert sorted(R.topics()) == [b"a/+/b", b"a/b/c"]
    assert R.engine().stats()["filters"] == 2
    R.delete_route(b"a/b/c")
    R.delete_route(b"a/+/b", R.NODE)
    assert R.topics() == [] and R.engine().empty()
    # shared-subscription dests aggregate to their group
    R.add_route(b"t/#", ("g1", "n1"))
    R.add_route(b"t/#", ("g1", "n2"))
    assert R.engine().stats()["filters"] == 1
    R.delete_route(b"t/#", ("g1", "n1"))
    assert not R.engine().empty()
    R.delete_route(b"t/#", ("g1", "n2"))
    assert R.engine().empty()
    R._engine = None


def test_routes_symbols_bound():
    for s in ("tm_route_add", "tm_route_delete", "tm_batch_routes", "tm_match_routes_batch"):
        assert s in N.SIGNATURES
