"""emqx_router mirror (src/emqx_router.erl) on top of the device trie.

The route table (the `emqx_route` bag, include/emqx.hrl:87-90) stays on the
host -- dests are Erlang terms.  Every routed topic, exact or wildcard, is put
into the device trie once (refcounted by its routes), so one device walk
returns M(t) = exact ∪ wildcard matches and `match_routes/1` is a lookup of the
routes of M(t).  The reference gets the same set from
`lookup_routes(Topic) ++ [lookup_routes(To) || To <- emqx_trie:match(Topic)]`
(src/emqx_router.erl:127-133); the order of the returned list differs (the
reference's callers treat it as a set: test/emqx_router_SUITE.erl:85-99 sorts).
"""

from __future__ import annotations

from collections import namedtuple

from . import _native as N
from .emqx_topic import wildcard
from .engine import Engine

Route = namedtuple("Route", "topic dest")   # #route{topic, dest}
NODE = "emqx@127.0.0.1"

_engine = None
_routes = {}   # topic -> [dest, ...] in insertion order (bag)
_agg_ids = {}  # aggregated destination (emqx_broker:aggre/1) -> u32 id of the device route table
_agg_of = []   # id -> aggregated destination


def aggregate(dest):
    """The aggre/1 destination of a route dest (src/emqx_broker.erl:250-261):
    a node stays the node, a shared-subscription dest {Group, Node} becomes Group."""
    return ("group", dest[0]) if isinstance(dest, tuple) else ("node", dest)


def _agg_id(dest) -> int:
    a = aggregate(dest)
    i = _agg_ids.get(a)
    if i is None:
        i = _agg_ids[a] = len(_agg_of)
        _agg_of.append(a)
    return i


def use(engine: Engine):
    global _engine
    _engine = engine


def engine() -> Engine:
    global _engine
    if _engine is None:
        _engine = Engine(device=0 if N.gpu_available() else -1)
    return _engine


def clear_tables():
    global _engine, _routes, _agg_ids, _agg_of
    dev = _engine.device if _engine is not None else (0 if N.gpu_available() else -1)
    if _engine is not None:
        _engine.close()
    _engine = Engine(device=dev)
    _routes = {}
    _agg_ids, _agg_of = {}, []


def add_route(topic: bytes, dest=NODE):
    """add_route/1,2 (:100-106); the gen_server hop is a direct call here."""
    return do_add_route(topic, dest)


def do_add_route(topic: bytes, dest=NODE):
    """do_add_route/1,2 (:108-124)"""
    if not isinstance(topic, (bytes, bytearray)):
        raise TypeError("function_clause")
    topic = bytes(topic)
    dests = _routes.setdefault(topic, [])
    if dest in dests:                      # lists:member(Route, lookup_routes(Topic)) (:116)
        return "ok"
    engine().route_add(topic, _agg_id(dest))   # first route of the topic inserts it into the trie
    dests.append(dest)
    return "ok"


def delete_route(topic: bytes, dest=NODE):
    return do_delete_route(topic, dest)


def do_delete_route(topic: bytes, dest=NODE):
    """do_delete_route/1,2 (:159-169) incl. delete_trie_route/1 (:239-247)"""
    topic = bytes(topic)
    dests = _routes.get(topic)
    if not dests or dest not in dests:
        return "ok"
    dests.remove(dest)
    if not dests:
        del _routes[topic]
    engine().route_delete(topic, _agg_id(dest))   # the last route deletes the trie entry
    return "ok"


def lookup_routes(topic: bytes):
    """lookup_routes/1 (:143-145)"""
    return [Route(topic, d) for d in _routes.get(bytes(topic), [])]


def has_routes(topic: bytes) -> bool:
    """has_routes/1 (:147-149)"""
    return bytes(topic) in _routes


def topics():
    """topics/0 (:171-173)"""
    return list(_routes.keys())


def match_routes(topic: bytes):
    """match_routes/1 (:127-133)"""
    if not isinstance(topic, (bytes, bytearray)):
        raise TypeError("function_clause")
    out = []
    for f in engine().match(bytes(topic)):
        out.extend(Route(f, d) for d in _routes.get(f, []))
    return out


def match_routes_batch(topic_list):
    """match_routes/1 over a batch of publishes in one device pipeline."""
    eng = engine()
    offs, ids = eng.match_batch(topic_list)
    cache = {}
    res = []
    for i in range(len(topic_list)):
        out = []
        for fid in ids[offs[i]:offs[i + 1]]:
            fid = int(fid)
            f = cache.get(fid)
            if f is None:
                f = cache[fid] = eng.filter_bytes(fid)
            out.extend(Route(f, d) for d in _routes.get(f, []))
        res.append(out)
    return res


def aggre_batch(topic_list):
    """emqx_broker:aggre(match_routes(T)) for a batch, resolved on the device:
    per topic the list of (To, Node) / (To, Group) pairs -- filters in Erlang
    binary order, each filter's destinations in first-added order, no pair
    twice (the reference's usort removes duplicate group pairs)."""
    eng = engine()
    offs, fids, dests = eng.match_routes_batch(topic_list)
    cache = {}
    out = []
    for i in range(len(topic_list)):
        row = []
        for k in range(int(offs[i]), int(offs[i + 1])):
            fid = int(fids[k])
            f = cache.get(fid)
            if f is None:
                f = cache[fid] = eng.filter_bytes(fid)
            row.append((f, _agg_of[int(dests[k])][1]))
        out.append(row)
    return out


def print_routes(topic: bytes):
    """print_routes/1 (:176-181)"""
    for r in match_routes(topic):
        print(f"{r.topic.decode(errors='replace')} -> {r.dest}")


def is_wildcard_route(topic: bytes) -> bool:
    """The reference stores only these in the trie (:120); kept for callers."""
    return wildcard(topic)
