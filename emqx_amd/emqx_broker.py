"""emqx_broker mirror (src/emqx_broker.erl): the local subscriber bag and
publish -> dispatch, resolved on the device.

subscribe/unsubscribe/subscriber_down keep the ?SUBSCRIBER / ?SUBSCRIPTION
bags inside the engine (tm_subscribe / tm_unsubscribe / tm_subscriber_down);
the first subscriber of a topic adds its node() route and the last one removes
it, as the broker pool does through emqx_router (:438-469).  publish_batch runs
the whole publish path of a batch on the device: match (emqx_router:
match_routes/1) then fan-out (dispatch/2 for every local route,
tm_batch_dispatch).  Shared subscriptions (emqx_shared_sub) are not mirrored.

Subscriber pids are arbitrary hashable terms here, mapped to u32 ids.
"""

from __future__ import annotations

from . import emqx_router as R

_ids = {}      # subscriber term -> u32 id
_terms = []    # id -> term


def _sid(pid) -> int:
    i = _ids.get(pid)
    if i is None:
        i = _ids[pid] = len(_terms)
        _terms.append(pid)
    return i


def _node_dest() -> int:
    return R._agg_id(R.NODE)


def clear_tables():
    global _ids, _terms, _topics_of, _nsubs
    R.clear_tables()
    _ids, _terms = {}, []
    _topics_of, _nsubs = {}, {}
    _order.clear()


_topics_of = {}   # subscriber id -> [topic]: which node() routes subscriptions hold
_nsubs = {}       # topic -> local subscriber count
_order = {}       # topic -> [subscriber term], subscription order


def subscribe(topic: bytes, pid="self"):
    """subscribe/1,2 -> do_subscribe/4, non-shared clause (:117-158)."""
    if not isinstance(topic, (bytes, bytearray)):
        raise TypeError("function_clause")
    topic, sid = bytes(topic), _sid(pid)
    R.engine().subscribe(topic, sid, _node_dest())
    ts = _topics_of.setdefault(sid, [])
    if topic not in ts:
        ts.append(topic)
        _nsubs[topic] = _nsubs.get(topic, 0) + 1
        _order.setdefault(topic, []).append(pid)
        dests = R._routes.setdefault(topic, [])
        if R.NODE not in dests:
            dests.append(R.NODE)
    return "ok"


def _dropped(topic: bytes, sid: int):
    _topics_of[sid].remove(topic)
    _nsubs[topic] -= 1
    _order[topic].remove(_terms[sid])
    if not _nsubs[topic]:
        del _nsubs[topic]
        del _order[topic]
        dests = R._routes.get(topic, [])
        if R.NODE in dests:
            dests.remove(R.NODE)
        if not dests:
            R._routes.pop(topic, None)


def unsubscribe(topic: bytes, pid="self"):
    """unsubscribe/1 -> do_unsubscribe/4 (:168-191); `ok` whether subscribed or not."""
    topic, sid = bytes(topic), _sid(pid)
    if R.engine().unsubscribe(topic, sid, _node_dest()):
        _dropped(topic, sid)
    return "ok"


def subscriber_down(pid) -> int:
    """subscriber_down/1 (:332-347): drops every subscription of pid."""
    sid = _sid(pid)
    n = R.engine().subscriber_down(sid, _node_dest())
    for t in list(_topics_of.get(sid, [])):
        _dropped(t, sid)
    return n


def subscribers(topic: bytes):
    """subscribers/1 (:320-325): the topic's local subscribers in subscription
    order (host view of the bag the engine holds)."""
    return list(_order.get(bytes(topic), []))


def topics():
    """topics/0 (:402-404) = emqx_router:topics/0."""
    return R.topics()


def publish_batch(topic_list):
    """publish/1 -> route/2 -> dispatch/2 for a batch: per publish the list of
    deliveries (To, SubPid); To in Erlang binary order, each To's subscribers
    in subscription order.  [] is {error, no_subscribers}."""
    eng = R.engine()
    b = eng.prepare(topic_list)
    b.launch()
    b.wait()
    roff, ids = b.result()
    offs, moff, subs = b.dispatch(match_offsets=True)
    b.free()
    cache = {}
    out = []
    for i in range(len(topic_list)):
        row = []
        for j in range(int(roff[i]), int(roff[i + 1])):
            if moff[j] == moff[j + 1]:
                continue
            fid = int(ids[j])
            f = cache.get(fid)
            if f is None:
                f = cache[fid] = eng.filter_bytes(fid)
            row.extend((f, _terms[int(s)]) for s in subs[moff[j]:moff[j + 1]])
        assert len(row) == offs[i + 1] - offs[i]
        out.append(row)
    return out
