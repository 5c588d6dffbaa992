"""emqx_router_helper mirror + the cluster route delta feed.

In the reference the emqx_route bag and the trie tables are mnesia ram_copies on
every node (src/emqx_router.erl:77-86, src/emqx_trie.erl:53-74): a route added
on any node replicates into every node's tables, and a node that goes down has
its routes removed by the survivors (emqx_router_helper: `{nodedown, Node}` ->
cleanup_routes/1, src/emqx_router_helper.erl:135-141, 173-177).

Here every node's engine is fed the same stream of route-table events.
`RouteFeed` takes them as mnesia table events -- `("write", Route)` and
`("delete_object", Route)`, the form `mnesia:subscribe({table, emqx_route,
simple})` delivers -- keeps the host route bag of `emqx_router` in step (an
identical record is stored once, an absent one is not deleted), and applies the
resulting changes to the device in one `tm_route_apply` call per flush, so a
burst of remote subscribes costs one engine lock and one delta upload instead of
one per route.
"""

from __future__ import annotations

from . import _native as N
from . import emqx_router as R
from .emqx_router import Route

WRITE, DELETE_OBJECT = "write", "delete_object"


class RouteFeed:
    """Batched consumer of emqx_route table events.

    `push(event)` queues one event; `flush()` applies the queued events in
    arrival order and returns how many changed the route bag.  `max_pending`
    bounds the queue (a full queue flushes itself), like emqx_batch's size
    threshold (src/emqx_batch.erl:60-73)."""

    def __init__(self, max_pending: int = 65536):
        self.max_pending = max_pending
        self._q = []
        self.applied = 0

    def push(self, event):
        kind, route = event
        if kind not in (WRITE, DELETE_OBJECT):
            raise ValueError(f"unexpected mnesia_table_event {kind!r}")
        if not isinstance(route.topic, (bytes, bytearray)):
            raise TypeError("function_clause")
        self._q.append((kind, bytes(route.topic), route.dest))
        if len(self._q) >= self.max_pending:
            self.flush()

    def extend(self, events):
        for ev in events:
            self.push(ev)
        return self

    def flush(self) -> int:
        q, self._q = self._q, []
        if not q:
            return 0
        ops = []
        for kind, topic, dest in q:
            dests = R._routes.get(topic)
            if kind == WRITE:
                if dests is not None and dest in dests:   # bag: identical record stored once
                    continue
                R._routes.setdefault(topic, []).append(dest)
                ops.append((N.TM_ROUTE_WRITE, topic, R._agg_id(dest)))
            else:
                if not dests or dest not in dests:        # delete_object of no record
                    continue
                dests.remove(dest)
                if not dests:
                    del R._routes[topic]
                ops.append((N.TM_ROUTE_DELETE, topic, R._agg_id(dest)))
        if ops:
            done = R.engine().route_apply(ops)
            if done != len(ops):
                raise N.TmError(N.TM_EIO, f"tm_route_apply applied {done} of {len(ops)}")
        self.applied += len(ops)
        return len(ops)


def cleanup_routes(node) -> int:
    """cleanup_routes/1 (src/emqx_router_helper.erl:173-177): deletes every route
    whose dest is `node` or `{_, node}`, in one device delta.  Returns how many."""
    feed = RouteFeed()
    for topic, dests in list(R._routes.items()):
        for d in list(dests):
            if d == node or (isinstance(d, tuple) and d[1] == node):
                feed.push((DELETE_OBJECT, Route(topic, d)))
    return feed.flush()


def nodedown(node) -> int:
    """handle_info({nodedown, Node}, _) (:135-141): the dead node's routes go."""
    return cleanup_routes(node)
