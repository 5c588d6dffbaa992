"""Pure-Python restatement of the reference hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module (or oracle/build/libtm_oracle.so through oracle/pyoracle.py).  The
product package `emqx_amd` never imports it.

Restates, clause by clause (reference = /root/reference, EMQ X 4.2.x):
  emqx_topic:words/1, word/1, tokens/1   src/emqx_topic.erl:150-164
  emqx_topic:match/2                     src/emqx_topic.erl:65-87
  emqx_topic:wildcard/1                  src/emqx_topic.erl:52-62
  emqx_topic:join/1                      src/emqx_topic.erl:183-195
  emqx_trie:insert/1, add_path/1         src/emqx_trie.erl:81-93, 145-158
  emqx_trie:match/1, match_node, 'match_#'  src/emqx_trie.erl:96-99, 162-186
  emqx_trie:delete/1, delete_path/1      src/emqx_trie.erl:107-116, 190-204
  emqx_trie:lookup/1, empty/0, triples/1 src/emqx_trie.erl:102-104, 119-136

Tables mirror the reference's ETS layout: node ids are prefix binaries
(`ROOT` for the atom root), edges are a dict keyed by (node_id, word).
Words are `bytes` for binaries and the singletons EMPTY / PLUS / HASH for the
atoms '' / '+' / '#'.
"""

from __future__ import annotations


class _Atom:
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return self.name


EMPTY = _Atom("''")
PLUS = _Atom("'+'")
HASH = _Atom("'#'")
ROOT = _Atom("root")


# ---------------------------------------------------------------- emqx_topic

def tokens(topic: bytes):
    """binary:split(Topic, <<"/">>, [global]) -- src/emqx_topic.erl:153-154"""
    return topic.split(b"/")


def word(w: bytes):
    """src/emqx_topic.erl:161-164"""
    if w == b"":
        return EMPTY
    if w == b"+":
        return PLUS
    if w == b"#":
        return HASH
    return w


def words(topic: bytes):
    """src/emqx_topic.erl:158-159"""
    return [word(w) for w in tokens(topic)]


def bin_(w) -> bytes:
    """src/emqx_topic.erl:140-144"""
    if w is EMPTY:
        return b""
    if w is PLUS:
        return b"+"
    if w is HASH:
        return b"#"
    return w


def join(ws) -> bytes:
    """src/emqx_topic.erl:183-195"""
    return b"/".join(bin_(w) for w in ws)


def wildcard(topic) -> bool:
    """src/emqx_topic.erl:52-62"""
    ws = words(topic) if isinstance(topic, (bytes, bytearray)) else topic
    return any(w is PLUS or w is HASH for w in ws)


def _match_words(n, f) -> bool:
    i = j = 0
    while True:
        if i == len(n) and j == len(f):
            return True                                   # match([], [])
        if i < len(n) and j < len(f) and (n[i] is f[j] or (isinstance(n[i], bytes) and n[i] == f[j])):
            i += 1; j += 1; continue                      # match([H|T1], [H|T2])
        if i < len(n) and j < len(f) and f[j] is PLUS:
            i += 1; j += 1; continue                      # match([_H|T1], ['+'|T2])
        if j + 1 == len(f) and f[j] is HASH:
            return True                                   # match(_, ['#'])
        return False


def match(name, flt) -> bool:
    """emqx_topic:match/2 -- src/emqx_topic.erl:65-87"""
    if isinstance(name, (bytes, bytearray)) and isinstance(flt, (bytes, bytearray)):
        if name[:1] == b"$" and flt[:1] in (b"+", b"#"):
            return False
        return _match_words(words(name), words(flt))
    return _match_words(name, flt)


# ----------------------------------------------------------------- emqx_trie

class Trie:
    """The two mnesia ram tables emqx_trie (edges) and emqx_trie_node."""

    def __init__(self):
        self.edges = {}   # (node_id, word) -> child node_id     (#trie{})
        self.nodes = {}   # node_id -> [edge_count, topic|None]  (#trie_node{})

    # triples/1 -- src/emqx_trie.erl:128-141
    @staticmethod
    def triples(topic: bytes):
        out, parent = [], ROOT
        for w in words(topic):
            node = bin_(w) if parent is ROOT else join([parent, w])
            out.append((parent, w, node))
            parent = node
        return out

    def insert(self, topic: bytes):
        """src/emqx_trie.erl:81-93"""
        tn = self.nodes.get(topic)
        if tn is not None:
            if tn[1] is None:
                tn[1] = topic
            return "ok"
        for (node, w, child) in self.triples(topic):       # add_path/1 :145-158
            pn = self.nodes.get(node)
            if pn is not None:
                if (node, w) not in self.edges:
                    pn[0] += 1
                    self.edges[(node, w)] = child
            else:
                self.nodes[node] = [1, None]
                self.edges[(node, w)] = child
        self.nodes[topic] = [0, topic]
        return "ok"

    def delete(self, topic: bytes):
        """src/emqx_trie.erl:107-116, delete_path/1 :190-204"""
        tn = self.nodes.get(topic)
        if tn is None:
            return "ok"
        if tn[0] != 0:
            tn[1] = None
            return "ok"
        del self.nodes[topic]
        for (node, w, _child) in reversed(self.triples(topic)):
            self.edges.pop((node, w), None)
            pn = self.nodes.get(node)
            if pn is None:
                raise RuntimeError(("node_not_found", node))
            if pn[0] == 1 and pn[1] is None:
                del self.nodes[node]
                continue
            if pn[0] == 1:
                pn[0] = 0
                break
            pn[0] -= 1
            break
        return "ok"

    def lookup(self, node_id):
        """src/emqx_trie.erl:102-104 -> [(node_id, edge_count, topic)]"""
        tn = self.nodes.get(node_id)
        return [] if tn is None else [(node_id, tn[0], tn[1])]

    def empty(self) -> bool:
        """src/emqx_trie.erl:119-121"""
        return len(self.edges) == 0

    def match(self, topic: bytes, stats=None):
        """emqx_trie:match/1 -- DFS order of the reference (src/emqx_trie.erl:96-99)."""
        ws = words(topic)
        if ws and isinstance(ws[0], bytes) and ws[0][:1] == b"$":
            res = self._match_node(ws[0], ws[1:], [], stats)     # :162-163
        else:
            res = self._match_node(ROOT, ws, [], stats)
        return [t for (_nid, _ec, t) in res if t is not None]

    def _read_node(self, nid):
        tn = self.nodes.get(nid)
        return [] if tn is None else [(nid, tn[0], tn[1])]

    def _match_hash(self, nid, acc, stats):
        """'match_#'/2 -- src/emqx_trie.erl:181-186"""
        child = self.edges.get((nid, HASH))
        if child is not None:
            if stats is not None:
                stats["H"] += 1
            return self._read_node(child) + acc
        return acc

    def _match_node(self, nid, ws, acc, stats):
        """match_node/3 -- src/emqx_trie.erl:168-177"""
        if stats is not None:
            stats["V"] += 1
        if not ws:
            return self._read_node(nid) + self._match_hash(nid, acc, stats)
        acc = self._match_hash(nid, acc, stats)
        for warg in (ws[0], PLUS):
            child = self.edges.get((nid, warg))
            if child is not None:
                acc = self._match_node(child, ws[1:], acc, stats)
        return acc


def erl_sorted(bins):
    """Erlang term order on binaries == Python bytes order (unsigned, prefix first)."""
    return sorted(bins)


def brute(topic: bytes, filters):
    """{f in F | emqx_topic:match(topic, f)}, sorted."""
    return sorted(f for f in filters if match(topic, f))


def match_routes(trie: Trie, routes: dict, topic: bytes):
    """emqx_router:match_routes/1 -- src/emqx_router.erl:127-145.

    `routes` maps a topic/filter binary to its list of dests (the emqx_route bag).
    """
    matched = [] if trie.empty() else trie.match(topic)
    if not matched:
        return [(topic, d) for d in routes.get(topic, [])]
    out = []
    for to in [topic] + matched:
        out.extend((to, d) for d in routes.get(to, []))
    return out


class Broker:
    """emqx_broker's local subscriber bag and dispatch, non-shared subscriptions.

    subscribe    do_subscribe/4 non-shared clause   src/emqx_broker.erl:145-158
                 (first subscriber -> do_add_route  :438-440, emqx_router:108-124)
    unsubscribe  do_unsubscribe/4                   :179-191
                 (last subscriber -> do_delete_route :463-469)
    subscriber_down/1                               :332-347
    publish      route/2 -> do_route/2 -> dispatch/2 (local node) :233-309
                 over emqx_router:match_routes/1

    publish() returns the deliveries [(To, SubPid)] of one message: its matched
    filters in Erlang binary order (the reference folds the route list in
    DFS/ETS order -- a set, its order is not part of the contract), each
    filter's subscribers in subscription order (ETS bag insertion order).
    len() == 0 is the reference's {error, no_subscribers}.
    """

    NODE = "node@local"

    def __init__(self):
        self.trie = Trie()
        self.routes = {}        # emqx_route bag: topic -> [dest]
        self.subscriber = {}    # ?SUBSCRIBER bag: topic -> [pid]
        self.subscription = {}  # ?SUBSCRIPTION bag: pid -> [topic]

    def _add_route(self, topic):
        dests = self.routes.setdefault(topic, [])
        if self.NODE in dests:
            return
        if not dests and wildcard(topic):
            self.trie.insert(topic)           # insert_trie_route/1 (src/emqx_router.erl:229-234)
        dests.append(self.NODE)

    def _delete_route(self, topic):
        dests = self.routes.get(topic, [])
        if self.NODE not in dests:
            return
        dests.remove(self.NODE)
        if not dests:
            del self.routes[topic]
            if wildcard(topic):
                self.trie.delete(topic)       # delete_trie_route/1 (:239-247)

    def subscribe(self, topic: bytes, pid):
        ts = self.subscription.setdefault(pid, [])
        if topic in ts:
            return
        ts.append(topic)
        subs = self.subscriber.setdefault(topic, [])
        first = not subs
        subs.append(pid)
        if first:
            self._add_route(topic)

    def unsubscribe(self, topic: bytes, pid) -> bool:
        ts = self.subscription.get(pid, [])
        if topic not in ts:
            return False                      # `[] -> ok` (:170-177)
        ts.remove(topic)
        if not ts:
            del self.subscription[pid]
        subs = self.subscriber[topic]
        subs.remove(pid)
        if not subs:
            del self.subscriber[topic]
            self._delete_route(topic)
        return True

    def subscriber_down(self, pid) -> int:
        ts = list(self.subscription.get(pid, []))
        for t in ts:
            self.unsubscribe(t, pid)
        return len(ts)

    def subscribers(self, topic: bytes):
        return list(self.subscriber.get(topic, []))

    def publish(self, topic: bytes):
        tos = sorted({to for to, d in match_routes(self.trie, self.routes, topic) if d == self.NODE})
        return [(to, pid) for to in tos for pid in self.subscriber.get(to, [])]


class RouteTable:
    """The replicated emqx_route bag as a node sees it through the cluster delta
    feed -- test infrastructure only.

    write         mnesia:write of #route{} into a bag: an identical record is
                  stored once (do_add_route/2's lists:member check,
                  src/emqx_router.erl:113-124); the first route of a wildcard
                  topic inserts it into the trie (insert_trie_route/1 :229-234)
    delete_object removes the record if present (do_delete_route/2 :163-169);
                  the last route of a wildcard topic deletes it from the trie
                  (delete_trie_route/1 :239-247)
    cleanup_routes(Node)  src/emqx_router_helper.erl:173-177: every route whose
                  dest is Node or {_, Node}
    aggre(topic)  emqx_broker:aggre(match_routes(T)) (src/emqx_broker.erl:250-261)
                  as a set of (To, Node | Group) pairs
    """

    def __init__(self):
        self.trie = Trie()
        self.routes = {}   # topic -> [dest] (bag, insertion order)

    def write(self, topic: bytes, dest):
        ds = self.routes.setdefault(topic, [])
        if dest in ds:
            return False
        if not ds and wildcard(topic):
            self.trie.insert(topic)
        ds.append(dest)
        return True

    def delete_object(self, topic: bytes, dest):
        ds = self.routes.get(topic)
        if not ds or dest not in ds:
            return False
        ds.remove(dest)
        if not ds:
            del self.routes[topic]
            if wildcard(topic):
                self.trie.delete(topic)
        return True

    def cleanup_routes(self, node):
        gone = [(t, d) for t, ds in self.routes.items() for d in ds
                if d == node or (isinstance(d, tuple) and d[1] == node)]
        for t, d in gone:
            self.delete_object(t, d)
        return gone

    def aggre(self, topic: bytes):
        out = set()
        for to, d in match_routes(self.trie, self.routes, topic):
            out.add((to, d[0] if isinstance(d, tuple) else d))
        return out
