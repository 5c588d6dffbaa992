"""emqx_trie mirror (src/emqx_trie.erl) over one device trie replica.

The reference keeps the trie in two mnesia ram tables; here the "tables" are a
tm_engine (host mirror + HBM replica).  `use(engine)` selects the engine the
module-level API acts on (default: a lazily created engine on device 0, or a
host-only engine when no GPU is visible -- then `match/1` raises, there is no
CPU fallback).
"""

from __future__ import annotations

from collections import namedtuple

from . import _native as N
from .emqx_topic import EMPTY, HASH, PLUS, join, words  # noqa: F401
from .engine import Engine

# #trie_node{} record (include/emqx.hrl:98-103)
TrieNode = namedtuple("TrieNode", "node_id edge_count topic flags")
ROOT = "root"

_engine = None


def use(engine: Engine):
    global _engine
    _engine = engine


def engine() -> Engine:
    global _engine
    if _engine is None:
        _engine = Engine(device=0 if N.gpu_available() else -1)
    return _engine


def clear_tables():
    """mnesia:clear_table/1 of both trie tables (test/emqx_trie_SUITE.erl:150-151)."""
    global _engine
    dev = _engine.device if _engine is not None else (0 if N.gpu_available() else -1)
    if _engine is not None:
        _engine.close()
    _engine = Engine(device=dev)


def insert(topic: bytes):
    """emqx_trie:insert/1 (:81-93)"""
    if not isinstance(topic, (bytes, bytearray)):
        raise TypeError("function_clause")
    engine().insert(bytes(topic))
    return "ok"


def delete(topic: bytes):
    """emqx_trie:delete/1 (:107-116)"""
    if not isinstance(topic, (bytes, bytearray)):
        raise TypeError("function_clause")
    try:
        engine().delete(bytes(topic))
    except N.TmError as e:
        if e.rc == N.TM_EABORT:
            raise RuntimeError(("aborted", ("node_not_found", topic))) from e
        raise
    return "ok"


def match(topic: bytes):
    """emqx_trie:match/1 (:96-99): filters matching `topic`, sorted, deduplicated
    (the reference returns the same set in its DFS order)."""
    if not isinstance(topic, (bytes, bytearray)):
        raise TypeError("function_clause")
    return engine().match(bytes(topic))


def lookup(node_id):
    """emqx_trie:lookup/1 (:102-104) -> [] | [TrieNode]"""
    r = engine().lookup(None if node_id == ROOT else node_id)
    if r is None:
        return []
    ec, topic = r
    return [TrieNode(node_id, ec, topic, None)]


def empty() -> bool:
    """emqx_trie:empty/0 (:119-121)"""
    return engine().empty()


def triples(topic: bytes):
    """emqx_trie:triples/1 (:128-136)"""
    out, parent = [], ROOT
    for w in words(topic):
        node = join([w]) if parent == ROOT else join([parent, w])
        out.append((parent, w, node))
        parent = node
    return out
