"""Pythonic wrapper of one tm_engine (one trie replica on one MI355X).

    eng = Engine(device=0)
    eng.insert(b"sensor/+/#")
    eng.match(b"sensor/1/temp")                  # -> [b"sensor/+/#"]
    offs, ids = eng.match_batch(topics)          # CSR over a whole batch
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N
from .gen import Strings


def _pack(topics) -> Strings:
    if isinstance(topics, Strings):
        return topics
    return Strings.from_list(list(topics))


class Batch:
    """A device-resident publish batch (tm_batch_prepare / launch / wait / result)."""

    def __init__(self, eng: "Engine", topics):
        self.eng = eng
        s = _pack(topics)
        self.n = len(s)
        buf = s.buf if s.buf.size else np.zeros(1, np.uint8)
        self._buf = np.ascontiguousarray(buf)
        self._offs = np.ascontiguousarray(s.offs.astype(np.uint64))
        h = C.c_void_p()
        N.check(eng.L.tm_batch_prepare(eng.h, self._buf.ctypes.data, self._offs.ctypes.data, self.n,
                                       C.byref(h)), "tm_batch_prepare")
        self.h = h

    def launch(self):
        N.check(self.eng.L.tm_batch_launch(self.eng.h, self.h), "tm_batch_launch")
        return self

    def wait(self):
        N.check(self.eng.L.tm_batch_wait(self.eng.h, self.h), "tm_batch_wait")
        return self

    def result(self):
        r = N.Result()
        N.check(self.eng.L.tm_batch_result(self.eng.h, self.h, C.byref(r)), "tm_batch_result")
        return _result_arrays(r)

    def stats(self) -> dict:
        st = N.BatchStats()
        N.check(self.eng.L.tm_batch_stats_get(self.eng.h, self.h, C.byref(st)), "tm_batch_stats_get")
        return st.asdict()

    def device_csr(self):
        row, ids, n = C.c_void_p(), C.c_void_p(), C.c_uint64()
        N.check(self.eng.L.tm_batch_device_csr(self.eng.h, self.h, C.byref(row), C.byref(ids), C.byref(n)),
                "tm_batch_device_csr")
        return row.value, ids.value, n.value

    def free(self):
        if self.h:
            self.eng.L.tm_batch_free(self.eng.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _result_arrays(r: N.Result):
    n = r.n_topics
    offs = np.ctypeslib.as_array(r.row_offsets, shape=(n + 1,)).copy()
    m = int(r.n_matches)
    ids = np.ctypeslib.as_array(r.filter_ids, shape=(max(m, 1),))[:m].copy() if m else np.zeros(0, np.uint32)
    return offs, ids


class Engine:
    def __init__(self, device: int = 0, init_slots: int = 0, host_threads: int = 0):
        self.L = N.lib()
        cfg = N.Config(device, init_slots, host_threads, 0)
        h = C.c_void_p()
        N.check(self.L.tm_create(C.byref(cfg), C.byref(h)), "tm_create")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            self.L.tm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- emqx_trie ---------------------------------------------------------
    def insert(self, f: bytes):
        N.check(self.L.tm_trie_insert(self.h, f, len(f)), "tm_trie_insert")

    def delete(self, f: bytes):
        N.check(self.L.tm_trie_delete(self.h, f, len(f)), "tm_trie_delete")

    def lookup(self, node_id):
        """-> None or (edge_count, topic_bytes_or_None)"""
        out = N.TrieNode()
        is_root = node_id is None
        nid = b"" if is_root else node_id
        rc = N.check(self.L.tm_trie_lookup(self.h, nid, len(nid), int(is_root), C.byref(out)), "tm_trie_lookup")
        if rc == 0:
            return None
        return out.edge_count, (self.filter_bytes(out.filter_id) if out.has_topic else None)

    def empty(self) -> bool:
        return bool(self.L.tm_trie_empty(self.h))

    def match_ids(self, topic: bytes):
        cap = 1024
        while True:
            ids = (C.c_uint32 * cap)()
            n = C.c_uint32()
            N.check(self.L.tm_trie_match(self.h, topic, len(topic), ids, cap, C.byref(n)), "tm_trie_match")
            if n.value <= cap:
                return list(ids[:n.value])
            cap = n.value

    def match(self, topic: bytes):
        return [self.filter_bytes(i) for i in self.match_ids(topic)]

    # ---- batches -----------------------------------------------------------
    def match_batch(self, topics):
        """-> (row_offsets uint32[n+1], filter_ids uint32[total]); rows sorted by filter bytes."""
        s = _pack(topics)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs.astype(np.uint64))
        r = N.Result()
        N.check(self.L.tm_match_batch(self.h, buf.ctypes.data, offs.ctypes.data, len(s), C.byref(r)),
                "tm_match_batch")
        return _result_arrays(r)

    def prepare(self, topics) -> Batch:
        return Batch(self, topics)

    # ---- filters -----------------------------------------------------------
    def filter_bytes(self, fid: int) -> bytes:
        n = C.c_size_t()
        p = self.L.tm_filter_bytes(self.h, fid, C.byref(n))
        if not p:
            raise KeyError(fid)
        return C.string_at(p, n.value)

    def filter_id(self, f: bytes) -> int:
        out = C.c_uint32()
        rc = self.L.tm_filter_id(self.h, f, len(f), C.byref(out))
        if rc == N.TM_ENOENT:
            raise KeyError(f)
        N.check(rc, "tm_filter_id")
        return out.value

    # ---- engine ------------------------------------------------------------
    @property
    def version(self) -> int:
        return int(self.L.tm_version(self.h))

    def stats(self) -> dict:
        st = N.EngineStats()
        N.check(self.L.tm_stats(self.h, C.byref(st)), "tm_stats")
        return st.asdict()

    def sync(self):
        N.check(self.L.tm_sync(self.h), "tm_sync")
