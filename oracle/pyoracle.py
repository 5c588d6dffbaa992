"""ctypes binding of oracle/build/libtm_oracle.so -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libtm_oracle.so")


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in
                ("topics", "visits", "hash_hits", "ets_probes", "words", "matches", "routes")]

    def asdict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P, U64, SZ = C.c_void_p, C.c_uint64, C.c_size_t
        L.tmo_create.restype = P
        L.tmo_destroy.argtypes = [P]
        L.tmo_insert.argtypes = [P, C.c_char_p, SZ]
        L.tmo_delete.argtypes = [P, C.c_char_p, SZ]
        L.tmo_register.argtypes = [P, C.c_char_p, SZ]
        L.tmo_register.restype = C.c_int64
        L.tmo_lookup.argtypes = [P, C.c_char_p, SZ, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_int64)]
        L.tmo_empty.argtypes = [P]
        L.tmo_topic_match.argtypes = [C.c_char_p, SZ, C.c_char_p, SZ]
        L.tmo_wildcard.argtypes = [C.c_char_p, SZ]
        L.tmo_match.argtypes = [P, C.c_char_p, SZ, C.POINTER(C.c_int64), SZ, C.POINTER(Stats)]
        L.tmo_match.restype = SZ
        L.tmo_match_batch.argtypes = [P, P, P, U64, C.c_int, C.c_int]
        L.tmo_match_batch.restype = P
        L.tmo_match_routes_batch.argtypes = [P, P, P, U64, C.c_int]
        L.tmo_match_routes_batch.restype = P
        L.tmo_brute_batch.argtypes = [P, P, U64, P, P, U64, C.c_int]
        L.tmo_brute_batch.restype = P
        L.tmo_batch_get.argtypes = [P, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.POINTER(C.c_int64)),
                                    C.POINTER(U64), C.POINTER(Stats)]
        L.tmo_batch_free.argtypes = [P]
        L.tmo_filter_bytes.argtypes = [P, C.c_int64, C.POINTER(C.c_uint32)]
        L.tmo_filter_bytes.restype = C.POINTER(C.c_uint8)
        L.tmo_route_add.argtypes = [P, C.c_char_p, SZ]
        L.tmo_add_route.argtypes = [P, C.c_char_p, SZ]
        L.tmo_edge_count_total.argtypes = [P]
        L.tmo_edge_count_total.restype = U64
        _lib = L
    return _lib


def pack(strings):
    """list[bytes] -> (uint8 buffer, uint64 offsets[n+1])"""
    offs = np.zeros(len(strings) + 1, dtype=np.uint64)
    if strings:
        offs[1:] = np.cumsum([len(s) for s in strings], dtype=np.uint64)
    buf = np.frombuffer(b"".join(strings), dtype=np.uint8) if strings else np.zeros(1, np.uint8)
    if buf.size == 0:
        buf = np.zeros(1, np.uint8)
    return np.ascontiguousarray(buf), offs


def _take_batch(b):
    L = lib()
    cnt = C.POINTER(C.c_uint32)()
    idx = C.POINTER(C.c_int64)()
    tot = C.c_uint64()
    st = Stats()
    L.tmo_batch_get(b, C.byref(cnt), C.byref(idx), C.byref(tot), C.byref(st))
    return cnt, idx, tot.value, st


class Oracle:
    """Faithful ETS-layout restatement (prefix-string node ids)."""

    def __init__(self):
        self.L = lib()
        self.h = self.L.tmo_create()

    def close(self):
        if self.h:
            self.L.tmo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def insert(self, f: bytes):
        return self.L.tmo_insert(self.h, f, len(f))

    def delete(self, f: bytes):
        return self.L.tmo_delete(self.h, f, len(f))

    def register(self, f: bytes) -> int:
        return self.L.tmo_register(self.h, f, len(f))

    def add_route(self, f: bytes):
        self.L.tmo_add_route(self.h, f, len(f))

    def empty(self) -> bool:
        return bool(self.L.tmo_empty(self.h))

    def lookup(self, node_id):
        ec = C.c_uint32()
        tp = C.c_int64()
        is_root = node_id is None
        nid = b"" if is_root else node_id
        if not self.L.tmo_lookup(self.h, nid, len(nid), int(is_root), C.byref(ec), C.byref(tp)):
            return []
        return [(node_id, ec.value, None if tp.value < 0 else self.filter_bytes(tp.value))]

    def filter_bytes(self, idx: int) -> bytes:
        n = C.c_uint32()
        p = self.L.tmo_filter_bytes(self.h, idx, C.byref(n))
        return C.string_at(p, n.value)

    def match(self, topic: bytes, with_stats=False):
        """DFS-order list like emqx_trie:match/1."""
        cap = 1 << 16
        out = (C.c_int64 * cap)()
        st = Stats()
        n = self.L.tmo_match(self.h, topic, len(topic), out, cap, C.byref(st))
        assert n <= cap
        res = [self.filter_bytes(out[i]) for i in range(n)]
        return (res, st.asdict()) if with_stats else res

    def match_batch(self, topics_buf, topics_offs, nthreads=1, sorted_=True):
        """Returns (counts[n] uint32, idx[total] int64 registry indices, stats)."""
        n = len(topics_offs) - 1
        b = self.L.tmo_match_batch(self.h, topics_buf.ctypes.data, topics_offs.ctypes.data, n,
                                   nthreads, int(sorted_))
        try:
            cnt, idx, tot, st = _take_batch(b)
            counts = np.ctypeslib.as_array(cnt, shape=(max(n, 1),))[:n].copy()
            ids = np.ctypeslib.as_array(idx, shape=(max(tot, 1),))[:tot].copy()
        finally:
            self.L.tmo_batch_free(b)
        return counts, ids, st.asdict()

    def match_routes_batch(self, topics_buf, topics_offs, nthreads=1):
        n = len(topics_offs) - 1
        b = self.L.tmo_match_routes_batch(self.h, topics_buf.ctypes.data, topics_offs.ctypes.data,
                                          n, nthreads)
        try:
            _, _, _, st = _take_batch(b)
        finally:
            self.L.tmo_batch_free(b)
        return st.asdict()


def topic_match(name: bytes, flt: bytes) -> bool:
    return bool(lib().tmo_topic_match(name, len(name), flt, len(flt)))


def brute_batch(filters, topics_buf, topics_offs, nthreads=1):
    fbuf, foffs = pack(filters)
    n = len(topics_offs) - 1
    L = lib()
    b = L.tmo_brute_batch(fbuf.ctypes.data, foffs.ctypes.data, len(filters),
                          topics_buf.ctypes.data, topics_offs.ctypes.data, n, nthreads)
    try:
        cnt, idx, tot, st = _take_batch(b)
        counts = np.ctypeslib.as_array(cnt, shape=(max(n, 1),))[:n].copy()
        ids = np.ctypeslib.as_array(idx, shape=(max(tot, 1),))[:tot].copy()
    finally:
        L.tmo_batch_free(b)
    return counts, ids
