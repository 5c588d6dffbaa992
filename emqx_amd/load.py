"""ctypes face of libemqx_load.so (emqx_amd/csrc/tm_load.cpp): the broker's
publishing processes played against the per-publish ABI (bench / tests only)."""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _native as N

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libemqx_load.so")

SYNC, ASYNC = 0, 1


class TmlResult(C.Structure):
    _fields_ = [("seconds", C.c_double), ("calls", C.c_uint64), ("errors", C.c_uint64), ("mean_us", C.c_double),
                ("p50_us", C.c_double), ("p99_us", C.c_double), ("max_us", C.c_double),
                ("max_at_s", C.c_double)]

    def asdict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


_lib = None


def lib():
    global _lib
    if _lib is None:
        N.lib()   # the engine library first (same file the load library links)
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built (python -m emqx_amd.build)")
        L = C.CDLL(LIB_PATH)
        L.tml_run.restype = C.c_int
        L.tml_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32,
                              C.c_void_p, C.c_void_p, C.POINTER(TmlResult)]
        L.tml_row_hashes.restype = None
        L.tml_row_hashes.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]
        _lib = L
    return _lib


def run(eng, topics, mode: int, threads: int, window: int = 1, hashes: bool = True):
    """Matches every topic once through tm_match_coalesced (SYNC) or
    tm_match_async (ASYNC, `window` calls in flight per thread).
    -> (stats dict, counts uint32[n], row hashes uint64[n] or None)"""
    from .engine import _pack
    s = _pack(topics)
    n = len(s)
    buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
    offs = np.ascontiguousarray(s.offs.astype(np.uint64))
    counts = np.zeros(max(n, 1), np.uint32)
    hs = np.zeros(max(n, 1), np.uint64) if hashes else None
    r = TmlResult()
    rc = lib().tml_run(eng.h, buf.ctypes.data, offs.ctypes.data, n, mode, threads, window, counts.ctypes.data,
                       hs.ctypes.data if hashes else None, C.byref(r))
    N.check(rc, "tml_run")
    return r.asdict(), counts[:n], (hs[:n] if hashes else None)


def row_hashes(offs, ids) -> np.ndarray:
    n = len(offs) - 1
    o = np.ascontiguousarray(offs.astype(np.uint32))
    i = np.ascontiguousarray(ids if len(ids) else np.zeros(1, np.uint32))
    out = np.zeros(max(n, 1), np.uint64)
    lib().tml_row_hashes(o.ctypes.data, i.ctypes.data, n, out.ctypes.data)
    return out[:n]
