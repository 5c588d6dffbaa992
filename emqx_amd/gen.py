"""Seeded synthetic workloads -- bench/test tooling.

`Params` mirrors `tm_gen_params` in csrc/tm_gen.c.  Two implementations exist:
the C one (`gen_filters` / `gen_topics`, used for the 1M-filter / 10M-topic
bench sets) and a pure-Python mirror (`py_gen_filters` / `py_gen_topics`, used
for small fixtures).  tests/test_gen.py checks they produce identical bytes.
"""

from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass, fields

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GEN_LIB = os.path.join(HERE, "libemqx_gen.so")


@dataclass
class Params:
    seed: int = 1
    n_filters: int = 10_000
    vocab: int = 64
    max_depth: int = 7
    zipf_s: float = 1.0
    p_plus: float = 0.2
    p_hash: float = 0.3
    p_final_plus: float = 0.1
    exact_frac: float = 0.1
    require_wildcard: int = 1
    p_dollar: float = 0.01
    p_empty: float = 0.01
    p_topic_dollar: float = 0.01
    p_topic_inst: float = 0.5
    p_unseen: float = 0.05


# Named configurations of BASELINE.json / SURVEY.md §8d.
C1 = Params(seed=1, n_filters=10_000, vocab=64, zipf_s=1.0, p_plus=0.2, p_hash=0.3, exact_frac=0.1)
C2 = Params(seed=2, n_filters=1_000_000, vocab=1024, zipf_s=1.1, p_plus=0.15, p_hash=0.25, exact_frac=0.0)
C1_TOPICS = 100_000
C2_TOPICS = 10_000_000


class _CParams(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64), ("n_filters", C.c_uint64), ("vocab", C.c_uint32), ("max_depth", C.c_uint32),
        ("zipf_s", C.c_double), ("p_plus", C.c_double), ("p_hash", C.c_double), ("p_final_plus", C.c_double),
        ("exact_frac", C.c_double), ("require_wildcard", C.c_int32), ("p_dollar", C.c_double),
        ("p_empty", C.c_double), ("p_topic_dollar", C.c_double), ("p_topic_inst", C.c_double),
        ("p_unseen", C.c_double),
    ]


class _CStrs(C.Structure):
    _fields_ = [("buf", C.c_void_p), ("offs", C.POINTER(C.c_uint64)), ("n", C.c_uint64)]


_glib = None


def _lib():
    global _glib
    if _glib is None:
        if not os.path.exists(GEN_LIB):
            raise RuntimeError(f"{GEN_LIB} missing: run __graft_entry__.build()")
        L = C.CDLL(GEN_LIB)
        L.tm_gen_filters.argtypes = [C.POINTER(_CParams), C.POINTER(_CStrs)]
        L.tm_gen_topics.argtypes = [C.POINTER(_CParams), C.POINTER(_CStrs), C.c_uint64, C.c_uint64,
                                    C.POINTER(_CStrs)]
        L.tm_gen_free.argtypes = [C.POINTER(_CStrs)]
        _glib = L
    return _glib


def _cparams(p: Params) -> _CParams:
    return _CParams(**{f.name: getattr(p, f.name) for f in fields(p)})


class Strings:
    """A packed string list: `buf` (uint8) + `offs` (uint64, n+1)."""

    def __init__(self, buf: np.ndarray, offs: np.ndarray):
        self.buf = buf
        self.offs = offs

    def __len__(self):
        return len(self.offs) - 1

    def __getitem__(self, i) -> bytes:
        return self.buf[int(self.offs[i]):int(self.offs[i + 1])].tobytes()

    def tolist(self):
        b = self.buf.tobytes()
        o = self.offs.tolist()
        return [b[o[i]:o[i + 1]] for i in range(len(o) - 1)]

    @classmethod
    def from_list(cls, strings):
        offs = np.zeros(len(strings) + 1, dtype=np.uint64)
        if strings:
            offs[1:] = np.cumsum([len(s) for s in strings], dtype=np.uint64)
        raw = b"".join(strings)
        buf = np.frombuffer(raw, dtype=np.uint8).copy() if raw else np.zeros(0, np.uint8)
        return cls(buf, offs)

    def slice(self, lo, hi) -> "Strings":
        a, b = int(self.offs[lo]), int(self.offs[hi])
        return Strings(self.buf[a:b].copy(), (self.offs[lo:hi + 1] - self.offs[lo]).astype(np.uint64))

    @classmethod
    def concat(cls, parts) -> "Strings":
        """parts[0] ++ parts[1] ++ ... as one packed list."""
        bufs, offs, base = [], [np.zeros(1, np.uint64)], 0
        for s in parts:
            bufs.append(s.buf[int(s.offs[0]):int(s.offs[-1])])
            offs.append((s.offs[1:] - s.offs[0] + base).astype(np.uint64))
            base += int(s.offs[-1] - s.offs[0])
        return cls(np.concatenate(bufs) if bufs else np.zeros(0, np.uint8), np.concatenate(offs))


def _take(cs: _CStrs) -> Strings:
    n = cs.n
    offs = np.ctypeslib.as_array(cs.offs, shape=(n + 1,)).copy()
    total = int(offs[-1])
    buf = np.frombuffer(C.string_at(cs.buf, total), dtype=np.uint8).copy() if total else np.zeros(0, np.uint8)
    _lib().tm_gen_free(C.byref(cs))
    return Strings(buf, offs)


def gen_filters(p: Params) -> Strings:
    cs = _CStrs()
    cp = _cparams(p)
    if _lib().tm_gen_filters(C.byref(cp), C.byref(cs)) != 0:
        raise RuntimeError("filter generation did not converge")
    return _take(cs)


def gen_topics(p: Params, filters: Strings, tseed: int, n: int) -> Strings:
    cs = _CStrs()
    cp = _cparams(p)
    fb = np.ascontiguousarray(filters.buf if filters.buf.size else np.zeros(1, np.uint8))
    fo = np.ascontiguousarray(filters.offs)
    fin = _CStrs(fb.ctypes.data, fo.ctypes.data_as(C.POINTER(C.c_uint64)), len(filters))
    _lib().tm_gen_topics(C.byref(cp), C.byref(fin), tseed, n, C.byref(cs))
    return _take(cs)


# ---------------------------------------------------------------- pure Python

M64 = (1 << 64) - 1
ALPH = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789!%"


class SplitMix64:
    def __init__(self, s):
        self.s = s & M64

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    def u01(self):
        return float(self.next() >> 11) * (1.0 / 9007199254740992.0)

    def below(self, n):
        return self.next() % n


def _vocab_word(seed, l, k) -> bytes:
    st = SplitMix64((seed * 0x9E3779B97F4A7C15 + ((l << 32) | k) + 1) & M64)
    if st.u01() < 0.05:
        ln = 1 + st.below(16)
        return bytes(ALPH[st.below(64)] for _ in range(ln))
    return b"w%d_%d" % (l, k)


class _Zipf:
    def __init__(self, p: Params):
        self.p = p
        acc = 0.0
        cdf = []
        for k in range(p.vocab):
            acc += math.pow(float(k + 1), -p.zipf_s)
            cdf.append(acc)
        self.cdf = [c / acc for c in cdf]

    def draw(self, s: SplitMix64):
        u = s.u01()
        lo, hi = 0, self.p.vocab - 1
        while lo < hi:
            mid = (lo + hi) // 2
            if u < self.cdf[mid]:
                hi = mid
            else:
                lo = mid + 1
        return lo


def _gen_filter(p, z, s, exact):
    depth = 1 + s.below(p.max_depth)
    dollar = s.u01() < p.p_dollar
    empty_at = s.below(depth) if s.u01() < p.p_empty else -1
    ws, wild = [], False
    for l in range(depth):
        if l == 0 and dollar:
            ws.append(b"$SYS"); continue
        if l == empty_at:
            ws.append(b""); continue
        if exact:
            ws.append(_vocab_word(p.seed, l, z.draw(s))); continue
        if l + 1 < depth:
            if s.u01() < p.p_plus:
                ws.append(b"+"); wild = True
            else:
                ws.append(_vocab_word(p.seed, l, z.draw(s)))
        else:
            r = s.u01()
            if r < p.p_hash:
                ws.append(b"#"); wild = True
            elif r < p.p_hash + p.p_final_plus:
                ws.append(b"+"); wild = True
            else:
                ws.append(_vocab_word(p.seed, l, z.draw(s)))
    return b"/".join(ws), wild


def py_gen_filters(p: Params):
    z = _Zipf(p)
    s = SplitMix64(p.seed)
    out, seen = [], set()
    while len(out) < p.n_filters:
        exact = s.u01() < p.exact_frac
        f, wild = _gen_filter(p, z, s, exact)
        if not exact and p.require_wildcard and not wild:
            continue
        if f in seen:
            continue
        seen.add(f)
        out.append(f)
    return out


def _unseen(s):
    return b"u%08x" % (s.next() & 0xFFFFFFFF)


def _instantiate(p, z, s, f: bytes):
    out, l = [], 0
    for w in f.split(b"/"):
        if w == b"#":
            extra = s.below(4)
            for _ in range(extra):
                out.append(_vocab_word(p.seed, l, z.draw(s)))
                l += 1
        else:
            if w == b"+":
                out.append(_vocab_word(p.seed, l, z.draw(s)) if s.u01() < 0.9 else _unseen(s))
            else:
                out.append(w)
            l += 1
    return b"/".join(out)


def py_gen_topics(p: Params, filters, tseed: int, n: int):
    z = _Zipf(p)
    s = SplitMix64(tseed)
    out = []
    for _ in range(n):
        r = s.u01()
        if filters and r < p.p_topic_dollar + p.p_topic_inst:
            dollar = r < p.p_topic_dollar
            f = filters[s.below(len(filters))]
            t = _instantiate(p, z, s, f)
            if t == b"":
                t = _vocab_word(p.seed, 0, z.draw(s))
            if dollar:
                k = t.find(b"/")
                t = b"$SYS" + (t[k:] if k >= 0 else b"")
        else:
            depth = 1 + s.below(p.max_depth)
            ws = []
            for l in range(depth):
                ws.append(_unseen(s) if s.u01() < p.p_unseen else _vocab_word(p.seed, l, z.draw(s)))
            t = b"/".join(ws)
        out.append(t)
    return out


# ---------------------------------------------------------------- C4 (IoT)

@dataclass
class IotParams:
    """Mirrors tm_iot_params (csrc/tm_gen.c): SURVEY.md §8d config C4."""
    seed: int = 4
    n_filters: int = 100_000_000
    n_ids: int = 10_000_000
    n_sensors: int = 16
    n_metrics: int = 8
    zipf_s: float = 1.05
    p_status: float = 0.2


C4 = IotParams()


class _CIot(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_filters", C.c_uint64), ("n_ids", C.c_uint32), ("n_sensors", C.c_uint32),
                ("n_metrics", C.c_uint32), ("pad", C.c_uint32), ("zipf_s", C.c_double), ("p_status", C.c_double)]


def _ciot(p: IotParams) -> _CIot:
    return _CIot(p.seed, p.n_filters, p.n_ids, p.n_sensors, p.n_metrics, 0, p.zipf_s, p.p_status)


def _iot_lib():
    L = _lib()
    if not getattr(L, "_iot_bound", False):
        L.tm_gen_iot_vocab.argtypes = [C.POINTER(_CIot), C.POINTER(_CStrs)]
        L.tm_gen_iot_filters.argtypes = [C.POINTER(_CIot), C.c_uint64, C.c_uint64, C.POINTER(_CStrs)]
        L.tm_gen_iot_topics.argtypes = [C.POINTER(_CIot), C.c_uint64, C.c_uint64, C.POINTER(_CStrs)]
        L._iot_bound = True
    return L


def gen_iot_vocab(p: IotParams) -> Strings:
    """The shared word dictionary of the sharded mode, in canonical order."""
    cs = _CStrs()
    cp = _ciot(p)
    _iot_lib().tm_gen_iot_vocab(C.byref(cp), C.byref(cs))
    return _take(cs)


def gen_iot_filters(p: IotParams, lo: int = 0, hi: int = None) -> Strings:
    hi = p.n_filters if hi is None else hi
    cs = _CStrs()
    cp = _ciot(p)
    if _iot_lib().tm_gen_iot_filters(C.byref(cp), lo, hi, C.byref(cs)) != 0:
        raise ValueError("IoT filter counts exceed the id/sensor/metric spaces")
    return _take(cs)


def iot_device_ids(s: Strings) -> np.ndarray:
    """The <X> of the second level d<X> of every IoT filter or topic (both
    generators put a literal d<X> there), vectorised: int64[len(s)]."""
    n = len(s)
    if n == 0:
        return np.zeros(0, np.int64)
    buf = s.buf
    slash = np.flatnonzero(buf == ord("/"))
    first = np.searchsorted(slash, s.offs[:-1])          # index of each string's first '/'
    a = slash[first] + 2                                  # after "/d"
    b = slash[first + 1]                                  # the second '/'
    out = np.zeros(n, np.int64)
    for k in range(int((b - a).max())):
        live = a + k < b
        digit = buf[np.minimum(a + k, len(buf) - 1)].astype(np.int64) - ord("0")
        out = np.where(live, out * 10 + digit, out)
    return out


def gen_iot_topics(p: IotParams, tseed: int, n: int) -> Strings:
    cs = _CStrs()
    cp = _ciot(p)
    _iot_lib().tm_gen_iot_topics(C.byref(cp), tseed, n, C.byref(cs))
    return _take(cs)


# ---------------------------------------------------------------- C5 (skew + churn)

@dataclass
class SkewParams:
    """Mirrors tm_skew_params (csrc/tm_gen.c): SURVEY.md §8d config C5."""
    seed: int = 5
    n_hot: int = 10_000
    hot_depth: int = 10
    vocab: int = 64
    k_per_hot: int = 100


class _CSkew(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_hot", C.c_uint32), ("hot_depth", C.c_uint32), ("vocab", C.c_uint32),
                ("k_per_hot", C.c_uint32)]


def _skew_lib():
    L = _lib()
    if not getattr(L, "_skew_bound", False):
        L.tm_gen_skew.argtypes = [C.POINTER(_CSkew), C.POINTER(_CStrs), C.POINTER(_CStrs)]
        L.tm_gen_derive_one.argtypes = [C.c_char_p, C.c_uint32, C.c_uint64, C.c_char_p, C.c_uint32]
        L.tm_gen_pick.argtypes = [C.POINTER(_CStrs), C.POINTER(_CStrs), C.c_uint64, C.c_uint64, C.c_double,
                                  C.c_double, C.POINTER(_CStrs)]
        L._skew_bound = True
    return L


def gen_skew(p: SkewParams):
    """-> (hot topics, filters derived from them: ~k_per_hot per hot topic)."""
    h, f = _CStrs(), _CStrs()
    cp = _CSkew(p.seed, p.n_hot, p.hot_depth, p.vocab, p.k_per_hot)
    if _skew_lib().tm_gen_skew(C.byref(cp), C.byref(h), C.byref(f)) != 0:
        raise ValueError("could not draw n_hot distinct hot topics")
    return _take(h), _take(f)


def derive_one(topic: bytes, seed: int) -> bytes:
    out = C.create_string_buffer(8192)
    n = _skew_lib().tm_gen_derive_one(topic, len(topic), seed, out, 8192)
    return out.raw[:n] if n > 0 else b""


def _cstrs(S: Strings):
    b = np.ascontiguousarray(S.buf if S.buf.size else np.zeros(1, np.uint8))
    o = np.ascontiguousarray(S.offs)
    return _CStrs(b.ctypes.data, o.ctypes.data_as(C.POINTER(C.c_uint64)), len(S)), (b, o)


def gen_pick(A: Strings, B: Strings, seed: int, n: int, p_a: float, zipf_s: float) -> Strings:
    ca, keep_a = _cstrs(A)
    cb, keep_b = _cstrs(B)
    out = _CStrs()
    _skew_lib().tm_gen_pick(C.byref(ca), C.byref(cb), seed, n, p_a, zipf_s, C.byref(out))
    return _take(out)
