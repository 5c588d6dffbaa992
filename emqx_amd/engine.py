"""Pythonic wrapper of one tm_engine (one host trie mirrored into an HBM
replica on each of its MI355X devices).

    eng = Engine(device=0)                       # one GPU
    eng = Engine(devices=[0, 1, 2, 3])           # one engine over four GPUs
    eng.insert(b"sensor/+/#")
    eng.match(b"sensor/1/temp")                  # -> [b"sensor/+/#"]
    offs, ids = eng.match_batch(topics)          # CSR over a whole batch
"""

from __future__ import annotations

import ctypes as C
import weakref

import numpy as np

from . import _native as N
from .gen import Strings


def _pack(topics) -> Strings:
    if isinstance(topics, Strings):
        return topics
    return Strings.from_list(list(topics))


class Tokens:
    """Tokenised publishes (tm_tokenize layout): words u32 = class << 29 | word id,
    toff u32[n+1], tflags u8[n]."""

    def __init__(self, words: np.ndarray, toff: np.ndarray, tflags: np.ndarray):
        self.words, self.toff, self.tflags = words, toff, tflags

    def __len__(self):
        return len(self.toff) - 1

    @property
    def nwords(self) -> int:
        return int(self.toff[-1])


class Batch:
    """A device-resident publish batch (tm_batch_prepare / launch / wait / result)."""

    def __init__(self, eng: "Engine", topics=None, handle=None, n=0, dedup=False, stream=False, replica=None):
        self.eng = eng
        if handle is not None:          # built by Engine.prepare_tokens
            self.h = handle
            self.n = n
            return
        s = _pack(topics)
        self.n = len(s)
        buf = s.buf if s.buf.size else np.zeros(1, np.uint8)
        self._buf = np.ascontiguousarray(buf)
        self._offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        h = C.c_void_p()
        flags = (N.TM_BATCH_DEDUP if dedup else 0) | (N.TM_BATCH_STREAM if stream else 0)
        if replica is None:
            N.check(eng.L.tm_batch_prepare_ex(eng.h, self._buf.ctypes.data, self._offs.ctypes.data, self.n,
                                              flags, C.byref(h)), "tm_batch_prepare_ex")
        else:
            N.check(eng.L.tm_batch_prepare_on(eng.h, replica, self._buf.ctypes.data, self._offs.ctypes.data,
                                              self.n, flags, C.byref(h)), "tm_batch_prepare_on")
        self.h = h

    @property
    def replica(self) -> int:
        return int(self.eng.L.tm_batch_replica(self.eng.h, self.h))

    def row_map(self):
        """-> (row_of uint32[n publishes], n_rows): result row of every publish."""
        p = C.POINTER(C.c_uint32)()
        nr = C.c_uint32()
        N.check(self.eng.L.tm_batch_row_map(self.eng.h, self.h, C.byref(p), C.byref(nr)), "tm_batch_row_map")
        return (np.ctypeslib.as_array(p, shape=(self.n,)).copy() if self.n else np.zeros(0, np.uint32)), nr.value

    def export(self, d_counts: int, d_ids: int, mul: int = 1, add: int = 0):
        """Per-topic counts and ids*mul+add into caller device buffers (tm_batch_export)."""
        N.check(self.eng.L.tm_batch_export(self.eng.h, self.h, d_counts, d_ids, mul, add), "tm_batch_export")

    def launch(self):
        N.check(self.eng.L.tm_batch_launch(self.eng.h, self.h), "tm_batch_launch")
        return self

    def wait(self):
        N.check(self.eng.L.tm_batch_wait(self.eng.h, self.h), "tm_batch_wait")
        return self

    def retokenize(self):
        """tm_batch_retokenize: the next launch tokenises the resident bytes again."""
        N.check(self.eng.L.tm_batch_retokenize(self.eng.h, self.h), "tm_batch_retokenize")
        return self

    def result(self):
        r = N.Result()
        N.check(self.eng.L.tm_batch_result(self.eng.h, self.h, C.byref(r)), "tm_batch_result")
        return _result_arrays(r)

    def result_packed(self):
        """tm_batch_result_packed -> (row_offsets u32[n+1], packed ids u8, id_bytes)."""
        r = N.ResultPacked()
        N.check(self.eng.L.tm_batch_result_packed(self.eng.h, self.h, C.byref(r)), "tm_batch_result_packed")
        n, m, ib = r.n_topics, int(r.n_matches), int(r.id_bytes)
        ro = np.ctypeslib.as_array(r.row_offsets, shape=(n + 1,)).copy()
        ids = np.ctypeslib.as_array(r.ids, shape=(m * ib,)).copy() if m else np.zeros(0, np.uint8)
        return ro, ids, ib

    def sample(self, rows):
        """tm_batch_sample: rows `rows` (row indices) of the waited batch,
        gathered on the device -> (offsets u32[k+1], ids) in that order."""
        idx = np.ascontiguousarray(np.asarray(rows, dtype=np.uint32))
        r = N.Result()
        N.check(self.eng.L.tm_batch_sample(self.eng.h, self.h, idx.ctypes.data, len(idx), C.byref(r)),
                "tm_batch_sample")
        return _result_arrays(r)

    def routes(self):
        """Device route resolution (tm_batch_routes) -> (row_offsets, filter_ids, dests)."""
        r = N.Routes()
        N.check(self.eng.L.tm_batch_routes(self.eng.h, self.h, C.byref(r)), "tm_batch_routes")
        return _routes_arrays(r)

    def dispatch(self, match_offsets: bool = False, counts_only: bool = False):
        """Device fan-out (tm_batch_dispatch): emqx_broker:dispatch/2 for every
        matched filter of every publish -> (row_offsets u64[n+1], match_offsets
        u64[m+1] or None, subscribers u32[deliveries] or None)."""
        d = self._dispatch((N.TM_DISPATCH_MATCH_OFFSETS if match_offsets else 0)
                           | (N.TM_DISPATCH_COUNT_ONLY if counts_only else 0))
        n, m, t = d.n_topics, int(d.n_matches), int(d.n_deliveries)
        offs = np.ctypeslib.as_array(d.row_offsets, shape=(n + 1,)).copy()
        moff = np.ctypeslib.as_array(d.match_offsets, shape=(m + 1,)).copy() if match_offsets else None
        if counts_only:
            subs = None
        else:
            subs = np.ctypeslib.as_array(d.subscribers, shape=(t,)).copy() if t else np.zeros(0, np.uint32)
        return offs, moff, subs

    def dispatch_device(self, match_offsets: bool = False):
        """Device-resident fan-out: -> (n_deliveries, fill kernel ms, device ptrs row/moff/subs);
        the moff pointer is None unless match_offsets."""
        d = self._dispatch(N.TM_DISPATCH_DEVICE | (N.TM_DISPATCH_MATCH_OFFSETS if match_offsets else 0))
        ptr = lambda p: C.cast(p, C.c_void_p).value  # noqa: E731
        return int(d.n_deliveries), float(d.fill_ms), ptr(d.row_offsets), ptr(d.match_offsets), ptr(d.subscribers)

    def dispatch_rows(self):
        """Fan-out over the walk's rows as it left them (TM_DISPATCH_ROWS), copied
        to the host for checking: (first delivery u64[n], deliveries u32[n],
        subscribers u32[total]); row i's deliveries are
        subscribers[first[i] : first[i] + count[i]]."""
        d = self._dispatch(N.TM_DISPATCH_ROWS)
        n, t = d.n_topics, int(d.n_deliveries)
        first = np.zeros(n, np.uint64)
        cnt = np.zeros(n, np.uint32)
        subs = np.zeros(t, np.uint32)
        ptr = lambda p: C.cast(p, C.c_void_p).value  # noqa: E731
        _d2h(first, ptr(d.row_offsets))
        _d2h(cnt, ptr(d.row_counts))
        _d2h(subs, ptr(d.subscribers))
        return first, cnt, subs

    def dispatch_rows_device(self):
        """TM_DISPATCH_ROWS kept in HBM: -> (n_deliveries, fill kernel ms)."""
        d = self._dispatch(N.TM_DISPATCH_ROWS)
        return int(d.n_deliveries), float(d.fill_ms)

    def _dispatch(self, flags: int) -> "N.Deliveries":
        d = N.Deliveries()
        N.check(self.eng.L.tm_batch_dispatch(self.eng.h, self.h, flags, C.byref(d)), "tm_batch_dispatch")
        return d

    def stats(self) -> dict:
        st = N.BatchStats()
        N.check(self.eng.L.tm_batch_stats_get(self.eng.h, self.h, C.byref(st)), "tm_batch_stats_get")
        return st.asdict()

    def device_csr(self):
        row, ids, n = C.c_void_p(), C.c_void_p(), C.c_uint64()
        N.check(self.eng.L.tm_batch_device_csr(self.eng.h, self.h, C.byref(row), C.byref(ids), C.byref(n)),
                "tm_batch_device_csr")
        return row.value, ids.value, n.value

    def device_rows(self):
        """Device pointers of the result as the walk left it (tm_batch_rows):
        (count u32[n], start u64[n], ids u32[...], n_matches); no CSR pass."""
        cnt, start, ids, n = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_uint64()
        N.check(self.eng.L.tm_batch_rows(self.eng.h, self.h, C.byref(cnt), C.byref(start), C.byref(ids),
                                         C.byref(n)), "tm_batch_rows")
        return cnt.value, start.value, ids.value, n.value

    def publish_rows_device(self):
        """tm_batch_publish_rows: device pointers of every PUBLISH's row
        (count u32[publishes], start u64[publishes], ids) and the delivered
        (publish, filter) matches; for a device-deduplicated batch the rows
        expanded behind the walk."""
        cnt, start, ids, n = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_uint64()
        N.check(self.eng.L.tm_batch_publish_rows(self.eng.h, self.h, C.byref(cnt), C.byref(start), C.byref(ids),
                                                 C.byref(n)), "tm_batch_publish_rows")
        return cnt.value, start.value, ids.value, n.value

    def rows(self, n_rows: int):
        """Host copy of the walk's rows (tm_batch_rows + hipMemcpy, for tests):
        (count u32[n_rows], start u64[n_rows], staging u32[max end])."""
        cnt, start, ids, _ = self.device_rows()
        c = np.zeros(n_rows, np.uint32)
        s = np.zeros(n_rows, np.uint64)
        _d2h(c, cnt)
        _d2h(s, start)
        end = int((s + c).max()) if n_rows else 0
        stg = np.zeros(max(end, 1), np.uint32)
        if end:
            _d2h(stg, ids)
        return c, s, stg[:end]

    def free(self):
        if self.h:
            self.eng.L.tm_batch_free(self.eng.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


_hip = None


def _d2h(dst: np.ndarray, src_ptr: int):
    """hipMemcpy device -> host through the HIP runtime the engine already
    loaded (same soname, so the same copy): test/diagnostic use only."""
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so.7")
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipMemcpy.restype = C.c_int
    if dst.nbytes:
        rc = _hip.hipMemcpy(dst.ctypes.data, src_ptr, dst.nbytes, 2)   # hipMemcpyDeviceToHost
        if rc:
            raise RuntimeError(f"hipMemcpy D2H failed: {rc}")


def _result_arrays(r: N.Result):
    n = r.n_topics
    offs = np.ctypeslib.as_array(r.row_offsets, shape=(n + 1,)).copy()
    m = int(r.n_matches)
    ids = np.ctypeslib.as_array(r.filter_ids, shape=(max(m, 1),))[:m].copy() if m else np.zeros(0, np.uint32)
    return offs, ids


def _routes_arrays(r: N.Routes):
    n, m = r.n_topics, int(r.n_routes)
    offs = np.ctypeslib.as_array(r.row_offsets, shape=(n + 1,)).copy()
    if not m:
        return offs, np.zeros(0, np.uint32), np.zeros(0, np.uint32)
    fids = np.ctypeslib.as_array(r.filter_ids, shape=(m,)).copy()
    dests = np.ctypeslib.as_array(r.dests, shape=(m,)).copy()
    return offs, fids, dests


def _invalidate(owner):
    """Borrowed Engine views of an owner that is being closed lose their handle."""
    for e in list(getattr(owner, "_borrowed", ())):
        e._h = None


class GroupBatch:
    """A publish batch split over a Group's replicas (tm_group_prepare ...)."""

    def __init__(self, grp: "Group", topics):
        self.grp = grp
        s = _pack(topics)
        self.n = len(s)
        self._buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        self._offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        h = C.c_void_p()
        N.check(grp.L.tm_group_prepare(grp.h, self._buf.ctypes.data, self._offs.ctypes.data, self.n, C.byref(h)),
                "tm_group_prepare")
        self.h = h

    def launch(self):
        N.check(self.grp.L.tm_group_launch(self.grp.h, self.h), "tm_group_launch")
        return self

    def wait(self):
        N.check(self.grp.L.tm_group_wait(self.grp.h, self.h), "tm_group_wait")
        return self

    def result(self):
        r = N.Result()
        N.check(self.grp.L.tm_group_result(self.grp.h, self.h, C.byref(r)), "tm_group_result")
        return _result_arrays(r)

    def sample(self, publishes):
        """tm_group_sample: the rows of `publishes` (indices into the whole
        batch), each gathered on its slice's device -> (offsets u32[k+1], ids)."""
        idx = np.ascontiguousarray(np.asarray(publishes, dtype=np.uint32))
        r = N.Result()
        N.check(self.grp.L.tm_group_sample(self.grp.h, self.h, idx.ctypes.data, len(idx), C.byref(r)),
                "tm_group_sample")
        return _result_arrays(r)

    def dispatch(self):
        """tm_group_dispatch -> (row_offsets u64[n+1], subscribers u32[deliveries])."""
        d = N.Deliveries()
        N.check(self.grp.L.tm_group_dispatch(self.grp.h, self.h, C.byref(d)), "tm_group_dispatch")
        n, t = d.n_topics, int(d.n_deliveries)
        offs = np.ctypeslib.as_array(d.row_offsets, shape=(n + 1,)).copy()
        subs = np.ctypeslib.as_array(d.subscribers, shape=(t,)).copy() if t else np.zeros(0, np.uint32)
        return offs, subs

    def stats(self) -> dict:
        st = N.BatchStats()
        N.check(self.grp.L.tm_group_batch_stats(self.grp.h, self.h, C.byref(st)), "tm_group_batch_stats")
        return st.asdict()

    def free(self):
        if self.h:
            self.grp.L.tm_group_batch_free(self.grp.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Group:
    """Replicated multi-device matching in one process (tm_group_*, config C3):
    a view of one replicated engine -- one host trie, one HBM replica per
    listed device, a mutation made once and uploaded to every replica, batches
    split into one contiguous slice per replica."""

    def __init__(self, devices, host_threads: int = 0):
        self.L = N.lib()
        devs = (C.c_int32 * len(devices))(*devices)
        cfg = N.Config(0, 0, host_threads, 0)
        h = C.c_void_p()
        N.check(self.L.tm_group_create(devs, len(devices), C.byref(cfg), C.byref(h)), "tm_group_create")
        self.h = h
        self.devices = list(devices)
        self._borrowed = weakref.WeakSet()

    def close(self):
        if getattr(self, "h", None):
            _invalidate(self)
            self.L.tm_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return int(self.L.tm_group_size(self.h))

    def insert(self, f: bytes):
        N.check(self.L.tm_group_trie_insert(self.h, f, len(f)), "tm_group_trie_insert")

    def delete(self, f: bytes):
        N.check(self.L.tm_group_trie_delete(self.h, f, len(f)), "tm_group_trie_delete")

    def insert_many(self, filters) -> int:
        s = _pack(filters)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        done = C.c_uint64()
        N.check(self.L.tm_group_insert_many(self.h, buf.ctypes.data, offs.ctypes.data, len(s), C.byref(done)),
                "tm_group_insert_many")
        return int(done.value)

    def route_apply(self, events) -> int:
        s = _pack([t for _, t, _ in events])
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        dests = np.ascontiguousarray(np.array([d for _, _, d in events] or [0], np.uint32))
        ops = np.ascontiguousarray(np.array([o for o, _, _ in events] or [0], np.uint8))
        done = C.c_uint64()
        N.check(self.L.tm_group_route_apply(self.h, buf.ctypes.data, offs.ctypes.data, dests.ctypes.data,
                                            ops.ctypes.data, len(events), C.byref(done)), "tm_group_route_apply")
        return int(done.value)

    def sync(self):
        N.check(self.L.tm_group_sync(self.h), "tm_group_sync")

    def prepare(self, topics) -> GroupBatch:
        return GroupBatch(self, topics)

    def engine(self) -> "Engine":
        """The group's engine (every tm_* call on it spans the replicas); the
        Group keeps ownership."""
        return Engine._borrow(self.L.tm_group_engine(self.h, 0), self.devices, owner=self)

    def match_batch(self, topics):
        s = _pack(topics)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        r = N.Result()
        N.check(self.L.tm_group_match_batch(self.h, buf.ctypes.data, offs.ctypes.data, len(s), C.byref(r)),
                "tm_group_match_batch")
        return _result_arrays(r)

    def filter_bytes(self, fid: int, replica: int = 0) -> bytes:
        e = self.L.tm_group_engine(self.h, replica)
        n = C.c_size_t()
        p = self.L.tm_filter_bytes(e, fid, C.byref(n))
        if not p:
            raise KeyError(fid)
        return C.string_at(p, n.value)


class Engine:
    def __init__(self, device: int = 0, init_slots: int = 0, host_threads: int = 0, frozen_dict: bool = False,
                 host_tokenize: bool = False, devices=None):
        self.L = N.lib()
        flags = (N.TM_CFG_FROZEN_DICT if frozen_dict else 0) | (N.TM_CFG_HOST_TOKENIZE if host_tokenize else 0)
        cfg = N.Config(device, init_slots, host_threads, flags)
        h = C.c_void_p()
        self._owned = True
        if devices is None:
            N.check(self.L.tm_create(C.byref(cfg), C.byref(h)), "tm_create")
            self.devices = [device] if device >= 0 else []
        else:
            devs = (C.c_int32 * max(len(devices), 1))(*devices)
            N.check(self.L.tm_create_replicated(C.byref(cfg), devs, len(devices), C.byref(h)), "tm_create_replicated")
            self.devices = list(devices)
        self._h = h
        self.device = self.devices[0] if self.devices else -1

    @classmethod
    def _borrow(cls, handle, devices, owner=None) -> "Engine":
        """A view of an engine another object owns: it keeps the owner alive,
        and the owner's close() invalidates it (calls then raise instead of
        reaching freed native memory)."""
        if not handle:
            raise ValueError("no such engine")
        e = cls.__new__(cls)
        e.L, e._h, e._owned = N.lib(), C.c_void_p(handle), False
        e.devices, e.device = list(devices), devices[0]
        e._owner = owner
        if owner is not None:
            owner._borrowed.add(e)
        return e

    @property
    def h(self):
        h = getattr(self, "_h", None)
        if h is None:
            raise RuntimeError("engine is closed (or its owner was)")
        return h

    @property
    def replicas(self) -> int:
        return int(self.L.tm_replica_count(self.h))

    def async_start(self):
        N.check(self.L.tm_async_start(self.h), "tm_async_start")

    def close(self):
        if getattr(self, "_h", None):
            if getattr(self, "_owned", True):
                self.L.tm_destroy(self._h)
            self._h = None

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

    def match_coalesced(self, topic: bytes):
        """emqx_trie:match/1 ids through tm_match_coalesced: concurrent callers
        (threads; ctypes drops the GIL) share device batches."""
        cap = 1024
        while True:
            ids = (C.c_uint32 * cap)()
            n = C.c_uint32()
            N.check(self.L.tm_match_coalesced(self.h, topic, len(topic), ids, cap, C.byref(n)), "tm_match_coalesced")
            if n.value <= cap:
                return list(ids[:n.value])
            cap = n.value

    def match_async(self, topic: bytes, done):
        """tm_match_async: done(rc, ids list) runs on the engine's completion
        thread.  The ctypes callback object is kept alive until it has run."""
        keep = getattr(self, "_async_keep", None)
        if keep is None:
            keep = self._async_keep = {}

        def cb(ctx, rc, ids, n, _key=[None]):
            try:
                done(rc, [ids[i] for i in range(n)] if rc == 0 else None)
            finally:
                keep.pop(_key[0], None)
        c = N.MATCH_CB(cb)
        key = id(c)
        cb.__defaults__[0][0] = key
        keep[key] = c
        rc = self.L.tm_match_async(self.h, topic, len(topic), c, None)
        if rc:
            keep.pop(key, None)
        N.check(rc, "tm_match_async")

    def async_stats(self) -> dict:
        st = N.AsyncStats()
        N.check(self.L.tm_async_stats_get(self.h, C.byref(st)), "tm_async_stats_get")
        return st.asdict()

    def coalesce_config(self, max_batch: int = 0, linger_us: int = N.TM_NONE):
        """-> (batches, requests) served by tm_match_coalesced so far."""
        b, r = C.c_uint64(), C.c_uint64()
        N.check(self.L.tm_coalesce_config(self.h, max_batch, linger_us, C.byref(b), C.byref(r)), "tm_coalesce_config")
        return int(b.value), int(r.value)

    # ---- batches -----------------------------------------------------------
    def match_batch(self, topics):
        """-> (row_offsets uint32[n+1], filter_ids uint32[total]); rows sorted by filter bytes."""
        s = _pack(topics)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        r = N.Result()
        N.check(self.L.tm_match_batch(self.h, buf.ctypes.data, offs.ctypes.data, len(s), C.byref(r)),
                "tm_match_batch")
        return _result_arrays(r)

    def match_batch_packed(self, topics):
        """tm_match_batch_packed -> (row_offsets uint32[n+1], packed ids uint8[total * id_bytes],
        id_bytes); id j = ids[j*id_bytes ...] little-endian."""
        s = _pack(topics)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        r = N.ResultPacked()
        N.check(self.L.tm_match_batch_packed(self.h, buf.ctypes.data, offs.ctypes.data, len(s), C.byref(r)),
                "tm_match_batch_packed")
        n, m, ib = r.n_topics, int(r.n_matches), int(r.id_bytes)
        ro = np.ctypeslib.as_array(r.row_offsets, shape=(n + 1,)).copy()
        ids = np.ctypeslib.as_array(r.ids, shape=(max(m * ib, 1),))[:m * ib].copy() if m else np.zeros(0, np.uint8)
        return ro, ids, ib

    def filters_copy_packed(self, ids, id_bytes: int) -> list:
        """tm_filters_copy_packed over packed ids: [(index, filter bytes)]."""
        a = np.ascontiguousarray(ids, dtype=np.uint8)
        n = len(a) // id_bytes
        offs = np.zeros(n + 1, np.uint64)
        keep = np.zeros(max(n, 1), np.uint32)
        k, need = C.c_uint32(), C.c_uint64()
        cap = 64 * max(n, 1)
        while True:
            buf = np.zeros(max(cap, 1), np.uint8)
            N.check(self.L.tm_filters_copy_packed(self.h, a.ctypes.data if n else None, id_bytes, n, buf.ctypes.data,
                                                  cap, offs.ctypes.data, keep.ctypes.data, C.byref(k),
                                                  C.byref(need)), "tm_filters_copy_packed")
            if need.value <= cap:
                break
            cap = need.value
        raw = buf.tobytes()
        return [(int(keep[j]), raw[int(offs[j]):int(offs[j + 1])]) for j in range(k.value)]

    def prepare(self, topics, dedup: bool = False, stream: bool = False, replica=None) -> Batch:
        """Device-resident batch; dedup=True matches identical topics once (TM_BATCH_DEDUP);
        stream=True gives it a HIP stream of its own, so launches of several
        batches overlap on the device (TM_BATCH_STREAM); replica = the device
        replica it runs on (default: the next one, round-robin)."""
        return Batch(self, topics, dedup=dedup, stream=stream, replica=replica)

    # ---- routes (emqx_router + emqx_broker:aggre/1) -------------------------
    def route_add(self, topic: bytes, dest: int):
        N.check(self.L.tm_route_add(self.h, topic, len(topic), dest), "tm_route_add")

    def route_delete(self, topic: bytes, dest: int) -> bool:
        rc = self.L.tm_route_delete(self.h, topic, len(topic), dest)
        if rc == N.TM_ENOENT:
            return False
        N.check(rc, "tm_route_delete")
        return True

    def route_apply(self, events) -> int:
        """tm_route_apply: [(op, topic, dest)] in order, op 1 = write (add), 0 =
        delete_object (absent = no-op).  Returns how many changed the table."""
        n = len(events)
        s = _pack([t for _, t, _ in events])
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        dests = np.ascontiguousarray(np.array([d for _, _, d in events] or [0], np.uint32))
        ops = np.ascontiguousarray(np.array([o for o, _, _ in events] or [0], np.uint8))
        done = C.c_uint64()
        N.check(self.L.tm_route_apply(self.h, buf.ctypes.data, offs.ctypes.data, dests.ctypes.data,
                                      ops.ctypes.data, n, C.byref(done)), "tm_route_apply")
        return int(done.value)

    # ---- subscribers (emqx_broker subscribe/unsubscribe/subscriber_down) ------
    def subscribe(self, topic: bytes, sub: int, node_dest: int = 0):
        N.check(self.L.tm_subscribe(self.h, topic, len(topic), sub, node_dest), "tm_subscribe")

    def unsubscribe(self, topic: bytes, sub: int, node_dest: int = 0) -> bool:
        rc = self.L.tm_unsubscribe(self.h, topic, len(topic), sub, node_dest)
        if rc == N.TM_ENOENT:
            return False
        N.check(rc, "tm_unsubscribe")
        return True

    def subscriber_down(self, sub: int, node_dest: int = 0) -> int:
        n = C.c_uint64()
        N.check(self.L.tm_subscriber_down(self.h, sub, node_dest, C.byref(n)), "tm_subscriber_down")
        return n.value

    def match_routes_batch(self, topics):
        """-> (row_offsets, filter_ids, dests): aggre(match_routes(T)) per topic."""
        s = _pack(topics)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        r = N.Routes()
        N.check(self.L.tm_match_routes_batch(self.h, buf.ctypes.data, offs.ctypes.data, len(s), C.byref(r)),
                "tm_match_routes_batch")
        return _routes_arrays(r)

    # ---- batched emqx_topic:match/2 (ACL / rewrite / tracer rules) -----------
    def rules_match(self, names, rules, dollar_rule: bool = True) -> np.ndarray:
        """-> bool[n, r]: emqx_topic:match(names[i], rules[j]) computed on the device
        (dollar_rule: the binary form's '$' rule; False = word-list form, as ACL)."""
        sn, sr = _pack(names), _pack(rules)
        n, r = len(sn), len(sr)
        if not n or not r:
            return np.zeros((n, r), bool)
        nb = np.ascontiguousarray(sn.buf if sn.buf.size else np.zeros(1, np.uint8))
        no = np.ascontiguousarray(sn.offs, dtype=np.uint64)
        rb = np.ascontiguousarray(sr.buf if sr.buf.size else np.zeros(1, np.uint8))
        ro = np.ascontiguousarray(sr.offs, dtype=np.uint64)
        wpr = (r + 31) // 32
        bits = np.zeros(n * wpr, np.uint32)
        N.check(self.L.tm_rules_match(self.h, nb.ctypes.data, no.ctypes.data, n, rb.ctypes.data, ro.ctypes.data, r,
                                      int(dollar_rule), bits.ctypes.data), "tm_rules_match")
        b = np.unpackbits(bits.view(np.uint8).reshape(n, wpr * 4), axis=1, bitorder="little")
        return b[:, :r].astype(bool)

    # ---- bulk load / filter-sharded mode -----------------------------------
    def insert_many(self, filters, shard: int = 0, nshards: int = 1) -> int:
        """emqx_trie:insert/1 over a filter list; with nshards > 1 only this
        shard's filters and the replicated ones.  Returns how many were inserted."""
        s = _pack(filters)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        done = C.c_uint64()
        N.check(self.L.tm_trie_insert_many(self.h, buf.ctypes.data, offs.ctypes.data, len(s), shard, nshards,
                                           C.byref(done)), "tm_trie_insert_many")
        return int(done.value)

    def delete_many(self, filters) -> int:
        """emqx_trie:delete/1 over a filter list (one C call)."""
        s = _pack(filters)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        done = C.c_uint64()
        N.check(self.L.tm_trie_delete_many(self.h, buf.ctypes.data, offs.ctypes.data, len(s), C.byref(done)),
                "tm_trie_delete_many")
        return int(done.value)

    def apply_many(self, dels, adds) -> tuple:
        """One subscription delta: delete_many(dels) then insert_many(adds),
        planned together (tm_trie_apply_many).  Returns (deleted, inserted)."""
        d, a = _pack(dels), _pack(adds)
        db = np.ascontiguousarray(d.buf if d.buf.size else np.zeros(1, np.uint8))
        do = np.ascontiguousarray(d.offs, dtype=np.uint64)
        ab = np.ascontiguousarray(a.buf if a.buf.size else np.zeros(1, np.uint8))
        ao = np.ascontiguousarray(a.offs, dtype=np.uint64)
        nd, ni = C.c_uint64(), C.c_uint64()
        N.check(self.L.tm_trie_apply_many(self.h, db.ctypes.data, do.ctypes.data, len(d), ab.ctypes.data,
                                          ao.ctypes.data, len(a), C.byref(nd), C.byref(ni)), "tm_trie_apply_many")
        return int(nd.value), int(ni.value)

    def dict_load(self, words):
        s = _pack(words)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        N.check(self.L.tm_dict_load(self.h, buf.ctypes.data, offs.ctypes.data, len(s)), "tm_dict_load")

    def filter_shard(self, f: bytes, nshards: int) -> int:
        return N.check(self.L.tm_filter_shard(self.h, f, len(f), nshards), "tm_filter_shard")

    def tokenize(self, topics) -> Tokens:
        s = _pack(topics)
        n = len(s)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        cap = int(n + np.count_nonzero(s.buf == ord("/"))) if n else 0
        words = np.zeros(max(cap, 1), np.uint32)
        toff = np.zeros(n + 1, np.uint32)
        tflags = np.zeros(max(n, 1), np.uint8)
        nw = C.c_uint64()
        N.check(self.L.tm_tokenize(self.h, buf.ctypes.data, offs.ctypes.data, n, words.ctypes.data, cap,
                                   toff.ctypes.data, tflags.ctypes.data, C.byref(nw)), "tm_tokenize")
        return Tokens(words[:nw.value], toff, tflags[:n])

    def tokenize_device(self, topics, words_cap: int = None):
        """tm_tokenize_device -> (words, toff, tflags) as torch tensors on this
        engine's GPU (the device tokeniser tm_match_batch uses)."""
        import torch
        s = _pack(topics)
        n = len(s)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        if words_cap is None:
            words_cap = int(n + np.count_nonzero(s.buf == ord("/"))) if n else 0
        dev = torch.device("cuda", self.device)
        words = torch.zeros(max(words_cap, 1), dtype=torch.int32, device=dev)
        toff = torch.zeros(n + 1, dtype=torch.int32, device=dev)
        tflags = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        nw = C.c_uint64()
        N.check(self.L.tm_tokenize_device(self.h, buf.ctypes.data, offs.ctypes.data, n, words.data_ptr(), words_cap,
                                          toff.data_ptr(), tflags.data_ptr(), C.byref(nw)), "tm_tokenize_device")
        return words[:nw.value], toff, tflags[:n]

    def prepare_tokens(self, words: int, toff: int, tflags: int, n: int, nwords: int, on_device: bool,
                       batch: Batch = None) -> Batch:
        """A batch from tokenised arrays given as raw pointers (device pointers when
        on_device, e.g. torch tensors' data_ptr()); `batch` is re-prepared in place."""
        h = C.c_void_p(batch.h.value if batch is not None else None)
        N.check(self.L.tm_batch_prepare_tokens(self.h, words, toff, tflags, n, nwords, int(on_device), C.byref(h)),
                "tm_batch_prepare_tokens")
        if batch is not None:
            batch.n = n
            return batch
        return Batch(self, handle=h, n=n)

    def prepare_tokens_host(self, tok: Tokens, batch: Batch = None) -> Batch:
        w = np.ascontiguousarray(tok.words if len(tok.words) else np.zeros(1, np.uint32))
        t = np.ascontiguousarray(tok.toff)
        f = np.ascontiguousarray(tok.tflags if len(tok.tflags) else np.zeros(1, np.uint8))
        return self.prepare_tokens(w.ctypes.data, t.ctypes.data, f.ctypes.data, len(tok), tok.nwords, False, batch)

    def gather_rows(self, d_src: int, d_src_off: int, d_idx: int, n: int, d_dst_off: int, d_dst: int):
        N.check(self.L.tm_gather_rows(self.h, d_src, d_src_off, d_idx, n, d_dst_off, d_dst), "tm_gather_rows")

    def tokens_shard(self, d_words: int, d_toff: int, n: int, nshards: int, d_shard: int):
        N.check(self.L.tm_tokens_shard(self.h, d_words, d_toff, n, nshards, d_shard), "tm_tokens_shard")

    # ---- filters -----------------------------------------------------------
    def filter_bytes(self, fid: int) -> bytes:
        n = C.c_size_t()
        p = self.L.tm_filter_bytes(self.h, fid, C.byref(n))
        if not p:
            raise KeyError(fid)
        return C.string_at(p, n.value)

    def filter_copy(self, fid: int) -> bytes:
        """tm_filter_copy: the filter's bytes copied under the engine lock."""
        n = C.c_size_t()
        buf = C.create_string_buffer(N.TM_MAX_TOPIC_LEN + 1)
        rc = self.L.tm_filter_copy(self.h, fid, buf, len(buf), C.byref(n))
        if rc == N.TM_ENOENT:
            raise KeyError(fid)
        N.check(rc, "tm_filter_copy")
        return buf.raw[:n.value]

    def filters_copy(self, ids) -> list:
        """tm_filters_copy: [(index in ids, filter bytes)] for the ids that
        still name a filter, copied under one acquisition of the engine lock."""
        a = np.ascontiguousarray(ids, dtype=np.uint32)
        n = len(a)
        offs = np.zeros(n + 1, np.uint64)
        keep = np.zeros(max(n, 1), np.uint32)
        k, need = C.c_uint32(), C.c_uint64()
        cap = 64 * max(n, 1)
        while True:
            buf = np.zeros(max(cap, 1), np.uint8)
            N.check(self.L.tm_filters_copy(self.h, a.ctypes.data, n, buf.ctypes.data, cap, offs.ctypes.data,
                                           keep.ctypes.data, C.byref(k), C.byref(need)), "tm_filters_copy")
            if need.value <= cap:
                break
            cap = need.value
        raw = buf.tobytes()
        return [(int(keep[j]), raw[int(offs[j]):int(offs[j + 1])]) for j in range(k.value)]

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

    def sync_async(self):
        """Queue the pending deltas' upload now, without waiting (tm_sync_async)."""
        N.check(self.L.tm_sync_async(self.h), "tm_sync_async")

    def debug_check(self) -> int:
        """tm_debug_check: edge-hash invariants; -> largest displacement."""
        md = C.c_uint64()
        N.check(self.L.tm_debug_check(self.h, C.byref(md)), "tm_debug_check")
        return int(md.value)


class ShardedBatch:
    """A publish batch of a ShardedGroup (tm_sharded_prepare / run / result)."""

    def __init__(self, grp: "ShardedGroup", topics):
        self.grp = grp
        s = _pack(topics)
        self.n = len(s)
        self._buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        self._offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        h = C.c_void_p()
        N.check(grp.L.tm_sharded_prepare(grp.h, self._buf.ctypes.data, self._offs.ctypes.data, self.n, C.byref(h)),
                "tm_sharded_prepare")
        self.h = h

    def run(self):
        N.check(self.grp.L.tm_sharded_run(self.grp.h, self.h), "tm_sharded_run")
        return self

    def reprepare(self, topics):
        """tm_sharded_prepare in place: new publishes (or the same ones again)."""
        s = _pack(topics)
        self.n = len(s)
        self._buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        self._offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        N.check(self.grp.L.tm_sharded_prepare(self.grp.h, self._buf.ctypes.data, self._offs.ctypes.data, self.n,
                                              C.byref(self.h)), "tm_sharded_prepare")
        return self

    def result(self):
        r = N.Result()
        N.check(self.grp.L.tm_sharded_result(self.grp.h, self.h, C.byref(r)), "tm_sharded_result")
        return _result_arrays(r)

    def stats(self) -> dict:
        st = N.ShardedStats()
        N.check(self.grp.L.tm_sharded_batch_stats(self.grp.h, self.h, C.byref(st)), "tm_sharded_batch_stats")
        out = st.match.asdict()
        out.update(ms_partition=st.ms_partition, ms_exchange=st.ms_exchange, ms_step=st.ms_step,
                   ms_unpartition=st.ms_unpartition, host_waits=st.host_waits,
                   part_topics=list(st.part_topics)[:len(self.grp)], ms_stage=st.ms_stage, ms_plan=st.ms_plan)
        return out

    def free(self):
        if self.h:
            self.grp.L.tm_sharded_batch_free(self.grp.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class ShardedGroup:
    """Filter-sharded matching in one process (tm_sharded_*, config C4 without
    torch or a collective): G shard engines, filters partitioned by their
    literal (w0, w1) prefix, publishes matched by their owner shard, rows in
    publish order with global ids (local id * G + shard)."""

    def __init__(self, devices, host_threads: int = 0):
        self.L = N.lib()
        devs = (C.c_int32 * len(devices))(*devices)
        cfg = N.Config(0, 0, host_threads, 0)
        h = C.c_void_p()
        N.check(self.L.tm_sharded_create(devs, len(devices), C.byref(cfg), C.byref(h)), "tm_sharded_create")
        self.h = h
        self.devices = list(devices)
        self._borrowed = weakref.WeakSet()

    def close(self):
        if getattr(self, "h", None):
            _invalidate(self)
            self.L.tm_sharded_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return int(self.L.tm_sharded_size(self.h))

    def link(self, i: int, j: int) -> str:
        """How shard i's memory reaches shard j's device: same / peer / staged."""
        return {N.TM_LINK_SAME: "same", N.TM_LINK_PEER: "peer", N.TM_LINK_STAGED: "staged"}[
            N.check(self.L.tm_sharded_link(self.h, i, j), "tm_sharded_link")]

    def dict_load(self, words):
        s = _pack(words)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        N.check(self.L.tm_sharded_dict_load(self.h, buf.ctypes.data, offs.ctypes.data, len(s)), "tm_sharded_dict_load")

    def insert_many(self, filters) -> int:
        s = _pack(filters)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        done = C.c_uint64()
        N.check(self.L.tm_sharded_insert_many(self.h, buf.ctypes.data, offs.ctypes.data, len(s), C.byref(done)),
                "tm_sharded_insert_many")
        return int(done.value)

    def delete_many(self, filters) -> int:
        s = _pack(filters)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        done = C.c_uint64()
        N.check(self.L.tm_sharded_delete_many(self.h, buf.ctypes.data, offs.ctypes.data, len(s), C.byref(done)),
                "tm_sharded_delete_many")
        return int(done.value)

    def prepare(self, topics) -> ShardedBatch:
        return ShardedBatch(self, topics)

    def match_batch(self, topics):
        s = _pack(topics)
        buf = np.ascontiguousarray(s.buf if s.buf.size else np.zeros(1, np.uint8))
        offs = np.ascontiguousarray(s.offs, dtype=np.uint64)
        r = N.Result()
        N.check(self.L.tm_sharded_match_batch(self.h, buf.ctypes.data, offs.ctypes.data, len(s), C.byref(r)),
                "tm_sharded_match_batch")
        return _result_arrays(r)

    def filter_bytes(self, gid: int) -> bytes:
        cap = 4096
        buf = C.create_string_buffer(cap)
        n = C.c_size_t()
        N.check(self.L.tm_sharded_filter_copy(self.h, gid, buf, cap, C.byref(n)), "tm_sharded_filter_copy")
        return buf.raw[:n.value]

    def engine(self, shard: int) -> "Engine":
        return Engine._borrow(self.L.tm_sharded_engine(self.h, shard), [self.devices[shard]], owner=self)
