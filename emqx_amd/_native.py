"""ctypes binding of libemqx_tm.so (include/emqx_tm.h).

The product path has no CPU fallback: if the HIP library is missing this module
raises at import, and match calls on an engine without a device fail with
TM_ENODEV.
"""

from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EMQX_TM_LIB") or os.path.join(HERE, "libemqx_tm.so")   # override: A/B builds
HEADER = os.path.join(os.path.dirname(HERE), "include", "emqx_tm.h")

TM_OK = 0
TM_ENOENT = -2
TM_EIO = -5
TM_ENOMEM = -12
TM_ENODEV = -19
TM_EINVAL = -22
TM_EOVERFLOW = -75
TM_EABORT = -125
TM_NONE = 0xFFFFFFFF
TM_MAX_TOPIC_LEN = 4096
TM_CFG_FROZEN_DICT = 1
TM_CFG_HOST_TOKENIZE = 2
TM_BATCH_DEDUP = 1
TM_BATCH_STREAM = 2
TM_ROUTE_DELETE = 0
TM_ROUTE_WRITE = 1
TM_LINK_SAME = 0
TM_LINK_PEER = 1
TM_LINK_STAGED = 2

_ERRNAMES = {TM_ENOENT: "ENOENT", TM_EIO: "EIO", TM_ENOMEM: "ENOMEM", TM_ENODEV: "ENODEV",
             TM_EINVAL: "EINVAL", TM_EOVERFLOW: "EOVERFLOW", TM_EABORT: "EABORT"}


class TmError(RuntimeError):
    def __init__(self, rc, what=""):
        self.rc = rc
        super().__init__(f"{what}: {_ERRNAMES.get(rc, rc)}")


class Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("init_slots", C.c_uint32), ("host_threads", C.c_uint32),
                ("flags", C.c_uint32)]


class TrieNode(C.Structure):
    _fields_ = [("edge_count", C.c_uint32), ("has_topic", C.c_uint32), ("filter_id", C.c_uint32)]


class Result(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("n_matches", C.c_uint64),
                ("row_offsets", C.POINTER(C.c_uint32)), ("filter_ids", C.POINTER(C.c_uint32))]


class ResultPacked(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("id_bytes", C.c_uint32), ("n_matches", C.c_uint64),
                ("row_offsets", C.POINTER(C.c_uint32)), ("ids", C.POINTER(C.c_uint8))]


class Routes(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("n_routes", C.c_uint64), ("row_offsets", C.POINTER(C.c_uint32)),
                ("filter_ids", C.POINTER(C.c_uint32)), ("dests", C.POINTER(C.c_uint32))]


class Deliveries(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("n_matches", C.c_uint64), ("n_deliveries", C.c_uint64),
                ("row_offsets", C.POINTER(C.c_uint64)), ("match_offsets", C.POINTER(C.c_uint64)),
                ("subscribers", C.POINTER(C.c_uint32)), ("fill_ms", C.c_float),
                ("row_counts", C.POINTER(C.c_uint32))]


TM_DISPATCH_COUNT_ONLY = 1
TM_DISPATCH_ROWS = 8
TM_DISPATCH_MATCH_OFFSETS = 2
TM_DISPATCH_DEVICE = 4


class BatchStats(C.Structure):
    _fields_ = [("topics", C.c_uint64), ("visits", C.c_uint64), ("hash_hits", C.c_uint64),
                ("words", C.c_uint64), ("matches", C.c_uint64), ("slow_topics", C.c_uint64),
                ("overflow_tiles", C.c_uint64), ("ms_match", C.c_float), ("ms_total", C.c_float),
                ("ms_tokenize", C.c_float), ("probes", C.c_uint64),
                ("ms_csr", C.c_float), ("ms_queue", C.c_float), ("iterations", C.c_uint64),
                ("publishes", C.c_uint64), ("delivered", C.c_uint64), ("ms_dedup", C.c_float),
                ("ms_expand", C.c_float)]

    def asdict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class EngineStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("version", "nodes", "edges", "filters", "words", "slots",
                                          "device_bytes", "uploads_full", "uploads_delta", "delta_slots",
                                          "graph_launches")]

    def asdict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class AsyncStats(C.Structure):
    _fields_ = [("batches", C.c_uint64), ("requests", C.c_uint64), ("recoveries", C.c_uint64),
                ("max_batch", C.c_uint64), ("depth", C.c_uint32), ("queued", C.c_uint32),
                ("us_launch", C.c_double), ("us_wait", C.c_double), ("us_deliver", C.c_double),
                ("inline_launches", C.c_uint64)]

    def asdict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class ShardedStats(C.Structure):
    _fields_ = [("match", BatchStats), ("ms_partition", C.c_float), ("ms_exchange", C.c_float),
                ("ms_step", C.c_float), ("ms_unpartition", C.c_float), ("host_waits", C.c_uint32),
                ("part_topics", C.c_uint32 * 64), ("ms_stage", C.c_float), ("ms_plan", C.c_float)]


# void (*tm_match_cb)(void* ctx, int rc, const uint32_t* ids, uint32_t n)
MATCH_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.POINTER(C.c_uint32), C.c_uint32)

# exported symbol -> (restype, argtypes); must cover every declaration in include/emqx_tm.h
P = C.c_void_p
SZ = C.c_size_t
U8P = C.c_char_p
SIGNATURES = {
    "tm_create": (C.c_int, [C.POINTER(Config), C.POINTER(P)]),
    "tm_create_replicated": (C.c_int, [C.POINTER(Config), P, C.c_uint32, C.POINTER(P)]),
    "tm_replica_count": (C.c_uint32, [P]),
    "tm_async_start": (C.c_int, [P]),
    "tm_destroy": (None, [P]),
    "tm_version": (C.c_uint64, [P]),
    "tm_stats": (C.c_int, [P, C.POINTER(EngineStats)]),
    "tm_sync": (C.c_int, [P]),
    "tm_sync_async": (C.c_int, [P]),
    "tm_trie_insert": (C.c_int, [P, U8P, SZ]),
    "tm_trie_delete": (C.c_int, [P, U8P, SZ]),
    "tm_trie_lookup": (C.c_int, [P, U8P, SZ, C.c_int, C.POINTER(TrieNode)]),
    "tm_trie_empty": (C.c_int, [P]),
    "tm_trie_match": (C.c_int, [P, U8P, SZ, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32)]),
    "tm_match_batch": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(Result)]),
    "tm_match_batch_packed": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(ResultPacked)]),
    "tm_match_coalesced": (C.c_int, [P, U8P, SZ, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32)]),
    "tm_coalesce_config": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "tm_match_async": (C.c_int, [P, U8P, SZ, MATCH_CB, P]),
    "tm_async_stats_get": (C.c_int, [P, C.POINTER(AsyncStats)]),
    "tm_batch_prepare": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(P)]),
    "tm_batch_prepare_ex": (C.c_int, [P, P, P, C.c_uint32, C.c_uint32, C.POINTER(P)]),
    "tm_batch_prepare_on": (C.c_int, [P, C.c_uint32, P, P, C.c_uint32, C.c_uint32, C.POINTER(P)]),
    "tm_batch_replica": (C.c_uint32, [P, P]),
    "tm_batch_row_map": (C.c_int, [P, P, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_uint32)]),
    "tm_batch_launch": (C.c_int, [P, P]),
    "tm_batch_wait": (C.c_int, [P, P]),
    "tm_batch_result": (C.c_int, [P, P, C.POINTER(Result)]),
    "tm_batch_result_packed": (C.c_int, [P, P, C.POINTER(ResultPacked)]),
    "tm_batch_sample": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(Result)]),
    "tm_batch_stats_get": (C.c_int, [P, P, C.POINTER(BatchStats)]),
    "tm_batch_device_csr": (C.c_int, [P, P, C.POINTER(P), C.POINTER(P), C.POINTER(C.c_uint64)]),
    "tm_batch_rows": (C.c_int, [P, P, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(C.c_uint64)]),
    "tm_batch_publish_rows": (C.c_int, [P, P, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(C.c_uint64)]),
    "tm_batch_free": (None, [P, P]),
    "tm_batch_retokenize": (C.c_int, [P, P]),
    "tm_route_add": (C.c_int, [P, U8P, SZ, C.c_uint32]),
    "tm_route_delete": (C.c_int, [P, U8P, SZ, C.c_uint32]),
    "tm_route_apply": (C.c_int, [P, P, P, P, P, C.c_uint32, C.POINTER(C.c_uint64)]),
    "tm_batch_routes": (C.c_int, [P, P, C.POINTER(Routes)]),
    "tm_subscribe": (C.c_int, [P, U8P, SZ, C.c_uint32, C.c_uint32]),
    "tm_unsubscribe": (C.c_int, [P, U8P, SZ, C.c_uint32, C.c_uint32]),
    "tm_subscriber_down": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64)]),
    "tm_batch_dispatch": (C.c_int, [P, P, C.c_uint32, C.POINTER(Deliveries)]),
    "tm_match_routes_batch": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(Routes)]),
    "tm_trie_insert_many": (C.c_int, [P, P, P, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64)]),
    "tm_trie_delete_many": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(C.c_uint64)]),
    "tm_trie_apply_many": (C.c_int, [P, P, P, C.c_uint32, P, P, C.c_uint32, C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint64)]),
    "tm_dict_load": (C.c_int, [P, P, P, C.c_uint32]),
    "tm_filter_shard": (C.c_int, [P, U8P, SZ, C.c_uint32]),
    "tm_tokenize": (C.c_int, [P, P, P, C.c_uint32, P, C.c_uint64, P, P, C.POINTER(C.c_uint64)]),
    "tm_tokenize_device": (C.c_int, [P, P, P, C.c_uint32, P, C.c_uint64, P, P, C.POINTER(C.c_uint64)]),
    "tm_batch_prepare_tokens": (C.c_int, [P, P, P, P, C.c_uint32, C.c_uint64, C.c_int, C.POINTER(P)]),
    "tm_gather_rows": (C.c_int, [P, P, P, P, C.c_uint32, P, P]),
    "tm_tokens_shard": (C.c_int, [P, P, P, C.c_uint32, C.c_uint32, P]),
    "tm_batch_export": (C.c_int, [P, P, P, P, C.c_uint32, C.c_uint32]),
    "tm_filter_bytes": (C.POINTER(C.c_uint8), [P, C.c_uint32, C.POINTER(SZ)]),
    "tm_filter_id": (C.c_int, [P, U8P, SZ, C.POINTER(C.c_uint32)]),
    "tm_filter_copy": (C.c_int, [P, C.c_uint32, P, SZ, C.POINTER(SZ)]),
    "tm_filters_copy": (C.c_int, [P, P, C.c_uint32, P, SZ, P, P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    "tm_filters_copy_packed": (C.c_int, [P, P, C.c_uint32, C.c_uint32, P, SZ, P, P, C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_uint64)]),
    "tm_topic_match": (C.c_int, [U8P, SZ, U8P, SZ]),
    "tm_topic_wildcard": (C.c_int, [U8P, SZ]),
    "tm_topic_validate": (C.c_int, [C.c_int, U8P, SZ, C.POINTER(C.c_char_p)]),
    "tm_rules_match": (C.c_int, [P, P, P, C.c_uint32, P, P, C.c_uint32, C.c_int, P]),
    "tm_group_create": (C.c_int, [P, C.c_uint32, C.POINTER(Config), C.POINTER(P)]),
    "tm_group_destroy": (None, [P]),
    "tm_group_size": (C.c_uint32, [P]),
    "tm_group_engine": (P, [P, C.c_uint32]),
    "tm_group_trie_insert": (C.c_int, [P, U8P, SZ]),
    "tm_group_trie_delete": (C.c_int, [P, U8P, SZ]),
    "tm_group_insert_many": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(C.c_uint64)]),
    "tm_group_route_apply": (C.c_int, [P, P, P, P, P, C.c_uint32, C.POINTER(C.c_uint64)]),
    "tm_group_sync": (C.c_int, [P]),
    "tm_group_prepare": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(P)]),
    "tm_group_launch": (C.c_int, [P, P]),
    "tm_group_wait": (C.c_int, [P, P]),
    "tm_group_result": (C.c_int, [P, P, C.POINTER(Result)]),
    "tm_group_sample": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(Result)]),
    "tm_group_batch_stats": (C.c_int, [P, P, C.POINTER(BatchStats)]),
    "tm_group_batch_free": (None, [P, P]),
    "tm_group_match_batch": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(Result)]),
    "tm_group_dispatch": (C.c_int, [P, P, C.POINTER(Deliveries)]),
    "tm_group_match_async": (C.c_int, [P, U8P, SZ, MATCH_CB, P]),
    "tm_group_match_coalesced": (C.c_int, [P, U8P, SZ, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32)]),
    "tm_group_match_routes_batch": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(Routes)]),
    "tm_group_rules_match": (C.c_int, [P, P, P, C.c_uint32, P, P, C.c_uint32, C.c_int, P]),
    "tm_sharded_create": (C.c_int, [P, C.c_uint32, C.POINTER(Config), C.POINTER(P)]),
    "tm_sharded_destroy": (None, [P]),
    "tm_sharded_size": (C.c_uint32, [P]),
    "tm_sharded_engine": (P, [P, C.c_uint32]),
    "tm_sharded_dict_load": (C.c_int, [P, P, P, C.c_uint32]),
    "tm_sharded_insert_many": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(C.c_uint64)]),
    "tm_sharded_delete_many": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(C.c_uint64)]),
    "tm_sharded_prepare": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(P)]),
    "tm_sharded_run": (C.c_int, [P, P]),
    "tm_sharded_result": (C.c_int, [P, P, C.POINTER(Result)]),
    "tm_sharded_device_csr": (C.c_int, [P, P, C.POINTER(P), C.POINTER(P), C.POINTER(C.c_uint64)]),
    "tm_sharded_batch_stats": (C.c_int, [P, P, C.POINTER(ShardedStats)]),
    "tm_sharded_link": (C.c_int, [P, C.c_uint32, C.c_uint32]),
    "tm_sharded_batch_free": (None, [P, P]),
    "tm_sharded_match_batch": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(Result)]),
    "tm_sharded_filter_copy": (C.c_int, [P, C.c_uint32, P, SZ, C.POINTER(SZ)]),
    "tm_debug_check": (C.c_int, [P, C.POINTER(C.c_uint64)]),
    "tm_last_error": (C.c_char_p, []),
    "tm_build_info": (C.c_char_p, []),
    "tm_device_count": (C.c_int, []),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built (run __graft_entry__.build()); "
                              "the HIP engine is required -- there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc < 0:
        detail = ""
        if rc == TM_EIO and _lib is not None:
            detail = " [" + (_lib.tm_last_error() or b"").decode(errors="replace") + "]"
        raise TmError(rc, what + detail)
    return rc


def gpu_available() -> bool:
    """True when a HIP device is visible, asked through the engine's own HIP
    runtime (torch.cuda.is_available() turns False once the engine has
    initialised HIP first in the process, so it is not asked)."""
    try:
        return lib().tm_device_count() > 0
    except (ImportError, OSError):
        return False
