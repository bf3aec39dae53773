"""ctypes binding of the zkagg C ABI (include/zkagg.h).

This is the same surface a JVM host binds through JNI/JNA; Python uses it for
the tests and the bench. Loading never falls back to anything: a missing or unloadable
libzkagg.so raises ZkLibraryError.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("ZKAGG_LIB", _PKG / "libzkagg.so"))

# status codes (zk_status)
ZK_OK = 0
ZK_ERR_INVALID_ARG = 1
ZK_ERR_HIP = 2
ZK_ERR_NO_SERVICE = 3
ZK_ERR_DURATION_RANGE = 4
ZK_ERR_TRACE_TOO_LARGE = 5
ZK_ERR_CAPACITY = 6
ZK_ERR_NOT_CLUSTERED = 7
ZK_ERR_NO_DEVICE = 8
ZK_ERR_SERVICE_RANGE = 9
ZK_ERR_UNSUPPORTED = 10
ZK_ERR_INVALID_SPAN = 11
ZK_ERR_RANK_FAILED = 12

# record flags
ZK_F_HAS_PARENT = 1 << 0
ZK_F_HAS_ANNOTATIONS = 1 << 1
ZK_F_SVC_CLIENT = 1 << 2
ZK_F_SVC_SERVER = 1 << 3
ZK_F_CS_SHIFT = 8
ZK_F_CR_SHIFT = 10
ZK_F_SR_SHIFT = 12
ZK_F_SS_SHIFT = 14

ZK_BATCH_DEVICE_PTRS = 1 << 0
ZK_BATCH_TRACE_CLUSTERED = 1 << 1
ZK_BATCH_VERIFY_TRACES = 1 << 2
ZK_BATCH_CONTINUES = 1 << 3

LIMBS_PER_CELL = 16
TABLE_TAIL_WORDS = 16  # the folded zk_stats counters after the S*S cells (ZK_TABLE_BYTES)


def table_words(num_services: int) -> int:
    """u64 words of the exact accumulator + counter tail: ZK_TABLE_BYTES(S) / 8."""
    return num_services * num_services * LIMBS_PER_CELL + TABLE_TAIL_WORDS


def xchg_words(num_services: int) -> int:
    """int64 words of the exchange buffer zk_deps_partial returns (ZK_XCHG_BYTES(S) / 8)."""
    return num_services * num_services * 12 + 16


class ZkLibraryError(RuntimeError):
    pass


class ZkError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"zk status {status}: {message}")
        self.status = status
        self.message = message


class zk_span_cols(C.Structure):
    _fields_ = [
        ("trace_id", C.c_void_p),
        ("span_id", C.c_void_p),
        ("parent_id", C.c_void_p),
        ("first_ts", C.c_void_p),
        ("last_ts", C.c_void_p),
        ("service_id", C.c_void_p),
        ("flags", C.c_void_p),
        ("n", C.c_uint64),
    ]


class zk_config(C.Structure):
    _fields_ = [
        ("num_services", C.c_uint32),
        ("device", C.c_int32),
        ("stream", C.c_void_p),
        ("strict", C.c_uint32),
        ("max_trace_records", C.c_uint32),
        ("timing", C.c_uint32),
        ("table", C.c_void_p),
        ("table_bytes", C.c_uint64),
        ("trace_pass", C.c_uint32),
        ("reserved", C.c_uint32 * 7),
    ]


class zk_stats(C.Structure):
    _fields_ = [
        (name, C.c_uint64)
        for name in (
            "records",
            "merged_spans",
            "valid_spans",
            "invalid_spans",
            "child_spans",
            "joined_links",
            "missing_parent",
            "no_service",
            "ambiguous",
            "spilled_traces",
            "duration_range",
            "service_range",
            "trace_too_large",
            "not_clustered",
        )
    ] + [("reserved", C.c_uint64 * 2)]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_ if k != "reserved"}


class zk_timing(C.Structure):
    _fields_ = [
        ("join_ms", C.c_double),
        ("reduce_ms", C.c_double),
        ("spill_ms", C.c_double),
        ("finalize_ms", C.c_double),
        ("join_calls", C.c_uint64),
        ("join_ms_total", C.c_double),
        ("reduce_ms_total", C.c_double),
        ("cluster_ms", C.c_double),
        ("cluster_ms_total", C.c_double),
        ("reserved", C.c_double * 2),
    ]


class zk_link_table(C.Structure):
    _fields_ = [
        ("m0", C.c_void_p),
        ("m1", C.c_void_p),
        ("m2", C.c_void_p),
        ("m3", C.c_void_p),
        ("m4", C.c_void_p),
        ("present", C.c_void_p),
        ("device_ptrs", C.c_uint32),
    ]


class zk_tracegen_params(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("num_traces", C.c_uint64),
        ("target_records", C.c_uint64),
        ("max_depth", C.c_uint32),
        ("num_services", C.c_uint32),
        ("base_ts", C.c_int64),
        ("rank", C.c_uint32),
        ("world", C.c_uint32),
        ("global_ids", C.c_uint32),
        ("reserved", C.c_uint32 * 3),
    ]


class zk_kv_config(C.Structure):
    _fields_ = [
        ("num_services", C.c_uint32),
        ("device", C.c_int32),
        ("stream", C.c_void_p),
        ("width", C.c_uint32),
        ("depth", C.c_uint32),
        ("candidates", C.c_uint32),
        ("seed", C.c_uint64),
        ("reserved", C.c_uint32 * 8),
    ]


class zk_rt_config(C.Structure):
    _fields_ = [
        ("num_services", C.c_uint32),
        ("device", C.c_int32),
        ("stream", C.c_void_p),
        ("hll_p", C.c_uint32),
        ("sub_bits", C.c_uint32),
        ("seed", C.c_uint64),
        ("reserved", C.c_uint32 * 8),
    ]


class zk_rl_config(C.Structure):
    _fields_ = [
        ("num_services", C.c_uint32),
        ("device", C.c_int32),
        ("stream", C.c_void_p),
        ("reserved", C.c_uint32 * 8),
    ]


ZK_RT_WITH_DEPS = 0
ZK_RT_ONLY = 1


class zk_ingest_items(C.Structure):
    _fields_ = [
        ("kv_service", C.c_void_p),
        ("kv_key", C.c_void_p),
        ("kv_cap", C.c_uint64),
        ("kv_n", C.c_uint64),
        ("ann_service", C.c_void_p),
        ("ann_value", C.c_void_p),
        ("ann_cap", C.c_uint64),
        ("ann_n", C.c_uint64),
    ]


ZK_CODEC_THRIFT = 0
ZK_CODEC_SNAPPY_THRIFT = 1
ZK_INGEST_STRICT = 1
ZK_INGEST_ONE_THREAD = 2


class zk_moments(C.Structure):
    _fields_ = [("m0", C.c_int64), ("m1", C.c_double), ("m2", C.c_double), ("m3", C.c_double), ("m4", C.c_double)]


class zk_dep_link(C.Structure):
    _fields_ = [("parent", C.c_uint32), ("child", C.c_uint32), ("moments", zk_moments)]


ZK_STORE_ANORM = 0
ZK_STORE_CASSANDRA = 1
ZK_STORE_HBASE = 2
ZK_TOP_ANNOTATIONS = 0
ZK_TOP_KV_ANNOTATIONS = 1
ZK_TIME_TOP = 2**63 - 1
ZK_TIME_BOTTOM = -(2**63)


# every symbol include/*.h declares: (name, restype, argtypes)
_P = C.c_void_p
_U64P = C.POINTER(C.c_uint64)
_U32P = C.POINTER(C.c_uint32)
_SIGNATURES = [
    ("zk_abi_version", C.c_uint32, []),
    ("zk_ctx_create", C.c_int, [C.POINTER(zk_config), C.POINTER(_P)]),
    ("zk_ctx_destroy", C.c_int, [_P]),
    ("zk_last_error", C.c_char_p, [_P]),
    ("zk_status_str", C.c_char_p, [C.c_int]),
    ("zk_ctx_sync", C.c_int, [_P]),
    ("zk_ctx_stats", C.c_int, [_P, C.POINTER(zk_stats)]),
    ("zk_ctx_timing", C.c_int, [_P, C.POINTER(zk_timing)]),
    ("zk_deps_reset", C.c_int, [_P]),
    ("zk_deps_accumulate", C.c_int, [_P, C.POINTER(zk_span_cols), C.c_uint32]),
    ("zk_deps_finalize", C.c_int, [_P, C.POINTER(zk_link_table)]),
    ("zk_deps_partial", C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_uint64)]),
    ("zk_deps_note_merged", C.c_int, [_P, C.c_uint64]),
    ("zk_deps_abort", C.c_int, [_P]),
    ("zk_trace_shard", C.c_uint32, [C.c_uint64, C.c_uint32]),
    (
        "zk_tracegen_host",
        C.c_int,
        [C.POINTER(zk_tracegen_params), C.POINTER(zk_span_cols), C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)],
    ),
    (
        "zk_tracegen_device",
        C.c_int,
        [_P, C.POINTER(zk_tracegen_params), C.POINTER(zk_span_cols), C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)],
    ),
    # include/zksketch.h: key-value count-min + top-K
    ("zk_kv_create", C.c_int, [C.POINTER(zk_kv_config), C.POINTER(_P)]),
    ("zk_kv_destroy", C.c_int, [_P]),
    ("zk_kv_last_error", C.c_char_p, [_P]),
    ("zk_kv_geometry", C.c_int, [_P, _U32P, _U32P, _U32P]),
    ("zk_kv_reset", C.c_int, [_P]),
    ("zk_kv_accumulate", C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint32]),
    ("zk_kv_topk_all", C.c_int, [_P, C.c_uint32, _P, _P, _P]),
    ("zk_kv_topk", C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, _P]),
    ("zk_kv_estimate", C.c_int, [_P, C.c_uint32, _P, C.c_uint64, _P]),
    ("zk_kv_totals", C.c_int, [_P, _P]),
    ("zk_kv_partial", C.c_int, [_P, C.POINTER(_P), _U64P, C.POINTER(_P), _U64P]),
    ("zk_kv_candidates", C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), _U64P, _U64P]),
    ("zk_kv_merge_candidates", C.c_int, [_P, _P, _P, C.c_uint32]),
    ("zk_kv_phase_ms", C.c_int, [_P, C.POINTER(C.c_double)]),
    # include/zksketch.h: realtime span sketches (HyperLogLog + duration histogram)
    ("zk_rt_create", C.c_int, [C.POINTER(zk_rt_config), C.POINTER(_P)]),
    ("zk_rt_destroy", C.c_int, [_P]),
    ("zk_rt_last_error", C.c_char_p, [_P]),
    ("zk_rt_geometry", C.c_int, [_P, _U32P, _U32P]),
    ("zk_rt_reset", C.c_int, [_P]),
    ("zk_rt_bind", C.c_int, [_P, _P, C.c_uint32]),
    ("zk_rt_accumulate_merged", C.c_int, [_P, _P, _P, _P, C.c_uint64, C.c_uint32]),
    ("zk_rt_distinct_traces", C.c_int, [_P, _P]),
    ("zk_rt_quantiles", C.c_int, [_P, C.c_uint32, _P, C.c_uint32, _P, _P, _U64P]),
    ("zk_rt_quantiles_all", C.c_int, [_P, _P, C.c_uint32, _P, _P, _U64P]),
    ("zk_rt_tdigest", C.c_int, [_P, C.c_uint32, C.c_double, _P, _P, C.c_uint32, C.POINTER(C.c_uint32), _P, C.c_uint32, _P, C.POINTER(C.c_uint64)]),
    ("zk_rt_partial", C.c_int, [_P, C.POINTER(_P), _U64P, C.POINTER(_P), _U64P]),
    ("zk_rt_read", C.c_int, [_P, _P, _P]),
    ("zk_rt_dropped", C.c_int, [_P, _U64P, _U64P]),
    # include/zksketch.h: realtime link store (RealtimeAggregates)
    ("zk_rl_create", C.c_int, [C.POINTER(zk_rl_config), C.POINTER(_P)]),
    ("zk_rl_destroy", C.c_int, [_P]),
    ("zk_rl_last_error", C.c_char_p, [_P]),
    ("zk_rl_reset", C.c_int, [_P]),
    ("zk_rl_bind", C.c_int, [_P, _P]),
    ("zk_rl_count", C.c_int, [_P, _U64P, _U64P]),
    ("zk_rl_server_links", C.c_int, [_P, C.c_uint32, _P, _P, _P, C.c_uint64, _U64P]),
    # include/zkcomm.h: RCCL communicator and the multi-GPU merges
    ("zk_comm_unique_id", C.c_int, [_P, C.c_uint64]),
    ("zk_comm_create", C.c_int, [_P, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int32, C.POINTER(_P)]),
    ("zk_comm_destroy", C.c_int, [_P]),
    ("zk_comm_last_error", C.c_char_p, [_P]),
    ("zk_deps_allreduce", C.c_int, [_P, _P, C.c_uint64]),
    ("zk_rt_allreduce", C.c_int, [_P, _P]),
    ("zk_kv_allreduce", C.c_int, [_P, _P]),
    # include/zkingest.h: stored span fragments -> columnar records
    ("zk_ingest_create", C.c_int, [C.POINTER(_P)]),
    ("zk_ingest_destroy", C.c_int, [_P]),
    ("zk_ingest_last_error", C.c_char_p, [_P]),
    (
        "zk_ingest_spans",
        C.c_int,
        [_P, _P, _P, C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(zk_span_cols), _U64P, _U64P,
         C.POINTER(zk_ingest_items)],
    ),
    ("zk_ingest_num_services", C.c_int, [_P, _U32P]),
    ("zk_ingest_service_id", C.c_int, [_P, C.c_char_p, C.c_uint64, _U32P]),
    ("zk_ingest_service_name", C.c_int, [_P, C.c_uint32, C.c_char_p, C.c_uint64, _U64P]),
    ("zk_ingest_string", C.c_int, [_P, C.c_uint64, C.c_char_p, C.c_uint64, _U64P]),
    ("zk_hash_string", C.c_uint64, [C.c_char_p, C.c_uint64]),
    ("zk_snappy_uncompress", C.c_int, [_P, C.c_uint64, _P, C.c_uint64, _U64P]),
    ("zk_dependencies_encode", C.c_int, [C.c_int64, C.c_int64, _P, C.c_uint64, _P, _P, C.c_uint32, _P, C.c_uint64,
                                         _U64P]),
    ("zk_dependencies_decode", C.c_int, [_P, _P, C.c_uint64, C.POINTER(C.c_int64), C.POINTER(C.c_int64), _P,
                                         C.c_uint64, _U64P]),
    ("zk_dependencies_row_key", C.c_int64, [C.c_int64]),
    ("zk_ingest_dev_create", C.c_int, [C.c_int32, _P, C.c_uint32, C.POINTER(_P)]),
    ("zk_ingest_dev_destroy", C.c_int, [_P]),
    ("zk_ingest_dev_last_error", C.c_char_p, [_P]),
    ("zk_ingest_dev_spans", C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint32, C.c_uint32, _P, _U64P, _U64P]),
    ("zk_ingest_dev_spans_items", C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint32, C.c_uint32, _P, _U64P, _U64P,
                                            C.POINTER(zk_ingest_items)]),
    ("zk_ingest_dev_spans_multi", C.c_int, [_P, C.c_uint32, _P, _P, _P, C.c_uint32, C.c_uint32, _P, _U64P, _U64P,
                                            C.POINTER(zk_ingest_items)]),
    ("zk_ingest_dev_string", C.c_int, [_P, C.c_uint64, C.c_char_p, C.c_uint64, _U64P]),
    ("zk_ingest_dev_num_services", C.c_int, [_P, C.POINTER(C.c_uint32)]),
    ("zk_ingest_dev_set_scratch", C.c_int, [_P, C.c_uint64]),
    ("zk_ingest_dev_service_name", C.c_int, [_P, C.c_uint32, C.c_char_p, C.c_uint64, _U64P]),
    # include/zkstore.h: the Aggregates store surface (host side)
    ("zk_store_create", C.c_int, [C.c_uint32, C.POINTER(_P)]),
    ("zk_store_destroy", C.c_int, [_P]),
    ("zk_store_last_error", C.c_char_p, [_P]),
    ("zk_store_put_dependencies", C.c_int, [_P, C.c_int64, C.c_int64, _P, C.c_uint64]),
    (
        "zk_store_get_dependencies",
        C.c_int,
        [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_int64, _P, C.c_uint64, _U64P,
         C.POINTER(C.c_int64), C.POINTER(C.c_int64)],
    ),
    ("zk_store_count", C.c_int, [_P, _U64P]),
    ("zk_store_watermark", C.c_int, [_P, C.POINTER(C.c_int64)]),
    ("zk_store_put_top", C.c_int, [_P, C.c_uint32, C.c_uint32, _P, C.c_uint64]),
    ("zk_store_get_top", C.c_int, [_P, C.c_uint32, C.c_uint32, _P, C.c_uint64, _U64P]),
    ("zk_moments_plus", C.c_int, [C.POINTER(zk_moments), C.POINTER(zk_moments), C.POINTER(zk_moments)]),
    ("zk_link_table_compact", C.c_int, [C.POINTER(zk_link_table), C.c_uint32, _P, C.c_uint64, _U64P]),
]

SYMBOLS = [s[0] for s in _SIGNATURES]

_lib = None


def lib() -> C.CDLL:
    """Load libzkagg.so (once). Raises ZkLibraryError if it is missing or lacks a symbol."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ZkLibraryError(f"{LIB_PATH} not built: run __graft_entry__.build() (no fallback exists)")
    try:
        L = C.CDLL(str(LIB_PATH))
    except OSError as e:  # pragma: no cover
        raise ZkLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    for name, res, args in _SIGNATURES:
        try:
            f = getattr(L, name)
        except AttributeError as e:
            raise ZkLibraryError(f"{LIB_PATH} does not export {name}") from e
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def status_str(s: int) -> str:
    return lib().zk_status_str(s).decode()
