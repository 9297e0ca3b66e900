"""ctypes binding of libgossip_hip.so (include/gossip.h).

The product path: there is no CPU fallback.  If the in-tree library is missing
or a GPU is absent, calls fail loudly (GossipError / OSError).
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# GS_LIB_PATH: an experimental build of the same ABI (A/B timing only)
LIB_PATH = os.environ.get("GS_LIB_PATH") or os.path.join(PKG_DIR, "libgossip_hip.so")
CLI_PATH = os.path.join(PKG_DIR, "bin", "gossip_sim")

GS_OK, GS_EINVAL, GS_ELIVELOCK, GS_EREJECT, GS_ENOMEM, GS_EDEVICE, GS_EOVERFLOW = (
    0, -1, -2, -3, -4, -5, -6)
GS_FLAG_TIMING = 1
GS_FLAG_TICK_ENGINE = 2
GS_FLAG_PP_L2_ONLY = 4
GS_FLAG_PP_DENSE = 8
GS_FLAG_PP_EARLY = 16
GS_FLAG_PP_TOPDOWN = 32
GS_FLAG_PP_BOTTOM = 64
GS_FLAG_PP_ANSWER = 128
GS_MODEL_FLOOD, GS_MODEL_PUSHPULL = 0, 1
GS_RUN_COVERED, GS_RUN_QUIESCENT, GS_RUN_MAX_TICKS, GS_RUN_RUNNING = 0, 1, 2, -1
GS_COMM_ID_BYTES = 128

# Every symbol include/gossip.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "gs_version", "gs_strerror", "gs_create", "gs_destroy", "gs_last_error",
    "gs_load_peers", "gs_load_peers_device", "gs_read_peers", "gs_build_overlay",
    "gs_set_failed", "gs_broadcast_begin", "gs_step", "gs_run", "gs_totals",
    "gs_read_received", "gs_read_crashed", "gs_timing_get", "gs_format_float32",
    "gs_format_float64", "gs_format_duration", "gs_threshold", "gs_philox",
    "gs_set_flags", "gs_reset", "gs_set_stream", "gs_create_multi", "gs_comm_unique_id",
    "gs_create_rank", "gs_shard_info", "gs_trial_results", "gs_set_trial",
    "gs_create_rank_exchange", "gs_shard_timing", "gs_trim", "gs_memory_stats",
)


class GossipError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} [code {code}]")
        self.code = code


class Params(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("fanout", C.c_int32),
        ("fanin", C.c_int32),
        ("delay_low", C.c_int32),
        ("delay_high", C.c_int32),
        ("drop_rate", C.c_double),
        ("crash_rate", C.c_double),
        ("seed", C.c_uint64),
        ("trial", C.c_uint32),
        ("device", C.c_int32),
        ("flags", C.c_uint32),
        ("model", C.c_uint32),  # GS_MODEL_FLOOD = 0 (reference), GS_MODEL_PUSHPULL = 1
        ("trials", C.c_uint32),  # batched independent trials (config C3); 0/1 = one
        ("reserved0_", C.c_uint32),
        ("reserved_", C.c_uint64 * 5),
    ]


class TickStats(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in
                ("tick", "fired", "sent", "messages", "received", "crashed", "pending")]


class TrialStats(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in
                ("trial", "tick_99", "tick", "fired", "sent", "messages", "received", "crashed")] + \
        [("status", C.c_int32), ("reserved_", C.c_int32)]


class Window(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("tick", "makeups", "breakups")]


class Timing(C.Structure):
    _fields_ = [("deliver_ms", C.c_double), ("resolve_ms", C.c_double),
                ("deliver_launches", C.c_uint64), ("resolve_launches", C.c_uint64),
                ("overlay_ms", C.c_double), ("expand_ms", C.c_double),
                ("part_ms", C.c_double), ("windows", C.c_uint64), ("exact_redos", C.c_uint64),
                ("prep_ms", C.c_double),
                ("pp_early_rounds", C.c_uint64), ("pp_bottom_rounds", C.c_uint64),
                ("pp_answer_rounds", C.c_uint64), ("dd_fallbacks", C.c_uint64), ("pp_rev_part", C.c_uint64),
                ("ov_part_ticks", C.c_uint64), ("ov_sort_ticks", C.c_uint64), ("ov_part_fallbacks", C.c_uint64),
                ("alloc_ms", C.c_double), ("largest_alloc_ms", C.c_double), ("free_ms", C.c_double),
                ("alloc_calls", C.c_uint64), ("alloc_cache_hits", C.c_uint64), ("cached_bytes", C.c_uint64),
                ("coarse_redos", C.c_uint64)]


# gs_exchange (gossip.h): host callbacks of a gs_create_rank_exchange rank
ALL_GATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)
ALL_REDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t)


ALL_TO_ALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p,
                             C.POINTER(C.c_size_t))


class Exchange(C.Structure):
    _fields_ = [("user", C.c_void_p), ("all_gather", ALL_GATHER_FN), ("all_reduce_sum_u64", ALL_REDUCE_FN),
                ("all_to_allv", ALL_TO_ALLV_FN)]


_lib = None


def load():
    """Load the in-tree library (raises OSError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    P, vp, sz = C.POINTER, C.c_void_p, C.c_size_t
    ctx = vp
    sig = {
        "gs_version": ([], C.c_int),
        "gs_strerror": ([C.c_int], C.c_char_p),
        "gs_create": ([P(Params), P(vp)], C.c_int),
        "gs_destroy": ([ctx], None),
        "gs_last_error": ([ctx], C.c_char_p),
        "gs_load_peers": ([ctx, vp, vp, C.c_uint32], C.c_int),
        "gs_load_peers_device": ([ctx, vp, vp, C.c_uint32], C.c_int),
        "gs_read_peers": ([ctx, vp, vp, P(C.c_uint32)], C.c_int),
        "gs_build_overlay": ([ctx, C.c_uint64, P(Window), sz, P(sz), P(C.c_uint64)], C.c_int),
        "gs_set_failed": ([ctx, vp, sz], C.c_int),
        "gs_broadcast_begin": ([ctx, C.c_int64], C.c_int),
        "gs_step": ([ctx, C.c_uint32, P(TickStats)], C.c_int),
        "gs_run": ([ctx, C.c_uint32, C.c_uint64, P(TickStats), sz, P(sz), P(C.c_int32)], C.c_int),
        "gs_totals": ([ctx, P(TickStats)], C.c_int),
        "gs_read_received": ([ctx, vp, sz], C.c_int),
        "gs_read_crashed": ([ctx, vp, sz], C.c_int),
        "gs_timing_get": ([ctx, P(Timing)], C.c_int),
        "gs_shard_timing": ([ctx, C.c_uint32, P(Timing)], C.c_int),
        "gs_format_float32": ([C.c_float, C.c_char_p, sz], sz),
        "gs_format_float64": ([C.c_double, C.c_char_p, sz], sz),
        "gs_format_duration": ([C.c_int64, C.c_char_p, sz], sz),
        "gs_threshold": ([C.c_double], C.c_int32),
        "gs_philox": ([P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)], None),
        "gs_set_flags": ([ctx, C.c_uint32], C.c_int),
        "gs_reset": ([ctx], C.c_int),
        "gs_set_stream": ([ctx, vp], C.c_int),
        "gs_create_multi": ([P(Params), P(C.c_int), C.c_int, P(vp)], C.c_int),
        "gs_comm_unique_id": ([C.c_char_p], C.c_int),
        "gs_create_rank": ([P(Params), C.c_int, C.c_int, C.c_int, C.c_char_p, P(vp)], C.c_int),
        "gs_create_rank_exchange": ([P(Params), C.c_int, C.c_int, C.c_int, P(Exchange), P(vp)], C.c_int),
        "gs_shard_info": ([ctx, C.c_uint32, P(C.c_uint32), P(C.c_uint64), P(C.c_uint64)], C.c_int),
        "gs_trial_results": ([ctx, P(TrialStats), sz, P(sz)], C.c_int),
        "gs_set_trial": ([ctx, C.c_uint32], C.c_int),
        "gs_trim": ([C.c_int, P(sz)], C.c_int),
        "gs_memory_stats": ([P(Timing)], C.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def format_float32(x: float) -> str:
    b = C.create_string_buffer(64)
    load().gs_format_float32(x, b, 64)
    return b.value.decode()


def format_float64(x: float) -> str:
    b = C.create_string_buffer(64)
    load().gs_format_float64(x, b, 64)
    return b.value.decode()


def format_duration(ns: int) -> str:
    b = C.create_string_buffer(64)
    load().gs_format_duration(ns, b, 64)
    return b.value.decode("utf-8")


def threshold(rate: float) -> int:
    return int(load().gs_threshold(rate))


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*[int(x) & 0xFFFFFFFF for x in ctr])
    k = (C.c_uint32 * 2)(*[int(x) & 0xFFFFFFFF for x in key])
    o = (C.c_uint32 * 4)()
    load().gs_philox(c, k, o)
    return [int(x) for x in o]
