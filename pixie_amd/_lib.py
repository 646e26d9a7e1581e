"""ctypes binding of libpxg.so (include/pxg.h).

Plumbing only: the product is the C ABI in libpxg.so.  Loading fails loudly if the library
is missing — there is no CPU fallback anywhere in pixie_amd.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PXG_LIB_PATH") or os.path.join(_HERE, "lib", "libpxg.so")  # (override: A/B builds in tools/)

# px.types.DataType (src/shared/types/typespb/types.proto:26-34)
BOOLEAN, INT64, UINT128, FLOAT64, STRING, TIME64NS = 1, 2, 3, 4, 5, 6
TYPE_NAMES = {BOOLEAN: "BOOLEAN", INT64: "INT64", UINT128: "UINT128", FLOAT64: "FLOAT64",
              STRING: "STRING", TIME64NS: "TIME64NS"}

# pxg_opcode
OP = dict(NOP=0, COL=1, CONST=2, I2F=3, B2I=4, I2B=5, F2I=6,
          ADD_I=10, SUB_I=11, MUL_I=12, MOD_I=13, BIN_I=14, NEG_I=15, INV_I=16,
          ADD_F=20, SUB_F=21, MUL_F=22, DIV_F=23, NEG_F=24,
          EQ_I=30, NE_I=31, LT_I=32, LE_I=33, GT_I=34, GE_I=35,
          EQ_F=40, NE_F=41, LT_F=42, LE_F=43, GT_F=44, GE_F=45, APPROX_EQ_F=46, APPROX_NE_F=47,
          EQ_S=50, NE_S=51, LT_S=52, LE_S=53, GT_S=54, GE_S=55,
          EQ_U=60, NE_U=61, AND=70, OR=71, NOT=72)

# pxg_uda_kind
UDA_COUNT, UDA_SUM, UDA_MEAN, UDA_MIN, UDA_MAX, UDA_QUANTILES, UDA_MINSUM = 1, 2, 3, 4, 5, 6, 100

HTTP_EVENTS_NCOLS = 10


class ColumnView(C.Structure):
    _fields_ = [("type", C.c_int32), ("reserved", C.c_int32), ("length", C.c_int64),
                ("values", C.c_void_p), ("offsets", C.c_void_p), ("data", C.c_void_p)]


class ColumnOut(C.Structure):
    _fields_ = [("type", C.c_int32), ("reserved", C.c_int32), ("length", C.c_int64),
                ("values", C.c_void_p), ("offsets", C.c_void_p), ("data", C.c_void_p),
                ("data_len", C.c_int64)]


class Insn(C.Structure):
    _fields_ = [("op", C.c_uint16), ("type", C.c_uint16), ("arg", C.c_int32), ("imm", C.c_int64)]


class Program(C.Structure):
    _fields_ = [("n_insns", C.c_int32), ("result_type", C.c_int32), ("insns", C.POINTER(Insn)),
                ("pool_len", C.c_int32), ("reserved", C.c_int32), ("pool", C.c_void_p)]


class UdaSpec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("arg_type", C.c_int32), ("arg", Program), ("arg2", Program),
                ("has_init", C.c_int32), ("reserved", C.c_int32), ("init_i64", C.c_int64)]


class AggSpec(C.Structure):
    _fields_ = [("n_keys", C.c_int32), ("n_udas", C.c_int32), ("keys", C.POINTER(Program)),
                ("udas", C.POINTER(UdaSpec)), ("filter", C.POINTER(Program)),
                ("expected_groups", C.c_int64), ("windowed", C.c_int32), ("emit_states", C.c_int32)]


class JoinSpec(C.Structure):
    _fields_ = [("n_keys", C.c_int32), ("emit_unmatched_probe", C.c_int32), ("emit_unmatched_build", C.c_int32),
                ("n_out", C.c_int32), ("build_keys", C.POINTER(C.c_int32)), ("probe_keys", C.POINTER(C.c_int32)),
                ("out_side", C.POINTER(C.c_int32)), ("out_col", C.POINTER(C.c_int32))]


class AggStats(C.Structure):
    _fields_ = [("table_capacity", C.c_int64), ("groups", C.c_int64), ("rows_selected", C.c_int64),
                ("key_arena_bytes", C.c_int64), ("staging_capacity", C.c_int64), ("fast_path_keys", C.c_int32),
                ("big_sort_groups", C.c_int32), ("hc_mode", C.c_int32), ("hc_partition_bits", C.c_int32),
                ("hc_reruns", C.c_int32)]


# Every symbol include/pxg.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "pxg_abi_version", "pxg_last_error", "pxg_device_count", "pxg_ctx_create", "pxg_ctx_destroy",
    "pxg_ctx_sync", "pxg_ctx_stream", "pxg_ctx_set_profiling", "pxg_ctx_profile_only", "pxg_ctx_kernel_stats",
    "pxg_ctx_reset_stats", "pxg_table_create", "pxg_table_destroy", "pxg_table_append",
    "pxg_table_append_device", "pxg_table_flush", "pxg_table_num_rows", "pxg_table_num_chunks",
    "pxg_table_device_bytes", "pxg_table_fetch", "pxg_table_time_bound", "pxg_table_pxrb_image",
    "pxg_pxrb_copy", "pxg_pxrb_destroy", "pxg_filter", "pxg_filter_split", "pxg_map", "pxg_agg_create",
    "pxg_agg_destroy", "pxg_agg_consume", "pxg_agg_finalize", "pxg_agg_result", "pxg_agg_result_skip", "pxg_agg_result_device", "pxg_agg_finalize_result", "pxg_agg_quantile_lanes", "pxg_result_free", "pxg_host_alloc", "pxg_host_free",
    "pxg_agg_reset", "pxg_agg_rows_selected", "pxg_agg_info", "pxg_agg_export_partial", "pxg_agg_import_partial", "pxg_agg_import_partials",
    "pxg_agg_export_partial_dev",
    "pxg_join", "pxg_datagen_http_events", "pxg_table_append_http_events", "pxg_digest_chains", "pxg_digest_merge",
    "pxg_comm_unique_id", "pxg_comm_init", "pxg_comm_init_host", "pxg_comm_destroy", "pxg_agg_alltoall", "pxg_agg_gather",
]

_lib = None


class Xfer(C.Structure):
    """pxg_xfer (include/pxg.h): one point-to-point transfer of a host-transport batch."""
    _fields_ = [("peer", C.c_int32), ("send", C.c_int32), ("buf", C.c_void_p), ("bytes", C.c_int64)]


# pxg_xfer_fn: int32_t (*)(void* user, int32_t n_ops, const pxg_xfer* ops)
XferFn = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, C.POINTER(Xfer))


class PxgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"pxg error {code}: {msg}")
        self.code = code


def load() -> C.CDLL:
    """Load libpxg.so.  torch (if importable) is imported first so that the process holds a
    single HIP runtime (torch ships its own libamdhip64.so.7)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C pixie_amd` "
                          "(or __graft_entry__.build()); pixie_amd has no CPU fallback")
    if "torch" not in sys.modules and os.environ.get("PXG_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401
        except Exception:
            pass
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    vp, i32, i64, p = C.c_void_p, C.c_int32, C.c_int64, C.POINTER
    sig = {
        "pxg_abi_version": (i32, []),
        "pxg_last_error": (C.c_char_p, []),
        "pxg_device_count": (i32, [p(i32)]),
        "pxg_ctx_create": (i32, [i32, p(vp)]),
        "pxg_ctx_destroy": (i32, [vp]),
        "pxg_ctx_sync": (i32, [vp]),
        "pxg_ctx_stream": (vp, [vp]),
        "pxg_ctx_set_profiling": (i32, [vp, i32]),
        "pxg_ctx_profile_only": (i32, [vp, C.c_char_p]),
        "pxg_ctx_kernel_stats": (i32, [vp, C.c_char_p, p(i64), p(C.c_double)]),
        "pxg_ctx_reset_stats": (i32, [vp]),
        "pxg_table_create": (i32, [vp, i32, p(i32), p(vp)]),
        "pxg_table_destroy": (i32, [vp]),
        "pxg_table_append": (i32, [vp, p(ColumnView), i64]),
        "pxg_table_append_device": (i32, [vp, p(ColumnView), i64]),
        "pxg_table_flush": (i32, [vp]),
        "pxg_table_num_rows": (i64, [vp]),
        "pxg_table_num_chunks": (i32, [vp]),
        "pxg_table_device_bytes": (i64, [vp, i32]),
        "pxg_table_fetch": (i32, [vp, i32, i64, i64, p(ColumnOut)]),
        "pxg_filter": (i32, [vp, p(Program), i32, p(i32), i64, i64, p(vp)]),
        "pxg_filter_split": (i32, [vp, p(Program), i32, p(i32), i64, i64, i32, p(i64), p(i64), p(vp)]),
        "pxg_map": (i32, [vp, i32, p(Program), i64, i64, p(vp)]),
        "pxg_agg_create": (i32, [vp, p(AggSpec), p(vp)]),
        "pxg_agg_destroy": (i32, [vp]),
        "pxg_agg_consume": (i32, [vp, vp, i64, i64]),
        "pxg_agg_finalize": (i32, [vp, p(i64)]),
        "pxg_agg_result": (i32, [vp, p(ColumnOut), i32]),
        "pxg_agg_result_skip": (i32, [vp, p(ColumnOut), i32, C.c_void_p]),
        "pxg_agg_result_device": (i32, [vp, C.c_void_p, i32, C.c_void_p]),
        "pxg_agg_finalize_result": (i32, [vp, C.c_void_p, p(ColumnOut), i32, C.c_void_p]),
        "pxg_agg_quantile_lanes": (i32, [vp, i32, C.c_uint32, C.c_void_p, C.c_void_p]),
        "pxg_result_free": (None, [p(ColumnOut), i32]),
        "pxg_host_alloc": (C.c_void_p, [C.c_int64]),
        "pxg_host_free": (None, [C.c_void_p]),
        "pxg_agg_reset": (i32, [vp]),
        "pxg_agg_rows_selected": (i32, [vp, p(i64)]),
        "pxg_agg_info": (i32, [vp, p(AggStats)]),
        "pxg_agg_export_partial": (i32, [vp, i32, vp, i64, p(i64), p(i64)]),
        "pxg_agg_import_partial": (i32, [vp, vp, i64]),
        "pxg_agg_import_partials": (i32, [vp, vp, i32, p(i64), p(i64)]),
        "pxg_agg_export_partial_dev": (i32, [vp, i32, p(vp), p(i64), vp]),
        "pxg_join": (i32, [vp, vp, p(JoinSpec), p(vp), p(i64)]),
        "pxg_table_time_bound": (i32, [vp, i32, i64, i32, p(i64)]),
        "pxg_table_pxrb_image": (i32, [vp, p(i64), i64, i32, i32, p(vp), p(i64)]),
        "pxg_pxrb_copy": (i32, [vp, vp]),
        "pxg_pxrb_destroy": (i32, [vp]),
        "pxg_datagen_http_events": (i32, [C.c_uint64, i64, i64, i64, i32, p(ColumnOut)]),
        "pxg_table_append_http_events": (i32, [vp, C.c_uint64, i64, i64, i64]),
        "pxg_digest_chains": (i32, [vp, vp, i32, i32, vp, i32, vp]),
        "pxg_digest_merge": (i32, [vp, vp, vp, i64, i32, vp]),
        "pxg_comm_unique_id": (i32, [vp, i32]),
        "pxg_comm_init": (i32, [vp, i32, i32, vp, i32, p(vp)]),
        "pxg_comm_init_host": (i32, [vp, i32, i32, XferFn, vp, p(vp)]),
        "pxg_comm_destroy": (i32, [vp]),
        "pxg_agg_alltoall": (i32, [vp, vp, p(i64), p(i64)]),
        "pxg_agg_gather": (i32, [vp, vp, i32, p(i64)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(code: int) -> None:
    if code != 0:
        msg = load().pxg_last_error()
        raise PxgError(code, msg.decode() if msg else "")
