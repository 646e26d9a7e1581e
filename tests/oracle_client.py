"""ctypes client of the CPU Carnot restatement (oracle/).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import subprocess
from typing import Dict, List, Sequence

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "build", "liboracle.so")

BOOLEAN, INT64, UINT128, FLOAT64, STRING, TIME64NS = 1, 2, 3, 4, 5, 6


class OColumn(C.Structure):
    _fields_ = [("type", C.c_int32), ("length", C.c_int64), ("values", C.c_void_p),
                ("offsets", C.c_void_p), ("data", C.c_void_p)]


class OTable(C.Structure):
    _fields_ = [("name", C.c_char_p), ("ncols", C.c_int32), ("col_names", C.POINTER(C.c_char_p)),
                ("col_types", C.POINTER(C.c_int32)), ("nbatches", C.c_int32), ("cols", C.POINTER(OColumn)),
                ("batch_flags", C.c_void_p)]


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_LIB):
        subprocess.run(["make", "-C", ORACLE_DIR, "-s"], check=True)
    lib = C.CDLL(ORACLE_LIB)
    lib.oracle_execute_plan.restype = C.c_int32
    lib.oracle_execute_plan.argtypes = [C.c_char_p, C.c_int32, C.POINTER(OTable), C.POINTER(C.c_void_p),
                                        C.POINTER(C.c_int64), C.c_char_p, C.c_int32]
    lib.oracle_execute_plan_timed.restype = C.c_int32
    lib.oracle_execute_plan_timed.argtypes = [C.c_char_p, C.c_int32, C.POINTER(OTable), C.POINTER(C.c_double),
                                              C.POINTER(C.c_int64), C.c_char_p, C.c_int32]
    lib.oracle_execute_plan_timed_rebatched.restype = C.c_int32
    lib.oracle_execute_plan_timed_rebatched.argtypes = [C.c_char_p, C.c_int32, C.POINTER(OTable), C.c_int64,
                                                        C.POINTER(C.c_double), C.POINTER(C.c_int64), C.c_char_p, C.c_int32]
    lib.oracle_execute_plan_rebatched.restype = C.c_int32
    lib.oracle_execute_plan_rebatched.argtypes = [C.c_char_p, C.c_int32, C.POINTER(OTable), C.c_int64, C.POINTER(C.c_double),
                                                  C.POINTER(C.c_void_p), C.POINTER(C.c_int64), C.c_char_p, C.c_int32]
    lib.oracle_free.argtypes = [C.c_void_p]
    lib.oracle_tdigest_quantiles.argtypes = [C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double)]
    lib.oracle_tdigest_merge_quantiles.argtypes = [C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double), C.c_int64,
                                                   C.POINTER(C.c_double)]
    lib.oracle_tdigest_centroids.argtypes = [C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                             C.c_int64, C.POINTER(C.c_int64)]
    lib.oracle_tdigest_batch_quantiles.argtypes = [C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_double),
                                                   C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.oracle_tdigest_batch_quantiles_mm.argtypes = [C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_double),
                                                      C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                                      C.POINTER(C.c_double)]
    lib.oracle_quantiles_json.argtypes = [C.POINTER(C.c_double), C.c_int64, C.c_char_p, C.c_int32]
    lib.oracle_quantiles_json.restype = C.c_int32
    lib.oracle_pluck_float64.argtypes = [C.c_char_p, C.c_char_p]
    lib.oracle_pluck_float64.restype = C.c_double
    _lib = lib
    return lib


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"oracle error {code}: {msg}")
        self.code = code


class AbsentColumn:
    """A table column the plan never reads: passed without buffers, never materialised."""

    def __init__(self, type_: int, length: int):
        self.type = type_
        self.length = length

    def __len__(self):
        return self.length


def _col_struct(col) -> OColumn:
    oc = OColumn()
    oc.type = col.type
    oc.length = len(col)
    if isinstance(col, AbsentColumn):
        return oc
    if col.type == STRING:
        oc.offsets = col.offsets.ctypes.data
        oc.data = col.data.ctypes.data
    else:
        oc.values = col.values.ctypes.data
    return oc


class _Tables:
    """Keeps the ctypes structures (and numpy buffers) alive for one call."""

    def __init__(self, tables: Dict[str, dict]):
        self.keep = []
        arr = (OTable * max(1, len(tables)))()
        for ti, (name, t) in enumerate(tables.items()):
            types = t["types"]
            names = t.get("names") or [f"c{i}" for i in range(len(types))]
            batches = t["batches"]
            cols = (OColumn * max(1, len(batches) * len(types)))()
            for b, batch in enumerate(batches):
                for c, col in enumerate(batch):
                    cols[b * len(types) + c] = _col_struct(col)
                    self.keep.append(col)
            cnames = (C.c_char_p * len(names))(*[n.encode() for n in names])
            ctypes_ = (C.c_int32 * len(types))(*types)
            self.keep += [cols, cnames, ctypes_]
            bname = name.encode()
            self.keep.append(bname)
            flags = None
            if t.get("flags") is not None:
                fl = np.array([(1 if eow else 0) | (2 if eos else 0) for eow, eos in t["flags"]], dtype=np.uint8)
                self.keep.append(fl)
                flags = fl.ctypes.data
            arr[ti] = OTable(bname, len(types), cnames, ctypes_, len(batches), cols, flags)
        self.arr = arr
        self.n = len(tables)


from pixie_amd.pxrb import parse_pxrb  # noqa: E402  (shared result decoder)


def execute_plan(plan, tables: Dict[str, dict]):
    """Run a planpb.Plan (message) on the oracle.  tables: name -> {types, batches, names}."""
    from google.protobuf import json_format
    lib = load()
    js = json_format.MessageToJson(plan).encode()
    t = _Tables(tables)
    out = C.c_void_p()
    n = C.c_int64()
    err = C.create_string_buffer(1024)
    code = lib.oracle_execute_plan(js, t.n, t.arr, C.byref(out), C.byref(n), err, 1024)
    if code != 0:
        raise OracleError(code, err.value.decode())
    try:
        buf = C.string_at(out.value, n.value)
    finally:
        lib.oracle_free(out)
    return parse_pxrb(buf)


def execute_plan_timed(plan, tables: Dict[str, dict], batch_rows: int = 0):
    """(execution-window seconds, result tables) of one oracle run; batch_rows > 0 re-slices
    every given batch into RowBatches of that many rows inside the oracle."""
    from google.protobuf import json_format
    lib = load()
    js = json_format.MessageToJson(plan).encode()
    t = _Tables(tables)
    secs = C.c_double()
    out = C.c_void_p()
    n = C.c_int64()
    err = C.create_string_buffer(1024)
    code = lib.oracle_execute_plan_rebatched(js, t.n, t.arr, batch_rows, C.byref(secs), C.byref(out), C.byref(n), err, 1024)
    if code != 0:
        raise OracleError(code, err.value.decode())
    try:
        buf = C.string_at(out.value, n.value)
    finally:
        lib.oracle_free(out)
    return secs.value, parse_pxrb(buf)


def time_plan(plan, tables: Dict[str, dict], batch_rows: int = 0):
    """Execution-window seconds of the plan (first GenerateNext .. last emit).  batch_rows > 0
    re-slices every given batch into RowBatches of that many rows inside the oracle."""
    from google.protobuf import json_format
    lib = load()
    js = json_format.MessageToJson(plan).encode()
    t = _Tables(tables)
    secs = C.c_double()
    rows = C.c_int64()
    err = C.create_string_buffer(1024)
    code = lib.oracle_execute_plan_timed_rebatched(js, t.n, t.arr, batch_rows, C.byref(secs), C.byref(rows), err, 1024)
    if code != 0:
        raise OracleError(code, err.value.decode())
    return secs.value, rows.value


def tdigest_quantiles(vals: Sequence[float]) -> List[float]:
    lib = load()
    a = np.ascontiguousarray(np.array(vals, dtype=np.float64))
    out = (C.c_double * 7)()
    lib.oracle_tdigest_quantiles(a.ctypes.data_as(C.POINTER(C.c_double)), len(a), out)
    return list(out)


def tdigest_merge_quantiles(a_vals, b_vals) -> List[float]:
    lib = load()
    a = np.ascontiguousarray(np.array(a_vals, dtype=np.float64))
    b = np.ascontiguousarray(np.array(b_vals, dtype=np.float64))
    out = (C.c_double * 7)()
    lib.oracle_tdigest_merge_quantiles(a.ctypes.data_as(C.POINTER(C.c_double)), len(a),
                                       b.ctypes.data_as(C.POINTER(C.c_double)), len(b), out)
    return list(out)


def tdigest_centroids(vals, cap: int = 8192):
    """TDigest::FromValuesOnce(vals): the single-pass digest a rank ships (means, weights)."""
    lib = load()
    a = np.ascontiguousarray(np.asarray(vals, dtype=np.float64))
    m = np.zeros(cap, np.float64)
    w = np.zeros(cap, np.float64)
    nc = C.c_int64()
    lib.oracle_tdigest_centroids(a.ctypes.data_as(C.POINTER(C.c_double)), len(a), m.ctypes.data_as(C.POINTER(C.c_double)),
                                 w.ctypes.data_as(C.POINTER(C.c_double)), cap, C.byref(nc))
    assert nc.value >= 0
    return m[:nc.value].copy(), w[:nc.value].copy()


def tdigest_batch_quantiles(parts, extremes=None) -> List[float]:
    """TDigest::merge_batch over parts = [("raw", values) | ("centroids", (means, weights))], then
    quantile() x7.  extremes: per part (true_min, true_max) carried with a centroid list into the
    merged digest (oracle_tdigest_batch_quantiles_mm), None = min / max from the centroid means."""
    lib = load()
    kinds, counts, data, weights = [], [], [], []
    for kind, payload in parts:
        if kind == "raw":
            v = np.asarray(payload, np.float64)
            kinds.append(0)
            counts.append(len(v))
            data.append(v)
            weights.append(np.zeros(len(v)))
        else:
            m, w = payload
            kinds.append(1)
            counts.append(len(m))
            data.append(np.asarray(m, np.float64))
            weights.append(np.asarray(w, np.float64))
    k = np.asarray(kinds, np.int32)
    c = np.asarray(counts, np.int64)
    d = np.ascontiguousarray(np.concatenate(data) if data else np.zeros(0))
    w = np.ascontiguousarray(np.concatenate(weights) if weights else np.zeros(0))
    out = (C.c_double * 7)()
    if extremes is not None:
        lo = np.ascontiguousarray([e[0] if e else np.inf for e in extremes], np.float64)
        hi = np.ascontiguousarray([e[1] if e else -np.inf for e in extremes], np.float64)
        lib.oracle_tdigest_batch_quantiles_mm(len(k), k.ctypes.data_as(C.POINTER(C.c_int32)), c.ctypes.data_as(C.POINTER(C.c_int64)),
                                              d.ctypes.data_as(C.POINTER(C.c_double)), w.ctypes.data_as(C.POINTER(C.c_double)),
                                              lo.ctypes.data_as(C.POINTER(C.c_double)), hi.ctypes.data_as(C.POINTER(C.c_double)), out)
        return list(out)
    lib.oracle_tdigest_batch_quantiles(len(k), k.ctypes.data_as(C.POINTER(C.c_int32)), c.ctypes.data_as(C.POINTER(C.c_int64)),
                                       d.ctypes.data_as(C.POINTER(C.c_double)), w.ctypes.data_as(C.POINTER(C.c_double)), out)
    return list(out)


def quantiles_json(vals) -> str:
    lib = load()
    a = np.ascontiguousarray(np.array(vals, dtype=np.float64))
    buf = C.create_string_buffer(1024)
    lib.oracle_quantiles_json(a.ctypes.data_as(C.POINTER(C.c_double)), len(a), buf, 1024)
    return buf.value.decode()


def pluck_float64(js: str, key: str) -> float:
    return load().oracle_pluck_float64(js.encode(), key.encode())
