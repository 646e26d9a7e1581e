"""ctypes binding of libpxcarnot.so (include/pxcarnot.h): the C++ host engine that runs a
binary planpb.Plan through the GPU ExecNode graph.  Plumbing only; the engine is C++."""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict

import numpy as np

from . import _lib
from ._lib import ColumnView
from .pxrb import parse_pxrb

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libpxcarnot.so")


class PxcTable(C.Structure):
    _fields_ = [("name", C.c_char_p), ("ncols", C.c_int32), ("nbatches", C.c_int32),
                ("col_types", C.POINTER(C.c_int32)), ("cols", C.POINTER(ColumnView)), ("batch_flags", C.c_void_p)]


_lib_h = None


def load() -> C.CDLL:
    global _lib_h
    if _lib_h is not None:
        return _lib_h
    _lib.load()  # libpxg first (one HIP runtime in the process)
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C pixie_amd`")
    lib = C.CDLL(LIB_PATH)
    vp, i32, i64, p = C.c_void_p, C.c_int32, C.c_int64, C.POINTER
    lib.pxc_engine_create.argtypes = [i32, p(vp)]
    lib.pxc_engine_create.restype = i32
    lib.pxc_engine_destroy.argtypes = [vp]
    lib.pxc_engine_destroy.restype = i32
    lib.pxc_execute_plan.argtypes = [vp, C.c_char_p, i64, i32, p(PxcTable), p(vp), p(i64)]
    lib.pxc_execute_plan.restype = i32
    lib.pxc_explain_plan.argtypes = [C.c_char_p, i64, i32, p(PxcTable), p(vp)]
    lib.pxc_explain_plan.restype = i32
    lib.pxc_engine_explain_plan.argtypes = [vp, C.c_char_p, i64, i32, p(PxcTable), p(vp)]
    lib.pxc_engine_explain_plan.restype = i32
    lib.pxc_store_create_table.argtypes = [vp, C.c_char_p, i32, p(i32), p(C.c_char_p)]
    lib.pxc_store_create_table.restype = i32
    lib.pxc_store_append.argtypes = [vp, C.c_char_p, p(ColumnView), i64]
    lib.pxc_store_append.restype = i32
    lib.pxc_store_drop_table.argtypes = [vp, C.c_char_p]
    lib.pxc_store_drop_table.restype = i32
    lib.pxc_store_num_rows.argtypes = [vp, C.c_char_p]
    lib.pxc_store_num_rows.restype = i64
    lib.pxc_store_device_table.argtypes = [vp, C.c_char_p]
    lib.pxc_store_device_table.restype = vp
    lib.pxc_engine_ctx.argtypes = [vp]
    lib.pxc_engine_ctx.restype = vp
    lib.pxc_free.argtypes = [vp]
    lib.pxc_free.restype = None
    lib.pxc_last_error.argtypes = []
    lib.pxc_last_error.restype = C.c_char_p
    _lib_h = lib
    return lib


class PxcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"pxc error {code}: {msg}")
        self.code = code


def _check(code: int) -> None:
    if code != 0:
        raise PxcError(code, load().pxc_last_error().decode())


class _Tables:
    """name -> {types, batches, flags?}; keeps every buffer alive for one call."""

    def __init__(self, tables: Dict[str, dict]):
        self.keep = []
        arr = (PxcTable * max(1, len(tables)))()
        for ti, (name, t) in enumerate(tables.items()):
            types = t["types"]
            batches = t["batches"]
            views = (ColumnView * max(1, len(batches) * len(types)))()
            for b, batch in enumerate(batches):
                for c, col in enumerate(batch):
                    v = ColumnView()
                    v.type = col.type
                    v.length = len(col)
                    if col.type == _lib.STRING:
                        v.offsets = col.offsets.ctypes.data
                        v.data = col.data.ctypes.data
                    else:
                        v.values = col.values.ctypes.data
                    views[b * len(types) + c] = v
                    self.keep.append(col)
            ty = (C.c_int32 * len(types))(*types)
            bname = name.encode()
            flags = None
            if t.get("flags") is not None:
                fl = np.array([(1 if eow else 0) | (2 if eos else 0) for eow, eos in t["flags"]], dtype=np.uint8)
                self.keep.append(fl)
                flags = fl.ctypes.data
            self.keep += [views, ty, bname]
            arr[ti] = PxcTable(bname, len(types), len(batches), ty, views, flags)
        self.arr = arr
        self.n = len(tables)


def explain(plan, tables: Dict[str, dict]) -> str:
    """Lowering only (no device): the node graph the operator switch builds."""
    lib = load()
    pb = plan.SerializeToString()
    t = _Tables(tables)
    out = C.c_void_p()
    _check(lib.pxc_explain_plan(pb, len(pb), t.n, t.arr, C.byref(out)))
    try:
        return C.string_at(out.value).decode()
    finally:
        lib.pxc_free(out)


class Engine:
    def __init__(self, device: int = 0):
        self.lib = load()
        self.h = C.c_void_p()
        _check(self.lib.pxc_engine_create(device, C.byref(self.h)))

    def ctx_handle(self) -> int:
        return int(self.lib.pxc_engine_ctx(self.h))

    def execute_raw(self, pb: bytes, tables: Dict[str, dict] = None) -> bytes:
        """pxc_execute_plan on serialized plan bytes; returns the PXRB result bytes."""
        t = _Tables(tables or {})
        out = C.c_void_p()
        n = C.c_int64()
        _check(self.lib.pxc_execute_plan(self.h, pb, len(pb), t.n, t.arr, C.byref(out), C.byref(n)))
        try:
            return C.string_at(out.value, n.value)
        finally:
            self.lib.pxc_free(out)

    def execute(self, plan, tables: Dict[str, dict] = None):
        """Run the plan's first fragment; returns {sink: [{'rows','eow','eos','cols'}]}."""
        pb = plan.SerializeToString()
        t = _Tables(tables or {})
        out = C.c_void_p()
        n = C.c_int64()
        _check(self.lib.pxc_execute_plan(self.h, pb, len(pb), t.n, t.arr, C.byref(out), C.byref(n)))
        try:
            buf = C.string_at(out.value, n.value)
        finally:
            self.lib.pxc_free(out)
        return parse_pxrb(buf)

    def explain(self, plan, tables: Dict[str, dict] = None) -> str:
        """Lowering with the engine's stored tables visible (no execution)."""
        pb = plan.SerializeToString()
        t = _Tables(tables or {})
        out = C.c_void_p()
        _check(self.lib.pxc_engine_explain_plan(self.h, pb, len(pb), t.n, t.arr, C.byref(out)))
        try:
            return C.string_at(out.value).decode()
        finally:
            self.lib.pxc_free(out)

    # HBM-resident table store (pxc_store_*).
    def create_table(self, name: str, types, names) -> None:
        ty = (C.c_int32 * len(types))(*types)
        nm = (C.c_char_p * len(names))(*[n.encode() for n in names])
        _check(self.lib.pxc_store_create_table(self.h, name.encode(), len(types), ty, nm))

    def append(self, name: str, cols) -> None:
        """Append one host RowBatch (a list of pixie_amd.device.Column) to a stored table."""
        views = (ColumnView * max(1, len(cols)))(*[c.view() for c in cols])
        _check(self.lib.pxc_store_append(self.h, name.encode(), views, len(cols[0]) if cols else 0))

    def drop_table(self, name: str) -> None:
        _check(self.lib.pxc_store_drop_table(self.h, name.encode()))

    def num_rows(self, name: str) -> int:
        return int(self.lib.pxc_store_num_rows(self.h, name.encode()))

    def device_table(self, name: str):
        return self.lib.pxc_store_device_table(self.h, name.encode())

    def close(self) -> None:
        if self.h:
            self.lib.pxc_engine_destroy(self.h)
            self.h = C.c_void_p()
