"""Thin Python handles over the libpxg C ABI (contexts, HBM tables, aggregations).

Columns are numpy arrays in Arrow layout:
  INT64/TIME64NS: int64[n]; FLOAT64: float64[n]; BOOLEAN: uint8[n];
  UINT128: uint64[n, 2] as (low, high); STRING: (int32 offsets[n+1], uint8 data[...]).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import (BOOLEAN, FLOAT64, INT64, STRING, TIME64NS, UINT128, AggSpec, ColumnOut,
                   ColumnView, check, load)

_NP = {INT64: np.int64, TIME64NS: np.int64, FLOAT64: np.float64, BOOLEAN: np.uint8}


@dataclass
class Column:
    """One Arrow-layout column (one RowBatch column, or a whole table column)."""
    type: int
    values: Optional[np.ndarray] = None
    offsets: Optional[np.ndarray] = None
    data: Optional[np.ndarray] = None

    def __len__(self) -> int:
        if self.type == STRING:
            return int(len(self.offsets) - 1)
        return int(self.values.shape[0])

    @staticmethod
    def from_values(type_: int, vals: Sequence) -> "Column":
        if type_ == STRING:
            bs = [v.encode() if isinstance(v, str) else bytes(v) for v in vals]
            offs = np.zeros(len(bs) + 1, dtype=np.int32)
            if bs:
                offs[1:] = np.cumsum([len(b) for b in bs])
            data = np.frombuffer(b"".join(bs) + b"\0" * 16, dtype=np.uint8).copy()
            return Column(STRING, offsets=offs, data=data)
        if type_ == UINT128:
            arr = np.array([[int(v) & (2**64 - 1), int(v) >> 64] for v in vals], dtype=np.uint64).reshape(-1, 2)
            return Column(UINT128, values=arr)
        return Column(type_, values=np.ascontiguousarray(np.array(vals, dtype=_NP[type_])))

    def to_list(self) -> list:
        if self.type == STRING:
            raw = self.data.tobytes()
            o = self.offsets
            return [raw[o[i]:o[i + 1]].decode(errors="surrogateescape") for i in range(len(o) - 1)]
        if self.type == UINT128:
            return [int(lo) | (int(hi) << 64) for lo, hi in self.values]
        if self.type == BOOLEAN:
            return [bool(x) for x in self.values]
        return self.values.tolist()

    def slice(self, a: int, b: int) -> "Column":
        if self.type == STRING:
            o = self.offsets[a:b + 1]
            data = self.data[o[0]:o[-1]]
            return Column(STRING, offsets=(o - o[0]).astype(np.int32), data=np.concatenate([data, np.zeros(16, np.uint8)]))
        return Column(self.type, values=self.values[a:b])

    def view(self) -> ColumnView:
        v = ColumnView()
        v.type = self.type
        v.length = len(self)
        if self.type == STRING:
            v.offsets = self.offsets.ctypes.data
            v.data = self.data.ctypes.data
        else:
            v.values = self.values.ctypes.data
        return v


def column_from_out(o: ColumnOut, per_row: int = 1) -> Column:
    """Copy a library-owned output column into numpy (caller frees the ColumnOut)."""
    n = int(o.length)
    t = int(o.type)
    if t == STRING:
        offs = np.ctypeslib.as_array(C.cast(o.offsets, C.POINTER(C.c_int32)), shape=(n + 1,)).copy()
        nb = int(o.data_len)
        data = (np.ctypeslib.as_array(C.cast(o.data, C.POINTER(C.c_uint8)), shape=(nb,)).copy()
                if nb > 0 else np.zeros(0, np.uint8))
        return Column(STRING, offsets=offs, data=np.concatenate([data, np.zeros(16, np.uint8)]))
    if t == UINT128:
        vals = np.ctypeslib.as_array(C.cast(o.values, C.POINTER(C.c_uint64)), shape=(n * 2,)).copy().reshape(n, 2)
        return Column(UINT128, values=vals)
    ct = {INT64: C.c_int64, TIME64NS: C.c_int64, FLOAT64: C.c_double, BOOLEAN: C.c_uint8}[t]
    cnt = n * per_row
    if cnt == 0:
        return Column(t, values=np.zeros(0, dtype=_NP[t]))
    arr = np.ctypeslib.as_array(C.cast(o.values, C.POINTER(ct)), shape=(cnt,)).copy()
    if per_row > 1:
        arr = arr.reshape(n, per_row)
    return Column(t, values=arr)


class Ctx:
    def __init__(self, device: int = 0, handle=None):
        """A new device context, or (handle given) a non-owning view of an existing pxg_ctx,
        e.g. the one a pxc_engine owns."""
        self.device = device
        lib = load()
        self.owned = handle is None
        if handle is None:
            h = C.c_void_p()
            check(lib.pxg_ctx_create(device, C.byref(h)))
        else:
            h = C.c_void_p(handle)
        self.h = h
        self.lib = lib

    def sync(self) -> None:
        check(self.lib.pxg_ctx_sync(self.h))

    def set_profiling(self, on: bool, only: str = None) -> None:
        """Time kernel launches with HIP events on the ctx stream (only: one kernel name)."""
        check(self.lib.pxg_ctx_profile_only(self.h, only.encode() if only else None))
        check(self.lib.pxg_ctx_set_profiling(self.h, 1 if on else 0))

    def kernel_stats(self, name: str):
        n = C.c_int64()
        ms = C.c_double()
        check(self.lib.pxg_ctx_kernel_stats(self.h, name.encode(), C.byref(n), C.byref(ms)))
        return int(n.value), float(ms.value)

    def reset_stats(self) -> None:
        check(self.lib.pxg_ctx_reset_stats(self.h))

    def close(self) -> None:
        if self.h and self.owned:
            self.lib.pxg_ctx_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Table:
    """HBM-resident table (pxg_table)."""

    def __init__(self, ctx: Ctx, types: Sequence[int], handle=None, owned: bool = True):
        self.ctx = ctx
        self.types = list(types)
        self.lib = ctx.lib
        self.owned = owned or handle is None
        if handle is None:
            h = C.c_void_p()
            arr = (C.c_int32 * len(types))(*types)
            check(self.lib.pxg_table_create(ctx.h, len(types), arr, C.byref(h)))
            self.h = h
        else:
            self.h = handle

    def append(self, cols: Sequence[Column]) -> None:
        n = len(cols[0]) if cols else 0
        views = (ColumnView * len(cols))(*[c.view() for c in cols])
        self._keep = cols
        check(self.lib.pxg_table_append(self.h, views, n))

    def append_device(self, views: Sequence[ColumnView], n: int) -> None:
        arr = (ColumnView * len(views))(*views)
        check(self.lib.pxg_table_append_device(self.h, arr, n))

    def flush(self) -> None:
        check(self.lib.pxg_table_flush(self.h))

    def append_http_events(self, seed: int, row_begin: int, nrows: int, n_pair_keys: int = 10_000_000) -> None:
        """Generate http_events rows on the device straight into this table (bit-identical to
        datagen_http_events)."""
        check(self.lib.pxg_table_append_http_events(self.h, seed, row_begin, nrows, n_pair_keys))

    @property
    def num_rows(self) -> int:
        return int(self.lib.pxg_table_num_rows(self.h))

    @property
    def num_chunks(self) -> int:
        return int(self.lib.pxg_table_num_chunks(self.h))

    def device_bytes(self, col: int) -> int:
        return int(self.lib.pxg_table_device_bytes(self.h, col))

    def fetch(self, col: int, begin: int = 0, end: Optional[int] = None) -> Column:
        end = self.num_rows if end is None else end
        o = ColumnOut()
        check(self.lib.pxg_table_fetch(self.h, col, begin, end, C.byref(o)))
        try:
            return column_from_out(o)
        finally:
            self.lib.pxg_result_free(C.byref(o), 1)

    def fetch_all(self) -> List[Column]:
        return [self.fetch(i) for i in range(len(self.types))]

    def filter(self, pred, select: Sequence[int], begin: int = 0, end: Optional[int] = None) -> "Table":
        end = self.num_rows if end is None else end
        h = C.c_void_p()
        sel = (C.c_int32 * max(1, len(select)))(*select)
        check(self.lib.pxg_filter(self.h, C.byref(pred.c), len(select), sel, begin, end, C.byref(h)))
        return Table(self.ctx, [self.types[i] for i in select], handle=h)

    def map(self, progs, begin: int = 0, end: Optional[int] = None) -> "Table":
        end = self.num_rows if end is None else end
        h = C.c_void_p()
        arr = (_lib.Program * max(1, len(progs)))(*[p.c for p in progs])
        check(self.lib.pxg_map(self.h, len(progs), arr, begin, end, C.byref(h)))
        return Table(self.ctx, [p.result_type for p in progs], handle=h)

    def join(self, probe: "Table", build_keys: Sequence[int], probe_keys: Sequence[int],
             outputs: Sequence[Tuple[int, int]], emit_unmatched_probe: bool = False,
             emit_unmatched_build: bool = False) -> Tuple["Table", int]:
        """pxg_join with this table as the build side.  outputs: (side, col), side 0 = probe,
        1 = build.  Returns (output table, rows produced by probe rows)."""
        n = len(build_keys)
        i32a = lambda xs: (C.c_int32 * max(1, len(xs)))(*xs)  # noqa: E731
        bk, pk = i32a(build_keys), i32a(probe_keys)
        side, col = i32a([o[0] for o in outputs]), i32a([o[1] for o in outputs])
        spec = _lib.JoinSpec(n, int(emit_unmatched_probe), int(emit_unmatched_build), len(outputs), bk, pk, side, col)
        h = C.c_void_p()
        nprobe = C.c_int64()
        check(self.lib.pxg_join(self.h, probe.h, C.byref(spec), C.byref(h), C.byref(nprobe)))
        types = [probe.types[c] if s == 0 else self.types[c] for s, c in outputs]
        return Table(self.ctx, types, handle=h), nprobe.value

    def close(self) -> None:
        # A table outliving its context (a test that failed before closing it) is not freed:
        # the context's device state is gone by then.
        if self.h and self.owned and getattr(self.ctx, "h", None):
            self.lib.pxg_table_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class _KindOnly:
    kind: int


class Agg:
    """pxg_agg: blocking (or windowed) group-by aggregation with device UDAs."""

    def __init__(self, ctx: Ctx, keys, udas, filt=None, expected_groups: int = 0, windowed: bool = False):
        self.ctx = ctx
        self.lib = ctx.lib
        self.keys = list(keys)
        self.udas = list(udas)
        self.filt = filt
        spec = AggSpec()
        spec.n_keys = len(self.keys)
        spec.n_udas = len(self.udas)
        self._karr = (_lib.Program * max(1, len(self.keys)))(*[k.c for k in self.keys])
        self._uarr = (_lib.UdaSpec * max(1, len(self.udas)))(*[u.c for u in self.udas])
        spec.keys = self._karr
        spec.udas = self._uarr
        spec.filter = C.pointer(filt.c) if filt is not None else None
        spec.expected_groups = expected_groups
        spec.windowed = 1 if windowed else 0
        h = C.c_void_p()
        check(self.lib.pxg_agg_create(ctx.h, C.byref(spec), C.byref(h)))
        self.h = h

    @classmethod
    def from_handle(cls, ctx: Ctx, handle, n_keys: int, uda_kinds) -> "Agg":
        """Wrap a pxg_agg created elsewhere (e.g. the engine's lowering, pxc_plan_create_agg)."""
        a = cls.__new__(cls)
        a.ctx, a.lib, a.h = ctx, ctx.lib, handle
        a.keys = [None] * n_keys
        a.udas = [_KindOnly(k) for k in uda_kinds]
        a.filt = None
        return a

    def consume(self, table: Table, begin: int = 0, end: Optional[int] = None) -> None:
        end = table.num_rows if end is None else end
        check(self.lib.pxg_agg_consume(self.h, table.h, begin, end))

    def finalize(self) -> int:
        n = C.c_int64()
        check(self.lib.pxg_agg_finalize(self.h, C.byref(n)))
        return int(n.value)

    def result(self) -> List[Column]:
        ncols = len(self.keys) + len(self.udas)
        outs = (ColumnOut * ncols)()
        check(self.lib.pxg_agg_result(self.h, outs, ncols))
        try:
            cols = [column_from_out(outs[i]) for i in range(len(self.keys))]
            for j, u in enumerate(self.udas):
                cols.append(column_from_out(outs[len(self.keys) + j], per_row=7 if u.kind == _lib.UDA_QUANTILES else 1))
            return cols
        finally:
            self.lib.pxg_result_free(outs, ncols)

    def reset(self) -> None:
        check(self.lib.pxg_agg_reset(self.h))

    # -- partial aggregation (PEM partial -> exchange by key hash -> Kelvin finalize) --------
    @property
    def device(self) -> str:
        return f"cuda:{self.ctx.device}"

    def export_partial(self, n_parts: int, dst=None):
        """Partition this agg's groups (and their staged values) by hash(key) % n_parts.
        With dst=None only sizes; otherwise dst is a uint8 device tensor (on this agg's GPU)
        of at least sum(aligned sizes) bytes.  Returns (part_offsets, part_bytes)."""
        offs = (C.c_int64 * n_parts)()
        nb = (C.c_int64 * n_parts)()
        ptr, cap = (None, 0) if dst is None else (C.c_void_p(dst.data_ptr()), dst.numel())
        check(self.lib.pxg_agg_export_partial(self.h, n_parts, ptr, cap, offs, nb))
        return list(offs), list(nb)

    def export_partial_dev(self, n_parts: int):
        """The export pxg_agg_alltoall sends, laid out on the device (pxg_agg_export_partial_dev):
        returns (device address of the parts, part byte counts, n_parts * 64 header bytes)."""
        ptr = C.c_void_p()
        nb = (C.c_int64 * n_parts)()
        hdr = (C.c_uint8 * (64 * n_parts))()
        check(self.lib.pxg_agg_export_partial_dev(self.h, n_parts, C.byref(ptr), nb, hdr))
        return int(ptr.value or 0), list(nb), bytes(hdr)

    def import_partial(self, src) -> None:
        """Merge one exported part (a contiguous uint8 device tensor) into this agg."""
        check(self.lib.pxg_agg_import_partial(self.h, C.c_void_p(src.data_ptr()), src.numel()))

    def info(self) -> dict:
        """pxg_agg_info: device-state sizes (table capacity, groups, staged rows, ...)."""
        st = _lib.AggStats()
        check(self.lib.pxg_agg_info(self.h, C.byref(st)))
        return {f: int(getattr(st, f)) for f, _ in st._fields_ if f != "reserved"}

    def import_partials(self, buf, offsets, sizes) -> None:
        """Merge several exported parts lying in one uint8 device tensor (pxg_agg_import_partials)."""
        n = len(offsets)
        o = (C.c_int64 * max(n, 1))(*offsets)
        z = (C.c_int64 * max(n, 1))(*sizes)
        check(self.lib.pxg_agg_import_partials(self.h, C.c_void_p(buf.data_ptr()), n, o, z))

    def rows_selected(self) -> int:
        n = C.c_int64()
        check(self.lib.pxg_agg_rows_selected(self.h, C.byref(n)))
        return int(n.value)

    def alltoall(self, comm: "Comm") -> Tuple[int, int]:
        """Re-partition this agg's state across the communicator's ranks by group-key hash over
        RCCL (pxg_agg_alltoall).  Collective.  Returns (bytes sent, bytes received)."""
        s, r = C.c_int64(), C.c_int64()
        check(self.lib.pxg_agg_alltoall(self.h, comm.h, C.byref(s), C.byref(r)))
        return int(s.value), int(r.value)

    def gather(self, comm: "Comm", root: int = 0) -> int:
        """Every rank's finalized rows to `root` over RCCL (pxg_agg_gather; after alltoall +
        finalize on every rank).  Collective.  Returns the gathered groups on the root, 0 elsewhere;
        the root's result() is then the whole result."""
        g = C.c_int64()
        check(self.lib.pxg_agg_gather(self.h, comm.h, root, C.byref(g)))
        return int(g.value)

    def close(self) -> None:
        if self.h and getattr(self.ctx, "h", None):
            self.lib.pxg_agg_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def datagen_http_events(seed: int, row_begin: int, nrows: int, n_pair_keys: int = 10_000_000,
                        threads: int = 8) -> List[Column]:
    """Synthetic http_events rows [row_begin, row_begin+nrows) (see include/pxg.h)."""
    lib = load()
    outs = (ColumnOut * _lib.HTTP_EVENTS_NCOLS)()
    code = lib.pxg_datagen_http_events(seed, row_begin, nrows, n_pair_keys, threads, outs)
    try:
        check(code)
        return [column_from_out(outs[i]) for i in range(_lib.HTTP_EVENTS_NCOLS)]
    finally:
        lib.pxg_result_free(outs, _lib.HTTP_EVENTS_NCOLS)


HTTP_EVENTS_SCHEMA = [("time_", TIME64NS), ("upid", UINT128), ("service", STRING), ("req_path", STRING),
                      ("remote_addr", STRING), ("resp_status", INT64), ("latency", INT64),
                      ("req_body_size", INT64), ("resp_body_size", INT64), ("pod", STRING)]


class Comm:
    """Communicator of libpxg (pxg_comm_*) over the ctx's device: RCCL (one rank per GPU), or
    with Comm.host() a caller-supplied byte mover (pxg_comm_init_host) that runs the same device
    exchange code with the bytes staged through host memory."""
    ID_BYTES = 128
    _transport = None

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * Comm.ID_BYTES)()
        check(load().pxg_comm_unique_id(buf, Comm.ID_BYTES))
        return bytes(buf)

    def __init__(self, ctx: "Ctx", rank: int, nranks: int, uid: bytes):
        self.lib = load()
        buf = (C.c_uint8 * Comm.ID_BYTES).from_buffer_copy(uid[:Comm.ID_BYTES])
        h = C.c_void_p()
        check(self.lib.pxg_comm_init(ctx.h, rank, nranks, buf, Comm.ID_BYTES, C.byref(h)))
        self.h = h
        self.rank, self.nranks = rank, nranks

    @classmethod
    def host(cls, ctx: "Ctx", rank: int, nranks: int, transport) -> "Comm":
        """A communicator whose bytes move through `transport(ops) -> None` (a list of
        (peer, is_send, memoryview) transfers, matched per peer in order; e.g.
        pixie_amd.dist.GlooTransport).  pxg_agg_alltoall / pxg_agg_gather keep their device
        code; only the byte mover differs from the RCCL communicator."""
        self = cls.__new__(cls)
        self.lib = load()

        def fn(_user, n, ops):
            try:
                batch = []
                for i in range(n):
                    o = ops[i]
                    buf = (C.c_uint8 * o.bytes).from_address(o.buf)
                    batch.append((int(o.peer), bool(o.send), memoryview(buf).cast("B")))
                transport(batch)
                return 0
            except Exception:  # reported to libpxg as a failed transfer batch
                import traceback
                traceback.print_exc()
                return 1

        self._transport = _lib.XferFn(fn)  # kept alive as long as the communicator
        h = C.c_void_p()
        check(self.lib.pxg_comm_init_host(ctx.h, rank, nranks, self._transport, None, C.byref(h)))
        self.h = h
        self.rank, self.nranks = rank, nranks
        return self

    def close(self) -> None:
        if self.h:
            self.lib.pxg_comm_destroy(self.h)
            self.h = None
