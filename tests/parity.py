"""Large-scale aggregate parity: the device result against the CPU Carnot restatement (oracle/)
on the same rows.  TEST INFRASTRUCTURE ONLY (used by tests/ and bench.py's parity leg).

Bars:
  * group set and counts, integer sums: bit-exact;
  * mean, float sum: 1e-6 relative;
  * quantiles of groups with <= 8000 values: <= 4 ULP (the reference digest is one process()
    over the sorted multiset, so it does not depend on row order);
  * quantiles of larger groups: |F(v_dev) - F(v_ref)| <= 2*pi*sqrt(q(1-q))/1000 + 1/n with F the
    group's midpoint empirical CDF (the reference's own result depends on insertion order).

Groups are matched by the exact bytes of their keys (RowTuple equality, row_tuple.h:109-153),
vectorised: every key row becomes one fixed-width byte string, both sides are sorted by it.
"""
from __future__ import annotations

import ctypes as C
import json
import math
from typing import Dict, List, Optional, Sequence

import numpy as np

import oracle_client as oc
from pixie_amd.device import Column

BOOLEAN, INT64, UINT128, FLOAT64, STRING, TIME64NS = 1, 2, 3, 4, 5, 6
QS = [0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99]
QNAMES = ["p01", "p10", "p25", "p50", "p75", "p90", "p99"]
EXACT_MAX = 8000


def rank_bound(q: float, n: int) -> float:
    return 2 * math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / n


def _str_width(c: Column) -> int:
    lens = np.diff(c.offsets)
    return int(lens.max()) if len(lens) else 0


def key_rows(cols: Sequence[Column], widths: Sequence[int]) -> np.ndarray:
    """One void scalar per row: the exact key bytes (STRING: u32 length + bytes zero-padded to
    widths[i]; fixed types: their value bytes)."""
    n = len(cols[0]) if cols else 0
    parts = []
    for c, w in zip(cols, widths):
        if c.type == STRING:
            starts = c.offsets[:-1].astype(np.int64)
            lens = np.diff(c.offsets).astype(np.int64)
            m = np.zeros((n, max(w, 1)), np.uint8)
            for j in range(w):
                s = lens > j
                m[s, j] = c.data[starts[s] + j]
            parts += [lens.astype("<u4").view(np.uint8).reshape(n, 4), m]
        elif c.type == UINT128:
            parts.append(np.ascontiguousarray(c.values, dtype=np.uint64).view(np.uint8).reshape(n, 16))
        elif c.type == BOOLEAN:
            parts.append(np.ascontiguousarray(c.values, dtype=np.uint8).reshape(n, 1))
        else:
            parts.append(np.ascontiguousarray(c.values).view(np.uint8).reshape(n, 8))
    if not parts:
        return np.zeros(n, dtype=np.dtype((np.void, 1)))
    M = np.ascontiguousarray(np.concatenate(parts, axis=1))
    return M.view(np.dtype((np.void, M.shape[1]))).ravel()


def encode_key(cols: Sequence[Column], i: int) -> bytes:
    """The oracle_group_ranks key encoding of row i (STRING: u32 len + bytes; fixed: value bytes)."""
    out = b""
    for c in cols:
        if c.type == STRING:
            a, b = int(c.offsets[i]), int(c.offsets[i + 1])
            out += (b - a).to_bytes(4, "little") + c.data[a:b].tobytes()
        elif c.type == UINT128:
            out += np.ascontiguousarray(c.values[i], dtype=np.uint64).tobytes()
        else:
            out += np.ascontiguousarray(c.values[i:i + 1]).tobytes().ljust(8, b"\0")[:8]
    return out


def ulp(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    ia, ib = a.view(np.int64).copy(), b.view(np.int64).copy()
    m = np.int64(0x7FFFFFFFFFFFFFFF)
    ia = np.where(ia < 0, -(ia & m), ia)
    ib = np.where(ib < 0, -(ib & m), ib)
    d = np.abs(ia - ib)
    both_nan = np.isnan(a) & np.isnan(b)
    return np.where((a == b) | both_nan, 0, d)


def quantile_matrix(col: Column) -> np.ndarray:
    """G x 7 doubles from a device quantiles column (raw 7 doubles per group) or a JSON column."""
    if col.type == STRING:
        out = np.full((len(col), 7), np.nan)
        for g, s in enumerate(col.to_list()):
            try:
                d = json.loads(s)
            except ValueError:
                continue
            out[g] = [float(d.get(k, np.nan)) for k in QNAMES]
        return out
    return np.asarray(col.values, dtype=np.float64).reshape(-1, 7)


class GroupValues:
    """The rows behind the aggregate, for rank checks of large groups: key columns, selection
    mask and the quantiles argument (one table, possibly a list of slices)."""

    def __init__(self, key_cols: List[List[Column]], sel: List[np.ndarray], vals: List[np.ndarray]):
        self.key_cols, self.sel, self.vals = key_cols, sel, vals

    def ranks(self, qkeys: List[bytes], qv: np.ndarray) -> (np.ndarray, np.ndarray):
        lib = oc.load()
        lib.oracle_group_ranks.restype = C.c_int32
        nq = len(qkeys)
        blob = b"".join(qkeys)
        offs = np.zeros(nq + 1, np.int64)
        offs[1:] = np.cumsum([len(k) for k in qkeys])
        bbuf = np.frombuffer(blob + b"\0", np.uint8)
        total_cnt = np.zeros(nq, np.int64)
        # lower/upper counts add over slices: rank = (lo + hi) / 2n; recover lo+hi per slice
        acc = np.zeros(qv.shape, np.float64)
        for kc, s, v in zip(self.key_cols, self.sel, self.vals):
            arr = (oc.OColumn * len(kc))(*[oc._col_struct(c) for c in kc])
            out = np.zeros(qv.shape, np.float64)
            cnt = np.zeros(nq, np.int64)
            sv = np.ascontiguousarray(s, dtype=np.uint8)
            vv = np.ascontiguousarray(v, dtype=np.float64)
            qq = np.ascontiguousarray(qv, dtype=np.float64)
            lib.oracle_group_ranks(arr, len(kc), sv.ctypes.data_as(C.c_void_p), vv.ctypes.data_as(C.c_void_p), len(vv),
                                   nq, bbuf.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p),
                                   qq.ctypes.data_as(C.c_void_p), qv.shape[1], out.ctypes.data_as(C.c_void_p),
                                   cnt.ctypes.data_as(C.c_void_p))
            acc += np.where(cnt[:, None] > 0, np.nan_to_num(out) * 2 * cnt[:, None], 0.0)
            total_cnt += cnt
        with np.errstate(invalid="ignore", divide="ignore"):
            return acc / (2 * np.maximum(total_cnt, 1)[:, None]), total_cnt


def compare_agg(dev: Sequence[Column], ref: Sequence[Column], nkeys: int, kinds: Sequence[str],
                values: Optional[GroupValues] = None, mean_rel: float = 1e-6) -> Dict:
    """Compare one aggregate output (groups, then values) of the device against the oracle.
    kinds[j] per value column: "count" / "exact" (bit-exact), "rel" (1e-6 relative),
    "quantiles" (§ bars above).  Returns a report dict with "ok"."""
    rep: Dict = {"groups_dev": len(dev[0]) if dev else 0, "groups_ref": len(ref[0]) if ref else 0}
    G = rep["groups_ref"]
    rep["ok"] = rep["groups_dev"] == G
    if not rep["ok"]:
        rep["error"] = "group counts differ"
        return rep
    widths = [max(_str_width(d), _str_width(r)) if d.type == STRING else 0 for d, r in zip(dev[:nkeys], ref[:nkeys])]
    kd, kr = key_rows(dev[:nkeys], widths), key_rows(ref[:nkeys], widths)
    od, orf = np.argsort(kd, kind="stable"), np.argsort(kr, kind="stable")
    if not np.array_equal(kd[od], kr[orf]):
        rep["ok"] = False
        rep["error"] = "group key sets differ"
        return rep
    if G and len(np.unique(kr)) != G:
        rep["ok"] = False
        rep["error"] = "duplicate groups"
        return rep
    counts = None
    for j, kind in enumerate(kinds):
        d, r = dev[nkeys + j], ref[nkeys + j]
        name = f"v{j}_{kind}"
        if kind in ("count", "exact"):
            a, b = np.asarray(d.values)[od], np.asarray(r.values)[orf]
            ok = np.array_equal(a.view(np.int64) if a.dtype == np.float64 else a,
                                b.view(np.int64) if b.dtype == np.float64 else b)
            rep[name] = {"bit_exact": bool(ok)}
            if kind == "count":
                counts = b.astype(np.int64)
                rep["rows_in_groups"] = int(counts.sum())
            rep["ok"] &= bool(ok)
        elif kind == "rel":
            a, b = np.asarray(d.values, np.float64)[od], np.asarray(r.values, np.float64)[orf]
            with np.errstate(invalid="ignore", divide="ignore"):
                rel = np.where(a == b, 0.0, np.abs(a - b) / np.abs(b))
            rel = np.where(np.isnan(a) & np.isnan(b), 0.0, rel)
            mx = float(np.nanmax(rel)) if G else 0.0
            if G and np.isnan(rel).any():
                mx = float("inf")
            rep[name] = {"max_rel": mx, "bar": mean_rel}
            rep["ok"] &= mx <= mean_rel
        elif kind == "quantiles":
            qd, qr = quantile_matrix(d)[od], quantile_matrix(r)[orf]
            if counts is None:
                raise ValueError("quantiles parity needs a count column before it")
            small = counts <= EXACT_MAX
            u = ulp(qd[small], qr[small]) if small.any() else np.zeros((0, 7), np.int64)
            q = {"groups_exact": int(small.sum()), "max_ulp": int(u.max()) if u.size else 0, "ulp_bar": 4}
            ok = q["max_ulp"] <= 4
            big = np.flatnonzero(~small)
            q["groups_rank"] = int(len(big))
            if len(big):
                if values is None:
                    raise ValueError("rank checks of groups above 8000 values need the group values")
                keys = [encode_key(ref[:nkeys], int(orf[i])) for i in big]
                both, cnt = values.ranks(keys, np.hstack([qd[big], qr[big]]))
                rd, rr = both[:, :7], both[:, 7:]
                bounds = np.array([[rank_bound(qq, int(n)) for qq in QS] for n in counts[big]])
                excess = np.abs(rd - rr) - bounds
                q["rank_counts_match"] = bool(np.array_equal(cnt, counts[big]))
                q["max_rank_diff"] = float(np.nanmax(np.abs(rd - rr)))
                q["max_rank_excess"] = float(np.nanmax(excess))  # <= 0: inside the bound
                ok &= q["rank_counts_match"] and q["max_rank_excess"] <= 0 and not np.isnan(excess).any()
            q["ok"] = bool(ok)
            rep[name] = q
            rep["ok"] &= bool(ok)
        else:
            raise ValueError(kind)
    rep["ok"] = bool(rep["ok"])
    return rep


def concat_columns(parts: List[List[Column]]) -> List[Column]:
    """Row-wise concatenation of several tables' columns (e.g. every rank's key partition)."""
    out = []
    for j in range(len(parts[0])):
        cs = [p[j] for p in parts]
        t = cs[0].type
        if t == STRING:
            offs, datas, base = [np.zeros(1, np.int64)], [], 0
            for c in cs:
                o = c.offsets.astype(np.int64)
                offs.append(o[1:] - o[0] + base)
                datas.append(c.data[int(o[0]):int(o[-1])])
                base += int(o[-1] - o[0])
            out.append(Column(STRING, offsets=np.concatenate(offs).astype(np.int32),
                              data=np.concatenate(datas + [np.zeros(16, np.uint8)])))
        else:
            out.append(Column(t, values=np.concatenate([np.asarray(c.values) for c in cs])))
    return out


def row_hash64(cols: Sequence[Column], rows: Optional[np.ndarray] = None) -> np.ndarray:
    """A 64-bit hash of each row's exact key bytes (for unique-count properties at scale)."""
    if rows is not None:
        cols = [take_rows(c, rows) for c in cols]
    widths = [_str_width(c) if c.type == STRING else 0 for c in cols]
    M = key_rows(cols, widths).view(np.uint8).reshape(len(cols[0]), -1)
    h = np.full(M.shape[0], np.uint64(0xCBF29CE484222325))
    with np.errstate(over="ignore"):
        for j in range(M.shape[1]):
            h = (h ^ M[:, j].astype(np.uint64)) * np.uint64(0x100000001B3)
            h ^= h >> np.uint64(29)
    return h


def take_rows(c: Column, idx: np.ndarray) -> Column:
    if c.type != STRING:
        return Column(c.type, values=np.ascontiguousarray(np.asarray(c.values)[idx]))
    starts = c.offsets[:-1].astype(np.int64)[idx]
    lens = np.diff(c.offsets).astype(np.int64)[idx]
    offs = np.zeros(len(idx) + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    flat = np.repeat(starts - offs[:-1], lens) + np.arange(int(offs[-1]))
    return Column(STRING, offsets=offs.astype(np.int32), data=np.concatenate([c.data[flat], np.zeros(16, np.uint8)]))
