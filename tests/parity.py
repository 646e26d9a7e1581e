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


# ---------------------------------------------------------------------------------------------
# Ground truth straight from the generator (oracle/http_events_truth.cc) for the C2 shape at the
# 1B-row north_star size, where the row-at-a-time restatement cannot hold the table.
# ---------------------------------------------------------------------------------------------
def http_events_key_tables():
    """(service strings, path strings) of the synthetic generator, as bytes, by index."""
    lib = oc.load()
    lib.oracle_http_events_tables.restype = None
    sb = C.create_string_buffer(64 * 16)
    so = (C.c_int32 * 65)()
    pb = C.create_string_buffer(1024 * 48)
    po = (C.c_int32 * 1025)()
    lib.oracle_http_events_tables(sb, so, pb, po)
    svc = [sb.raw[so[k]:so[k + 1]] for k in range(64)]
    paths = [pb.raw[po[k]:po[k + 1]] for k in range(1024)]
    return svc, paths


def c2_truth(seed: int, row0: int, n: int, collect: Optional[np.ndarray] = None, n_pair_keys: int = 10_000_000,
             threads: int = 16, status_min: int = 400):
    """Per (service index, canonical path index) group g = s * 1024 + p of rows [row0, row0 + n):
    counts, exact int64 latency sums and (groups flagged in `collect`) the values latency/1e6 in
    row order, as (counts, lat_sum, voff, vals)."""
    lib = oc.load()
    lib.oracle_http_events_c2_truth.restype = C.c_int64
    G = 64 * 1024
    counts = np.zeros(G, np.int64)
    sums = np.zeros(G, np.int64)
    vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    if collect is None:
        r = lib.oracle_http_events_c2_truth(C.c_uint64(seed), C.c_int64(row0), C.c_int64(n), C.c_int64(n_pair_keys),
                                            C.c_int32(threads), C.c_int64(status_min), vp(counts), vp(sums), None, None,
                                            None, C.c_int64(0))
        if r < 0:
            raise RuntimeError("oracle_http_events_c2_truth failed")
        return counts, sums, None, None
    flags = np.ascontiguousarray(collect, dtype=np.uint8)
    voff = np.zeros(G + 1, np.int64)
    cap = int(collect.astype(bool).sum()) and int(n)  # upper bound refined below
    # Capacity: a first counts-only pass would double the scan; size from the flagged groups'
    # expected share instead and retry once with the exact total if it was too small.
    cap = min(cap, max(1 << 20, int(n // 4)))
    for _ in range(2):
        vals = np.empty(max(cap, 1), np.float64)
        r = lib.oracle_http_events_c2_truth(C.c_uint64(seed), C.c_int64(row0), C.c_int64(n), C.c_int64(n_pair_keys),
                                            C.c_int32(threads), C.c_int64(status_min), vp(counts), vp(sums), vp(flags),
                                            vp(voff), vp(vals), C.c_int64(cap))
        if r >= 0:
            return counts, sums, voff, vals[:r]
        cap = int(counts[flags.astype(bool)].sum())
    raise RuntimeError("oracle_http_events_c2_truth: value capacity")


def check_c2_against_truth(dev: Sequence[Column], seed: int, row0: int, n: int, n_big: int = 20, n_small: int = 200,
                           rng_seed: int = 7, threads: int = 16) -> Dict:
    """Full-size parity of a device C2 aggregate (service, req_path, count, mean, quantiles raw 7
    doubles) over generator rows [row0, row0 + n) against generator ground truth:
      * every group's key and count bit-exact (the group set is the set of distinct selected
        (service, req_path) byte strings), so also sum(count) = selected rows;
      * every mean within 1e-6 relative of (exact int64 latency sum) / 1e6 / count, and
        sum(mean * count) within 1e-9 relative of sum(latency) / 1e6;
      * quantiles of the n_big largest groups (millions of values at 1B rows) within the
        midpoint-rank bound of the oracle t-digest fed the group's values in row order
        (TDigest(1000).add per row, math_sketches.h:36-54), and of n_small seeded groups of
        <= 8000 values within 4 ULP of it."""
    t0 = __import__("time").time()
    svc, paths = http_events_key_tables()
    svc_id = {s: i for i, s in enumerate(svc)}
    path_id: Dict[bytes, int] = {}
    for i, p in enumerate(paths):
        path_id.setdefault(p, i)
    rep: Dict = {"rows": n, "groups_dev": len(dev[0])}
    raw = [dev[0].data.tobytes(), dev[1].data.tobytes()]
    offs = [dev[0].offsets, dev[1].offsets]
    G = len(dev[0])
    gid = np.empty(G, np.int64)
    for i in range(G):
        s = raw[0][offs[0][i]:offs[0][i + 1]]
        p = raw[1][offs[1][i]:offs[1][i + 1]]
        if s not in svc_id or p not in path_id:
            rep.update(ok=False, error=f"device group key not in the generator's tables: {s!r}, {p!r}")
            return rep
        gid[i] = svc_id[s] * 1024 + path_id[p]
    if len(np.unique(gid)) != G:
        rep.update(ok=False, error="duplicate device groups")
        return rep
    dcount = np.asarray(dev[2].values, np.int64)
    dmean = np.asarray(dev[3].values, np.float64)
    dq = quantile_matrix(dev[4])
    rng = np.random.default_rng(rng_seed)
    big = np.argsort(-dcount, kind="stable")[:n_big]
    small_pool = np.flatnonzero(dcount <= EXACT_MAX)
    small = rng.choice(small_pool, size=min(n_small, len(small_pool)), replace=False) if len(small_pool) else small_pool
    flags = np.zeros(64 * 1024, np.uint8)
    flags[gid[big]] = 1
    flags[gid[small]] = 1
    counts, sums, voff, vals = c2_truth(seed, row0, n, flags, threads=threads)
    rep["truth_s"] = round(__import__("time").time() - t0, 2)
    tg = np.flatnonzero(counts)
    rep["groups_ref"] = int(len(tg))
    rep["selected_rows_ref"] = int(counts.sum())
    rep["selected_rows_dev"] = int(dcount.sum())
    ok = rep["groups_ref"] == G and np.array_equal(np.sort(gid), tg)
    rep["group_set_exact"] = bool(ok)
    cnt_ok = bool(ok and np.array_equal(dcount, counts[gid]))
    rep["counts_bit_exact"] = cnt_ok
    ok &= cnt_ok
    ref_mean = sums[gid].astype(np.float64) / 1e6 / np.maximum(counts[gid], 1)
    rel = np.abs(dmean - ref_mean) / np.abs(ref_mean)
    rep["mean_max_rel"] = float(rel.max()) if G else 0.0
    ok &= rep["mean_max_rel"] <= 1e-6
    tot_dev = float(np.sum(dmean * dcount))
    tot_ref = float(sums.sum()) / 1e6
    rep["sum_mean_count_rel"] = abs(tot_dev - tot_ref) / tot_ref if tot_ref else 0.0
    ok &= rep["sum_mean_count_rel"] <= 1e-9
    # quantiles
    lib = oc.load()
    max_ulp, worst_excess, big_sizes = 0, -1.0, []
    for i in small:
        g = gid[i]
        v = vals[voff[g]:voff[g] + counts[g]]
        ref = np.zeros(7)
        lib.oracle_tdigest_quantiles(v.ctypes.data_as(C.POINTER(C.c_double)), len(v), ref.ctypes.data_as(C.POINTER(C.c_double)))
        max_ulp = max(max_ulp, int(ulp(dq[i], ref).max()))
    for i in big:
        g = gid[i]
        v = vals[voff[g]:voff[g] + counts[g]]
        big_sizes.append(int(len(v)))
        ref = np.zeros(7)
        lib.oracle_tdigest_quantiles(v.ctypes.data_as(C.POINTER(C.c_double)), len(v), ref.ctypes.data_as(C.POINTER(C.c_double)))
        sv = np.sort(v)
        nn = len(sv)

        def rank(x):
            return (np.searchsorted(sv, x, "left") + np.searchsorted(sv, x, "right")) / (2.0 * nn)
        for j, q in enumerate(QS):
            ex = abs(rank(dq[i][j]) - rank(ref[j])) - rank_bound(q, nn)
            worst_excess = max(worst_excess, float(ex)) if not np.isnan(ex) else float("inf")
    rep["quantiles"] = {"groups_exact": int(len(small)), "max_ulp": max_ulp, "ulp_bar": 4,
                        "groups_rank": int(len(big)), "largest_group": max(big_sizes) if big_sizes else 0,
                        "rank_checked_values": int(sum(big_sizes)), "max_rank_excess": worst_excess,
                        "rank_bar": "2*pi*sqrt(q(1-q))/1000 + 1/n vs the oracle digest fed row order"}
    ok &= max_ulp <= 4 and worst_excess <= 0
    rep["ok"] = bool(ok)
    rep["check_s"] = round(__import__("time").time() - t0, 2)
    return rep
