"""Big-group quantiles by selection (pxg_finalize.hip BigSample..BigSelDigest) against the full
sort + merge path (PXG_BIG_SORT=1) and the CPU restatement, and the per-wave speculative
boundary chain against the sequential one.  Bars: identical digests (bit-exact) for groups
whose centroids all hold <= 16 values (W <= ~10000, incremental means in sorted order on both
paths); 1e-12 relative above that (centroid sums in a different fixed order); groups the
selection path cannot serve (NaN values, heavy duplicates) fall back to the sort path and are
bit-exact again."""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest

import oracle_client as oc
import parity
from device_runner import run_plan
from kat import rows, ulp_diff
from pixie_amd import _lib
from pixie_amd import plans as P
from pixie_amd.device import Column

pytestmark = pytest.mark.gpu
NAMES = ["p01", "p10", "p25", "p50", "p75", "p90", "p99"]
QS = [0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99]


def _chains(ctx, ws, wave, cap=2048):
    import torch
    w = torch.tensor(ws, dtype=torch.int64, device="cuda")
    starts = torch.zeros(len(ws) * cap, dtype=torch.int32, device="cuda")
    nc = torch.zeros(len(ws), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _lib.check(_lib.load().pxg_digest_chains(ctx.h, C.c_void_p(w.data_ptr()), len(ws), wave, C.c_void_p(starts.data_ptr()), cap,
                                             C.c_void_p(nc.data_ptr())))
    return starts.view(len(ws), cap).cpu().numpy(), nc.cpu().numpy()


def test_speculative_chain_matches_sequential(ctx):
    rng = np.random.default_rng(3)
    ws = list(range(1, 4200)) + list(range(7900, 10300, 7)) + [int(x) for x in rng.integers(10_000, 3_000_000, 400)] + \
        [2**20, 2**24 - 1, 123_456_789]
    s_seq, n_seq = _chains(ctx, ws, 0)
    s_wave, n_wave = _chains(ctx, ws, 1)
    assert (n_seq == n_wave).all(), [(w, a, b) for w, a, b in zip(ws, n_seq, n_wave) if a != b][:5]
    for i, n in enumerate(n_seq):
        if n > 0:
            assert (s_seq[i, :n] == s_wave[i, :n]).all(), ws[i]
    # a chain longer than its capacity reports -1 on both builders
    s1, n1 = _chains(ctx, [5000, 50_000], 1, cap=64)
    s0, n0 = _chains(ctx, [5000, 50_000], 0, cap=64)
    assert list(n1) == list(n0) == [-1, -1]


FALLBACK_GROUPS = ("dup", "few", "nan")


def _groups(fallback):
    rng = np.random.default_rng(11)
    spec = [
        ("u4097", rng.uniform(0, 1, 4097)),
        ("l5000", rng.lognormal(2.0, 1.3, 5000)),
        ("n8000", rng.normal(-3, 2, 8000)),
        ("l9999", rng.lognormal(0.5, 0.7, 9999)),
        ("l12000", rng.lognormal(3.0, 0.9, 12_000)),   # (<= 16384 values: the mid LDS-sort classes)
        ("l17000", rng.lognormal(1.2, 0.8, 17_000)),   # the smallest groups the selection path takes
        ("n40000", rng.normal(0, 1e6, 40_000)),
        ("l250000", rng.lognormal(1.6, 1.0, 250_000)),
        ("grid", np.round(rng.lognormal(4, 1, 90_000), 1)),     # many ties
        ("m2000", rng.normal(0, 1, 2000)),
        ("t10", rng.normal(0, 1, 10)),
        # a dense spike inside a huge range: most splitters share a few guide buckets (the
        # guided bin search's wide-bracket steps)
        ("spike", np.concatenate([rng.normal(100, 1e-6, 40_000), rng.uniform(-1e9, 1e9, 300)])),
    ]
    if fallback == "dup":
        spec.append(("dup", np.full(20_000, 7.25)))                          # one value
        spec.append(("few", rng.integers(0, 4, 30_000).astype(np.float64)))  # four values
    elif fallback == "nan":
        spec.append(("nan", np.where(rng.uniform(size=20_000) < 0.01, np.nan, rng.normal(5, 1, 20_000))))
    keys, vals = [], []
    for k, v in spec:
        keys += [k] * len(v)
        vals.append(v)
    vals = np.concatenate(vals)
    perm = rng.permutation(len(keys))
    return [keys[i] for i in perm], vals[perm], {k: len(v) for k, v in spec}


def _run(ctx, keys, vals, force_sort):
    plan = P.linear_plan([P.source_op("t", [5, 4], ["k", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("quantiles", [P.col(1)], [4]), P.agg_expr("count", [P.col(1)], [4], fid=1)]),
                          P.sink_op("out")])
    tables = {"t": {"types": [5, 4], "batches": [[Column.from_values(5, keys), Column(4, values=vals)]]}}
    old = os.environ.get("PXG_BIG_SORT")
    if force_sort:
        os.environ["PXG_BIG_SORT"] = "1"
    else:
        os.environ.pop("PXG_BIG_SORT", None)
    try:
        out = run_plan(ctx, plan, tables)
    finally:
        if old is None:
            os.environ.pop("PXG_BIG_SORT", None)
        else:
            os.environ["PXG_BIG_SORT"] = old
    return plan, tables, {r[0]: (json.loads(r[1]), r[2]) for r in rows(out[0]["cols"])}


@pytest.mark.parametrize("fallback", [None, "dup", "nan"])
def test_selection_path_matches_sort_path(ctx, fallback):
    """The two paths differ only in big-centroid summation order; a fallback group (duplicates
    beyond a bin's capacity, NaN values) is handed to the sort path on its own (one quantile
    UDA), so its results are identical and the others' stay the selection path's."""
    keys, vals, sizes = _groups(fallback)
    _, _, sel = _run(ctx, keys, vals, force_sort=False)
    _, _, srt = _run(ctx, keys, vals, force_sort=True)
    assert set(sel) == set(srt) == set(sizes)
    for k, n in sizes.items():
        qa, ca = sel[k]
        qb, cb = srt[k]
        assert ca == cb == n
        for name in NAMES:
            a, b = qa[name], qb[name]
            if n <= 10_000 or k in FALLBACK_GROUPS:
                assert a == b or (a != a and b != b), (k, name, a, b)
            else:
                assert abs(a - b) <= 1e-12 * max(abs(a), abs(b)), (k, name, a, b)


def test_selection_path_against_restatement(ctx):
    keys, vals, sizes = _groups(None)
    plan, tables, dev = _run(ctx, keys, vals, force_sort=False)
    ref = {r[0]: (json.loads(r[1]), r[2]) for r in rows(oc.execute_plan(plan, tables)["out"][0]["cols"])}
    karr = np.array(keys, dtype=object)
    for k, n in sizes.items():
        rq, dq = ref[k][0], dev[k][0]
        assert ref[k][1] == dev[k][1] == n
        if n <= 8000:
            for name in NAMES:
                assert (rq[name] != rq[name] and dq[name] != dq[name]) or ulp_diff(rq[name], dq[name]) <= 4, (k, name, rq[name], dq[name])
        else:
            s = np.sort(vals[karr == k])
            s = s[~np.isnan(s)]
            for q, name in zip(QS, NAMES):
                bound = 2 * math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / len(s)
                r_dev = (np.searchsorted(s, dq[name], "left") + np.searchsorted(s, dq[name], "right")) / 2 / len(s)
                r_ref = (np.searchsorted(s, rq[name], "left") + np.searchsorted(s, rq[name], "right")) / 2 / len(s)
                assert abs(r_dev - r_ref) <= bound, (k, name, dq[name], rq[name])


def _run_info(ctx, keys, vals, force_sort):
    """Like _run, but through the aggregation handle so its stats are visible."""
    from device_runner import _upload
    from pixie_amd.pipeline import LinearQuery
    plan = P.linear_plan([P.source_op("t", [5, 4], ["k", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("quantiles", [P.col(1)], [4]), P.agg_expr("count", [P.col(1)], [4], fid=1)]),
                          P.sink_op("out")])
    old = os.environ.pop("PXG_BIG_SORT", None)
    if force_sort:
        os.environ["PXG_BIG_SORT"] = "1"
    try:
        q = LinearQuery(plan, [5, 4])
        agg = q.make_agg(ctx)
        kc = keys if isinstance(keys, Column) else Column.from_values(5, keys)
        t = _upload(ctx, [5, 4], [[kc, Column(4, values=vals)]])
        agg.consume(t)
        agg.finalize()
        out = {r[0]: (json.loads(r[1]), r[2]) for r in rows(q.emit(agg.result()))}
        info = agg.info()
        agg.close()
        t.close()
    finally:
        os.environ.pop("PXG_BIG_SORT", None)
        if old is not None:
            os.environ["PXG_BIG_SORT"] = old
    return out, info


def test_selection_serves_multi_million_groups(ctx):
    """Groups of millions of values on a 4096-point grid (the shape of the 1B-row north_star
    table's largest groups: ~6.9M values, latency from a 4096-interval inverse CDF) are served by
    selection — no gathered bin beyond the 16384-key LDS sort — and agree with the sort path."""
    rng = np.random.default_rng(29)
    grid = np.sort(rng.lognormal(3.0, 1.0, 4096))
    spec = [("g7m", grid[rng.integers(0, 4096, 7_000_000)]),
            ("l2m", rng.lognormal(1.0, 0.8, 2_000_000)),
            ("g300k", grid[np.minimum(rng.geometric(0.01, 300_000), 4095)]),
            ("s5000", rng.normal(0, 1, 5000))]
    keys = np.concatenate([np.full(len(v), i) for i, (_, v) in enumerate(spec)])
    vals = np.concatenate([v for _, v in spec])
    perm = rng.permutation(len(keys))
    names = [k for k, _ in spec]
    kp = keys[perm]
    lens = np.array([len(k) for k in names], dtype=np.int32)[kp]
    offs = np.zeros(len(kp) + 1, dtype=np.int32)
    np.cumsum(lens, out=offs[1:])
    pool = np.frombuffer("".join(names).encode(), dtype=np.uint8)
    starts = np.cumsum([0] + [len(k) for k in names])[:-1]
    idx = np.repeat(starts[kp] - offs[:-1], lens) + np.arange(offs[-1])
    keys_s = Column(5, offsets=offs, data=np.ascontiguousarray(pool[idx]))
    vals_p = vals[perm]
    sel, info = _run_info(ctx, keys_s, vals_p, force_sort=False)
    assert info["big_sort_groups"] == 0, info
    srt, info_s = _run_info(ctx, keys_s, vals_p, force_sort=True)
    assert info_s["big_sort_groups"] == 3, info_s  # (s5000 takes the mid LDS-sort class)
    for k, v in spec:
        assert sel[k][1] == srt[k][1] == len(v)
        for name in NAMES:
            a, b = sel[k][0][name], srt[k][0][name]
            assert abs(a - b) <= 1e-12 * max(abs(a), abs(b)), (k, name, a, b)
    # Against the oracle, not only the sort path: each group's values in row order through the
    # restated TDigest(1000) (math_sketches.h:36-54); <= 8000 values 4 ULP, above the rank bound.
    for i, (k, _) in enumerate(spec):
        v = vals_p[kp == i]
        ref = oc.tdigest_quantiles(v)
        sv = np.sort(v)
        for j, name in enumerate(NAMES):
            d = sel[k][0][name]
            if len(v) <= parity.EXACT_MAX:
                assert parity.ulp(np.array([d]), np.array([ref[j]]))[0] <= 4, (k, name, d, ref[j])
            else:
                rank = lambda x: (np.searchsorted(sv, x, "left") + np.searchsorted(sv, x, "right")) / (2.0 * len(sv))  # noqa: E731
                assert abs(rank(d) - rank(ref[j])) <= parity.rank_bound(parity.QS[j], len(sv)), (k, name, d, ref[j])


def test_selection_path_int64_values_match_sort_path(ctx):
    """INT64 quantile arguments (the selection passes are compiled per argument type): the
    selection path against the full sort path on the same integer values."""
    rng = np.random.default_rng(31)
    spec = [("i9000", np.round(rng.lognormal(8, 1, 9000))), ("i60000", np.round(rng.lognormal(6, 2, 60_000))),
            ("neg30000", rng.integers(-10**12, 10**12, 30_000).astype(np.float64)), ("i500", np.arange(500.0))]
    keys = sum(([k] * len(v) for k, v in spec), [])
    vals = np.concatenate([v for _, v in spec]).astype(np.int64)
    perm = rng.permutation(len(keys))
    keys = [keys[i] for i in perm]
    vals = vals[perm]
    plan = P.linear_plan([P.source_op("t", [5, 2], ["k", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("quantiles", [P.col(1)], [2]), P.agg_expr("count", [P.col(1)], [2], fid=1)]),
                          P.sink_op("out")])
    tables = {"t": {"types": [5, 2], "batches": [[Column.from_values(5, keys), Column(2, values=vals)]]}}
    res = {}
    for force in (False, True):
        old = os.environ.pop("PXG_BIG_SORT", None)
        if force:
            os.environ["PXG_BIG_SORT"] = "1"
        try:
            out = run_plan(ctx, plan, tables)
        finally:
            os.environ.pop("PXG_BIG_SORT", None)
            if old is not None:
                os.environ["PXG_BIG_SORT"] = old
        res[force] = {r[0]: (json.loads(r[1]), r[2]) for r in rows(out[0]["cols"])}
    for k, v in spec:
        (qa, ca), (qb, cb) = res[False][k], res[True][k]
        assert ca == cb == len(v)
        for name in NAMES:
            a, b = qa[name], qb[name]
            if len(v) <= 10_000:
                assert a == b, (k, name, a, b)
            else:
                assert abs(a - b) <= 1e-12 * max(abs(a), abs(b)), (k, name, a, b)


@pytest.mark.parametrize("fallback", [None, "nan"])
def test_early_set_matches_late_set(ctx, monkeypatch, fallback):
    """Fused split (forced on, > 256 groups): the designated big groups take the selection path
    as their own early set, started before the rest sort finishes (PXG_EARLY_BIG; off, they are
    class 3 of the classification).  Same values, same kernels: the same quantiles (big groups to
    the last bits of their inside-bin sums), and a fallback group in either set goes to the sort
    path on its own (identical)."""
    keys, vals, sizes = _groups(fallback)
    rng = np.random.default_rng(77)
    small = {f"s{i}": rng.lognormal(1, 1, 100) for i in range(400)}
    keys = keys + [k for k, v in small.items() for _ in v]
    vals = np.concatenate([vals] + list(small.values()))
    sizes.update({k: len(v) for k, v in small.items()})
    monkeypatch.setenv("PXG_FSPLIT", "1")
    monkeypatch.setenv("PXG_EARLY_BIG", "0")
    late, info_l = _run_info(ctx, keys, vals, force_sort=False)
    monkeypatch.setenv("PXG_EARLY_BIG", "1")
    early, info_e = _run_info(ctx, keys, vals, force_sort=False)
    assert set(late) == set(early) == set(sizes)
    assert info_l["big_sort_groups"] == info_e["big_sort_groups"], (info_l, info_e)
    if fallback:
        assert info_e["big_sort_groups"] >= 1
    for k, n in sizes.items():
        assert late[k][1] == early[k][1] == n
        for name in NAMES:
            a, b = late[k][0][name], early[k][0][name]
            if n <= 10_000 or k in FALLBACK_GROUPS:
                assert a == b or (a != a and b != b), (k, name, a, b)
            else:  # (inside-bin sums: atomics, last bits run to run, as in the late set alone)
                assert abs(a - b) <= 1e-12 * max(abs(a), abs(b)), (k, name, a, b)


def test_two_quantile_udas_with_a_fallback_group_sort_every_big_group(ctx):
    """Two quantile UDAs (over the value and its negation) and a fallback group: the selection
    plans keep the last UDA's flags only, so finalize hands every big group to the sort path
    and both UDAs' results equal the forced sort path's exactly."""
    keys, vals, sizes = _groups("dup")
    plan = P.linear_plan([P.source_op("t", [5, 4], ["k", "v"], [0, 1]),
                          P.map_op([P.col(0), P.col(1), P.func("multiply", [P.col(1), P.const(4, -1.0)], [4, 4])], ["k", "v", "w"]),
                          P.agg_op([0], [P.agg_expr("quantiles", [P.col(1)], [4]), P.agg_expr("quantiles", [P.col(2)], [4], fid=1)]),
                          P.sink_op("out")])
    tables = {"t": {"types": [5, 4], "batches": [[Column.from_values(5, keys), Column(4, values=vals)]]}}
    out = {}
    for force in (False, True):
        old = os.environ.pop("PXG_BIG_SORT", None)
        if force:
            os.environ["PXG_BIG_SORT"] = "1"
        try:
            res = run_plan(ctx, plan, tables)
        finally:
            os.environ.pop("PXG_BIG_SORT", None)
            if old is not None:
                os.environ["PXG_BIG_SORT"] = old
        out[force] = {r[0]: (json.loads(r[1]), json.loads(r[2])) for r in rows(res[0]["cols"])}
    assert set(out[False]) == set(out[True]) == set(sizes)
    for k in sizes:
        for j in range(2):
            for name in NAMES:
                a, b = out[False][k][j][name], out[True][k][j][name]
                assert a == b or (a != a and b != b), (k, j, name, a, b)
