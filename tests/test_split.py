"""The large-group designation of the fused split (pxg_finalize.hip SplitSampleKernel ..
FsHistKernel): groups a sample says are large get their own bucket in the sort's first pass and
only the rest go through the remaining pass.  The designation decides cost only, never results,
so every case here is checked against the oracle and against the same aggregation finalized with
the plain radix sort (PXG_FSPLIT=0; PXG_FSPLIT=1 forces the fused split at small sizes)."""
import json
import math

import numpy as np
import pytest

import oracle_client as oc
from device_runner import run_plan
from kat import rows, rows_match, ulp_diff
from pixie_amd import plans as P
from pixie_amd.device import Column, datagen_http_events

pytestmark = pytest.mark.gpu
NAMES = ["p01", "p10", "p25", "p50", "p75", "p90", "p99"]
QS = [0.01, 0.10, 0.25, 0.50, 0.75, 0.90, 0.99]


def _by_key(cols, nkeys):
    return {t[:nkeys]: t[nkeys:] for t in rows(cols)}


def _run(ctx, plan, tables, monkeypatch, split):
    monkeypatch.setenv("PXG_FSPLIT", "1" if split else "0")
    return run_plan(ctx, plan, tables)


def test_c2_split_matches_oracle_and_unsplit(ctx, monkeypatch):
    n = 400_000
    cols = datagen_http_events(20250117, 0, n, threads=8)
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}}
    plan = P.c2_plan(with_pluck=False)
    R = _by_key(oc.execute_plan(plan, tables)["output"][0]["cols"], 2)
    S = _by_key(_run(ctx, plan, tables, monkeypatch, True)[0]["cols"], 2)
    U = _by_key(_run(ctx, plan, tables, monkeypatch, False)[0]["cols"], 2)
    assert set(R) == set(S) == set(U)
    sel = cols[5].values >= 400
    svc = np.array(cols[2].to_list(), dtype=object)[sel]
    path = np.array(cols[3].to_list(), dtype=object)[sel]
    lat = cols[6].values[sel] / 1e6
    groups = {}
    for s, p, v in zip(svc, path, lat):
        groups.setdefault((s, p), []).append(v)
    for k in R:
        rc, rm, rq = R[k]
        sc, sm, sq = S[k]
        assert rc == sc == U[k][0], k
        assert abs(rm - sm) <= 1e-6 * abs(rm), k
        assert abs(sm - U[k][1]) <= 1e-12 * abs(sm), k
        rq, sq, uq = json.loads(rq), json.loads(sq), json.loads(U[k][2])
        if rc <= 8000:
            for name in NAMES:
                assert ulp_diff(rq[name], sq[name]) <= 4, (k, name)
                assert sq[name] == uq[name], (k, name)  # same multiset, same digest
        else:
            s = sorted(groups[k])
            for q, name in zip(QS, NAMES):
                bound = 2 * math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / rc
                lo, hi = np.searchsorted(s, sq[name], "left"), np.searchsorted(s, sq[name], "right")
                rlo, rhi = np.searchsorted(s, rq[name], "left"), np.searchsorted(s, rq[name], "right")
                assert abs((lo + hi) / 2 / rc - (rlo + rhi) / 2 / rc) <= bound, (k, name)


def test_designated_overflow_and_integer_udas(ctx, monkeypatch):
    """600 groups of ~5000 rows, every one large enough to be designated: more than the 255
    designated buckets, so the overflow goes through the rest sort; count / sum / min / max
    exact, mean to 1e-12 against the unsplit run."""
    rng = np.random.default_rng(77)
    g = rng.integers(0, 600, 3_000_000)
    v = rng.integers(-(1 << 40), 1 << 40, len(g))
    types = [2, 2]
    plan = P.linear_plan([P.source_op("t", types, ["g", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("count", [P.col(1)], [2]), P.agg_expr("sum", [P.col(1)], [2], fid=1),
                                         P.agg_expr("min", [P.col(1)], [2], fid=2), P.agg_expr("max", [P.col(1)], [2], fid=3),
                                         P.agg_expr("mean", [P.col(1)], [2], fid=4)]),
                          P.sink_op("out")])
    tables = {"t": {"types": types, "batches": [[Column.from_values(2, g.tolist()), Column.from_values(2, v.tolist())]]}}
    S = _by_key(_run(ctx, plan, tables, monkeypatch, True)[0]["cols"], 1)
    U = _by_key(_run(ctx, plan, tables, monkeypatch, False)[0]["cols"], 1)
    assert set(S) == set(U) and len(S) == 600
    for k in S:
        assert S[k][:4] == U[k][:4], k
        assert abs(S[k][4] - U[k][4]) <= 1e-12 * abs(U[k][4]) + 1e-9, k
    # and the oracle, on the exact columns
    ref = oc.execute_plan(plan, tables)["out"][0]["cols"]
    R = _by_key(ref, 1)
    for k in R:
        assert R[k][:4] == S[k][:4], k


def test_split_with_one_dominant_group_and_strings(ctx, monkeypatch):
    """One group holds most rows (designated), hundreds of small STRING-keyed groups stay in the
    sort; quantiles of the small groups bit-identical to the unsplit run, the large one within
    the rank bound of the oracle's."""
    rng = np.random.default_rng(12)
    n = 300_000
    small = [f"s{i:03d}" for i in range(400)]
    keys = ["HOT"] * 240_000 + [small[i] for i in rng.integers(0, len(small), n - 240_000)]
    vals = rng.lognormal(1.0, 1.0, n)
    perm = rng.permutation(n)
    keys = [keys[i] for i in perm]
    vals = vals[perm]
    plan = P.linear_plan([P.source_op("t", [5, 4], ["k", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("quantiles", [P.col(1)], [4]), P.agg_expr("count", [P.col(1)], [4], fid=1),
                                         P.agg_expr("mean", [P.col(1)], [4], fid=2)]),
                          P.sink_op("out")])
    tables = {"t": {"types": [5, 4], "batches": [[Column.from_values(5, keys), Column(4, values=vals)]]}}
    R = _by_key(oc.execute_plan(plan, tables)["out"][0]["cols"], 1)
    S = _by_key(_run(ctx, plan, tables, monkeypatch, True)[0]["cols"], 1)
    U = _by_key(_run(ctx, plan, tables, monkeypatch, False)[0]["cols"], 1)
    assert set(R) == set(S) == set(U)
    hot = np.sort(vals[[i for i, k in enumerate(keys) if k == "HOT"]])
    for k in R:
        assert R[k][1] == S[k][1] == U[k][1]
        assert abs(R[k][2] - S[k][2]) <= 1e-6 * abs(R[k][2])
        rq, sq, uq = json.loads(R[k][0]), json.loads(S[k][0]), json.loads(U[k][0])
        if R[k][1] <= 8000:
            assert sq == uq, k
            for name in NAMES:
                assert ulp_diff(rq[name], sq[name]) <= 4, (k, name)
        else:
            for q, name in zip(QS, NAMES):
                bound = 2 * math.pi * math.sqrt(q * (1 - q)) / 1000 + 1 / len(hot)
                rk = lambda x: (np.searchsorted(hot, x, "left") + np.searchsorted(hot, x, "right")) / 2 / len(hot)
                assert abs(rk(sq[name]) - rk(rq[name])) <= bound, (k, name)
