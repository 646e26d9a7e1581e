"""Finalize grouping by counting placement (pixie_amd/csrc/pxg_place.hip) against the stable radix
sort it replaces, on the same staged records (one consume, two finalizes), and against the CPU
restatement.  Bars: group keys, counts and integer results bit-exact; means 1e-12 relative
(a float sum in another order); quantiles of groups <= 8000 values bit-exact (the digest sorts
them); above that 1e-12 relative (big-group centroid sums in another fixed order), and the
oracle's rank bound via tests/parity.py."""
import numpy as np
import pytest

import oracle_client as oc
import parity
from device_runner import run_plan
from kat import rows, rows_match
from pixie_amd import plans as P
from pixie_amd.device import Column, Table, datagen_http_events
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu
SEED = 20250117


def _finalize_with(monkeypatch, agg, place):
    monkeypatch.setenv("PXG_PLACE", "1" if place else "0")
    agg.finalize()
    return agg.result()


def _by_key(cols, nk):
    keys = [c.to_list() for c in cols[:nk]]
    out = {}
    for i in range(len(cols[0])):
        out[tuple(k[i] for k in keys)] = i
    return out


def test_place_matches_radix_on_the_same_staging(ctx, monkeypatch):
    n = 6_000_000
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(SEED, 0, n, 10_000_000)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    a.consume(t)
    R = _finalize_with(monkeypatch, a, False)
    D = _finalize_with(monkeypatch, a, True)
    kr, kd = _by_key(R, 2), _by_key(D, 2)
    assert set(kr) == set(kd) and len(kr) == len(R[0])
    big = 0
    for k, i in kr.items():
        j = kd[k]
        assert R[2].values[i] == D[2].values[j], k
        assert abs(R[3].values[i] - D[3].values[j]) <= 1e-12 * abs(R[3].values[i]), k
        qa, qb = R[4].values[i], D[4].values[j]
        if R[2].values[i] <= 8000:
            assert np.array_equal(qa.view(np.int64), qb.view(np.int64)), (k, qa, qb)
        else:
            big += 1
            assert np.all(np.abs(qa - qb) <= 1e-12 * np.abs(qa)), (k, qa, qb)
    assert big > 0
    a.close()
    t.close()


def test_place_c2_matches_oracle(ctx, monkeypatch):
    monkeypatch.setenv("PXG_PLACE", "1")
    n = 3_000_000
    cols = datagen_http_events(SEED, 0, n, threads=8)
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}}
    plan = P.c2_plan(with_pluck=False)
    ref = oc.execute_plan(plan, tables)["output"][0]["cols"]
    t = Table(ctx, P.HTTP_TYPES)
    t.append(cols)
    q = LinearQuery(plan, P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    a.consume(t)
    a.finalize()
    dev = a.result()
    gv = parity.GroupValues([[cols[2], cols[3]]], [cols[5].values >= 400], [cols[6].values / 1e6])
    rep = parity.compare_agg(dev, ref, 2, ["count", "rel", "quantiles"], gv)
    assert rep["ok"], rep
    a.close()
    t.close()


def test_place_many_groups_table_path_matches_oracle(ctx, monkeypatch):
    """~100K groups on the global-table path (high-cardinality mode off): thousands of distinct
    slots per 4096-record tile."""
    monkeypatch.setenv("PXG_PLACE", "1")
    monkeypatch.setenv("PXG_NO_HC", "1")
    cols = datagen_http_events(SEED, 0, 1_000_000, n_pair_keys=300_000, threads=8)
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}}
    ref = oc.execute_plan(P.c3_plan(), tables)["output"][0]["cols"]
    dev = run_plan(ctx, P.c3_plan(), tables, expected_groups=200_000)[0]["cols"]
    R, D = {t[:2]: t[2:] for t in rows(ref)}, {t[:2]: t[2:] for t in rows(dev)}
    assert set(R) == set(D) and len(R) > 50_000
    for k in R:
        assert R[k][0] == D[k][0] and R[k][2] == D[k][2], k
        assert abs(R[k][1] - D[k][1]) <= 1e-9 * abs(R[k][1]), k


def test_place_long_keys_and_mixed_udas(ctx, monkeypatch):
    """String keys past the fast path's 48 bytes (deferred inserts), count / sum / min / max /
    mean / quantiles over INT64 and FLOAT64, several batches."""
    monkeypatch.setenv("PXG_PLACE", "1")
    rng = np.random.default_rng(5)
    n = 120_000
    base = [("k" * int(rng.integers(1, 90))) + str(i) for i in range(700)]
    ks = [base[i] for i in rng.integers(0, len(base), n)]
    iv = rng.integers(-1000, 1000, n)
    fv = rng.normal(0, 10, n)
    types = [5, 2, 4]
    batches = [[Column.from_values(5, ks[a:a + 30_000]), Column.from_values(2, iv[a:a + 30_000].tolist()),
                Column.from_values(4, fv[a:a + 30_000].tolist())] for a in range(0, n, 30_000)]
    tables = {"t": {"types": types, "batches": batches}}
    plan = P.linear_plan([P.source_op("t", types, ["k", "i", "f"], [0, 1, 2]),
                          P.agg_op([0], [P.agg_expr("count", [P.col(1)], [2]), P.agg_expr("sum", [P.col(1)], [2], fid=1),
                                         P.agg_expr("min", [P.col(2)], [4], fid=2), P.agg_expr("max", [P.col(1)], [2], fid=3),
                                         P.agg_expr("mean", [P.col(2)], [4], fid=4), P.agg_expr("quantiles", [P.col(2)], [4], fid=5)]),
                          P.sink_op("out")])
    ref = oc.execute_plan(plan, tables)["out"][0]["cols"]
    dev = run_plan(ctx, plan, tables, expected_groups=1000)[0]["cols"]
    assert rows_match(rows(dev), rows(ref), ordered=False, tol_ulp=4, rel=1e-9), "placement result differs from the oracle"
