"""The large-scale parity checker (tests/parity.py) on the CPU: the oracle against itself must
pass, and every kind of divergence the bars forbid must be caught."""
import copy

import numpy as np

import oracle_client as oc
import parity
from pixie_amd import plans as P
from pixie_amd.device import Column, datagen_http_events


def _c2(n=200_000):
    cols = datagen_http_events(20250117, 0, n, threads=4)
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [cols], "names": P.HTTP_NAMES}}
    out = oc.execute_plan(P.c2_plan(with_pluck=False), tables)["output"][0]["cols"]
    sel = cols[5].values >= 400
    vals = GV = parity.GroupValues([[cols[2], cols[3]]], [sel], [cols[6].values / 1e6])
    return out, GV


def test_oracle_vs_itself_passes_with_rank_groups():
    out, gv = _c2(1_500_000)
    rep = parity.compare_agg(out, out, 2, ["count", "rel", "quantiles"], gv)
    assert rep["ok"], rep
    q = rep["v2_quantiles"]
    assert q["groups_exact"] > 100 and q["groups_rank"] >= 1 and q["max_ulp"] == 0
    assert q["rank_counts_match"]


def test_checker_catches_divergence():
    out, gv = _c2(120_000)
    # reorder the device side: order must not matter
    perm = np.random.default_rng(1).permutation(len(out[0]))
    def take(c):
        if c.type == 5:
            vals = c.to_list()
            return Column.from_values(5, [vals[i] for i in perm])
        return Column(c.type, values=np.ascontiguousarray(c.values[perm]))
    shuffled = [take(c) for c in out]
    assert parity.compare_agg(shuffled, out, 2, ["count", "rel", "quantiles"], gv)["ok"]
    bad = copy.deepcopy(shuffled)
    bad[2].values = bad[2].values.copy(); bad[2].values[3] += 1
    assert not parity.compare_agg(bad, out, 2, ["count", "rel", "quantiles"], gv)["ok"]
    bad = copy.deepcopy(shuffled)
    bad[3].values = bad[3].values * (1 + 1e-5)
    assert not parity.compare_agg(bad, out, 2, ["count", "rel", "quantiles"], gv)["ok"]
    q = parity.quantile_matrix(shuffled[4]).copy()
    q[:, 3] = np.nextafter(np.nextafter(np.nextafter(np.nextafter(np.nextafter(q[:, 3], np.inf), np.inf), np.inf), np.inf), np.inf)
    bad = shuffled[:4] + [Column(4, values=q.ravel())]
    assert not parity.compare_agg(bad, out, 2, ["count", "rel", "quantiles"], gv)["ok"]
    bad = [Column.from_values(5, ["x"] + shuffled[0].to_list()[1:])] + shuffled[1:]
    assert not parity.compare_agg(bad, out, 2, ["count", "rel", "quantiles"], gv)["ok"]


def test_rank_bound_catches_a_wrong_big_group_quantile():
    rng = np.random.default_rng(2)
    n = 20_000
    keys = Column.from_values(5, ["big"] * n + ["s"] * 10)
    vals = np.concatenate([rng.normal(0, 1, n), rng.normal(0, 1, 10)])
    plan = P.linear_plan([P.source_op("t", [5, 4], ["k", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("count", [P.col(1)], [4]), P.agg_expr("quantiles", [P.col(1)], [4], fid=1)]),
                          P.sink_op("out")])
    out = oc.execute_plan(plan, {"t": {"types": [5, 4], "batches": [[keys, Column(4, values=vals)]]}})["out"][0]["cols"]
    gv = parity.GroupValues([[keys]], [np.ones(n + 10, bool)], [vals])
    assert parity.compare_agg(out, out, 1, ["count", "quantiles"], gv)["ok"]
    q = parity.quantile_matrix(out[2]).copy()
    big = [i for i, k in enumerate(out[0].to_list()) if k == "big"][0]
    q[big, 3] += 0.05   # p50 moved by ~2% of the rank: outside 0.0031 + 1/n
    rep = parity.compare_agg(out[:2] + [Column(4, values=q.ravel())], out, 1, ["count", "quantiles"], gv)
    assert not rep["ok"] and rep["v1_quantiles"]["max_rank_excess"] > 0
