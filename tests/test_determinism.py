"""Run-to-run determinism of the per-group floating-point reductions (pixie_amd/csrc/
pxg_finalize.hip ChunkReduce / GroupCombine: double-double sums).  The staging order of a
group's values is the consume's tile completion order, which differs between runs; plain double
sums then differed in the last bits (the reference, one sequential loop, is deterministic).
With the sums carried in double-double and rounded once, count, sum and mean are bit-identical
across runs, and agree with an exact (math.fsum) restatement to the last bit.  The big groups'
selection path sums the values inside its centroid ranges the same way, so their quantiles are
bit-identical across runs as well."""
import math

import numpy as np
import pytest

from pixie_amd import plans as P
from pixie_amd.device import Column, Table
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu


def _rows(res, nk, widths):
    keys = [c.to_list() for c in res[:nk]]
    vals = [np.asarray(c.values).reshape(-1, w) for c, w in zip(res[nk:], widths)]
    return {tuple(k[g] for k in keys): tuple(v[g].tobytes() for v in vals) for g in range(len(keys[0]))}


def test_c2_results_are_bit_identical_across_runs(ctx):
    """count, mean and all 7 quantiles of every group, big groups (selection path: its inside-bin
    centroid sums are double-double too) included."""
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(20250117, 0, 20_000_000, 10_000_000)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    runs = []
    for _ in range(3):
        a.reset()
        a.consume(t)
        a.finalize()
        r = a.result()
        runs.append(_rows(r, 2, [1, 1, 7]))  # keys; count, mean, quantiles
    assert len(runs[0]) > 20_000
    assert runs[0] == runs[1] == runs[2]
    a.close()
    t.close()


def test_float_sum_and_mean_equal_the_exact_sum(ctx):
    """Values spanning 30 orders of magnitude with cancellation: sum = fsum rounded once, mean =
    that / count, for every group, bit for bit."""
    rng = np.random.default_rng(9)
    n = 400_000
    keys = rng.integers(0, 300, n)
    vals = rng.standard_normal(n) * np.power(10.0, rng.integers(-15, 15, n))
    plan = P.linear_plan([P.source_op("t", [2, 4], ["k", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("sum", [P.col(1)], [4]), P.agg_expr("mean", [P.col(1)], [4], fid=1)]),
                          P.sink_op("out")])
    q = LinearQuery(plan, [2, 4])
    t = Table(ctx, [2, 4])
    t.append([Column(2, values=keys.astype(np.int64)), Column(4, values=vals)])
    a = q.make_agg(ctx)
    a.consume(t)
    a.finalize()
    r = a.result()
    ks = np.asarray(r[0].values)
    sums = np.asarray(r[1].values)
    means = np.asarray(r[2].values)
    for g, k in enumerate(ks):
        sel = vals[keys == k]
        exact = math.fsum(sel.tolist())
        assert sums[g] == exact, (k, sums[g], exact)
        assert means[g] == exact / len(sel), (k, means[g], exact / len(sel))
    a.close()
    t.close()
