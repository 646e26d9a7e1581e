"""pxg_agg_result_skip + pxg_agg_quantile_lanes (pluck on the device) against pxg_agg_result:
the packed lanes equal the selected columns of the 7-double quantiles, the finiteness flag is
set exactly when all 7 are finite, and a skipped column comes back without buffers."""
import ctypes as C

import numpy as np
import pytest

from pixie_amd import _lib
from pixie_amd import plans as P
from pixie_amd.device import Column, Table
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu


def test_quantile_lanes_match_full_result(ctx):
    rng = np.random.default_rng(4)
    n = 20_000
    keys = [f"g{int(i)}" for i in rng.integers(0, 300, n)]
    vals = rng.lognormal(0.0, 1.0, n)
    vals[rng.integers(0, n, 40)] = np.nan          # skipped by the digest
    karr = np.array(keys)
    vals[karr == "g7"] = np.inf                     # every quantile of g7 is infinite
    vals[(karr == "g8") & (rng.random(n) < 0.5)] = -np.inf
    plan = P.linear_plan([P.source_op("t", [5, 4], ["k", "v"], [0, 1]),
                          P.agg_op([0], [P.agg_expr("count", [P.col(1)], [4]), P.agg_expr("quantiles", [P.col(1)], [4], fid=1)]),
                          P.sink_op("out")])
    q = LinearQuery(plan, [5, 4])
    t = Table(ctx, [5, 4])
    t.append([Column.from_values(5, keys), Column(4, values=vals)])
    a = q.make_agg(ctx)
    a.consume(t)
    G = a.finalize()
    full = a.result()
    qv = np.asarray(full[2].values, dtype=np.float64).reshape(G, 7)
    lib = ctx.lib
    for mask in (0b1001000, 0b0000001, 0b1111111, 0):
        nsel = bin(mask).count("1")
        out = np.zeros(max(G * nsel, 1), dtype=np.float64)
        fin = np.zeros(G, dtype=np.uint8)
        rc = lib.pxg_agg_quantile_lanes(a.h, 1, mask, out.ctypes.data_as(C.c_void_p), fin.ctypes.data_as(C.c_void_p))
        assert rc == 0
        sel = [k for k in range(7) if (mask >> k) & 1]
        got = out[:G * nsel].reshape(G, nsel)
        want = qv[:, sel]
        assert np.array_equal(np.isnan(got), np.isnan(want)) and np.array_equal(got[~np.isnan(got)], want[~np.isnan(want)])
        assert np.array_equal(fin.astype(bool), np.isfinite(qv).all(axis=1))
    assert (~np.isfinite(qv).all(axis=1)).sum() > 0
    # skip: the quantiles column comes back typed and sized, without buffers
    outs = (_lib.ColumnOut * 3)()
    skip = (C.c_uint8 * 3)(0, 0, 1)
    assert lib.pxg_agg_result_skip(a.h, outs, 3, skip) == 0
    assert outs[2].length == G and not outs[2].values and outs[0].length == G
    lib.pxg_result_free(outs, 3)
    # a non-quantiles UDA is refused
    assert lib.pxg_agg_quantile_lanes(a.h, 0, 1, None, fin.ctypes.data_as(C.c_void_p)) != 0
    a.close()
    t.close()
