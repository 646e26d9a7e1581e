"""pxg_agg_result_skip + pxg_agg_quantile_lanes (pluck on the device) against pxg_agg_result:
the lane-major lanes equal the selected columns of the 7-double quantiles (0.0 for a group with a
non-finite quantile, as pluck_float64 of its JSON), the finiteness flag is set exactly when all 7
are finite, and a skipped column comes back without buffers."""
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
        got = out[:G * nsel].reshape(nsel, G).T      # lane-major
        finite = np.isfinite(qv).all(axis=1)
        want = np.where(finite[:, None], qv[:, sel], 0.0)  # pluck_float64 of an unparsable JSON: 0.0
        assert np.array_equal(got, want)
        assert np.array_equal(fin.astype(bool), finite)
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


def _cols_bytes(outs, n, per_row=None):
    """Every column of a pxg_column_out array as raw bytes (values / offsets / payload)."""
    from pixie_amd.device import column_from_out
    res = []
    for j in range(n):
        if not outs[j].values and not outs[j].offsets:
            res.append((outs[j].type, None, None, None))
            continue
        c = column_from_out(outs[j], (per_row or {}).get(j, 1))
        res.append((c.type, None if c.values is None else np.asarray(c.values).tobytes(),
                    None if c.offsets is None else np.asarray(c.offsets).tobytes(),
                    None if c.data is None else np.asarray(c.data)[:int(np.asarray(c.offsets)[-1])].tobytes() if c.offsets is not None else None))
    return res


@pytest.mark.parametrize("skip_q", [0, 1])
def test_finalize_result_equals_finalize_then_result(ctx, skip_q):
    """pxg_agg_finalize_result (result copies issued inside the finalize, overlapping it) gives
    the same rows as pxg_agg_finalize followed by pxg_agg_result_skip (group order is the
    table's, which differs run to run, so rows are compared by key); a skipped quantiles column
    comes back typed and sized without buffers."""
    from pixie_amd.device import column_from_out
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(20250117, 0, 3_000_000, 10_000_000)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    lib = ctx.lib
    skip = (C.c_uint8 * 5)(0, 0, 0, 0, skip_q)

    def rows_of(outs, G):
        cols = [column_from_out(outs[j]).to_list() for j in range(4)]
        qv = None
        if not skip_q:
            qv = column_from_out(outs[4], 7).values
        out = {}
        for g in range(G):
            out[(cols[0][g], cols[1][g])] = (cols[2][g], cols[3][g], None if qv is None else tuple(qv[g]))
        return out

    a.consume(t)
    ng = C.c_int64(0)
    assert lib.pxg_agg_finalize(a.h, C.byref(ng)) == 0
    ref = (_lib.ColumnOut * 5)()
    assert lib.pxg_agg_result_skip(a.h, ref, 5, skip) == 0
    want = rows_of(ref, ng.value)
    lib.pxg_result_free(ref, 5)
    a.reset()
    a.consume(t)
    got_o = (_lib.ColumnOut * 5)()
    ng2 = C.c_int64(0)
    assert lib.pxg_agg_finalize_result(a.h, C.byref(ng2), got_o, 5, skip) == 0
    assert ng2.value == ng.value > 20_000
    if skip_q:
        assert got_o[4].length == ng.value and not got_o[4].values
    got = rows_of(got_o, ng2.value)
    lib.pxg_result_free(got_o, 5)
    assert set(got) == set(want)
    for k, (c, m, qq) in want.items():
        gc, gm, gq = got[k]
        assert gc == c and abs(gm - m) <= 1e-12 * abs(m), k
        if qq is not None and c <= 8000:
            assert gq == qq, k
    a.close()
    t.close()


@pytest.mark.parametrize("via", ["result_skip", "finalize_result"])
def test_lanes_result_mode_equals_quantile_lanes(ctx, via):
    """skip[c] = 0x80 | mask returns the quantiles column as its plucked lanes (values) and the
    finiteness bytes (data), identical to pxg_agg_quantile_lanes; through pxg_agg_finalize_result
    the lanes are issued inside the finalize, before its last synchronisation."""
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(20250117, 0, 3_000_000, 10_000_000)
    q = LinearQuery(P.c2_plan(with_pluck=False), P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    lib = ctx.lib
    mask = 0b1001000  # p50, p99
    a.consume(t)
    ng = C.c_int64(0)
    outs = (_lib.ColumnOut * 5)()
    skip = (C.c_uint8 * 5)(0, 0, 0, 0, 0x80 | mask)
    if via == "result_skip":
        assert lib.pxg_agg_finalize(a.h, C.byref(ng)) == 0
        assert lib.pxg_agg_result_skip(a.h, outs, 5, skip) == 0
    else:
        assert lib.pxg_agg_finalize_result(a.h, C.byref(ng), outs, 5, skip) == 0
    G = ng.value
    assert G > 20_000 and outs[4].length == G and outs[4].data_len == G
    got = np.ctypeslib.as_array(C.cast(outs[4].values, C.POINTER(C.c_double)), shape=(2 * G,)).copy()
    got_fin = np.ctypeslib.as_array(C.cast(outs[4].data, C.POINTER(C.c_uint8)), shape=(G,)).copy()
    want = np.zeros(2 * G, dtype=np.float64)
    fin = np.zeros(G, dtype=np.uint8)
    assert lib.pxg_agg_quantile_lanes(a.h, 2, mask, want.ctypes.data_as(C.c_void_p), fin.ctypes.data_as(C.c_void_p)) == 0
    assert np.array_equal(got, want) and np.array_equal(got_fin, fin)
    lib.pxg_result_free(outs, 5)
    a.close()
    t.close()
