"""The consume kernel's integer range filter (FilterRange, pxg_device.h; DESIGN.md §4.1 "Phase 1
as issued loads"): every integer comparison against a constant, including the constants at the
ends of the int64 range where `>` / `<` become empty or full ranges, against numpy on a column
holding those values.  The reference semantics are the comparison UDFs' (comparison_ops.h:
GreaterThanUDF etc., plain int64 compares)."""
import numpy as np
import pytest

from pixie_amd import plans as P
from pixie_amd.device import Column, Table
from pixie_amd.pipeline import LinearQuery

pytestmark = pytest.mark.gpu
I64 = 2
MIN, MAX = np.iinfo(np.int64).min, np.iinfo(np.int64).max
OPS = {"equal": np.equal, "notEqual": np.not_equal, "lessThan": np.less, "lessThanEqual": np.less_equal,
       "greaterThan": np.greater, "greaterThanEqual": np.greater_equal}
CONSTS = [int(MIN), int(MIN) + 1, -1, 0, 1, 400, int(MAX) - 1, int(MAX)]


@pytest.fixture(scope="module")
def table(ctx):
    rng = np.random.default_rng(23)
    n = 300_001  # odd: a ragged last tile
    special = np.array(CONSTS + [int(MIN) + 2, int(MAX) - 2, 399, 401, -2, 2], dtype=np.int64)
    x = np.where(rng.random(n) < 0.5, rng.choice(special, n), rng.integers(MIN, MAX, n, dtype=np.int64, endpoint=True))
    k = rng.integers(0, 37, n).astype(np.int64)
    t = Table(ctx, [I64, I64])
    t.append([Column(I64, values=k), Column(I64, values=x)])
    yield t, k, x
    t.close()


@pytest.mark.parametrize("op", sorted(OPS))
def test_integer_range_filter_matches_numpy(ctx, table, op):
    t, k, x = table
    for c in CONSTS:
        pred = P.func(op, [P.col(1), P.const(I64, c)], [I64, I64])
        plan = P.linear_plan([P.source_op("t", [I64, I64], ["k", "x"], [0, 1]),
                              P.filter_op(pred, [0, 1]),
                              P.agg_op([0], [P.agg_expr("count", [P.col(1)], [I64]), P.agg_expr("sum", [P.col(1)], [I64], fid=1)]),
                              P.sink_op("out")])
        q = LinearQuery(plan, [I64, I64])
        a = q.make_agg(ctx)
        a.consume(t)
        a.finalize()
        r = a.result()
        a.close()
        sel = OPS[op](x, c)
        keys, cnt = np.unique(k[sel], return_counts=True)
        got = dict(zip(np.asarray(r[0].values).tolist(), np.asarray(r[1].values).tolist()))
        assert got == dict(zip(keys.tolist(), cnt.tolist())), (op, c)
        wrap = lambda v: (int(v) + 2 ** 63) % 2 ** 64 - 2 ** 63  # noqa: E731  (int64 sums wrap)
        sums = {int(g): wrap(sum(int(v) for v in x[sel & (k == g)])) for g in keys}
        got_s = dict(zip(np.asarray(r[0].values).tolist(), np.asarray(r[2].values).astype(np.int64).tolist()))
        assert got_s == sums, (op, c)
