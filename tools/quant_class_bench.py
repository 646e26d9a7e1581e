#!/usr/bin/env python3
"""The quantile digests of one group-size class alone (tools/, GPU box): a synthetic table of G
groups of exactly `size` rows each (INT64 key, FLOAT64 lognormal value), group by key ->
quantiles(value), finalized `reps` times.  Run under `rocprofv3 --kernel-trace --stats` so the
class's kernel (quant_tiny / quant_small / quant_mid / the selection path) is timed without the
other classes' kernels sharing the chip.  Usage: quant_class_bench.py size [total_values reps]."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pixie_amd import plans as P  # noqa: E402
from pixie_amd.device import Column, Ctx, Table  # noqa: E402
from pixie_amd.pipeline import LinearQuery  # noqa: E402

size = int(sys.argv[1])
total = int(sys.argv[2]) if len(sys.argv) > 2 else 15_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
G = max(1, total // size)
rng = np.random.default_rng(size)
keys = rng.permutation(np.repeat(np.arange(G, dtype=np.int64), size))
vals = rng.lognormal(1.0, 1.0, len(keys))
types = [2, 4]
plan = P.linear_plan([P.source_op("t", types, ["k", "v"], [0, 1]),
                      P.agg_op([0], [P.agg_expr("quantiles", [P.col(1)], [4])]),
                      P.sink_op("out")])
ctx = Ctx(0)
t = Table(ctx, types)
t.append([Column(2, values=keys), Column(4, values=vals)])
t.flush()
q = LinearQuery(plan, types, expected_groups=G)
a = q.make_agg(ctx)
a.consume(t)
for _ in range(reps):
    g = a.finalize()
ctx.sync()
print(f"quant_class_bench: size {size} groups {g} values {len(keys)}", flush=True)
a.close()
t.close()
ctx.close()
