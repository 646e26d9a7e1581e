#!/usr/bin/env python3
"""Consume-only timing (event-bracketed agg_consume + agg_consume_prefix, median of steps) for
the probe-record prefix sizing: run once per PXG_PREFIX_DIV / PXG_PREFIX_MIN setting
(tools/, GPU box).  argv: rows steps."""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from pixie_amd import plans as P  # noqa: E402
from pixie_amd.device import Ctx, Table  # noqa: E402
from pixie_amd.host_engine import plan_agg  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ctx = Ctx(0)
t = Table(ctx, P.HTTP_TYPES)
t.append_http_events(bench.SEED, 0, rows, bench.N_PAIR_KEYS)
a = plan_agg(ctx, P.c2_plan(with_pluck=True), "http_events", P.HTTP_TYPES, expected_groups=65536)
for _ in range(2):
    a.reset(); a.consume(t); a.finalize()
ctx.sync()
cons, walls, steps_ms = [], [], []
for _ in range(steps):
    ctx.reset_stats()
    ctx.set_profiling(True, only="agg_consume")
    ctx.sync()
    t0 = time.perf_counter()
    a.reset()
    a.consume(t)
    ctx.sync()
    t1 = time.perf_counter()
    a.finalize()
    ctx.sync()
    t2 = time.perf_counter()
    ctx.set_profiling(False)
    l, ms = ctx.kernel_stats("agg_consume")
    l0, ms0 = ctx.kernel_stats("agg_consume_prefix")
    cons.append(ms + ms0)
    walls.append((t1 - t0) * 1e3)
    steps_ms.append((t2 - t0) * 1e3)
print(json.dumps({"div": os.environ.get("PXG_PREFIX_DIV", "32"), "min": os.environ.get("PXG_PREFIX_MIN", str(1 << 20)),
                  "no_prec": os.environ.get("PXG_NO_PREC", "0"), "rows": rows,
                  "consume_kernel_ms": round(statistics.median(cons), 4), "consume_wall_ms": round(statistics.median(walls), 4),
                  "step_wall_ms": round(statistics.median(steps_ms), 4)}), flush=True)
