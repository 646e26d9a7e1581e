#!/usr/bin/env python3
"""Which big groups fall back to the full sort path in the north_star step (tools/, GPU box):
the bench's n1 aggregation (plan_agg, the engine's lowering of the C2 plan with pluck) and the
pipeline's (LinearQuery), a few steps each, printing the finalize's big_sort_groups."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pixie_amd import plans as P  # noqa: E402
from pixie_amd.device import Ctx, Table  # noqa: E402
from pixie_amd.host_engine import plan_agg  # noqa: E402
from pixie_amd.pipeline import LinearQuery  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
ctx = Ctx(0)
t = Table(ctx, P.HTTP_TYPES)
t.append_http_events(20250117, 0, rows, 10_000_000)
t.flush()
for name, mk in [("plan_agg", lambda: plan_agg(ctx, P.c2_plan(with_pluck=True), "http_events", P.HTTP_TYPES, expected_groups=65536)),
                 ("linear", lambda: LinearQuery(P.c2_plan(with_pluck=True), P.HTTP_TYPES, expected_groups=65536).make_agg(ctx))]:
    a = mk()
    for i in range(int(os.environ.get("N1_STEPS", "3"))):
        ctx.sync()
        t0 = time.perf_counter()
        a.reset()
        a.consume(t)
        g = a.finalize()
        ctx.sync()
        info = a.info()
        print(f"{name} step {i}: {(time.perf_counter() - t0) * 1000:.2f} ms groups {g} big_sort_groups {info['big_sort_groups']}", flush=True)
    a.close()
t.close()
ctx.close()
