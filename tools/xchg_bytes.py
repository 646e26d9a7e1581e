#!/usr/bin/env python3
"""Exchange bytes per rank at the bench's C2 shape: one rank's 100M-row shard (device-generated),
exported for N owners as exchange v2 parts (partial states) and as v1 row parts
(PXG_XCHG_V1=1), plus the export / import kernel time of v2 (tools/, GPU box)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from pixie_amd import plans as P  # noqa: E402
from pixie_amd.device import Ctx, Table  # noqa: E402
from pixie_amd.host_engine import plan_agg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
ctx = Ctx(0)
t = Table(ctx, P.HTTP_TYPES)
t.append_http_events(bench.SEED, 0, n, bench.N_PAIR_KEYS)
a = plan_agg(ctx, P.c2_plan(with_pluck=True), "http_events", P.HTTP_TYPES, expected_groups=65536)
out = {"rows_per_rank": n}
for world in (2, 8):
    for v1 in (False, True):
        if v1:
            os.environ["PXG_XCHG_V1"] = "1"
        a.reset()
        a.consume(t)
        ctx.sync()
        t0 = time.perf_counter()
        offs, nb = a.export_partial(world)
        ctx.sync()
        dt = time.perf_counter() - t0
        os.environ.pop("PXG_XCHG_V1", None)
        out[f"n{world}_{'v1_rows' if v1 else 'v2_states'}"] = {"bytes": int(sum(nb)), "sizing_ms": dt * 1e3}
print(json.dumps(out), flush=True)
