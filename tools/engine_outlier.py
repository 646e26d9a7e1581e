#!/usr/bin/env python3
"""The bench's engine leg alone (bench.py engine_query: the binary C2 plan through
pxc_execute_plan over the HBM-resident stored table, 10 queries after one untimed one), with
per-query wall time and the engine / library stage logs (PXC_TIMING=1, PXG_TIMING=1 lines on
stderr).  Run under `rocprofv3 --kernel-trace --memory-copy-trace` to put the kernels and copies
of a slow query beside its host stages (tools/, GPU box)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("PXC_TIMING", "1")
os.environ.setdefault("PXG_TIMING", "1")
from pixie_amd import plans as P  # noqa: E402
from pixie_amd.device import Ctx, Table  # noqa: E402
from pixie_amd.host_engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
e = Engine(0)
ctx = Ctx(0, handle=e.ctx_handle())
e.create_table("http_events", P.HTTP_TYPES, P.HTTP_NAMES)
Table(ctx, P.HTTP_TYPES, handle=e.device_table("http_events"), owned=False).append_http_events(20250117, 0, n, 10_000_000)
pb = P.c2_plan(with_pluck=True).SerializeToString()
e.execute_raw(pb)
ctx.sync()
times = []
for i in range(reps):
    print(f"=== query {i} start {time.perf_counter():.6f}", file=sys.stderr, flush=True)
    t = time.perf_counter()
    e.execute_bytes_len(pb)
    times.append((time.perf_counter() - t) * 1000.0)
    print(f"=== query {i} end {time.perf_counter():.6f} {times[-1]:.3f} ms", file=sys.stderr, flush=True)
print(json.dumps({"ms": [round(x, 3) for x in times], "median": sorted(times)[len(times) // 2], "max": max(times)}), flush=True)
e.close()
