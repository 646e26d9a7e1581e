#!/usr/bin/env python3
"""The bench's C5 leg alone (bench.py c5_leg: conn_stats bin x (upid, remote_addr) sums joined to
pod_metadata through pxc_execute_plan over stored tables), with per-query wall time and the
engine / library stage logs (PXC_TIMING=1, PXG_TIMING=1 lines on stderr), to split the query's
host time from its kernels (tools/, GPU box)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("PXC_TIMING", "1")
os.environ.setdefault("PXG_TIMING", "1")
from pixie_amd import plans as P  # noqa: E402
from pixie_amd import synth  # noqa: E402
from pixie_amd.device import Ctx  # noqa: E402
from pixie_amd.host_engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
e = Engine(0)
ctx = Ctx(0, handle=e.ctx_handle())
tabs = synth.c5_tables(20250117, n, rows_per_batch=1 << 20, n_pods=1000, n_addrs=100, span_s=300)
for name, t in tabs.items():
    e.create_table(name, t["types"], t["names"])
    for b in t["batches"]:
        e.append(name, b)
del tabs
pb = P.c5_plan().SerializeToString()
e.execute_raw(pb)
ctx.sync()
times = []
for i in range(reps):
    print(f"=== query {i} start", file=sys.stderr, flush=True)
    t = time.perf_counter()
    nbytes = e.execute_bytes_len(pb)
    times.append((time.perf_counter() - t) * 1000.0)
    print(f"=== query {i} end {times[-1]:.3f} ms ({nbytes} result bytes)", file=sys.stderr, flush=True)
print(json.dumps({"ms": [round(x, 3) for x in times], "median": sorted(times)[len(times) // 2]}), flush=True)
e.close()
