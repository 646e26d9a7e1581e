#!/usr/bin/env python3
"""C5 engine query diagnosis: per-query wall time, per-kernel device time and the agg's table
state for the bench's C5 shape over stored tables (tools/, GPU box)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pixie_amd import plans as P, synth  # noqa: E402
from pixie_amd.device import Ctx  # noqa: E402
from pixie_amd.host_engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
shape = json.loads(sys.argv[2]) if len(sys.argv) > 2 else dict(n_pods=1000, n_addrs=100, span_s=300)
eng = Engine(0)
ctx = Ctx(0, handle=eng.ctx_handle())
tabs = synth.c5_tables(20250117, n, rows_per_batch=1 << 20, **shape)
for name, t in tabs.items():
    eng.create_table(name, t["types"], t["names"])
    for b in t["batches"]:
        eng.append(name, b)
pb = P.c5_plan().SerializeToString()
eng.set_analyze(os.environ.get("C5_ANALYZE", "1") == "1")
names = ["agg_consume", "agg_consume_list", "agg_rehash", "stage_remap", "agg_publish_sizes", "agg_publish_write"]
for q in range(4):
    ctx.sync()
    ctx.reset_stats()
    ctx.set_profiling(True)
    t0 = time.perf_counter()
    res = eng.execute_raw(pb)
    ctx.sync()
    wall = time.perf_counter() - t0
    ctx.set_profiling(False)
    ks = {k: ctx.kernel_stats(k) for k in names if ctx.kernel_stats(k)[0]}
    st = eng.last_stats()
    print(json.dumps({"query": q, "wall_ms": wall * 1e3, "kernels": ks, "bytes": len(res),
                      "stats": {k: v for k, v in st.items() if k != "nodes"} if isinstance(st, dict) else None}), flush=True)
    if isinstance(st, dict):
        for nd in st.get("nodes", []):
            print("   ", json.dumps(nd)[:400], flush=True)
eng.close()
