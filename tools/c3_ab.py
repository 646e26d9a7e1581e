"""C3 step time, table mode against high-cardinality mode (PXG_NO_HC toggles it per agg), on the
100M-row table with 10M (pod, remote_addr) pairs; both modes must agree on groups and totals."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pixie_amd import plans as P  # noqa: E402
from pixie_amd.device import Ctx, Table  # noqa: E402
from pixie_amd.host_engine import plan_agg  # noqa: E402

ctx = Ctx(0)
t = Table(ctx, P.HTTP_TYPES)
t.append_http_events(20250117, 0, 100_000_000, 10_000_000)
res = {}
for mode in ("table", "hc", "table", "hc"):
    if mode == "table":
        os.environ["PXG_NO_HC"] = "1"
    else:
        os.environ.pop("PXG_NO_HC", None)
    a = plan_agg(ctx, P.c3_plan(), "http_events", P.HTTP_TYPES, expected_groups=5_100_000)
    ms = []
    for _ in range(6):
        ctx.sync()
        t0 = time.perf_counter()
        a.reset()
        a.consume(t)
        g = a.finalize()
        ctx.sync()
        ms.append((time.perf_counter() - t0) * 1e3)
    cols = a.result() if hasattr(a, "result") else None
    tot = None
    if cols is not None:
        tot = (int(np.sum(cols[2].values)), int(np.sum(cols[4].values)))
    print(mode, "groups", g, "ms", [round(x, 2) for x in ms], "median", round(float(np.median(ms[1:])), 3), "totals", tot, flush=True)
    res.setdefault(mode, []).append((g, tot))
    a.close()
print("agree", res["table"][0] == res["hc"][0], flush=True)
