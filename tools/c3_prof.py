"""C3 (group by (pod, remote_addr), 100M rows, ~5M groups) steps for a kernel profile."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pixie_amd import plans as P  # noqa: E402
from pixie_amd.device import Ctx, Table  # noqa: E402
from pixie_amd.host_engine import plan_agg  # noqa: E402

ctx = Ctx(0)
t = Table(ctx, P.HTTP_TYPES)
t.append_http_events(20250117, 0, 100_000_000, 10_000_000)
a = plan_agg(ctx, P.c3_plan(), "http_events", P.HTTP_TYPES, expected_groups=5_100_000)
for _ in range(4):
    a.reset()
    a.consume(t)
    g = a.finalize()
ctx.sync()
print("groups", g)
