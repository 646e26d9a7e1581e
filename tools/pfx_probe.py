import os, sys
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import bench
from pixie_amd import plans as P
from pixie_amd.device import Ctx, Table
from pixie_amd.host_engine import plan_agg
ctx = Ctx(0)
t = Table(ctx, P.HTTP_TYPES)
t.append_http_events(bench.SEED, 0, 100_000_000, bench.N_PAIR_KEYS)
a = plan_agg(ctx, P.c2_plan(with_pluck=True), "http_events", P.HTTP_TYPES, expected_groups=65536)
for i in range(3):
    print("--- step", i, file=sys.stderr, flush=True)
    a.reset(); a.consume(t); a.finalize()
print(a.info(), file=sys.stderr)
