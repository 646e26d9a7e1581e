#!/usr/bin/env python3
"""The bench's Filter -> Map leg alone (bench.filter_map_leg over the 100M-row device table),
for iterating on the standalone operators (tools/, GPU box)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from pixie_amd import plans as P  # noqa: E402
from pixie_amd.device import Ctx, Table  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
ctx = Ctx(0)
t = Table(ctx, P.HTTP_TYPES)
t.append_http_events(bench.SEED, 0, n, bench.N_PAIR_KEYS)
t.flush()
print(json.dumps(bench.filter_map_leg(ctx, t, n, P)), flush=True)
t.close()
ctx.close()
