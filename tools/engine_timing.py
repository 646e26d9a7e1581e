"""Stage timing of the C2 plan through the C++ engine over an HBM-resident stored table
(PXC_TIMING=1 makes libpxcarnot print one line per stage)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("PXC_TIMING", "1")
from pixie_amd import plans as P  # noqa: E402
from pixie_amd.device import Ctx, Table, datagen_http_events  # noqa: E402
from pixie_amd.host_engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 100_000_000
e = Engine(0)
e.create_table("http_events", P.HTTP_TYPES, P.HTTP_NAMES)
if "--host-gen" in sys.argv:
    for a in range(0, n, 16_000_000):
        e.append("http_events", datagen_http_events(20250117, a, min(16_000_000, n - a), n_pair_keys=10_000_000, threads=16))
else:
    ctx = Ctx(0, handle=e.ctx_handle())
    Table(ctx, P.HTTP_TYPES, handle=e.device_table("http_events"), owned=False).append_http_events(20250117, 0, n)
print("rows", e.num_rows("http_events"), flush=True)
pb = P.c2_plan(with_pluck=True).SerializeToString()
ctx = Ctx(0, handle=e.ctx_handle())
names = ["agg_consume", "agg_consume_list", "agg_rehash", "stage_remap", "agg_publish_sizes", "agg_publish_write",
         "radix_scatter", "quant_big_merge", "digest_chain"]
for i in range(5):
    ctx.reset_stats()
    ctx.set_profiling(True)
    t = time.perf_counter()
    r = e.execute_raw(pb)
    ms = 1000 * (time.perf_counter() - t)
    ctx.set_profiling(False)
    ks = {k: ctx.kernel_stats(k) for k in names}
    ks = {k: (v[0], round(v[1], 3)) for k, v in ks.items() if v[0]}
    print(f"query {i}: {ms:.2f} ms, {len(r)} bytes, kernels {ks}", file=sys.stderr, flush=True)
e.close()
