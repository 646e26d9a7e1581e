"""Consume-kernel experiment: times agg_consume for plan variants that isolate phase 1
(filter stream), phase 2 (key hash + probe + staging) and group cardinality."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pixie_amd import plans as P
from pixie_amd._lib import INT64, FLOAT64
from pixie_amd.device import Ctx, Table, datagen_http_events
from pixie_amd.pipeline import LinearQuery

HE = P.HE
def plan(thr, groups, vals):
    src = P.source_op("http_events", P.HTTP_TYPES, P.HTTP_NAMES, list(range(10)))
    flt = P.filter_op(P.func("greaterThanEqual", [P.col(HE["resp_status"]), P.const(INT64, thr)], [INT64, INT64]), list(range(10)))
    aggs = []
    for i, (name, c) in enumerate(vals):
        aggs.append(P.agg_expr(name, [P.col(c)], [INT64], fid=i))
    agg = P.agg_op([HE[g] for g in groups], aggs)
    return P.linear_plan([src, flt, agg, P.sink_op("output")])

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
ctx = Ctx(0)
t = Table(ctx, P.HTTP_TYPES)
for a in range(0, n, 16_000_000):
    m = min(16_000_000, n - a)
    t.append(datagen_http_events(20250117, a, m, n_pair_keys=10_000_000, threads=16))
t.flush()
V = {
  "c2like": (400, ["service", "req_path"], [("count", HE["latency"]), ("mean", HE["latency"])]),
  "nopass": (1000, ["service", "req_path"], [("count", HE["latency"]), ("mean", HE["latency"])]),
  "svc_only": (400, ["service"], [("count", HE["latency"]), ("mean", HE["latency"])]),
  "count_only": (400, ["service", "req_path"], [("count", HE["latency"])]),
  "allpass_svc": (0, ["service"], [("count", HE["latency"])]),
  "allpass_status": (0, ["resp_status"], [("count", HE["latency"])]),
  "c3like": (400, ["pod", "remote_addr"], [("count", HE["latency"])]),
  "int_key_hot": (400, ["resp_status"], [("count", HE["latency"])]),
}
res = {}
for name, (thr, g, v) in V.items():
    q = LinearQuery(plan(thr, g, v), P.HTTP_TYPES, expected_groups=65536)
    agg = q.make_agg(ctx)
    for _ in range(2):
        agg.reset(); agg.consume(t)
    ctx.sync(); ctx.reset_stats(); ctx.set_profiling(True)
    for _ in range(3):
        agg.reset(); agg.consume(t)
    ctx.sync(); ctx.set_profiling(False)
    l, ms = ctx.kernel_stats("agg_consume")
    res[name] = {"ms": ms / max(l, 1), "selected": agg.rows_selected()}
    print(name, res[name], flush=True)
    agg.close()
json.dump(res, open("gpurun_out/exp_consume.json", "w"), indent=1)
