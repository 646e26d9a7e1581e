#!/usr/bin/env python3
"""Partition-count A/B of the high-cardinality path (pxg_hc.hip) on the C3 table:
`python3 tools/hc_pbits_ab.py PLAN ROUNDS PBITS...` with PLAN c3 or c3_full; PBITS 0 = the
library's own choice.  Variants interleaved round by round; prints median step ms and the
partition pass's kernel times (event-bracketed step) per variant."""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    plan_name, rounds = sys.argv[1], int(sys.argv[2])
    pbits = [int(x) for x in sys.argv[3:]]
    from pixie_amd import plans as P
    from pixie_amd.device import Ctx, Table
    from pixie_amd.host_engine import plan_agg
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(20250117, 0, 100_000_000, 10_000_000)
    plan = P.c3_full_plan() if plan_name == "c3_full" else P.c3_plan()
    probe = plan_agg(ctx, plan, "http_events", P.HTTP_TYPES, expected_groups=0)
    probe.consume(t)
    hint = probe.finalize()
    probe.close()
    a = plan_agg(ctx, plan, "http_events", P.HTTP_TYPES, expected_groups=hint)
    res = {b: [] for b in pbits}
    kern = {}
    for r in range(rounds):
        for b in pbits:
            if b:
                os.environ["PXG_HC_PBITS"] = str(b)
            else:
                os.environ.pop("PXG_HC_PBITS", None)
            for i in range(3):
                prof = r == 0 and i == 0
                if prof:
                    ctx.reset_stats()
                    ctx.set_profiling(True)
                ctx.sync()
                t0 = time.perf_counter()
                a.reset()
                a.consume(t)
                g = a.finalize()
                ctx.sync()
                ms = (time.perf_counter() - t0) * 1000
                if prof:
                    ctx.set_profiling(False)
                    kern[b] = {k: round(ctx.kernel_stats(k)[1], 3) for k in ("agg_consume", "radix_scatter", "radix_hist", "hc_agg",
                                                                             "hc_part_starts", "hc_key_copy")}
                    kern[b]["pbits"] = a.info().get("hc_partition_bits")
                    kern[b]["reruns"] = a.info().get("hc_reruns")
                elif i > 0:
                    res[b].append(ms)
        print(f"round {r}: " + " ".join(f"{b}:{statistics.median(v):.3f}" for b, v in res.items()), flush=True)
    for b in pbits:
        print(f"pbits {b}: median {statistics.median(res[b]):.3f} ms, groups {g}, kernels {kern[b]}", flush=True)


if __name__ == "__main__":
    main()
