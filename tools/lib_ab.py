#!/usr/bin/env python3
"""One side of a library A/B (run it once per build, alternating, with PXG_LIB_PATH naming the
other build's libpxg.so): `python3 tools/lib_ab.py LABEL ROWS STEPS [c2|c3|c3_full]` prints the
median step (reset -> consume -> finalize) and the agg_consume time of one event-bracketed step.
C3 plans get their group-count hint from a first untimed run, as the bench does."""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    label, rows, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    plan_name = sys.argv[4] if len(sys.argv) > 4 else "c2"
    from pixie_amd import plans as P
    from pixie_amd.device import Ctx, Table
    from pixie_amd.pipeline import LinearQuery
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(20250117, 0, rows, 10_000_000)
    t.flush()
    if plan_name == "c2":
        a = LinearQuery(P.c2_plan(with_pluck=True), P.HTTP_TYPES, expected_groups=65536).make_agg(ctx)
    else:
        from pixie_amd.host_engine import plan_agg
        plan = P.c3_full_plan() if plan_name == "c3_full" else P.c3_plan()
        probe = plan_agg(ctx, plan, "http_events", P.HTTP_TYPES, expected_groups=0)
        probe.consume(t)
        hint = probe.finalize()
        probe.close()
        a = plan_agg(ctx, plan, "http_events", P.HTTP_TYPES, expected_groups=hint)
    ms = []
    for i in range(steps + 2):
        ctx.sync()
        t0 = time.perf_counter()
        a.reset()
        a.consume(t)
        g = a.finalize()
        ctx.sync()
        if i >= 2:
            ms.append((time.perf_counter() - t0) * 1000)
    ctx.reset_stats()
    ctx.set_profiling(True)
    a.reset()
    a.consume(t)
    a.finalize()
    ctx.sync()
    ctx.set_profiling(False)
    ks = {k: round(ctx.kernel_stats(k)[1], 3) for k in ("agg_consume", "radix_scatter", "hc_agg", "hc_part_starts", "hc_key_copy")}
    print(f"{label} {plan_name} rows {rows}: step median {statistics.median(ms):.3f} min {min(ms):.3f} ms, groups {g}, kernels {ks}",
          flush=True)
    a.close()
    t.close()
    ctx.close()


if __name__ == "__main__":
    main()
