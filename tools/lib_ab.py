#!/usr/bin/env python3
"""One side of a library A/B (run it once per build, alternating, with PXG_LIB_PATH naming the
other build's libpxg.so): `python3 tools/lib_ab.py LABEL ROWS STEPS` prints the median C2 step
(reset -> consume -> finalize) and the agg_consume time of one event-bracketed step."""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    label, rows, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    from pixie_amd import plans as P
    from pixie_amd.device import Ctx, Table
    from pixie_amd.pipeline import LinearQuery
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(20250117, 0, rows, 10_000_000)
    t.flush()
    q = LinearQuery(P.c2_plan(with_pluck=True), P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
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
    cons = ctx.kernel_stats("agg_consume")[1]
    print(f"{label} rows {rows}: step median {statistics.median(ms):.3f} min {min(ms):.3f} ms, agg_consume {cons:.3f} ms, groups {g}",
          flush=True)
    a.close()
    t.close()
    ctx.close()


if __name__ == "__main__":
    main()
