#!/usr/bin/env python3
"""The north_star step alone (1B http_events rows on one GPU, C2 plan: reset -> consume ->
finalize), for `rocprofv3 --kernel-trace --stats -- python3 tools/n1_prof.py [steps]`: every
kernel launch in the trace is a 1B-row launch (one warm-up step + `steps` steps), so the stats'
averages are the per-step kernel times of the north_star configuration."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    rows = int(os.environ.get("N1_ROWS", "1000000000"))
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
    for i in range(steps + 1):
        ctx.sync()
        t0 = time.perf_counter()
        a.reset()
        a.consume(t)
        g = a.finalize()
        ctx.sync()
        ms.append((time.perf_counter() - t0) * 1000)
    print(f"n1_prof: rows {rows} groups {g} step ms {' '.join(f'{x:.2f}' for x in ms)} (first is the warm-up)", flush=True)
    a.close()
    t.close()
    ctx.close()


if __name__ == "__main__":
    main()
