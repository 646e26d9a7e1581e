#!/usr/bin/env python3
"""Timing-only diagnosis of agg_consume on the C2 table: runs reset + consume (no finalize)
under each PXG_DIAG_CONSUME mode (0 production, 2 filter only,
3 keys + hash without probe) in a child process per mode and prints kernel ms per launch."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(rows, steps):
    sys.path.insert(0, REPO)
    from pixie_amd import plans as P
    from pixie_amd.device import Ctx, Table
    from pixie_amd.pipeline import LinearQuery
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(20250117, 0, rows, 10_000_000)
    t.flush()
    q = LinearQuery(P.c2_plan(with_pluck=True), P.HTTP_TYPES, expected_groups=65536)
    agg = q.make_agg(ctx)
    for _ in range(2):
        agg.reset(); agg.consume(t)
    ctx.sync(); ctx.reset_stats(); ctx.set_profiling(True)
    for _ in range(steps):
        agg.reset(); agg.consume(t)
    ctx.sync(); ctx.set_profiling(False)
    n, ms = ctx.kernel_stats("agg_consume")
    n0, ms0 = ctx.kernel_stats("agg_consume_prefix")  # the probe-record prefix launch, when it runs
    print(json.dumps({"mode": os.environ.get("PXG_DIAG_CONSUME", "0"), "launches_per_step": (n + n0) / steps,
                      "consume_ms_per_step": (ms + ms0) / steps, "prefix_ms_per_step": ms0 / steps,
                      "ms_per_launch": ms / max(n, 1)}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(int(sys.argv[2]), int(sys.argv[3]))
        sys.exit(0)
    for mode in sys.argv[1:] or ["0", "1", "2", "3"]:
        env = dict(os.environ, PXG_DIAG_CONSUME=mode)
        r = subprocess.run([sys.executable, __file__, "child", "100000000", "5"], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)
