#!/usr/bin/env python3
"""A/B of libpxg environment knobs on one table in one process (variants interleaved round by
round, so box drift cancels): `python3 tools/step_ab.py ROWS ROUNDS label:ENV=1,ENV2=0 label2: ...`.
Each round runs every variant for 3 steps (reset -> consume -> finalize of the C2 plan) and keeps
the last 2; prints per-variant median / min step ms.  Knobs are read by libpxg at call time
(std::getenv), so os.environ changes between steps take effect."""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    rows = int(sys.argv[1])
    rounds = int(sys.argv[2])
    variants = []
    for spec in sys.argv[3:]:
        label, _, envs = spec.partition(":")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
        variants.append((label, env))
    from pixie_amd import plans as P
    from pixie_amd.device import Ctx, Table
    from pixie_amd.pipeline import LinearQuery
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(20250117, 0, rows, 10_000_000)
    t.flush()
    q = LinearQuery(P.c2_plan(with_pluck=True), P.HTTP_TYPES, expected_groups=65536)
    a = q.make_agg(ctx)
    keys = sorted({k for _, e in variants for k in e})
    res = {label: [] for label, _ in variants}
    groups = {}
    kern_names = [k for k in os.environ.get("STEP_AB_KERNELS", "").split(",") if k]
    kern = {}
    for r in range(rounds):
        for label, env in variants:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            if kern_names and r == 0:  # one event-bracketed step per variant, untimed
                ctx.reset_stats()
                ctx.set_profiling(True)
                a.reset()
                a.consume(t)
                a.finalize()
                ctx.sync()
                ctx.set_profiling(False)
                kern[label] = {k: round(ctx.kernel_stats(k)[1], 4) for k in kern_names}
            for i in range(3):
                ctx.sync()
                t0 = time.perf_counter()
                a.reset()
                a.consume(t)
                g = a.finalize()
                ctx.sync()
                if i > 0:
                    res[label].append((time.perf_counter() - t0) * 1000)
            groups[label] = g
        print(f"round {r}: " + " ".join(f"{lb} {statistics.median(v):.3f}" for lb, v in res.items()), flush=True)
    for label, v in res.items():
        print(f"{label}: median {statistics.median(v):.3f} ms min {min(v):.3f} ms over {len(v)} steps, groups {groups[label]}"
              + (f", kernels {kern.get(label)}" if kern_names else ""), flush=True)
    a.close()
    t.close()
    ctx.close()


if __name__ == "__main__":
    main()
