#!/usr/bin/env python3
"""Benchmark: http_events Filter(resp_status>=400) -> Map(latency_ms) -> BlockingAgg by
(service, req_path) with count / mean / quantiles (BASELINE.json configs[1], "C2"), on HBM-
resident synthetic data, one process per GPU.

One step = one full pass of the fused hot path over the rank's table: pxg_agg_reset ->
pxg_agg_consume (filter + map + group-key hash + staging) -> [N>1: export partial states,
RCCL all-to-all by key hash, import] -> pxg_agg_finalize (group sort, count/mean reductions,
t-digest quantiles, key extraction) — finalized result columns on device.

Legs after the timed region (none of them is inside it):
  * engine_query: the unmodified binary C2 plan through the C++ engine (pxc_execute_plan).
  * cpu_baseline + parity (rank 0, N=1): the CPU Carnot restatement (oracle/) runs the C2 plan
    over the SAME rows (regenerated on the host, bit-identical to the device generator) as
    1024-row RowBatches; its execution window is the baseline and its result is compared with
    the device result (tests/parity.py bars) -> "parity".
  * n1 (N=1): the north-star configuration, 1B rows of http_events on one GPU, same step.

Prints ONE JSON line on rank 0 (the driver's contract).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
SEED = 20250117
N_PAIR_KEYS = 10_000_000
KERNELS = ["agg_consume", "agg_consume_prefix", "agg_records", "agg_publish_sizes", "agg_publish_write", "finalize_init", "slot_flags", "slot_gslot", "group_heads",
           "radix_hist_rank", "radix_hist", "radix_scan", "radix_scatter",
           "run_heads", "group_starts", "group_chunk_count", "chunk_reduce", "group_combine", "classify_groups",
           "digest_chain", "quant_tiny", "quant_small", "quant_mid", "big_setup", "quant_big_chunk_sort", "quant_big_merge", "quant_big_digest",
           "quant_sel_sample", "quant_sel_hist", "quant_sel_plan", "quant_sel_collect", "quant_sel_bin_sort", "quant_sel_digest",
           "key_extract", "key_string_copy", "scan_reduce", "scan_spine", "scan_downsweep",
           "export_slot_part", "export_group_rank", "export_row_digit", "export_centroids", "export_write_groups", "export_write_rows",
           "part_hist", "part_scatter", "part_starts", "import_keys", "import_rows",
           "hc_part_starts", "hc_agg", "hc_key_copy", "hc_spill",
           "split_sample", "split_ids", "split_hist", "split_scan", "split_scatter"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows-per-gpu", type=int, default=None,
                    help="default: 100M at N=1 (configs[1], C2); 125M per GPU at N>1 (configs[3], C4: 1B rows at N=8)")
    ap.add_argument("--n1-rows", type=int, default=1_000_000_000,
                    help="rows of the north-star 1-GPU leg (N=1 only; 0 disables)")
    ap.add_argument("--n1-steps", type=int, default=5)
    ap.add_argument("--no-n1-parity", action="store_true",
                    help="skip the n1 leg's full-size parity check against the generator ground truth")
    ap.add_argument("--gen-slice", type=int, default=16_000_000)
    ap.add_argument("--cpu-batch-rows", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the oracle leg (cpu_baseline and parity)")
    ap.add_argument("--no-engine-leg", action="store_true",
                    help="skip the engine query leg (profiling runs: keeps per-kernel averages to the timed steps)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 (bin + join) leg")
    ap.add_argument("--no-c3-full", action="store_true", help="skip the full-cardinality C3 leg (no filter, 10M groups)")
    ap.add_argument("--no-c3-parity", action="store_true", help="skip the full-cardinality C3 leg's oracle parity (20M rows)")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 (carnot_csv, CSV parse included) leg")
    ap.add_argument("--c5-rows", type=int, default=20_000_000)
    ap.add_argument("--host-gen", action="store_true", help="generate on the host and upload (default: device generator)")
    ap.add_argument("--backend", default="nccl",
                    help="N>1 data path: nccl = libpxg's RCCL communicator over xGMI (pxg_agg_alltoall); "
                         "gloo = torch.distributed all_to_all on the host (CPU rehearsal). The control plane is gloo.")
    ap.add_argument("--rank-timeout", type=float, default=1500.0,
                    help="N>1 launcher: wall-clock limit in seconds after which every rank still running is killed and the "
                         "launcher exits non-zero (0 = none)")
    ap.add_argument("--share-gpu0", action="store_true",
                    help="rehearsal only: every rank uses cuda:0 (a 1-GPU box; pair it with --backend gloo, since RCCL "
                         "refuses two ranks on one GPU)")
    ap.add_argument("--standin", action="store_true", help=argparse.SUPPRESS)  # tests only: N>1 protocol on CPU
    ap.add_argument("--standin-hang-rank", type=int, default=-1, help=argparse.SUPPRESS)  # tests only: that rank never returns
    ap.add_argument("--pmc-file",default=os.path.join(REPO, "profiles", "pmc_agg_consume.json"),
                    help="committed PMC summary used for roofline.traffic only when the live PMC leg cannot run")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the live PMC leg (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child runs of this build's consume)")
    ap.add_argument("--pmc-child", type=int, default=0, metavar="ROWS",
                    help=argparse.SUPPRESS)  # internal: the consume-only workload the PMC leg profiles
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="shard processes of the supplementary CPU baseline (SURVEY.md §8d: P PEMs + merge); "
                         "16 = the GPU box's CPU share; 0 disables")
    ap.add_argument("--cpu-timing-rows", type=int, default=25_000_000,
                    help="rows of the pinned 1-core CPU baseline sample (median of --cpu-timing-reps runs after a warm-up)")
    ap.add_argument("--cpu-timing-reps", type=int, default=5)
    ap.add_argument("--cpu-timing-child", type=int, nargs=3, default=None, metavar=("ROWS", "REPS", "BATCH"),
                    help=argparse.SUPPRESS)  # internal: the pinned CPU baseline process
    ap.add_argument("--cpu-shard-child", type=int, nargs=3, default=None, metavar=("ROW0", "ROWS", "BATCH"),
                    help=argparse.SUPPRESS)  # internal: one shard process of the parallel CPU baseline
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def consume_stats(ctx):
    """agg_consume launches of the profiled region: a fresh large run consumes a short prefix
    first ("agg_consume_prefix", whose publication writes the probe records) and then the rest
    ("agg_consume"); both are the consume kernel.  Returns (launches, ms of both, prefix ms)."""
    l, ms = ctx.kernel_stats("agg_consume")
    l0, ms0 = ctx.kernel_stats("agg_consume_prefix")
    return l + l0, ms + ms0, ms0


def alg_bytes_of(table, n):
    """every referenced input column once, Arrow layout (INT64 8 B; STRING 4 B
    offset + payload, from the table's own offsets)."""
    from pixie_amd import plans as P
    return 8 * n + 8 * n + table.device_bytes(P.HE["service"]) + table.device_bytes(P.HE["req_path"])


PMC_STEPS = 3


def pmc_child(rows):
    """The workload the PMC leg profiles: the C2 consume (reset + consume, the timed step's
    dominant kernel) over `rows` device-generated rows, 3 launches."""
    from pixie_amd import plans as P
    from pixie_amd.device import Ctx, Table
    from pixie_amd.host_engine import plan_agg
    ctx = Ctx(0)
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(SEED, 0, rows, N_PAIR_KEYS)
    a = plan_agg(ctx, P.c2_plan(with_pluck=True), "http_events", P.HTTP_TYPES, expected_groups=65536)
    for _ in range(PMC_STEPS):
        a.reset()
        a.consume(t)
    ctx.sync()
    a.close()
    t.close()
    ctx.close()


def pmc_leg(n):
    """roofline.traffic measured for THIS build: two rocprofv3 --pmc passes (FETCH_SIZE and
    WRITE_SIZE do not fit one TCC pass) over a child process running the consume on n rows,
    summarised per launch by tools/pmc_summary.py (FETCH_SIZE doubled: the gfx950 correction of
    MI355X_MICROARCH.md §HBM).  Returns the summary dict or None."""
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return None
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import pmc_summary as ps
    d = tempfile.mkdtemp(prefix="pxg_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        res = {}
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(d, counter)
            cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--pmc", counter, "-d", out, "-o", "run", "--output-format", "csv",
                   "--", sys.executable, os.path.abspath(__file__), "--pmc-child", str(n)]
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=200)
            if r.returncode != 0:
                return {"error": f"rocprofv3 --pmc {counter} exited {r.returncode}"}
            res[counter], res[counter + "_launches"] = ps.counter_per_step(out, r"AggConsume(Fast)?Kernel", counter, PMC_STEPS)
        # per consume step (prefix + main launch when the probe-record prefix runs)
        return {"hbm_bytes_per_launch": (2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024,
                "hbm_read_bytes_per_launch": 2 * res["FETCH_SIZE"] * 1024, "hbm_write_bytes_per_launch": res["WRITE_SIZE"] * 1024,
                "launches": [res["FETCH_SIZE_launches"], res["WRITE_SIZE_launches"]], "steps": PMC_STEPS, "rows": n,
                "per": "consume step (every agg_consume / agg_consume_prefix launch of one consume summed)",
                "source": "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this build (bench.py --pmc-child), "
                          "FETCH_SIZE x2 (gfx950), KiB -> bytes"}
    except Exception as e:  # the legs must never break the bench line
        return {"error": f"pmc leg failed: {e}"}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def pmc_traffic(args, n):
    """HBM bytes per agg_consume launch from a committed PMC summary for this row count
    (tools/pmc_summary.py output): the fallback when the live PMC leg cannot run."""
    for path in (args.pmc_file, os.path.join(REPO, "profiles", "pmc_agg_consume_n1.json")):
        if not os.path.exists(path):
            continue
        try:
            pm = json.load(open(path))
        except Exception:
            continue
        if pm.get("rows_per_gpu") == n and pm.get("kernel") == "agg_consume":
            return pm.get("hbm_bytes_per_launch")
    return None


def main():
    args = parse()
    if args.pmc_child:
        pmc_child(args.pmc_child)
        return
    if args.cpu_timing_child:
        cpu_timing_child(*args.cpu_timing_child)
        return
    if args.cpu_shard_child:
        cpu_shard_child(*args.cpu_shard_child)
        return
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # No external launcher: start the N ranks here (fresh interpreters; this process never
        # touches the GPU) and pass rank 0's JSON line through.
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"[bench] refusing to run: WORLD_SIZE={world} but --gpus {args.gpus} (launch one rank per GPU with "
              f"--gpus equal to the world size, or run `bench.py --gpus N` alone and it starts the N ranks itself)",
              file=sys.stderr, flush=True)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        return multi_main(args, rank, world, local_rank)
    import torch

    from pixie_amd import plans as P
    from pixie_amd.device import Ctx, Table, datagen_http_events
    from pixie_amd.host_engine import Engine, plan_agg

    n = args.rows_per_gpu or 100_000_000
    row0 = 0
    # The table lives in the C++ engine's HBM-resident table store; the timed step runs the
    # libpxg ABI on that device table, and the engine leg runs the whole plan over it.
    engine = Engine(local_rank)
    ctx = Ctx(local_rank, handle=engine.ctx_handle())
    engine.create_table("http_events", P.HTTP_TYPES, P.HTTP_NAMES)
    t0 = time.time()
    table = Table(ctx, P.HTTP_TYPES, handle=engine.device_table("http_events"), owned=False)
    if args.host_gen:
        for a in range(0, n, args.gen_slice):
            m = min(args.gen_slice, n - a)
            engine.append("http_events", datagen_http_events(SEED, row0 + a, m, n_pair_keys=N_PAIR_KEYS, threads=16))
    else:
        table.append_http_events(SEED, row0, n, N_PAIR_KEYS)
    assert engine.num_rows("http_events") == n
    log(rank, f"[bench] {'host-generated + uploaded' if args.host_gen else 'device-generated'} {n} rows "
              f"in {time.time() - t0:.1f}s ({table.num_chunks} chunks)")
    alg_bytes = alg_bytes_of(table, n)

    # The engine's own lowering of the C2 plan (the drop-in path's fused Filter/Map/Agg), driven
    # directly on the HBM-resident table so the timed step is exactly the device hot path.
    agg = plan_agg(ctx, P.c2_plan(with_pluck=True), "http_events", P.HTTP_TYPES, expected_groups=65536)

    def step():
        agg.reset()
        agg.consume(table)
        return agg.finalize()

    for _ in range(args.warmup):
        ngroups = step()
    ctx.sync()
    # Per-kernel breakdown from one untimed, fully event-bracketed pass (the event records
    # themselves cost time, so the timed region brackets agg_consume only).
    kernel_ms = profiled_kernels(ctx, step)
    step_launches = launches_of(ctx, step)
    ctx.reset_stats()
    ctx.set_profiling(True, only="agg_consume")
    torch.cuda.synchronize()
    ctx.sync()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        ngroups = step()
    ctx.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    ctx.set_profiling(False)
    launches, cons_ms, pre_ms = consume_stats(ctx)
    ms_per_step = elapsed * 1000.0 / args.steps
    selected = agg.rows_selected()
    world = 1
    total_rows = n
    value = total_rows * args.steps / elapsed
    # The consume kernel's time per step (both launches when the prefix runs): the algorithmic
    # bytes of one step are read by the two launches together.
    avg_launch_ms = cons_ms / args.steps
    achieved = alg_bytes / (avg_launch_ms / 1000.0) / 1e9 if launches else None
    dev_result = agg.result() if not args.no_cpu_baseline else None
    traffic = pmc_traffic(args, n)

    # Engine leg (N=1): the unmodified binary C2 plan through pxc_execute_plan over the stored
    # table: fused consume + finalize + result D2H + quantile JSON + pluck + PXRB serialisation.
    engine_query = None
    if world == 1 and not args.no_engine_leg:
        pb = P.c2_plan(with_pluck=True).SerializeToString()
        engine.execute_raw(pb)
        ctx.sync()
        reps = max(3, min(args.steps, 10))
        times = []
        for _ in range(reps):
            tq = time.perf_counter()
            res_len = engine.execute_bytes_len(pb)
            times.append(time.perf_counter() - tq)
        te = sum(times)
        st = sorted(times)
        # Per-query spread: some boxes stall an occasional query start by 10-30 ms while every
        # kernel's own time is unchanged, so the median is reported beside the mean.
        engine_query = {"ms_per_query": te * 1000.0 / reps, "ms_median": st[len(st) // 2] * 1000.0,
                        "ms_min": st[0] * 1000.0, "ms_max": st[-1] * 1000.0, "rows_per_s": n * reps / te, "queries": reps,
                        "result_bytes": res_len, "over_abi_step_ms": st[len(st) // 2] * 1000.0 - ms_per_step,
                        "path": "pxc_execute_plan (C++ engine, include/pxcarnot.h) over the HBM-resident stored table: "
                                "fused consume + finalize + result D2H + quantiles JSON + pluck_float64 + PXRB "
                                "(the PXRB buffer is released unread: the Python copy of it is not engine work)"}

    filter_map = None
    if world == 1 and not args.no_engine_leg:
        filter_map = filter_map_leg(ctx, table, n, P)
    c3 = c3_full = None
    if world == 1 and not args.no_engine_leg:
        c3 = c3_leg(args, ctx, table, n, P, plan_agg)
        if not args.no_c3_full:
            c3_full = c3_leg(args, ctx, table, n, P, plan_agg, full=True)

    c5 = None
    if world == 1 and not args.no_engine_leg and not args.no_c5:
        c5 = c5_leg(args, engine, ctx, P)
    c1 = None
    if world == 1 and not args.no_engine_leg and not args.no_c1:
        c1 = c1_leg(args, P)

    cpu, par = None, None
    if not args.no_cpu_baseline:
        cpu, par = oracle_leg(args, n, row0, dev_result)
        if cpu is not None and args.cpu_procs > 0:
            cpu["parallel"] = cpu_parallel_leg(args, n, row0)

    # North-star leg (N=1): the same step over 1B rows on one GPU.
    n1 = None
    if world == 1 and args.n1_rows > 0:
        agg.close()
        engine.drop_table("http_events")
        n1 = n1_leg(args, ctx, P, Table, plan_agg)

    # Live PMC traffic of this build's consume kernel (N=1, after every timed leg; child
    # processes under rocprofv3, so nothing of it touches the timed region).
    traffic_src = "committed file " + os.path.relpath(args.pmc_file, REPO) if traffic is not None else None
    pmc = None
    if world == 1 and not args.no_pmc:
        pmc = pmc_leg(n)
        if pmc and "hbm_bytes_per_launch" in pmc:
            traffic, traffic_src = pmc["hbm_bytes_per_launch"], pmc["source"]
        if n1 is not None:
            p1 = pmc_leg(args.n1_rows)
            if p1 and "hbm_bytes_per_launch" in p1:
                n1["roofline"]["traffic"] = p1["hbm_bytes_per_launch"]
                n1["roofline"]["traffic_source"] = p1["source"]
            n1["roofline"]["traffic_detail"] = p1

    if rank == 0:
        line = {
            "metric": "rows/sec + achieved HBM GB/s, http_events filter+group-by agg, 1/2/4/8 MI355X",
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": "synthetic http_events (counter-based splitmix64, seed 20250117; SURVEY.md §8d spec), generated in HBM",
            "config": {
                "workload": "C2: Filter(resp_status>=400) -> Map(latency_ms=latency/1e6) -> BlockingAgg by (service, req_path): "
                            "count, mean, quantiles -> pluck p50/p99",
                "rows_per_gpu": n, "total_rows": total_rows, "groups": ngroups, "selected_rows_per_gpu": selected,
                "parallelism": "single GPU",
                "algorithmic_bytes_per_row": alg_bytes / n,
                "kernel_ms_per_step": kernel_ms,
                "kernel_launches_per_step": step_launches,
                "step_rate_gbs_algorithmic": alg_bytes / (ms_per_step / 1000.0) / 1e9,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "agg_consume",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_detail": pmc,
                "algorithmic_bytes_per_launch": alg_bytes,
                "avg_launch_ms": avg_launch_ms,
                "consume_ms_per_step": avg_launch_ms,
                "launches_per_step": launches / args.steps,
                "prefix_ms_per_step": pre_ms / args.steps,
            },
            "cpu_baseline": cpu,
            "parity": par,
            "engine_query": engine_query,
            "filter_map": filter_map,
            "c3": c3,
            "c3_full": c3_full,
            "c5": c5,
            "c1": c1,
            "n1": n1,
        }
        print(json.dumps(line), flush=True)
    if args.n1_rows <= 0:
        agg.close()
    table.close()
    ctx.close()
    engine.close()


def profiled_kernels(ctx, step):
    """kernel -> summed ms of one untimed step with every library launch event-bracketed."""
    ctx.reset_stats()
    ctx.set_profiling(True)
    step()
    ctx.sync()
    ctx.set_profiling(False)
    out = {}
    for name in KERNELS + ["gather_rebase"]:
        l, ms = ctx.kernel_stats(name)
        if l:
            out[name] = round(ms, 4)
    return out


def launches_of(ctx, step):
    """Kernel launches of one step (every libpxg launch, counted with profiling on), without
    the runtime's copy / fill operations."""
    ctx.reset_stats()
    ctx.set_profiling(True)
    step()
    ctx.sync()
    ctx.set_profiling(False)
    return ctx.kernel_stats("*")[0]


def launch_ranks(args):
    """`bench.py --gpus N` with no external launcher: start N rank processes of this script
    (fresh interpreters, env RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1), wait for
    them, and return the worst exit code.  This process never initialises the GPU.  Rank 0
    inherits stdout, so its JSON line is the only one printed; the other ranks' stdout is
    discarded.  A rank that fails takes the others down with it."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    n = args.gpus
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    print(f"[bench] starting {n} ranks (one process per GPU, rendezvous 127.0.0.1:{port})", file=sys.stderr, flush=True)
    procs = []

    def stop_all(sig=signal.SIGTERM):
        for q in procs:
            if q.poll() is None:
                try:
                    os.killpg(q.pid, sig)
                except ProcessLookupError:
                    pass

    # A Ctrl-C / kill of the launcher takes the ranks (each in its own session) with it.
    def on_signal(signum, _frame):
        print(f"[bench] launcher got signal {signum}: stopping the ranks", file=sys.stderr, flush=True)
        stop_all()
        raise SystemExit(128 + signum)

    old_handlers = {sg: signal.signal(sg, on_signal) for sg in (signal.SIGINT, signal.SIGTERM)}
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL, start_new_session=True))
    codes = [None] * n
    failed = False
    deadline = time.time() + args.rank_timeout if args.rank_timeout > 0 else None
    try:
        while any(c is None for c in codes):
            for r, p in enumerate(procs):
                if codes[r] is None:
                    c = p.poll()
                    if c is not None:
                        codes[r] = c
                        if c != 0 and not failed:
                            failed = True
                            print(f"[bench] rank {r} exited {c}: stopping the other ranks", file=sys.stderr, flush=True)
                            stop_all()
            if deadline is not None and time.time() > deadline and any(c is None for c in codes):
                print(f"[bench] ranks still running after --rank-timeout {args.rank_timeout}s: killing them", file=sys.stderr, flush=True)
                stop_all(signal.SIGKILL)
                for r, p in enumerate(procs):
                    if codes[r] is None:
                        p.wait()
                        codes[r] = 124
                break
            time.sleep(0.05)
    finally:
        for sg, h in old_handlers.items():
            signal.signal(sg, h)
    return max((c if c > 0 else 1 if c != 0 else 0) for c in codes)


class DeviceRank:
    """One rank of the N > 1 bench (BASELINE configs[3], C4): its contiguous row shard
    [rank * n, (rank + 1) * n) generated in HBM, the engine's C2 lowering, libpxg's own RCCL
    communicator (backend nccl) or torch.distributed gloo (CPU-hosted rehearsal)."""

    def __init__(self, args, rank, world, local_rank):
        import torch
        from pixie_amd import plans as P
        from pixie_amd.device import Ctx, Table
        from pixie_amd.host_engine import Engine, plan_agg
        torch.cuda.set_device(local_rank)
        self.torch = torch
        self.rank, self.world, self.backend = rank, world, args.backend
        self.n = args.rows_per_gpu or 125_000_000
        self.engine = Engine(local_rank)
        self.ctx = Ctx(local_rank, handle=self.engine.ctx_handle())
        self.engine.create_table("http_events", P.HTTP_TYPES, P.HTTP_NAMES)
        self.table = Table(self.ctx, P.HTTP_TYPES, handle=self.engine.device_table("http_events"), owned=False)
        t0 = time.time()
        self.table.append_http_events(SEED, rank * self.n, self.n, N_PAIR_KEYS)
        log(rank, f"[bench] device-generated {self.n} rows/rank in {time.time() - t0:.1f}s ({self.table.num_chunks} chunks)")
        self.alg_bytes = alg_bytes_of(self.table, self.n)
        self.agg = plan_agg(self.ctx, P.c2_plan(with_pluck=True), "http_events", P.HTTP_TYPES, expected_groups=65536)
        self.comm = None
        self.parts = None
        self.exch = {"bytes_sent": 0, "bytes_recv": 0, "via": None, "gather": None}
        if args.backend == "nccl":
            import torch.distributed as dist
            from pixie_amd.device import Comm
            # every rank is on this node (--nnodes=1): RCCL's bootstrap socket stays on loopback
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            obj = [Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            self.comm = Comm(self.ctx, rank, world, obj[0])

    def step(self):
        """reset -> consume -> exchange partial states by key hash -> finalize -> gather the
        final rows on rank 0.  Returns the gathered groups on rank 0 (0 elsewhere).  Both
        backends run libpxg's exchange (pxg_agg_alltoall: device part layout, {bytes, header}
        records, import) and pxg_agg_gather (device rebase of the STRING offsets); backend gloo
        moves the bytes through a host communicator (pxg_comm_init_host over torch gloo) instead
        of RCCL."""
        a = self.agg
        a.reset()
        a.consume(self.table)
        # rows this rank selected (read before the exchange: the import resets the staging)
        self.selected_rows = a.rows_selected()
        if self.comm is not None:
            s, r = a.alltoall(self.comm)
            a.finalize()
            g = a.gather(self.comm, 0)
            self.exch.update(via="pxg_agg_alltoall (RCCL grouped send/recv on the ctx stream)",
                             gather="pxg_agg_gather (RCCL send/recv of the result columns to rank 0)")
        else:
            from pixie_amd.dist import exchange_partials, gather_device_results
            s, r = exchange_partials(a)
            a.finalize()
            g = gather_device_results(a)
            self.exch.update(via=f"pxg_agg_alltoall over a host communicator (pxg_comm_init_host; bytes over torch.distributed "
                                 f"{self.backend}, same device export / import code as RCCL)",
                             gather="pxg_agg_gather over the host communicator (device rebase of the STRING offsets)")
        self.exch["bytes_sent"], self.exch["bytes_recv"] = s, r
        return g

    def sync(self):
        self.ctx.sync()
        self.torch.cuda.synchronize()

    def profile(self):
        return profiled_kernels(self.ctx, self.step)

    def start_timing(self):
        self.ctx.reset_stats()
        self.ctx.set_profiling(True, only="agg_consume")

    def consume_ms(self):
        self.ctx.set_profiling(False)
        return consume_stats(self.ctx)

    def selected(self):
        return self.selected_rows

    def result(self):
        """Rank 0: the whole gathered result (service, req_path, count, mean, quantiles)."""
        return self.agg.result()

    def close(self):
        if self.comm is not None:
            self.comm.close()
        else:
            from pixie_amd.dist import close_host_comms
            close_host_comms()
        self.agg.close()
        self.table.close()
        self.ctx.close()
        self.engine.close()


def multi_main(args, rank, world, local_rank):
    """N > 1 (BASELINE configs[3] "C4": 1B rows over 8 GPUs = 125M rows per rank):
    one process per GPU, row shards, partial UDA states exchanged by hash(key) with one
    all-to-all(v), local finalize, final rows gathered to rank 0 -- all inside the timed step.
    Control plane (unique id, barriers, max over ranks) on torch.distributed gloo.  After the
    timed region rank 0 checks the gathered result of the last step against the generator's
    ground truth over all world * n rows (tests/parity.py::check_c2_against_truth: group set and
    counts bit-exact, means 1e-6, quantiles 4 ULP / rank bound)."""
    import torch.distributed as dist
    if args.share_gpu0:
        local_rank = 0
    # gloo's connection banner goes to the C-level stdout; keep stdout for the one JSON line.
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo", init_method="env://")
        dist.barrier()
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    runner = None
    try:
        if args.standin:
            # TEST ONLY (tests/test_bench_launch.py): the launcher / rendezvous / timing / gather /
            # parity protocol on CPU, with a numpy + oracle stand-in for the device step.
            sys.path.insert(0, os.path.join(REPO, "tests"))
            from bench_standin import StandinRank
            runner = StandinRank(args, rank, world, SEED, N_PAIR_KEYS)
            if rank == args.standin_hang_rank:  # TEST ONLY: a rank stuck before the first collective
                while True:
                    time.sleep(1)
        else:
            runner = DeviceRank(args, rank, world, local_rank)
        n = runner.n
        for _ in range(args.warmup):
            runner.step()
        runner.sync()
        kernel_ms = runner.profile()
        runner.start_timing()
        dist.barrier()
        runner.sync()
        t_start = time.perf_counter()
        for _ in range(args.steps):
            ngroups = runner.step()
        runner.sync()
        dist.barrier()
        elapsed = time.perf_counter() - t_start
        launches, cons_ms, pre_ms = runner.consume_ms()
        import torch
        tt = torch.tensor([elapsed, cons_ms / args.steps], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, avg_launch_ms = float(tt[0]), float(tt[1])
        sel = torch.tensor([runner.selected()], dtype=torch.int64)
        dist.all_reduce(sel, op=dist.ReduceOp.SUM)
        selected_total = int(sel[0])
        ms_per_step = elapsed * 1000.0 / args.steps
        total_rows = n * world
        value = total_rows * args.steps / elapsed
        alg_bytes = runner.alg_bytes
        achieved = alg_bytes / (avg_launch_ms / 1000.0) / 1e9 if launches and avg_launch_ms > 0 else None
        par = None
        pmc = None
        if rank == 0 and not args.standin and not args.no_pmc:
            # rank 0's consume (its shard = rows [0, n), the same consume as the timed one) under
            # two rocprofv3 --pmc passes in a child process; the other ranks wait at the barrier
            pmc = pmc_leg(n)
        if rank == 0:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            try:
                import parity
                par = parity.check_c2_against_truth(runner.result(), SEED, 0, total_rows, threads=16)
                par["scope"] = (f"the rank-0 gathered result of the last timed step against the generator's ground truth over "
                                f"all {total_rows} rows of the {world} shards")
            except Exception as e:  # the legs must never break the bench line
                import traceback
                traceback.print_exc()
                par = {"ok": False, "error": f"N>1 parity failed: {e}"}
        if rank == 0:
            line = {
                "metric": "rows/sec + achieved HBM GB/s, http_events filter+group-by agg, 1/2/4/8 MI355X",
                "value": value, "unit": "rows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": "int64/f64",
                "data": ("STAND-IN (test of the launcher protocol; numpy + oracle step, not the product)" if args.standin else
                         "synthetic http_events (counter-based splitmix64, seed 20250117; SURVEY.md §8d spec), generated in HBM"),
                "config": {
                    "workload": "C4: per-rank Filter(resp_status>=400) -> Map(latency_ms=latency/1e6) -> partial BlockingAgg by "
                                "(service, req_path): count, mean, quantiles; partial states exchanged by hash(key) % N; "
                                "finalize; final rows gathered on rank 0",
                    "rows_per_gpu": n, "total_rows": total_rows, "groups": ngroups, "selected_rows_per_gpu": runner.selected(),
                    "selected_rows_all_ranks": selected_total,
                    "parallelism": f"dp{world} (row shards, partial UDA states exchanged by key hash, rows gathered on rank 0)",
                    "algorithmic_bytes_per_row": alg_bytes / n if n else None,
                    "kernel_ms_per_step_rank0": kernel_ms,
                    "step_rate_gbs_algorithmic": alg_bytes * world / (ms_per_step / 1000.0) / 1e9,
                    "exchange_bytes_per_rank": runner.exch, "backend": args.backend, "share_gpu0": bool(args.share_gpu0),
                },
                "roofline": {
                    "bound": "hbm", "kernel": "agg_consume", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                    "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                    "traffic_detail": pmc,
                    "algorithmic_bytes_per_launch": alg_bytes, "avg_launch_ms": avg_launch_ms if launches else None,
                    "per": "one rank's consume step (the slowest rank's event-timed consume); traffic: rank 0's consume of "
                           "its shard under rocprofv3 --pmc after the timed region",
                },
                "cpu_baseline": None,
                "parity": par,
            }
            print(json.dumps(line), flush=True)
        dist.barrier()
    finally:
        if runner is not None:
            runner.close()
        dist.destroy_process_group()


def filter_map_leg(ctx, table, n, P, reps=5):
    """The non-fused operator shape: standalone FilterNode (resp_status >= 400, keeping service,
    req_path, latency) then MapNode (service, req_path, latency / 1e6) over the whole table, as
    pxg_filter + pxg_map into new device tables.  Roofline of the filter kernels: the predicate
    column streamed (8 B/row) plus the kept rows' columns read and written once each."""
    from pixie_amd.compile import ExprCompiler
    comp = ExprCompiler(P.HTTP_TYPES)
    pred = comp.compile(P.func("greaterThanEqual", [P.col(P.HE["resp_status"]), P.const(2, 400)], [2, 2]))
    sel = [P.HE["service"], P.HE["req_path"], P.HE["latency"]]
    mcomp = ExprCompiler([5, 5, 2])
    progs = [mcomp.compile(P.col(0)), mcomp.compile(P.col(1)), mcomp.compile(P.func("divide", [P.col(2), P.const(4, 1e6)], [2, 4]))]
    f = table.filter(pred, sel)
    m = f.map(progs)
    kept = f.num_rows
    kept_bytes = f.device_bytes(0) + f.device_bytes(1) + 8 * kept
    m.close()
    f.close()
    names = ["filter_count", "filter_scan", "filter_write", "map_eval", "map_rebase"]
    ctx.sync()
    ctx.reset_stats()
    ctx.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        f = table.filter(pred, sel)
        m = f.map(progs)
        m.close()
        f.close()
    ctx.sync()
    wall = (time.perf_counter() - t0) / reps
    ctx.set_profiling(False)
    kms = {k: ctx.kernel_stats(k)[1] / reps for k in names if ctx.kernel_stats(k)[0]}
    filt_ms = sum(v for k, v in kms.items() if k.startswith("filter"))
    alg = 8 * n + 2 * kept_bytes
    # SURVEY.md §8d's definition (the one agg_consume is priced by): every referenced input column
    # once in Arrow layout, plus the kept rows written.
    cols_bytes = 8 * n + table.device_bytes(P.HE["service"]) + table.device_bytes(P.HE["req_path"]) + 8 * n + kept_bytes
    return {"workload": "Filter(resp_status>=400; service, req_path, latency) -> Map(service, req_path, latency/1e6) "
                        "over the HBM table (pxg_filter + pxg_map, non-fused operators)",
            "rows": n, "kept_rows": kept, "ms_per_query_wall": wall * 1000.0, "rows_per_s": n / wall,
            "kernel_ms": {k: round(v, 4) for k, v in kms.items()},
            "roofline": {"bound": "hbm", "kernels": "filter_count + filter_scan + filter_write",
                         "algorithmic_bytes": alg, "achieved": alg / (filt_ms / 1000.0) / 1e9 if filt_ms else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / (filt_ms / 1000.0) / 1e9 / HBM_PEAK_GBS if filt_ms else None,
                         "algorithmic_bytes_input_columns": cols_bytes,
                         "frac_input_columns": cols_bytes / (filt_ms / 1000.0) / 1e9 / HBM_PEAK_GBS if filt_ms else None,
                         "bytes_note": "frac counts the predicate column and the kept rows read + written once; a 12%-selective "
                                       "gather touches most 128-byte lines of every gathered column, so the measured traffic "
                                       "(profiles/r05_filter_pmc.json) is ~2.5x that; frac_input_columns uses SURVEY.md §8d's "
                                       "definition (every referenced input column once + the output), as agg_consume does"}}


def c3_leg(args, ctx, table, n, P, plan_agg, steps=3, full=False):
    """BASELINE config C3: the high-cardinality group-by, (pod, remote_addr) over the same
    100M-row table (10M distinct pairs): count, mean(latency), sum(resp_body_size).  Default:
    SURVEY §8d's query, behind Filter(resp_status >= 400) (~5M groups; parity for this shape is
    tests/test_scale_parity.py).  full=True: no filter, every row, all 10M pairs as groups
    (plans.c3_full_plan), with its own parity block against the oracle on a 20M-row prefix."""
    plan = P.c3_full_plan() if full else P.c3_plan()
    alg = (16 if full else 24) * n + table.device_bytes(P.HE["pod"]) + table.device_bytes(P.HE["remote_addr"])
    # The group-count hint comes from a first, untimed run without one, as the engine's
    # group-count statistics size the next run of the same plan.
    probe = plan_agg(ctx, plan, "http_events", P.HTTP_TYPES, expected_groups=0)
    probe.reset()
    probe.consume(table)
    hint = probe.finalize()
    probe.close()
    a = plan_agg(ctx, plan, "http_events", P.HTTP_TYPES, expected_groups=hint)

    def step():
        a.reset()
        a.consume(table)
        return a.finalize()

    g = step()
    ctx.sync()
    # per-kernel breakdown from one untimed, event-bracketed step
    ctx.reset_stats()
    ctx.set_profiling(True)
    step()
    ctx.sync()
    ctx.set_profiling(False)
    kernel_ms = {}
    for name in KERNELS:
        kl, kms = ctx.kernel_stats(name)
        if kl:
            kernel_ms[name] = round(kms, 4)
    mode = a.info()
    ctx.reset_stats()
    ctx.set_profiling(True, only="agg_consume")
    ctx.sync()
    ts = time.perf_counter()
    for _ in range(steps):
        g = step()
    ctx.sync()
    el = time.perf_counter() - ts
    ctx.set_profiling(False)
    l, ms, _pre = consume_stats(ctx)
    avg = ms / steps
    achieved = alg / (avg / 1000.0) / 1e9
    wl = ("C3 full cardinality: Agg by (pod, remote_addr) over every row (no filter; 10M distinct pairs): count, mean(latency), "
          "sum(resp_body_size)" if full else
          "C3: Filter(resp_status>=400) -> Agg by (pod, remote_addr): count, mean(latency), sum(resp_body_size)")
    out = {"workload": wl,
           "mode": "high-cardinality (partition records + LDS tables, pxg_hc.hip)" if mode.get("hc_mode") else "global table",
           "partition_bits": mode.get("hc_partition_bits"), "kernel_ms_per_step": kernel_ms,
           "rows": n, "steps": steps, "groups": g, "selected_rows": a.rows_selected(), "ms_per_step": el * 1000.0 / steps,
           "value": n * steps / el, "unit": "rows/s", "algorithmic_bytes_per_row": alg / n,
           "roofline": {"bound": "hbm", "kernel": "agg_consume", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": alg, "avg_launch_ms": avg}}
    a.close()
    if full and not args.no_c3_parity:
        out["parity"] = c3_full_parity(ctx, P, plan_agg, plan)
    return out


def c3_full_parity(ctx, P, plan_agg, plan, n=20_000_000):
    """The full-cardinality C3 plan on the table's first n rows (device table generated in HBM,
    bit-identical to the host generator) against the oracle over the same rows: group keys and
    counts and sums bit-exact, means 1e-6 (tests/parity.py bars)."""
    try:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_client as oc
        import parity
        from pixie_amd.device import Table, datagen_http_events
        t = Table(ctx, P.HTTP_TYPES)
        t.append_http_events(SEED, 0, n, N_PAIR_KEYS)
        a = plan_agg(ctx, plan, "http_events", P.HTTP_TYPES, expected_groups=n // 2)
        a.reset()
        a.consume(t)
        a.finalize()
        mode = a.info().get("hc_mode")
        dev = a.result()
        a.close()
        t.close()
        cols = datagen_http_events(SEED, 0, n, n_pair_keys=N_PAIR_KEYS, threads=16)
        need = {P.HE[c] for c in ("pod", "remote_addr", "latency", "resp_body_size")}
        ocols = [c if i in need else oc.AbsentColumn(c.type, len(c)) for i, c in enumerate(cols)]
        tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [ocols], "names": P.HTTP_NAMES}}
        t0 = time.time()
        ref = oc.execute_plan(plan, tables)["output"][0]["cols"]
        rep = parity.compare_agg(dev, ref, 2, ["count", "rel", "exact"])
        rep.update(rows=n, oracle_s=round(time.time() - t0, 2), device_mode="high-cardinality" if mode else "global table",
                   scope=f"the full-cardinality C3 plan over rows [0, {n}) of the same generator, device vs the oracle")
        return rep
    except Exception as e:  # the legs must never break the bench line
        import traceback
        traceback.print_exc()
        return {"ok": False, "error": f"C3 full parity failed: {e}"}


def c5_leg(args, engine, ctx, P, reps=5):
    """BASELINE config C5: conn_stats bin(time_, 10 s) x (upid, remote_addr) sums joined to pod
    metadata (plans.c5_plan: MemorySource -> Map(bin) -> Agg -> Equijoin <- MemorySource), the
    unmodified plan through the C++ engine over HBM-resident stored tables (pxc_execute_plan):
    fused consume with the bin key, finalize, device equijoin, result D2H + PXRB.  Timed at
    --c5-rows rows; parity and the CPU baseline (oracle, one thread) on a 1M-row table of the
    same shape (the restated agg + join runs ~0.2M rows/s).  Roofline: agg_consume over the
    five referenced conn_stats columns (time_ 8 + upid 16 + remote_addr 4 + payload + two INT64)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    try:
        from pixie_amd import synth
        shape = dict(n_pods=1000, n_addrs=100, span_s=300)

        def store(n, rpb):
            tabs = synth.c5_tables(SEED, n, rows_per_batch=rpb, **shape)
            for name, t in tabs.items():
                engine.create_table(name, t["types"], t["names"])
                for b in t["batches"]:
                    engine.append(name, b)
            return tabs

        def drop():
            engine.drop_table("conn_stats")
            engine.drop_table("pod_metadata")

        pb = P.c5_plan().SerializeToString()
        # parity + CPU baseline at 1M rows
        import oracle_client as oc
        from kat import rows as kat_rows
        small = 1_000_000
        tabs = store(small, 1 << 16)
        dev = engine.execute(P.c5_plan())["output"]
        secs, ref = oc.execute_plan_timed(P.c5_plan(), tabs)
        ref = ref["output"]
        rows_d = sorted(r for b in dev for r in kat_rows(b["cols"]))
        rows_r = sorted(r for b in ref for r in kat_rows(b["cols"]))
        parity = {"rows": small, "output_rows": len(rows_r), "ok": rows_d == rows_r,
                  "bar": "output rows (time bin, upid, remote_addr, pod, namespace, sums) identical as a multiset"}
        cpu = {"value": small / secs, "unit": "rows/s", "cores": 1, "kind": "port",
               "sample": f"{small} conn_stats rows as 65536-row RowBatches, C5 plan, oracle/ one thread, {secs:.2f} s window"}
        drop()
        del tabs
        n = args.c5_rows
        store(n, 1 << 20)
        t = engine.device_table("conn_stats")
        from pixie_amd.device import Table
        tt = Table(ctx, P.CONN_TYPES, handle=t, owned=False)
        c = {nm: i for i, nm in enumerate(P.CONN_NAMES)}
        alg = 8 * n + 16 * n + tt.device_bytes(c["remote_addr"]) + 16 * n
        engine.execute_raw(pb)
        ctx.sync()
        ctx.reset_stats()
        ctx.set_profiling(True)
        times = []
        res_len = 0
        for _ in range(reps):
            tq = time.perf_counter()
            res_len = engine.execute_bytes_len(pb)
            times.append(time.perf_counter() - tq)
        ctx.sync()
        ctx.set_profiling(False)
        kms = {k: round(ctx.kernel_stats(k)[1] / reps, 4) for k in KERNELS + ["join_build", "join_slot_flags", "join_probe_count", "join_unprobed_count", "join_probe_write", "join_unprobed_write", "join_gather",
                                                                               "agg_consume_list"]
               if ctx.kernel_stats(k)[0]}
        l, ms = ctx.kernel_stats("agg_consume")
        avg = ms / max(l, 1)
        st = sorted(times)
        out = {"workload": "C5: conn_stats bin(time_, 10s) x (upid, remote_addr) sum(bytes_sent), sum(bytes_recv), "
                           "inner equijoin on upid to pod_metadata (pxc_execute_plan over stored tables)",
               "rows": n, "queries": reps, "ms_per_query": sum(times) * 1000 / reps, "ms_median": st[len(st) // 2] * 1000,
               "ms_min": st[0] * 1000, "value": n * reps / sum(times), "unit": "rows/s", "result_bytes": int(res_len),
               "kernel_ms_per_query": kms, "algorithmic_bytes_per_row": alg / n,
               "roofline": {"bound": "hbm", "kernel": "agg_consume", "achieved": alg / (avg / 1000.0) / 1e9, "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": alg / (avg / 1000.0) / 1e9 / HBM_PEAK_GBS, "avg_launch_ms": avg},
               "parity": parity, "cpu_baseline": cpu, "shape": shape}
        drop()
        return out
    except Exception as e:  # the legs must never break the bench line
        import traceback
        traceback.print_exc()
        return {"error": f"c5 leg failed: {e}"}


def c1_leg(args, P, n=1_000_000, reps=3):
    """BASELINE config C1: carnot_executable's shape -- a 1M-row http_events CSV (type row, name
    row), groupby(service).agg(count, mean(latency)) -- through pixie_amd/lib/carnot_csv (CSV
    parse into --rowbatch_size 100-row RowBatches, the reference default, then the engine), wall
    time including the CSV parse (carnot_executable.cc:232-277), next to the oracle's execution
    window over the same parsed rows (one thread)."""
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tests"))
    try:
        import oracle_client as oc
        from pixie_amd.device import datagen_http_events
        exe = os.path.join(REPO, "pixie_amd", "lib", "carnot_csv")
        cols = datagen_http_events(SEED, 0, n, threads=16)
        svc, lat = cols[P.HE["service"]], cols[P.HE["latency"]]
        d = tempfile.mkdtemp(prefix="pxg_c1_", dir=os.environ.get("TMPDIR", "/tmp"))
        csv, pbf, outf = os.path.join(d, "in.csv"), os.path.join(d, "plan.pb"), os.path.join(d, "out.csv")
        raw = svc.data.tobytes()
        o = svc.offsets
        with open(csv, "w") as f:
            f.write("string,int64\nservice,latency\n")
            f.write("".join(f"{raw[o[i]:o[i + 1]].decode()},{int(lat.values[i])}\n" for i in range(n)))
        types, names = [P.STRING, P.INT64], ["service", "latency"]
        plan = P.linear_plan([P.source_op("csv_table", types, names, [0, 1]),
                              P.agg_op([0], [P.agg_expr("count", [P.col(1)], [P.INT64]), P.agg_expr("mean", [P.col(1)], [P.INT64], fid=1)],
                                       ["service"], ["count", "mean"]),
                              P.sink_op("output")])
        with open(pbf, "wb") as f:
            f.write(plan.SerializeToString())
        walls, stats = [], []
        for _ in range(reps + 1):
            t0 = time.perf_counter()
            r = subprocess.run([exe, f"--input_file={csv}", f"--output_file={outf}", f"--plan_file={pbf}", "--rowbatch_size=100"],
                               capture_output=True, text=True, timeout=300)
            walls.append(time.perf_counter() - t0)
            if r.returncode != 0:
                return {"error": r.stderr[-500:]}
            stats.append(json.loads([ln for ln in r.stderr.splitlines() if ln.startswith("{")][-1]))
        walls, stats = walls[1:], stats[1:]
        groups = sum(1 for _ in open(outf))
        batches = [[c.slice(a, min(a + 100, n)) for c in (svc, lat)] for a in range(0, n, 100)]
        secs, _ = oc.execute_plan_timed(plan, {"csv_table": {"types": types, "names": names, "batches": batches}})
        best = min(range(reps), key=lambda i: walls[i])
        return {"workload": "C1: carnot_csv (carnot_executable harness) 1M-row http_events CSV, groupby(service): count, mean(latency), "
                            "--rowbatch_size 100",
                "rows": n, "groups": groups, "runs": reps, "wall_s_median": sorted(walls)[reps // 2], "wall_s_min": walls[best],
                "harness_stats_best": stats[best], "rows_per_s_wall": n / sorted(walls)[reps // 2],
                "cpu_baseline": {"value": n / secs, "unit": "rows/s", "cores": 1, "kind": "port",
                                 "sample": f"oracle over the same {n} parsed rows as 100-row RowBatches (execution window "
                                           f"{secs:.3f} s, CSV parse excluded)"}}
    except Exception as e:  # the legs must never break the bench line
        import traceback
        traceback.print_exc()
        return {"error": f"c1 leg failed: {e}"}


def n1_leg(args, ctx, P, Table, plan_agg):
    """BASELINE north_star: 1B-row filter + group-by(service, req_path) with count/mean/p50/p99
    on ONE GPU (the config the >= 60% of HBM roofline target is quoted on)."""
    n = args.n1_rows
    t0 = time.time()
    t = Table(ctx, P.HTTP_TYPES)
    t.append_http_events(SEED, 0, n, N_PAIR_KEYS)
    gen_s = time.time() - t0
    alg = alg_bytes_of(t, n)
    a = plan_agg(ctx, P.c2_plan(with_pluck=True), "http_events", P.HTTP_TYPES, expected_groups=65536)

    def step():
        a.reset()
        a.consume(t)
        return a.finalize()

    g = step()
    ctx.sync()
    # Per-kernel breakdown of the 1B-row step from one untimed, fully event-bracketed step
    # (sum of launch durations per kernel name; finalize runs on three streams, so the kernels
    # overlap and their sum exceeds the step's span).
    ctx.reset_stats()
    ctx.set_profiling(True)
    t_prof = time.perf_counter()
    step()
    ctx.sync()
    prof_step_ms = (time.perf_counter() - t_prof) * 1000.0
    fallback_groups = [a.info()["big_sort_groups"]]  # big groups the selection path handed to the sort path
    ctx.set_profiling(False)
    kernel_ms = {}
    for name in KERNELS:
        l, ms = ctx.kernel_stats(name)
        if l:
            kernel_ms[name] = round(ms, 4)
    ctx.reset_stats()
    ctx.set_profiling(True, only="agg_consume")
    ctx.sync()
    ts = time.perf_counter()
    for _ in range(args.n1_steps):
        g = step()
    ctx.sync()
    el = time.perf_counter() - ts
    fallback_groups.append(a.info()["big_sort_groups"])
    ctx.set_profiling(False)
    l, ms, pre = consume_stats(ctx)
    avg = ms / args.n1_steps
    achieved = alg / (avg / 1000.0) / 1e9
    par = None
    if not args.no_n1_parity:
        # Outside the timed region: the result of the last timed step against the generator's
        # ground truth for all n rows (tests/parity.py::check_c2_against_truth).
        par = n1_parity(a.result(), n)
    out = {
        "workload": "north_star: 1B-row http_events on 1 GPU, Filter(resp_status>=400) -> Map -> Agg by (service, req_path): "
                    "count, mean, quantiles (p50/p99 plucked)",
        "rows": n, "steps": args.n1_steps, "ms_per_step": el * 1000.0 / args.n1_steps,
        "value": n * args.n1_steps / el, "unit": "rows/s", "groups": g, "selected_rows": a.rows_selected(),
        "algorithmic_bytes_per_row": alg / n, "generate_s": gen_s,
        "kernel_ms_per_step": kernel_ms, "profiled_step_ms": round(prof_step_ms, 3),
        "finalize_ms_per_step": round(el * 1000.0 / args.n1_steps - avg, 3),
        "sort_fallback_groups": {"profiled_step": fallback_groups[0], "last_timed_step": fallback_groups[1]},
        # the whole query (consume + finalize, HBM-resident inputs to finalized results) against
        # the HBM roofline: algorithmic bytes / step time -- the north_star's >= 0.60 target
        "roofline_step": {"achieved": alg / (el / args.n1_steps) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": alg / (el / args.n1_steps) / 1e9 / HBM_PEAK_GBS,
                          "per": "whole step: reset + consume + finalize, timed over the steps"},
        "roofline": {"bound": "hbm", "kernel": "agg_consume", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(args, n),
                     "traffic_source": "committed file (replaced by the live PMC leg when it runs)", "algorithmic_bytes_per_launch": alg,
                     "avg_launch_ms": avg, "consume_ms_per_step": avg, "launches_per_step": l / args.n1_steps,
                     "prefix_ms_per_step": pre / args.n1_steps},
        "cpu_baseline": "same CPU Carnot restatement as the top-level cpu_baseline (rows/s of one thread; the plan is per-row linear)",
        "parity": par,
    }
    a.close()
    t.close()
    return out


def n1_parity(dev, n):
    """Full-size parity of the 1B-row result: every group key and count bit-exact, every mean
    within 1e-6 (sum(mean*count) within 1e-9) of the generator's exact sums, quantiles of the 20
    largest groups within the rank bound and of 200 seeded <= 8000-value groups within 4 ULP of
    the oracle t-digest fed each group's values in row order (test infrastructure, tests/parity.py)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    try:
        import parity
        return parity.check_c2_against_truth(dev, SEED, 0, n, threads=16)
    except Exception as e:  # the legs must never break the bench line
        import traceback
        traceback.print_exc()
        return {"ok": False, "error": f"n1 parity failed: {e}"}


def cpu_shard_child(row0, rows, batch_rows):
    """One shard process of the parallel CPU baseline: the C2 plan over rows [row0, row0+rows)
    through the CPU Carnot restatement (one thread); prints its execution window."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_client as oc
    from pixie_amd import plans as P
    from pixie_amd.device import datagen_http_events
    need = {P.HE["service"], P.HE["req_path"], P.HE["resp_status"], P.HE["latency"]}
    cols = datagen_http_events(SEED, row0, rows, n_pair_keys=N_PAIR_KEYS, threads=1)
    batch = [c if i in need else oc.AbsentColumn(c.type, len(c)) for i, c in enumerate(cols)]
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [batch], "names": P.HTTP_NAMES}}
    secs, res = oc.execute_plan_timed(P.c2_plan(with_pluck=False), tables, batch_rows=batch_rows)
    print(json.dumps({"secs": secs, "rows": rows, "groups": len(res["output"][0]["cols"][0])}), flush=True)


def cpu_timing_child(rows, reps, batch_rows):
    """The primary CPU baseline: this process pins itself to core 0 before it
    builds anything, generates `rows` rows of the bench table, runs the C2 plan through the CPU
    Carnot restatement once as a warm-up and `reps` more times, and prints every execution
    window (first GenerateNext .. last emit)."""
    os.sched_setaffinity(0, {0})
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_client as oc
    from pixie_amd import plans as P
    from pixie_amd.device import datagen_http_events
    need = {P.HE["service"], P.HE["req_path"], P.HE["resp_status"], P.HE["latency"]}
    cols = datagen_http_events(SEED, 0, rows, n_pair_keys=N_PAIR_KEYS, threads=1)
    batch = [c if i in need else oc.AbsentColumn(c.type, len(c)) for i, c in enumerate(cols)]
    tables = {"http_events": {"types": P.HTTP_TYPES, "batches": [batch], "names": P.HTTP_NAMES}}
    secs = []
    for _ in range(reps + 1):
        s, _res = oc.execute_plan_timed(P.c2_plan(with_pluck=False), tables, batch_rows=batch_rows)
        secs.append(s)
    print(json.dumps({"warmup_secs": secs[0], "secs": secs[1:], "rows": rows, "cpus": sorted(os.sched_getaffinity(0))}), flush=True)


def cpu_timing_leg(args):
    """Runs cpu_timing_child in a fresh interpreter (never a fork of this GPU process)."""
    import subprocess
    try:
        kid = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-timing-child", str(args.cpu_timing_rows),
                              str(args.cpu_timing_reps), str(args.cpu_batch_rows)], stdout=subprocess.PIPE,
                             stderr=subprocess.DEVNULL, timeout=900)
        if kid.returncode != 0:
            return {"error": f"cpu timing process exited {kid.returncode}"}
        return json.loads(kid.stdout.decode().strip().splitlines()[-1])
    except Exception as e:  # the legs must never break the bench line
        return {"error": f"cpu timing leg failed: {e}"}


def cpu_parallel_leg(args, n, row0):
    """Supplementary CPU baseline (P PEMs): P processes, each running the C2
    plan over its own 1/P row shard with the CPU Carnot restatement, started together; the value
    is n / the slowest shard's execution window.  The PEM -> Kelvin merge is left out (quantiles
    have no Serialize in the reference, udf.h:367, so it cannot be split at all), which makes this
    an upper bound for the CPU.  Processes are children (fresh interpreters), never forks."""
    import subprocess
    procs = args.cpu_procs
    try:
        per = (n + procs - 1) // procs
        kids = []
        for p in range(procs):
            a = p * per
            k = min(per, n - a)
            if k <= 0:
                break
            kids.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-shard-child", str(row0 + a), str(k),
                                          str(args.cpu_batch_rows)], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL))
        outs = []
        for kp in kids:
            o, _ = kp.communicate(timeout=600)
            if kp.returncode != 0:
                return {"error": f"shard process exited {kp.returncode}"}
            outs.append(json.loads(o.decode().strip().splitlines()[-1]))
        slow = max(o["secs"] for o in outs)
        return {"value": n / slow, "unit": "rows/s", "cores": len(outs), "kind": "port",
                "sample": f"all {n} rows in {len(outs)} shard processes of {per} rows (one thread each, started together), "
                          f"C2 plan per shard; slowest execution window {slow:.2f} s (mean {sum(o['secs'] for o in outs) / len(outs):.2f} s); "
                          f"PEM-side only, no merge (quantiles have no Serialize, udf.h:367): an upper bound for P PEMs"}
    except Exception as e:  # the legs must never break the bench line
        return {"error": f"parallel cpu leg failed: {e}"}


def oracle_leg(args, n, row0, dev_result):
    """The CPU Carnot restatement (oracle/, one thread) over the same n rows as the GPU table, as
    cpu_batch_rows-row RowBatches, C2 plan: its execution window is cpu_baseline; its result is
    the parity reference for the device result of the timed steps (tests/parity.py)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    try:
        import numpy as np
        import oracle_client as oc
        import parity
        from pixie_amd import plans as P
        from pixie_amd.device import datagen_http_events
        need = {P.HE["service"], P.HE["req_path"], P.HE["resp_status"], P.HE["latency"]}
        batches, keys, sel, vals = [], [], [], []
        for a in range(0, n, args.gen_slice):
            k = min(args.gen_slice, n - a)
            cols = datagen_http_events(SEED, row0 + a, k, n_pair_keys=N_PAIR_KEYS, threads=16)
            batches.append([c if i in need else oc.AbsentColumn(c.type, len(c)) for i, c in enumerate(cols)])
            keys.append([cols[P.HE["service"]], cols[P.HE["req_path"]]])
            sel.append(cols[P.HE["resp_status"]].values >= 400)
            vals.append(cols[P.HE["latency"]].values / 1e6)
            del cols
        tables = {"http_events": {"types": P.HTTP_TYPES, "batches": batches, "names": P.HTTP_NAMES}}
        secs, res = oc.execute_plan_timed(P.c2_plan(with_pluck=False), tables, batch_rows=args.cpu_batch_rows)
        cpu_model = ""
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
        cpu = {"value": n / secs, "unit": "rows/s", "cores": 1, "kind": "port",
               "sample": f"all {n} rows of the bench table (regenerated on the host, bit-identical to the device generator) "
                         f"as {args.cpu_batch_rows}-row RowBatches, C2 plan (quantiles JSON, no pluck), 1 thread of "
                         f"{cpu_model or 'host CPU'}; {secs:.2f} s execution window (first GenerateNext .. last emit); "
                         f"CPU Carnot restated in oracle/ (reference unbuildable, SURVEY.md §8c)"}
        # the primary number is the median of 5 runs after a warm-up, on core 0.
        if args.cpu_timing_reps > 0:
            tm = cpu_timing_leg(args)
            if "secs" in tm and tm["secs"]:
                med = sorted(tm["secs"])[len(tm["secs"]) // 2]
                k = tm["rows"]
                cpu = {"value": k / med, "unit": "rows/s", "cores": 1, "kind": "port",
                       "sample": f"the first {k} rows of the bench table (bit-identical host regeneration) as {args.cpu_batch_rows}-row "
                                 f"RowBatches, C2 plan (quantiles JSON, no pluck), one process pinned to core {tm['cpus']} of "
                                 f"{cpu_model or 'host CPU'}: median of {len(tm['secs'])} execution windows after 1 warm-up "
                                 f"({', '.join(f'{x:.2f}' for x in tm['secs'])} s; first GenerateNext .. last emit); "
                                 f"CPU Carnot restated in oracle/ (reference unbuildable, SURVEY.md §8c)",
                       "runs_s": tm["secs"], "warmup_s": tm["warmup_secs"],
                       "full_table": {"rows": n, "secs": secs, "value": n / secs, "pinned": False}}
            else:
                cpu["timing_error"] = tm.get("error")
        par = None
        if dev_result is not None:
            ref = res["output"][0]["cols"]
            t0 = time.time()
            rep = parity.compare_agg(dev_result, ref, 2, ["count", "rel", "quantiles"], parity.GroupValues(keys, sel, vals))
            rep["rows"] = n
            rep["check_s"] = round(time.time() - t0, 2)
            rep["bars"] = ("groups/counts bit-exact; mean 1e-6 rel; quantiles <= 4 ULP for groups <= 8000 values, "
                           "midpoint-rank bound 2*pi*sqrt(q(1-q))/1000 + 1/n above")
            par = rep
        return cpu, par
    except Exception as e:  # the legs must never break the bench line
        import traceback
        traceback.print_exc()
        return ({"value": None, "unit": "rows/s", "cores": 1, "kind": "port", "sample": f"failed: {e}"},
                {"ok": False, "error": f"oracle leg failed: {e}"})


if __name__ == "__main__":
    main()
