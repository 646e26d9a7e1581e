"""bench.py's N > 1 contract on CPU: `bench.py --gpus N` with no external launcher starts its own
N ranks (gloo rendezvous on 127.0.0.1), runs the barrier-bracketed timed loop, takes the max over
ranks, gathers the final rows on rank 0 and prints ONE JSON line with n_gpus = N and a parity
block checked against the generator's ground truth.  The device step is replaced by the CPU
stand-in of tests/bench_standin.py (--standin); the device step itself runs in the GPU tests and
on the driver's node.  A WORLD_SIZE that disagrees with --gpus is refused before anything runs."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    return env


def test_bench_gpus_2_launches_its_own_ranks_and_checks_parity():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--backend", "gloo", "--standin", "--steps", "2", "--warmup", "1",
                        "--rows-per-gpu", "40000"], env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["config"]["total_rows"] == 80_000
    assert "STAND-IN" in line["data"]
    par = line["parity"]
    assert par["ok"], par
    assert par["group_set_exact"] and par["counts_bit_exact"]
    assert line["config"]["groups"] == par["groups_ref"]
    assert line["value"] > 0 and line["ms_per_step"] > 0


def test_bench_three_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--backend", "gloo", "--standin", "--steps", "1", "--warmup", "0",
                        "--rows-per-gpu", "20000"], env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 3 and line["parity"]["ok"], line["parity"]


def test_bench_refuses_world_size_that_disagrees_with_gpus():
    env = dict(_env(), WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--standin"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "refusing" in r.stderr
    assert r.stdout.strip() == ""


def test_launcher_kills_ranks_after_rank_timeout():
    """a rank stuck in a collective must not hang `bench.py --gpus N` forever; after
    --rank-timeout the launcher kills every rank's process group and exits non-zero."""
    import time
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--backend", "gloo", "--standin", "--steps", "1", "--warmup", "0",
                        "--rows-per-gpu", "20000", "--standin-hang-rank", "1", "--rank-timeout", "20"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "rank-timeout" in r.stderr
    assert r.stdout.strip() == ""
    assert time.time() - t0 < 200
