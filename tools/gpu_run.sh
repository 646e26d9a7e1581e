# One documented runner for the GPU box (gpurun -- 'bash tools/gpu_run.sh MODE...'): each mode is
# one step with its own time limit, steps chained with && so the first failure ends the call.
# Output goes under gpurun_out/ (merged back by gpurun); copy what is judged into profiles/.
#   tests  : pytest -m gpu (one process) + __graft_entry__.smoke()
#   bench  : bench.py default line (C2 + legs + n1 with parity) -> gpurun_out/bench.json
#   prof   : rocprofv3 --kernel-trace --stats over the bench's timed C2 steps only
#   n1prof : the same over the 1B-row n1 steps (no C2 legs)
#   n1only : rocprofv3 stats of tools/n1_prof.py alone (every launch a 1B-row launch)
#   pmc    : FETCH_SIZE / WRITE_SIZE passes over the consume kernel (C2) + summary JSON
#   c3prof : rocprofv3 stats of the C3 leg
#   diag   : tools/consume_diag.py timing modes (0 production, 2 filter only, 3 keys + hash)
#   filterpmc: the Filter -> Map leg alone + FETCH_SIZE / WRITE_SIZE passes of its filter kernels
#   c5pmc  : FETCH_SIZE / WRITE_SIZE passes over the C5 query's consume kernel (tools/c5_timing.py)
#   multi2 : bench.py --gpus 2 --share-gpu0 --backend gloo (the N>1 line, both ranks on GPU 0)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="--no-cpu-baseline --no-engine-leg"
step() {
  case "$1" in
    tests) timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 &&
           timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench) timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 $B --n1-rows 0 --no-pmc > gpurun_out/prof.log 2>&1 ;;
    n1prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_n1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 $B --no-n1-parity --no-pmc --rows-per-gpu 1000000 > gpurun_out/prof_n1.log 2>&1 ;;
    pmc) timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --pmc-child 100000000 > gpurun_out/pmc_fetch.log 2>&1 &&
         timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --pmc-child 100000000 > gpurun_out/pmc_write.log 2>&1 &&
         python3 tools/pmc_summary.py --steps 3 --rows 100000000 --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --out gpurun_out/pmc_agg_consume.json > gpurun_out/pmc_summary.log 2>&1 ;;
    n1only) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_n1only -o run --output-format csv -- python3 tools/n1_prof.py 3 > gpurun_out/prof_n1only.log 2>&1 ;;
    c3prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 tools/c3_prof.py > gpurun_out/prof_c3.log 2>&1 ;;
    diag) timeout -k 10 300 python3 tools/consume_diag.py 0 2 3 > gpurun_out/diag.log 2>&1 ;;
    filterpmc) timeout -k 10 200 python3 tools/ops_bench.py > gpurun_out/ops_bench.json 2> gpurun_out/ops_bench.err &&
         timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fpmc_fetch -o run --output-format csv -- python3 tools/ops_bench.py > gpurun_out/fpmc_fetch.log 2>&1 &&
         timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/fpmc_write -o run --output-format csv -- python3 tools/ops_bench.py > gpurun_out/fpmc_write.log 2>&1 &&
         python3 tools/pmc_summary.py --kernel FilterWriteKernel --name filter_write --rows 100000000 --fetch gpurun_out/fpmc_fetch --write gpurun_out/fpmc_write --out gpurun_out/fpmc_write.json > /dev/null 2>&1 &&
         python3 tools/pmc_summary.py --kernel FilterCountKernel --name filter_count --rows 100000000 --fetch gpurun_out/fpmc_fetch --write gpurun_out/fpmc_write --out gpurun_out/fpmc_count.json > /dev/null 2>&1 ;;
    c5pmc) timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/c5pmc_fetch -o run --output-format csv -- python3 tools/c5_timing.py 20000000 2 > gpurun_out/c5pmc_fetch.log 2>&1 &&
         timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/c5pmc_write -o run --output-format csv -- python3 tools/c5_timing.py 20000000 2 > gpurun_out/c5pmc_write.log 2>&1 &&
         python3 tools/pmc_summary.py --kernel AggConsumeFastKernel --name c5_agg_consume --rows 20000000 --fetch gpurun_out/c5pmc_fetch --write gpurun_out/c5pmc_write --out gpurun_out/c5pmc_consume.json > gpurun_out/c5pmc_summary.log 2>&1 ;;
    multi2) timeout -k 10 400 python3 -u bench.py --gpus 2 --share-gpu0 --backend gloo --steps 3 --warmup 1 > gpurun_out/bench_multi2.json 2> gpurun_out/bench_multi2.err ;;
    *) echo "unknown mode $1" >&2; return 2 ;;
  esac
}
for m in "$@"; do
  step "$m" || { echo "step $m failed ($?)" >&2; exit 1; }
done
