# Profiling evidence only: rocprofv3 kernel stats of the timed bench steps (no engine leg, so the
# per-kernel averages match bench.py's roofline.avg_launch_ms) and the two PMC traffic passes.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-engine-leg > gpurun_out/prof.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-engine-leg > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-engine-leg > gpurun_out/pmc_write.log 2>&1 && \
python3 tools/pmc_summary.py --rows 100000000 --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --out gpurun_out/pmc_agg_consume.json > gpurun_out/pmc_summary.log 2>&1
