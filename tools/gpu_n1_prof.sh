# North-star (1B rows, 1 GPU) profile evidence: rocprofv3 kernel stats of the timed 1B-row steps
# and the two PMC traffic passes over its consume kernel.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="bench.py --rows-per-gpu 1000000000 --no-cpu-baseline --no-engine-leg --n1-rows 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_n1 -o run --output-format csv -- python3 $B --steps 5 --warmup 1 > gpurun_out/prof_n1.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_n1_fetch -o run --output-format csv -- python3 $B --steps 1 --warmup 1 > gpurun_out/pmc_n1_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_n1_write -o run --output-format csv -- python3 $B --steps 1 --warmup 1 > gpurun_out/pmc_n1_write.log 2>&1 && \
python3 tools/pmc_summary.py --rows 1000000000 --fetch gpurun_out/pmc_n1_fetch --write gpurun_out/pmc_n1_write --out gpurun_out/pmc_agg_consume_n1.json > gpurun_out/pmc_n1_summary.log 2>&1 && \
cp gpurun_out/pmc_agg_consume_n1.json profiles/ && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-engine-leg > gpurun_out/bench_n1chk.json 2> gpurun_out/bench_n1chk.err
