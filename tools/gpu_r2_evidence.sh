# Round-2 evidence pass: full GPU suite, smoke, bench line, rocprofv3 kernel stats of the timed C2
# steps (no N1 / engine / oracle legs, so the consume average matches the bench line's), the
# two PMC traffic passes over the consume kernel, and a 2-rank rehearsal of the bench N>1 path
# (both ranks on GPU 0, gloo exchange: RCCL refuses two ranks on one device).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-engine-leg --n1-rows 0 > gpurun_out/prof.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-engine-leg --n1-rows 0 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-engine-leg --n1-rows 0 > gpurun_out/pmc_write.log 2>&1 && \
python3 tools/pmc_summary.py --rows 100000000 --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --out gpurun_out/pmc_agg_consume.json > gpurun_out/pmc_summary.log 2>&1 && \
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --share-gpu0 --backend gloo --steps 5 --warmup 2 --rows-per-gpu 50000000 > gpurun_out/bench_2rank_gloo.json 2> gpurun_out/bench_2rank_gloo.err
