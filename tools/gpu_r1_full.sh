# Round-1 evidence run: GPU tests, smoke, rocprof kernel stats, PMC traffic passes, a 2-rank
# gloo rehearsal of the multi-GPU exchange on one GPU, and the default bench line.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-engine-leg > gpurun_out/prof.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-engine-leg > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-engine-leg > gpurun_out/pmc_write.log 2>&1 && \
python3 tools/pmc_summary.py --rows 100000000 --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --out profiles/pmc_agg_consume.json > gpurun_out/pmc_summary.log 2>&1 && \
cp profiles/pmc_agg_consume.json gpurun_out/ && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --rows-per-gpu 20000000 --backend gloo --share-gpu0 --no-cpu-baseline > gpurun_out/bench_2r.json 2> gpurun_out/bench_2r.err && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
