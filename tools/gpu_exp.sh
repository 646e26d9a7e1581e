cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_big_select.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_q.log 2>&1 && \
timeout -k 10 300 python -u bench.py --rows-per-gpu 1000000000 --steps 3 --warmup 1 --no-cpu-baseline --no-engine-leg --n1-rows 0 > gpurun_out/bench_1b.json 2> gpurun_out/bench_1b.err && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-engine-leg --n1-rows 0 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
