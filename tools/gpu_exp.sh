cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PXG_CONSUME_TILE=32768 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_parity.py tests/test_partial.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_q.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-engine-leg --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
