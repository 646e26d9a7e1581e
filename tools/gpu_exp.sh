cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_big_select.py tests/test_gpu_parity.py tests/test_scale_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_q.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-engine-leg --n1-rows 0 > gpurun_out/tl.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-engine-leg > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
