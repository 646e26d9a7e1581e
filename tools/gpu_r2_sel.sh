# Finalize rework check: selection-path + chain tests, quantile/join parity suites, bench line, kernel timeline.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_big_select.py tests/test_gpu_parity.py tests/test_split_agg.py tests/test_scale_parity.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_sel.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tl -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-engine-leg --n1-rows 0 > gpurun_out/tl.log 2>&1
