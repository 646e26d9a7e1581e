# Scratch GPU experiment runner (edited per experiment; the last one: full GPU suite, engine stage
# timing, and a C2 bench line without the oracle leg).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_q.log 2>&1 && \
PXC_TIMING=1 timeout -k 10 200 python -u tools/engine_timing.py > gpurun_out/engine_timing.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --n1-rows 0 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
