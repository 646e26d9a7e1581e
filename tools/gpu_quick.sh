# Quick GPU iteration: gpu tests, a short bench, and a kernel-trace profile.
# usage: bash tools/gpu_quick.sh [pytest-args...]
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-engine-leg > gpurun_out/prof.log 2>&1
