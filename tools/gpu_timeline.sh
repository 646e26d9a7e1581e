# Kernel timeline of the bench's timed steps (rocprofv3 kernel trace; no oracle / engine / N1 legs).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tl -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-engine-leg --n1-rows 0 > gpurun_out/tl.log 2>&1
