# Full GPU suite + chain timing + selection stats + bench line.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u tools/chain_timing.py > gpurun_out/chain_timing.log 2>&1 && \
PXG_DIAG_SEL=1 PXC_TIMING=0 timeout -k 10 200 python -u tools/engine_timing.py > gpurun_out/sel_diag.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
