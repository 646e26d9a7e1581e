cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_big_select.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_chain.log 2>&1 && \
timeout -k 10 200 python -u tools/chain_timing.py > gpurun_out/chain_timing.log 2>&1 && \
PXG_DIAG_SEL=1 PXC_TIMING=0 timeout -k 10 200 python -u tools/engine_timing.py > gpurun_out/sel_diag.log 2>&1
