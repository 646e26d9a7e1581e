cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag3
PXG_TIMING=1 timeout -k 10 120 python -u tools/engine_timing.py > gpurun_out/diag3/engine_dev.log 2>&1 && \
timeout -k 10 300 python -u tools/consume_diag.py 0 > gpurun_out/diag3/consume_diag.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/diag3/pytest_gpu.log 2>&1
