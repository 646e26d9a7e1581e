cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_comm_gpu.py -v --timeout 400 --timeout-method thread -m gpu > gpurun_out/pytest_comm.log 2>&1
