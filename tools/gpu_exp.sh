cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_consume_tiles.py tests/test_comm_gpu.py -v -rs --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_q.log 2>&1
