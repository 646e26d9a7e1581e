cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_exec_stats.py tests/test_host_engine.py -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_stats.log 2>&1
