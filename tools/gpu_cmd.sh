# Ad-hoc GPU command of the current session (gpurun -- 'bash tools/gpu_cmd.sh'): each step has its
# own time limit and the steps are chained with &&.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_big_select.py tests/test_fsplit.py tests/test_n1_parity.py tests/test_gpu_parity.py > gpurun_out/t.log 2>&1 &&
true
rc=$?; tail -5 gpurun_out/t.log; exit $rc
