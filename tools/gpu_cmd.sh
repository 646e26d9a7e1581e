# Ad-hoc GPU command of the current session (gpurun -- 'bash tools/gpu_cmd.sh'): each step has its
# own time limit and the steps are chained with &&.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_host_engine.py > gpurun_out/t.log 2>&1 &&
timeout -k 10 300 python3 tools/c5_timing.py 20000000 5 > gpurun_out/c5t.json 2> gpurun_out/c5t.log &&
true
rc=$?; tail -3 gpurun_out/t.log; cat gpurun_out/c5t.json; exit $rc
