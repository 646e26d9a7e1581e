# Ad-hoc GPU command of the current session (gpurun -- 'bash tools/gpu_cmd.sh'): each step has its
# own time limit and the steps are chained with &&.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_host_engine.py -k "past_one_chunk or result_image" > gpurun_out/t.log 2>&1 &&
true
rc=$?; tail -8 gpurun_out/t.log; exit $rc
