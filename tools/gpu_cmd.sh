# Ad-hoc GPU command of the current session (gpurun -- 'bash tools/gpu_cmd.sh'): each step has its
# own time limit and the steps are chained with &&.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_n1only -o run --output-format csv -- python3 tools/n1_prof.py 4 > gpurun_out/prof_n1only.log 2>&1 &&
true
rc=$?; tail -3 gpurun_out/t.log; grep n1_prof gpurun_out/prof_n1only.log; exit $rc
