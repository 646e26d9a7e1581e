# Ad-hoc GPU command of the current session (gpurun -- 'bash tools/gpu_cmd.sh'): each step has its
# own time limit and the steps are chained with &&.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_n1only -o run --output-format csv -- python3 tools/n1_prof.py 4 > gpurun_out/prof_n1only.log 2>&1 &&
true
rc=$?; grep n1_prof gpurun_out/prof_n1only.log; exit $rc
