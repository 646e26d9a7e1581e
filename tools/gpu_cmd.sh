# Ad-hoc GPU command of the current session (gpurun -- 'bash tools/gpu_cmd.sh'): each step has its
# own time limit and the steps are chained with &&.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_quant_lanes.py tests/test_host_engine.py > gpurun_out/t.log 2>&1 &&
timeout -k 10 300 python3 -u tools/engine_outlier.py 100000000 10 > gpurun_out/eo.json 2> gpurun_out/eo.log &&
PXC_TIMING= PXG_TIMING= timeout -k 10 300 python3 -u tools/engine_outlier.py 100000000 10 > gpurun_out/eo_plain.json 2> gpurun_out/eo_plain.err &&
true
rc=$?; tail -2 gpurun_out/t.log; cat gpurun_out/eo.json gpurun_out/eo_plain.json; exit $rc
