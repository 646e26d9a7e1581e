# Ad-hoc GPU command of the current session (gpurun -- 'bash tools/gpu_cmd.sh'): each step has its
# own time limit and the steps are chained with &&.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="--steps 30 --warmup 3 --no-cpu-baseline --no-engine-leg --no-c5 --no-c1 --no-pmc --n1-rows 0"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/t.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 300 python3 -u bench.py $B > gpurun_out/b_4_$r.json 2>/dev/null || exit 1
PXG_CONSUME_BPC=5 timeout -k 10 300 python3 -u bench.py $B > gpurun_out/b_5_$r.json 2>/dev/null || exit 1
done
tail -1 gpurun_out/t.log
for f in 4_1 5_1 4_2 5_2; do python3 -c "
import json;d=json.load(open('gpurun_out/b_$f.json'));print('$f', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), (d.get('c3') or {}).get('ms_per_step'))"; done
