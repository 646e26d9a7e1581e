# Ad-hoc GPU command of the current session (gpurun -- 'bash tools/gpu_cmd.sh'): each step has its
# own time limit and the steps are chained with &&.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="--steps 30 --warmup 3 --no-cpu-baseline --no-c5 --no-c1 --no-pmc --n1-rows 0"
for r in 1 2; do
timeout -k 10 300 python3 -u bench.py $B > gpurun_out/b_o$r.json 2> gpurun_out/b_o$r.err || exit 1
PXG_SPIN_EXP=1 timeout -k 10 300 python3 -u bench.py $B > gpurun_out/b_s$r.json 2> gpurun_out/b_s$r.err || exit 1
done
for f in o1 s1 o2 s2; do python3 -c "
import json;d=json.load(open('gpurun_out/b_$f.json'));print('$f', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['engine_query']['ms_median'], d['c3']['ms_per_step'])"; done
