# A/B of finalize variants at 1B rows: bash tools/n1_env_ab.sh "label:ENV=1" "label2:" (on the GPU box).
# Each variant: rocprofv3 kernel stats over one warm n1 step -> gpurun_out/n1env_<label>/.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/n1env_$label -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-engine-leg --no-n1-parity --no-pmc --rows-per-gpu 1000000 > gpurun_out/n1env_$label.log 2>&1 || exit 1
done
