# A/B timing of consume variants on the GPU box (tools/): the GPU parity
# subset under each variant that changes results-relevant code, then tools/consume_diag.py
# children (C2 100M rows and the 1B-row north_star table) under each variant's env.
#   usage: bash tools/ab_run.sh "label:ENV=1 ENV2=1" "label2:X=1" ...   (X=1 = no-op env)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/ab_consume.log
PAR="tests/test_gpu_parity.py tests/test_scale_parity.py tests/test_consume_tiles.py tests/test_n1_parity.py"
for v in "$@"; do
  label=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 400 python -u -m pytest $PAR -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_$label.log 2>&1 || { echo "parity failed under $label" >&2; exit 1; }
done
for ROWS in 100000000 1000000000; do
  STEPS=5; [ $ROWS = 1000000000 ] && STEPS=3
  for i in 1 2; do
    for v in "$@"; do
      label=${v%%:*}; envs=${v#*:}
      env $envs timeout -k 10 150 python3 tools/consume_diag.py child $ROWS $STEPS | sed "s/^/$ROWS $label /" >> gpurun_out/ab_consume.log 2>&1 || exit 1
    done
  done
done
