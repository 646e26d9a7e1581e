# A/B timing of consume variants on the GPU box (tools/): GPU parity subset,
# then tools/consume_diag.py children under PXG_NO_PAIRS / PXG_NO_HOT.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/ab_consume.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_parity.py tests/test_consume_tiles.py tests/test_n1_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || exit 1
run() { # label env... rows steps
  local label=$1; shift
  env "$@" timeout -k 10 150 python3 tools/consume_diag.py child $ROWS $STEPS | sed "s/^/$label /" >> gpurun_out/ab_consume.log 2>&1
}
for ROWS in 100000000 1000000000; do
  STEPS=5; [ $ROWS = 1000000000 ] && STEPS=3
  for i in 1 2; do
    run "$ROWS base" PXG_NO_PAIRS=1 PXG_NO_HOT=1 || exit 1
    run "$ROWS pairs" PXG_NO_HOT=1 || exit 1
    run "$ROWS hot" PXG_NO_PAIRS=1 || exit 1
    run "$ROWS pairs+hot" X=1 || exit 1
  done
done
timeout -k 10 300 python3 tools/c5_diag.py 20000000 > gpurun_out/c5_diag.log 2>&1
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
