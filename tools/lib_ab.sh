# Library A/B on the GPU box: ab_alt/libpxg_base.so (the committed build) against the working
# build, alternating processes (tools/lib_ab.py), then a parity subset.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/lib_ab.log
for spec in "100000000 20 c3" "100000000 5 c3_full"; do
  for i in 1 2 3; do
    PXG_LIB_PATH=$PWD/ab_alt/libpxg_base.so timeout -k 10 200 python3 tools/lib_ab.py base $spec >> $L 2>&1 || exit 1
    timeout -k 10 200 python3 tools/lib_ab.py new $spec >> $L 2>&1 || exit 1
  done
done
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_hc_agg.py tests/test_scale_parity.py tests/test_comm_gpu.py tests/test_partial.py tests/test_exchange_states.py tests/test_gpu_parity.py tests/test_filter_range.py -m gpu > gpurun_out/lib_ab_tests.log 2>&1
