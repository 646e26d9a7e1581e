set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  PXG_LIB_PATH=$PWD/ab_alt/libpxg_base.so timeout -k 10 120 python3 tools/lib_ab.py base 100000000 20 >> gpurun_out/prevals_ab.log 2>&1 || exit 1
  timeout -k 10 120 python3 tools/lib_ab.py prevals 100000000 20 >> gpurun_out/prevals_ab.log 2>&1 || exit 1
done
for i in 1 2; do
  PXG_LIB_PATH=$PWD/ab_alt/libpxg_base.so timeout -k 10 180 python3 tools/lib_ab.py base 1000000000 5 >> gpurun_out/prevals_ab.log 2>&1 || exit 1
  timeout -k 10 180 python3 tools/lib_ab.py prevals 1000000000 5 >> gpurun_out/prevals_ab.log 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py tests/test_row_records.py tests/test_n1_parity.py tests/test_hc_agg.py tests/test_consume_tiles.py -m gpu > gpurun_out/prevals_tests.log 2>&1
