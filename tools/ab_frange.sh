# Library A/B on the GPU box: ab_alt/libpxg_base.so against ab_alt/libpxg_b16.so and the working
# build, alternating processes (tools/lib_ab.py).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/lib_ab.log
for spec in "100000000 20 c2" "1000000000 5 c2" "100000000 5 c3_full"; do
  for i in 1 2; do
    PXG_LIB_PATH=$PWD/ab_alt/libpxg_base.so timeout -k 10 200 python3 tools/lib_ab.py b32 $spec >> $L 2>&1 || exit 1
    PXG_LIB_PATH=$PWD/ab_alt/libpxg_b16.so timeout -k 10 200 python3 tools/lib_ab.py b16 $spec >> $L 2>&1 || exit 1
  done
done
