# Library A/B on the GPU box: ab_alt/libpxg_base.so against ab_alt/libpxg_hc.so, alternating
# processes (tools/lib_ab.py).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/lib_ab.log
for spec in "100000000 20 c3" "100000000 5 c3_full"; do
  for i in 1 2 3; do
    PXG_LIB_PATH=$PWD/ab_alt/libpxg_base.so timeout -k 10 200 python3 tools/lib_ab.py base $spec >> $L 2>&1 || exit 1
    PXG_LIB_PATH=$PWD/ab_alt/libpxg_hc.so timeout -k 10 200 python3 tools/lib_ab.py hc $spec >> $L 2>&1 || exit 1
  done
done
