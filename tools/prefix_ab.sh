cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && : > gpurun_out/prefix_ab.log
for cfg in "32 1048576" "64 1048576" "128 524288" "256 262144" "32 1048576 NOPREC"; do
  set -- $cfg
  if [ "$3" = "NOPREC" ]; then export PXG_NO_PREC=1; else unset PXG_NO_PREC; fi
  PXG_PREFIX_DIV=$1 PXG_PREFIX_MIN=$2 timeout -k 10 120 python3 tools/prefix_ab.py 100000000 10 >> gpurun_out/prefix_ab.log 2>/dev/null || exit 1
done
unset PXG_NO_PREC
for cfg in "32 1048576" "128 1048576" "512 1048576"; do
  set -- $cfg
  PXG_PREFIX_DIV=$1 PXG_PREFIX_MIN=$2 timeout -k 10 200 python3 tools/prefix_ab.py 1000000000 4 >> gpurun_out/prefix_ab.log 2>/dev/null || exit 1
done
