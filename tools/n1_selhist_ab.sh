# A/B of quant_sel_hist chunks per block at 1B rows: CAPS="8 32" bash tools/n1_selhist_ab.sh (on the GPU box)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ${CAPS:-8 32}; do
  PXG_SEL_HIST_CPB=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/n1ab_$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-engine-leg --no-n1-parity --no-pmc --rows-per-gpu 1000000 > gpurun_out/n1ab_$v.log 2>&1 || exit 1
  grep -E "BigHist|BigCollect" gpurun_out/n1ab_$v/run_kernel_stats.csv | cut -d, -f2-4 | sed "s/^/cap $v: /" >> gpurun_out/n1ab.txt
done
