cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for m in 0 1 2; do PXG_DIAG_QUANT=$m timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/qd_$m.json 2>/dev/null || exit 1; done
