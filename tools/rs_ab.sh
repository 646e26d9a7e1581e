cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && : > gpurun_out/rs_ab.log
timeout -k 10 200 python3 tools/n1_prof.py 3 >> gpurun_out/rs_ab.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-engine-leg --no-c5 --no-c1 --no-pmc --n1-rows 0 > gpurun_out/rs_bench.json 2>>gpurun_out/rs_ab.log || exit 1
