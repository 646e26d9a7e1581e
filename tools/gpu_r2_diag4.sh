cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag4
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/diag4/prof -o run --output-format csv -- python3 tools/engine_timing.py > gpurun_out/diag4/engine_dev.log 2>&1
