cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag2
timeout -k 10 120 python -u tools/engine_timing.py > gpurun_out/diag2/engine_dev.log 2>&1 && \
timeout -k 10 200 python -u tools/engine_timing.py --host-gen > gpurun_out/diag2/engine_host.log 2>&1
