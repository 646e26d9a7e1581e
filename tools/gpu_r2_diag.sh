# Diagnosis: engine stage timing (device- and host-generated tables), consume phase breakdown,
# FETCH_SIZE calibration for 8 B / 16 B per lane streams.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag
timeout -k 10 120 python -u tools/engine_timing.py > gpurun_out/diag/engine_dev.log 2>&1 && \
timeout -k 10 200 python -u tools/engine_timing.py --host-gen > gpurun_out/diag/engine_host.log 2>&1 && \
timeout -k 10 300 python -u tools/consume_diag.py 0 2 3 > gpurun_out/diag/consume_diag.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/diag/calib_fetch -o run --output-format csv -- ./tools/pmc_calib > gpurun_out/diag/calib.log 2>&1
