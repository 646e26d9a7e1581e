cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcc
run() { timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmcc/$1 -o run --output-format csv -- python3 tools/consume_diag.py child 100000000 2 > gpurun_out/pmcc/$1.log 2>&1; }
run TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum && \
run TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum && \
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU
