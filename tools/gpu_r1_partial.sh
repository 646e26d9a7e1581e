cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_partial.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_partial.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --rows-per-gpu 20000000 --backend gloo --share-gpu0 --no-cpu-baseline > gpurun_out/bench_2r.json 2> gpurun_out/bench_2r.err && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
