cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --share-gpu0 --backend gloo --steps 5 --warmup 2 --rows-per-gpu 50000000 > gpurun_out/bench_2rank_gloo.json 2> gpurun_out/bench_2rank_gloo.err
