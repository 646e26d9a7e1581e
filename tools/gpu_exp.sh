cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 200 python -u ab_v5/eng_ab.py $GRAFT_REPO_ROOT/ab_v5 >> gpurun_out/ab_v5.log 2>&1 || exit 1
timeout -k 10 200 python -u ab_v5/eng_ab.py $GRAFT_REPO_ROOT >> gpurun_out/ab_head.log 2>&1 || exit 1
done
