cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
 for pkg in $GRAFT_REPO_ROOT/ab_sub $GRAFT_REPO_ROOT; do
  timeout -k 10 120 python -u ab_sub/diag.py $pkg 100000000 5 >> gpurun_out/ab_sub.log 2>&1 || exit 1
  timeout -k 10 200 python -u ab_sub/diag.py $pkg 1000000000 3 >> gpurun_out/ab_sub.log 2>&1 || exit 1
 done
done
