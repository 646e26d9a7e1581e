# rocprofv3 kernel stats of the north_star step under env variants (on the GPU box):
#   bash tools/n1_prof_ab.sh "label:ENV=1 ENV2=2" "label2:X=1" ...   -> gpurun_out/n1prof_<label>/
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/n1prof_$label -o run --output-format csv -- python3 tools/n1_prof.py 3 > gpurun_out/n1prof_$label.log 2>&1 || exit 1
done
