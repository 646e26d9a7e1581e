cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_carnot_csv.py tests/test_union_ordered.py tests/test_streaming_source.py tests/test_rowbatch_grpc.py -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_new.log 2>&1
