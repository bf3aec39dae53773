cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kv.py tests/test_realtime.py tests/test_gpu_sketch_shards.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/kv_tests.log 2>&1; rc=$?; tail -3 gpurun_out/kv_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/c4_ab.sh cur px0
