# round-4 session 24: C4 partition with the next chunk's loads in two halves (cur) vs one burst (ps0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kv.py tests/test_realtime.py tests/test_gpu_sketch_shards.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s24_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s24_tests.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/c4_ab.sh cur ps0 2>&1 | tee gpurun_out/s24_ab.txt
