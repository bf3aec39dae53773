# round-4 session 6: partition without cursor claims (ZK_PART_BASES) -- sketch tests + C4 A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kv.py tests/test_realtime.py tests/test_gpu_sketch_shards.py tests/test_launch.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sk_tests.log 2>&1; rc=$?
tail -3 gpurun_out/sk_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/c4_ab.sh cur pb0 r03 2>&1 | tee gpurun_out/ab_c4_bases.txt
