# round-4 session 31: P0 histogram with 1024 threads and two load buffers (cur) vs 256 threads, one buffer (base)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s31_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s31_tests.log)"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=3 BENCH_ARGS="--order shuffled --pipeline 0" timeout -k 10 900 bash tools/ab.sh cur base 2>&1 | tee gpurun_out/s31_ab.txt
