# round-4 session 32: + software-pipelined P1/P2 chunks (next claim and traceIds in flight) (cur) vs HEAD (base)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s32_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s32_tests.log)"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=3 BENCH_ARGS="--order shuffled --pipeline 0" timeout -k 10 900 bash tools/ab.sh cur base 2>&1 | tee gpurun_out/s32_ab.txt
