# round-4 session 30: K1 with the next window's early columns in three groups (cur) vs one (k1s0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_continuation.py tests/test_realtime.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s30_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s30_tests.log)"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=3 BENCH_ARGS="--pipeline 0" timeout -k 10 900 bash tools/ab.sh cur k1s0 2>&1 | tee gpurun_out/s30_ab.txt
