cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--pipeline 0" AB_ROUNDS=3 timeout -k 10 500 bash tools/ab.sh cur e0 r03 2>&1 | tee gpurun_out/ab1.txt
