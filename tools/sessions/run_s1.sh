# round-4 session 1: GPU tests, K1 A/B (epoch slots vs pruned 3-barrier vs round-3 library), C4 + C3 lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--pipeline 0" AB_ROUNDS=3 timeout -k 10 400 bash tools/ab.sh cur e0 r03 2>&1 | tee gpurun_out/ab1.txt || exit 1
timeout -k 10 300 python bench.py --workload c4 > gpurun_out/bench_c4.log 2>&1 || { tail -5 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-300
timeout -k 10 400 python bench.py --workload c3 --cpu-sample 20000000 > gpurun_out/bench_c3.log 2>&1 || { tail -5 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log | cut -c1-300
