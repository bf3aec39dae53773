# round-4 session 4: GPU tests after the prune, smoke, default bench + shuffled bench + C4/C5 lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
timeout -k 10 300 python bench.py --order shuffled --cpu-sample 0 > gpurun_out/bench_shuffled.log 2>&1 || { tail -5 gpurun_out/bench_shuffled.log; exit 1; }
tail -1 gpurun_out/bench_shuffled.log | cut -c1-200
timeout -k 10 300 python bench.py --workload c4 > gpurun_out/bench_c4.log 2>&1 || { tail -5 gpurun_out/bench_c4.log; exit 1; }
timeout -k 10 300 python bench.py --workload c5 > gpurun_out/bench_c5.log 2>&1 || { tail -5 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log | cut -c1-200
