# round-4 session 5: GPU tests incl. batch continuation; C4 query latency
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_continuation.py -x -v --timeout 120 --timeout-method thread > gpurun_out/cont_tests.log 2>&1; rc=$?
tail -15 gpurun_out/cont_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c4 --cpu-sample 0 > gpurun_out/bench_c4.log 2>&1 || { tail -5 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['detail'])"
