cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/order_tests.log 2>&1; rc=$?; tail -3 gpurun_out/order_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/diag/cl_ab.sh cur xcd0 || exit 1
timeout -k 10 250 python bench.py --order shuffled --cpu-sample 0 > gpurun_out/bench_shuffled.log 2>&1; rc=$?; tail -1 gpurun_out/bench_shuffled.log | cut -c1-300; exit $rc
