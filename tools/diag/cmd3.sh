cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_order.py tests/test_incremental.py tests/test_gpu_sharded.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1; echo "tests rc $?"
tail -3 gpurun_out/t3.log
timeout -k 10 200 python -u tools/diag/shuffle_parity.py 100000000 > gpurun_out/diag_shuffle.log 2>&1; echo "diag rc $?"
timeout -k 10 200 python -u bench.py --order shuffled --cpu-sample 0 --steps 10 > gpurun_out/bench_shuffled.log 2>&1; echo "bench rc $?"
tail -1 gpurun_out/bench_shuffled.log | cut -c1-300
