cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_sharded.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t8.log 2>&1; echo "tests rc $?"
tail -2 gpurun_out/t8.log
timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- python3 bench.py --order shuffled --steps 5 --warmup 1 --pipeline 0 --cpu-sample 0 > gpurun_out/prof8.log 2>&1; echo "prof rc $?"
timeout -k 10 200 python -u bench.py --order shuffled --cpu-sample 0 --steps 10 > gpurun_out/bs8.log 2>&1; echo "shuffled rc $?"
