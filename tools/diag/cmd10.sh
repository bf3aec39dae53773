cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ZKAGG_LIB=$PWD/zipkin_amd/libzkagg_slot16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_vectors.py tests/test_gpu_order.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t10_slot16.log 2>&1; echo "slot16 tests rc $?"
tail -2 gpurun_out/t10_slot16.log
timeout -k 10 100 python -u tools/k1_stamps.py > gpurun_out/stamps10.log 2>&1; echo "stamps rc $?"
BENCH_ARGS="--pipeline 0" timeout -k 10 500 bash tools/ab.sh cur slot16 > gpurun_out/ab_slot16.txt 2>&1; echo "ab rc $?"
cat gpurun_out/ab_slot16.txt
