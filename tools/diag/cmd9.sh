cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t9.log 2>&1; echo "all gpu tests rc $?"
tail -2 gpurun_out/t9.log
ZKAGG_LIB=$PWD/zipkin_amd/libzkagg_pair.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_vectors.py tests/test_gpu_order.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t9_pair.log 2>&1; echo "pair tests rc $?"
tail -2 gpurun_out/t9_pair.log
timeout -k 10 100 python -u tools/k1_stamps.py > gpurun_out/stamps9.log 2>&1; echo "stamps rc $?"
BENCH_ARGS="--pipeline 0" timeout -k 10 500 bash tools/ab.sh cur pair > gpurun_out/ab_pair.txt 2>&1; echo "ab rc $?"
cat gpurun_out/ab_pair.txt
timeout -k 10 200 python -u bench.py --order shuffled --cpu-sample 0 --steps 10 > gpurun_out/bs9.log 2>&1; echo "shuffled rc $?"
timeout -k 10 200 python -u bench.py --workload ingest > gpurun_out/bi9.log 2>&1; echo "ingest rc $?"
timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof9 -o run --output-format csv -- python3 bench.py --order shuffled --steps 5 --warmup 1 --pipeline 0 --cpu-sample 0 > gpurun_out/prof9.log 2>&1; echo "prof rc $?"
