cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_order.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t12_order.log 2>&1; echo "order tests rc $?"
tail -2 gpurun_out/t12_order.log
AB_ROUNDS=2 AB_TIMEOUT=200 BENCH_ARGS="--order shuffled --pipeline 0 --steps 6" timeout -k 10 700 bash tools/ab.sh cur sg1 tr4k > gpurun_out/ab_cl12.txt 2>&1; echo "ab rc $?"
cat gpurun_out/ab_cl12.txt
ZK_CL_B1=9 timeout -k 10 200 python bench.py --cpu-sample 0 --order shuffled --pipeline 0 --steps 6 > gpurun_out/b12_b19.log 2>&1; echo "b1=9 rc $?"
python -c "import json;j=json.loads(open('gpurun_out/b12_b19.log').read().strip().splitlines()[-1]);print('B1=9', j['ms_per_step'], j['detail']['cluster_ms_avg'], j['parity']['shuffled_vs_clustered']['result'])"
timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof12 -o run --output-format csv -- python3 bench.py --order shuffled --steps 5 --warmup 1 --pipeline 0 --cpu-sample 0 > gpurun_out/prof12.log 2>&1; echo "prof rc $?"
