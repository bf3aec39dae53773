# round-4 session 20: C4 candidates -- keys whose row-0 counter is below the threshold skip the other rows and the set probes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kv.py tests/test_gpu_sketch_shards.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s20_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s20_tests.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/c4_ab.sh cur kvr0 2>&1 | tee gpurun_out/s20_ab.txt
timeout -k 10 300 python bench.py --workload c4 --steps 10 > gpurun_out/s20_c4.log 2>&1; echo "c4 parity rc=$?"
tail -1 gpurun_out/s20_c4.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['ms_per_step'], j['parity']['result'], j['kernels'])"
