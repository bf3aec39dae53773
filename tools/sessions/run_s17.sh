# round-4 session 17: C4 -- the sketch pass writes per-unit key lists with most repeats dropped; the candidate pass reads them
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kv.py tests/test_gpu_sketch_shards.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s17_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s17_tests.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/c4_ab.sh cur kvold 2>&1 | tee gpurun_out/s17_ab.txt
timeout -k 10 300 python bench.py --workload c4 --steps 10 --cpu-sample 100000000 > gpurun_out/s17_c4.log 2>&1; echo "c4 parity rc=$?"
tail -1 gpurun_out/s17_c4.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['ms_per_step'], j['parity'], j['cpu_baseline'])"
