# round-4 session 3: GPU tests; A/B of the list-major K1 histogram (cur) vs bucket-major (ht0), grid multiples; K1 vs batch size
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--pipeline 0" AB_ROUNDS=3 timeout -k 10 400 bash tools/ab.sh cur ht0 gm2 gm8 2>&1 | tee gpurun_out/ab3.txt || exit 1
AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh cur ht0 2>&1 | tee gpurun_out/ab3_pipelined.txt || exit 1
for r in 200000000 400000000; do
  timeout -k 10 200 python bench.py --pipeline 0 --records $r --cpu-sample 0 --steps 10 > gpurun_out/bench_n$r.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/bench_n$r.log').read().strip().splitlines()[-1]); r=d['roofline']; print($r, d['ms_per_step'], r['avg_launch_ms'], r['frac'])"
done
