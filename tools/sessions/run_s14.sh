# round-4 session 14: group join hash factor 8 + a 512-digit scatter instance -- order tests, A/B vs hash factor 4, kernel stats
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s14_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s14_tests.log)"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in cur hf4; do
    if [ $v = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
    ZKAGG_LIB=$L timeout -k 10 200 python bench.py --order shuffled --pipeline 0 --steps 10 --cpu-sample 0 > gpurun_out/s14_v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/s14_v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
j = json.loads(open("gpurun_out/s14_v.log").read().strip().splitlines()[-1])
d = j.get("detail", {})
print(f"{v:6s} step {j['ms_per_step']:.3f} ms  cluster {d.get('cluster_ms_avg', 0):.3f}  join {j['roofline']['avg_launch_ms']:.3f}  reduce {d.get('reduce_avg_ms', 0):.3f}  parity {((j.get('parity') or {}).get('shuffled_vs_clustered') or {}).get('result')}")
PY
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/s14_prof -o s14 -- python $GRAFT_REPO_ROOT/bench.py --order shuffled --pipeline 0 --steps 5 --cpu-sample 0 > $GRAFT_REPO_ROOT/gpurun_out/s14_prof.log 2>&1
echo prof rc=$?
