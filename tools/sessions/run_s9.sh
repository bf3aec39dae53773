# round-4 session 9: group join (k_group_join) -- shuffled-order GPU tests, then the shuffled C2 A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_order.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s9_order_tests.log 2>&1; rc=$?
tail -5 gpurun_out/s9_order_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in group trace b19; do
    case $v in
      group) E="";;
      trace) E="ZK_GROUP_JOIN=0";;
      b19) E="ZK_CL_B1=9";;
    esac
    env $E timeout -k 10 200 python bench.py --order shuffled --steps 10 --cpu-sample 0 > gpurun_out/s9_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/s9_$v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
j = json.loads(open(f"gpurun_out/s9_{v}.log").read().strip().splitlines()[-1])
d = j.get("detail", {})
print(f"{v:6s} step {j['ms_per_step']:.3f} ms  cluster {d.get('cluster_ms_avg', 0):.3f}  join(K1 events) {j['roofline']['avg_launch_ms']:.3f}  reduce {d.get('reduce_avg_ms', 0):.3f}  parity {((j.get('parity') or {}).get('shuffled_vs_clustered') or {}).get('result')}")
PY
  done
done
