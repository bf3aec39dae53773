# round-4 session 10: group join with batched sub-buckets -- order tests, serial shuffled A/B, kernel stats
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_order.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s10_order_tests.log 2>&1; rc=$?
tail -3 gpurun_out/s10_order_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in group trace b19; do
    case $v in
      group) E="";;
      trace) E="ZK_GROUP_JOIN=0";;
      b19) E="ZK_CL_B1=9";;
    esac
    env $E timeout -k 10 200 python bench.py --order shuffled --pipeline 0 --steps 10 --cpu-sample 0 > gpurun_out/s10_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/s10_$v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
j = json.loads(open(f"gpurun_out/s10_{v}.log").read().strip().splitlines()[-1])
d = j.get("detail", {})
print(f"{v:6s} step {j['ms_per_step']:.3f} ms  cluster {d.get('cluster_ms_avg', 0):.3f}  join {j['roofline']['avg_launch_ms']:.3f}  reduce {d.get('reduce_avg_ms', 0):.3f}  parity {((j.get('parity') or {}).get('shuffled_vs_clustered') or {}).get('result')}")
PY
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s10_prof -o s10 -- python $GRAFT_REPO_ROOT/bench.py --order shuffled --pipeline 0 --steps 5 --cpu-sample 0 > $GRAFT_REPO_ROOT/gpurun_out/s10_prof.log 2>&1
echo prof rc=$?
find $GRAFT_REPO_ROOT/gpurun_out/s10_prof -name "*kernel_stats.csv" | head -3
