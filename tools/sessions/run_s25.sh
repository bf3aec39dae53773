# round-4 session 25: P2 chunk lookup by a wave-parallel bucket search (cur) vs the binary search (xc0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s25_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s25_tests.log)"
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in cur xc0; do
    if [ $v = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
    ZKAGG_LIB=$L timeout -k 10 200 python bench.py --order shuffled --pipeline 0 --steps 10 --cpu-sample 0 > gpurun_out/s25_v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/s25_v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
j = json.loads(open("gpurun_out/s25_v.log").read().strip().splitlines()[-1])
d = j.get("detail", {})
print(f"{v:6s} step {j['ms_per_step']:.3f} ms  cluster {d.get('cluster_ms_avg', 0):.3f}  join {j['roofline']['avg_launch_ms']:.3f}  reduce {d.get('reduce_avg_ms', 0):.3f}  parity {((j.get('parity') or {}).get('shuffled_vs_clustered') or {}).get('result')}")
PY
  done
done
