# round-4 session 11: group join workgroup size (256 / 512 / 1024) x digit split -- order tests, serial shuffled A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in libzkagg.so libzkagg_gj256.so; do
  ZKAGG_LIB=$PWD/zipkin_amd/$L timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s11_order_$L.log 2>&1; rc=$?
  echo "$L: $(tail -1 gpurun_out/s11_order_$L.log)"
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in cur:8 cur:9 cur:10 gj256:8 gj256:10 gj256:11 gj1024:8; do
    lib=${v%%:*}; b1=${v##*:}
    if [ $lib = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$lib.so; fi
    ZKAGG_LIB=$L ZK_CL_B1=$b1 timeout -k 10 200 python bench.py --order shuffled --pipeline 0 --steps 10 --cpu-sample 0 > gpurun_out/s11_v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/s11_v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
j = json.loads(open("gpurun_out/s11_v.log").read().strip().splitlines()[-1])
d = j.get("detail", {})
print(f"{v:9s} step {j['ms_per_step']:.3f} ms  cluster {d.get('cluster_ms_avg', 0):.3f}  join {j['roofline']['avg_launch_ms']:.3f}  reduce {d.get('reduce_avg_ms', 0):.3f}  parity {((j.get('parity') or {}).get('shuffled_vs_clustered') or {}).get('result')}")
PY
  done
done
