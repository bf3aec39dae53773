# round-4 session 13: group join -- hash factor 8, sub-bucket target (1536 = one 256-digit P2), WG 512; kernel stats
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ZKAGG_LIB=$PWD/zipkin_amd/libzkagg_hf8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s13_order_hf8.log 2>&1; rc=$?
echo "hf8 tests: $(tail -1 gpurun_out/s13_order_hf8.log)"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in cur:0 cur:1536 hf8:0 hf8:1536 gj512:0; do
    lib=${v%%:*}; t=${v##*:}
    if [ $lib = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$lib.so; fi
    if [ $t = 0 ]; then E=""; else E="ZK_CL_GROUP_TARGET=$t"; fi
    env ZKAGG_LIB=$L $E timeout -k 10 200 python bench.py --order shuffled --pipeline 0 --steps 10 --cpu-sample 0 > gpurun_out/s13_v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/s13_v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
j = json.loads(open("gpurun_out/s13_v.log").read().strip().splitlines()[-1])
d = j.get("detail", {})
print(f"{v:11s} step {j['ms_per_step']:.3f} ms  cluster {d.get('cluster_ms_avg', 0):.3f}  join {j['roofline']['avg_launch_ms']:.3f}  reduce {d.get('reduce_avg_ms', 0):.3f}  parity {((j.get('parity') or {}).get('shuffled_vs_clustered') or {}).get('result')}")
PY
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/s13_prof -o s13 -- python $GRAFT_REPO_ROOT/bench.py --order shuffled --pipeline 0 --steps 5 --cpu-sample 0 > $GRAFT_REPO_ROOT/gpurun_out/s13_prof.log 2>&1
echo prof rc=$?
