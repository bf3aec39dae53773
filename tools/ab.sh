#!/bin/bash
# A/B of library variants on the default bench: tools/ab.sh v1 v2 ... ("cur" = libzkagg.so).
# Prints ms/step and K1 avg launch ms per variant, two rounds interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${AB_ROUNDS:-3}); do
  for v in "$@"; do
    if [ "$v" = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
    ZKAGG_LIB=$L timeout -k 10 ${AB_TIMEOUT:-120} python bench.py --cpu-sample 0 --steps 40 ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
j = json.loads(open(f"gpurun_out/ab_{v}.log").read().strip().splitlines()[-1])
d = j.get("detail", {})
print(f"{v:10s} step {j['ms_per_step']:.4f} ms  K1 {j['roofline']['avg_launch_ms']:.4f} ms  frac {j['roofline']['frac']:.3f}"
      f"  K1-isolated {j['roofline'].get('isolated_avg_launch_ms') or 0:.4f}  reduce {d.get('reduce_avg_ms', 0):.4f}"
      + (f"  cluster {d['cluster_ms_avg']:.3f}" if 'cluster_ms_avg' in d else "")
      + (f"  parity {j['parity']['shuffled_vs_clustered']['result']}" if (j.get('parity') or {}).get('shuffled_vs_clustered') else ""))
PY
  done
done
