#!/bin/bash
# Step-schedule A/B on the default bench, three rounds interleaved. VARIANTS is a ';'-separated list of
# bench argument strings (default: pipeline depths 1, 2, 3).
#   VARIANTS="--pipeline 0;--pipeline 1 --overlap tail;--pipeline 1 --overlap full" bash tools/pipe_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -r -a VS <<< "${VARIANTS:---pipeline 1;--pipeline 2;--pipeline 3}"
for r in 1 2 3; do
  i=0
  for v in "${VS[@]}"; do
    i=$((i+1))
    timeout -k 10 120 python bench.py --cpu-sample 0 --steps 40 $v > gpurun_out/pipe_$i.log 2>&1 || { echo "[$v] failed"; tail -5 gpurun_out/pipe_$i.log; exit 1; }
    python - "$v" "gpurun_out/pipe_$i.log" <<'PY'
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = j["roofline"]
print(f"{sys.argv[1]:32s} step {j['ms_per_step']:.4f} ms  K1 timed {r['avg_launch_ms']:.4f} ms (frac {r['frac']:.3f})"
      f"  K1 isolated {r.get('isolated_avg_launch_ms') or 0:.4f}")
PY
  done
done
