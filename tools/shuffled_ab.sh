#!/bin/bash
# Shuffled C2 A/B: bench --order shuffled per library variant ("cur" = libzkagg.so), 2 rounds interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
    ZKAGG_LIB=$L timeout -k 10 300 python bench.py --order shuffled --steps 10 --cpu-sample 0 > gpurun_out/sh_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/sh_$v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
j = json.loads(open(f"gpurun_out/sh_{v}.log").read().strip().splitlines()[-1])
print(v, round(j["ms_per_step"], 3), "ms")
PY
  done
done
