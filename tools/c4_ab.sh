#!/bin/bash
# C4 A/B: bench --workload c4 per library variant ("cur" = libzkagg.so), 2 rounds interleaved;
# prints ms/step and the per-phase kernel times of the line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
    ZKAGG_LIB=$L timeout -k 10 200 python bench.py --workload c4 --steps 10 --cpu-sample 0 > gpurun_out/c4_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/c4_$v.log; exit 1; }
    python -c "
import json; j=json.loads(open('gpurun_out/c4_$v.log').read().strip().splitlines()[-1]); k=j['kernels']
print('$v', round(j['ms_per_step'],3), 'ms', ' '.join(f'{n} {k[n][\"ms\"]:.3f}' for n in k))"
  done
done
