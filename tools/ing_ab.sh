#!/bin/bash
# ingest A/B: bench --workload ingest per library variant, 3 rounds interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 ${AB_ROUNDS:-3}); do
  for v in "$@"; do
    if [ "$v" = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
    ZKAGG_LIB=$L timeout -k 10 200 python bench.py --workload ingest --steps 10 > gpurun_out/ing_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ing_$v.log; exit 1; }
    python -c "import json,sys; j=json.loads(open('gpurun_out/ing_$v.log').read().strip().splitlines()[-1]); print('$v', round(j['ms_per_step'],3), 'ms', '%.3g'%j['value'])"
  done
done
