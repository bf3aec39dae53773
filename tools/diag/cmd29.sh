#!/bin/bash
# C2 pipelined step vs number of table sets in flight (--pipeline N = N + 1 sets), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for p in 1 2 3; do
    timeout -k 10 150 python bench.py --cpu-sample 0 --steps 40 --pipeline $p > gpurun_out/pl_$p.log 2>&1 || { echo "p$p failed"; tail -5 gpurun_out/pl_$p.log; exit 1; }
    python3 -c "
import json; j=json.loads(open('gpurun_out/pl_$p.log').read().strip().splitlines()[-1])
print('pipeline $p', round(j['ms_per_step'],4), 'ms', 'K1 isolated', round(j['roofline']['avg_launch_ms'],4), 'frac', round(j['roofline']['frac'],3), 'step_frac', round(j['roofline']['step_frac'],3))"
  done
done
