#!/bin/bash
# A/B: the C2 columns as seven allocations vs one packed block (DeviceColumns(packed=True)), pipelined
# and serial steps, interleaved. Prints ms_per_step and K1's event ms per line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for lay in separate packed; do
    for pipe in 3 0; do
      timeout -k 10 200 python -u bench.py --layout $lay --pipeline $pipe --cpu-sample 0 --steps 20 > gpurun_out/lay_${lay}_${pipe}_$r.json 2> gpurun_out/lay_${lay}_${pipe}_$r.err || { echo "bench failed"; tail gpurun_out/lay_${lay}_${pipe}_$r.err; exit 1; }
      python - "$lay" "$pipe" "$r" gpurun_out/lay_${lay}_${pipe}_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print(sys.argv[1], "pipe", sys.argv[2], "round", sys.argv[3], "ms/step %.4f" % d["ms_per_step"],
      "k1_ms", r.get("avg_launch_ms"), "frac %.4f" % r.get("frac", 0), "isolated", r.get("isolated_frac"), flush=True)
PY
    done
  done
done
