#!/bin/bash
# K1 probe: PC sampling of the clustered C2 accumulate (stochastic, else host-trap), then an A/B
# of library variants named in $AB (default: cur).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 65536 -d gpurun_out/pcs -o k1 --output-format csv -- python3 tools/diag/k1_run.py 100000000 5 \
  > gpurun_out/pcs_stoch.log 2>&1 || echo "stochastic pc sampling failed: $?" >> gpurun_out/pcs_stoch.log
if ! ls gpurun_out/pcs/*/*pc_sampling* >/dev/null 2>&1; then
  timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 10 -d gpurun_out/pcs_ht -o k1 --output-format csv -- python3 tools/diag/k1_run.py 100000000 5 \
    > gpurun_out/pcs_ht.log 2>&1 || echo "host-trap pc sampling failed: $?" >> gpurun_out/pcs_ht.log
fi
AB_ROUNDS=3 timeout -k 10 600 bash tools/ab.sh ${AB:-cur} > gpurun_out/ab_k1_probe.txt 2>&1
