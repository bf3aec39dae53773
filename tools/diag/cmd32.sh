#!/bin/bash
# ingest LDS budget per wave: decode time per variant (tools/diag/ing_stamps.py timing mode)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
ZK_STAMP_VARIANTS= ZK_TIME_VARIANTS=cur,ib16,ib26,ib32,cur,ib16,ib26,ib32 timeout -k 10 400 python3 tools/diag/ing_stamps.py > gpurun_out/ib.log 2>&1 || { tail -20 gpurun_out/ib.log; exit 1; }
cat gpurun_out/ib.log | grep ms_per
