#!/bin/bash
# PMC of the C4 candidate pass: current (cur) vs no set work (kd1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -rf gpurun_out/pmckv; mkdir -p gpurun_out/pmckv
for v in cur kd1; do
  if [ "$v" = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA"; do
    i=$((i+1))
    ZKAGG_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmckv/${v}_p$i -o run --output-format csv -- python3 bench.py --workload c4 --steps 2 --warmup 1 > gpurun_out/pmckv/${v}_p$i.log 2>&1
    rc=$?; echo "$v pass $i exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmckv/${v}_p$i.log; exit $rc; }
  done
  python3 - $v <<'PY'
import csv, glob, sys
from collections import defaultdict
v = sys.argv[1]
acc = defaultdict(list)
for f in glob.glob(f"gpurun_out/pmckv/{v}_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_kv_candidates" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(v, {c: round(sum(x) / len(x)) for c, x in sorted(acc.items())})
PY
done
