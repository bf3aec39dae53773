#!/bin/bash
# PMC of K2 (k_link_scatter vs k_link_xscatter) on the clustered C2 accumulate (tools/diag/k1_run.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -rf gpurun_out/pmck2; mkdir -p gpurun_out/pmck2
for v in cur xk0; do
  if [ "$v" = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum"; do
    i=$((i+1))
    ZKAGG_LIB=$L timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmck2/${v}_p$i -o run --output-format csv -- python3 tools/diag/k1_run.py 100000000 3 > gpurun_out/pmck2/${v}_p$i.log 2>&1
    rc=$?; echo "$v pass $i exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmck2/${v}_p$i.log; exit $rc; }
  done
  python3 - $v <<'PY'
import csv, glob, sys
from collections import defaultdict
v = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/pmck2/{v}_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "link_scatter" in k or "link_xscatter" in k:
            acc[k[:24]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(v, k, {c: round(sum(x) / len(x)) for c, x in sorted(d.items())})
PY
done
