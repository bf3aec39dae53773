# PMC passes of the ingest decode (k_ing_decode_lds) for the round-2 decoder (ingold) and the current one
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -rf gpurun_out/pmci; mkdir -p gpurun_out/pmci
for v in ingold cur; do
  if [ "$v" = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SMEM" \
             "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    ZKAGG_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmci/${v}_p$i -o run --output-format csv -- python3 bench.py --workload ingest --steps 2 --warmup 1 --fragments 4000000 > gpurun_out/pmci/${v}_p$i.log 2>&1
    rc=$?; echo "$v pass $i exit $rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_summary.py gpurun_out/pmci/ > /dev/null
  python3 - $v <<'PY'
import csv, glob, sys
from collections import defaultdict
v = sys.argv[1]
acc = defaultdict(list)
for f in glob.glob(f"gpurun_out/pmci/{v}_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "decode_lds" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(v, {c: round(sum(x) / len(x)) for c, x in sorted(acc.items())})
PY
done
