#!/bin/bash
# A/B of clustering-pass variants (tools/build_variant.py): per variant one rocprofv3 kernel-stats
# run of tools/diag/cl_time.py; prints the clustering kernels' average durations.
# usage: tools/diag/cl_ab.sh cur v1 v2 ...   (cur = libzkagg.so; CL_SCRIPT=tools/diag/k1_run.py for K1/K2/K3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
  rm -rf gpurun_out/clab_$v
  ZKAGG_LIB=$L timeout -k 10 ${CL_TIMEOUT:-150} rocprofv3 --kernel-trace --stats -d gpurun_out/clab_$v -o run --output-format csv \
    -- python3 ${CL_SCRIPT:-tools/diag/cl_time.py} ${CL_ARGS:-} > gpurun_out/clab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/clab_$v.log; exit 1; }
  grep "cluster\|K1" gpurun_out/clab_$v.log | tail -1
  python3 - gpurun_out/clab_$v/run_kernel_stats.csv <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_cl_", "k_span_join_stream", "k_link_scatter", "k_link_xscatter", "k_bucket_base", "k_bucket_colscan", "k_bucket_lds")):
        m = re.search(r"(k_\w+(?:<[^>]*>)?)", n)
        print(f"    {(m.group(1) if m else n)[:48]:48s} {int(r['Calls']):4d} x {float(r['AverageNs']) / 1e6:8.4f} ms")
PY
done
