#!/bin/bash
# K1 A/B: tools/diag/k1_run.py (1e8 clustered records, serial accumulates, K1 launch time from HIP
# events) for each library variant in "$@" ("cur" = libzkagg.so), ROUNDS rounds interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in "$@"; do
    if [ "$v" = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
    ZKAGG_LIB=$L timeout -k 10 ${K1_TIMEOUT:-90} python tools/diag/k1_run.py ${K1_RECORDS:-100000000} ${K1_STEPS:-10} \
      > gpurun_out/k1_ab_$v.log 2>&1 || { echo "$v failed ($?)"; tail -5 gpurun_out/k1_ab_$v.log; exit 1; }
    echo "round $r $(tail -1 gpurun_out/k1_ab_$v.log)"
  done
done
