#!/bin/bash
# Round 6: K1 wait breakdown. The counter list, a baseline C2 line, then one rocprofv3 --pmc pass per
# counter set over tools/diag/k1_run.py (K1-dominated, counters for K1 only). Every GPU step has its
# own time limit and the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06_k1pmc}
mkdir -p $OUT
export TMPDIR=/tmp
LIB=${ZKAGG_LIB:-$PWD/zipkin_amd/libzkagg.so}
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || echo "counter list failed: $?"
timeout -k 10 150 python bench.py --cpu-sample 0 --steps 20 > $OUT/bench_c2.log 2>&1 || exit $?
tail -c 600 $OUT/bench_c2.log
i=0
for set in "$@"; do
  i=$((i+1))
  ZKAGG_LIB=$LIB timeout -s KILL 90 rocprofv3 --kernel-trace --kernel-include-regex k_span_join_stream --pmc $set \
    -d $OUT/p$i -o run --output-format csv -- python3 tools/diag/k1_run.py 100000000 4 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($set): exit $rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
