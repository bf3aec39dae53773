#!/bin/bash
# PMC passes (each its own rocprofv3 run, counters only + kernel trace) on a short bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --cpu-sample 0 ${BENCH_ARGS:-}"
i=0
for set in "${@}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i ($set): exit $rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
