#!/bin/bash
# One GPU-box session that regenerates the round's measurement artifacts under gpurun_out/:
# GPU tests, smoke, default bench (C2), C4/C5 bench lines, rocprofv3 kernel stats and the K1 HBM
# PMC passes. Every GPU step has its own time limit; a crash or timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc"
  if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
step gpu_tests 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tail -1 gpurun_out/gpu_tests.log
step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
step bench 250 python bench.py
step bench_c4 250 python bench.py --workload c4
step bench_c5 250 python bench.py --workload c5
step bench_ingest 250 python bench.py --workload ingest
step prof 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0
rm -rf gpurun_out/pmc
step pmc 300 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt
python3 tools/pmc_latest.py gpurun_out/pmc k_span_join 99999986 gpurun_out/pmc_latest.json > /dev/null
tail -1 gpurun_out/bench.log
