#!/bin/bash
# Round-6 validation session, part A (PART=a): the whole -m gpu suite, smoke, the default bench (C2), its
# rocprof kernel stats (serial steps) and K1's HBM counters (two --pmc passes); part B (PART=b): the
# other bench lines and the job drivers. Every GPU step has its own limit; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06m}
if [ "${PART:-a}" = a ]; then
  timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${T}_gpu_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
  timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; tail gpurun_out/${T}_bench.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o c2 --output-format csv -- python3 bench.py --pipeline 0 --steps 20 --cpu-sample 0 > gpurun_out/${T}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
  rm -rf gpurun_out/pmc
  BENCH_ARGS="--pipeline 0" timeout -k 10 600 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE > gpurun_out/${T}_pmc.log 2>&1 || { echo "pmc failed"; cat gpurun_out/${T}_pmc.log; exit 1; }
else
  timeout -k 10 500 python -u bench.py --workload ingest --ingest-items 1 > gpurun_out/${T}_ingest_items.json 2> gpurun_out/${T}_ingest_items.err || { echo "ingest items failed"; tail gpurun_out/${T}_ingest_items.err; exit 1; }
  timeout -k 10 300 python -u tools/diag/run_device_timing.py > gpurun_out/${T}_run_device.txt 2>&1 || { echo "run_device timing failed"; exit 1; }
  for w in c3 c4 c5 ingest; do
    timeout -k 10 500 python -u bench.py --workload $w > gpurun_out/${T}_$w.json 2> gpurun_out/${T}_$w.err || { echo "$w failed"; tail gpurun_out/${T}_$w.err; exit 1; }
  done
  timeout -k 10 400 python -u bench.py --order shuffled > gpurun_out/${T}_shuffled.json 2> gpurun_out/${T}_shuffled.err || { echo "shuffled failed"; tail gpurun_out/${T}_shuffled.err; exit 1; }
  timeout -k 10 500 python -u -m pytest -q -s --timeout 400 --timeout-method thread tests/test_gpu_jobs.py > gpurun_out/${T}_jobs.txt 2>&1 || { echo "jobs failed"; tail -20 gpurun_out/${T}_jobs.txt; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_ingest -o ingest --output-format csv -- python3 bench.py --workload ingest --steps 10 --cpu-sample 0 > gpurun_out/${T}_prof_ingest.log 2>&1 || { echo "ingest rocprof failed"; exit 1; }
fi
echo "part ${PART:-a} done"
