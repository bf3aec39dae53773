#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout (exit >= 124 or signal) stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() {  # $1 = exit code, $2 = step name; assertion failures (1) continue, crashes stop
  local rc=$1
  echo "[$2] exit $rc" | tee -a gpurun_out/steps.log
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $2" | tee -a gpurun_out/steps.log; exit "$rc"; fi
}
STEPS="${STEPS:-tests smoke bench prof}"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 500 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
      ok_or_stop $? tests; tail -5 gpurun_out/gpu_tests.log ;;
    smoke)
      timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      ok_or_stop $? smoke; tail -3 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 250 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
      ok_or_stop $? bench; tail -2 gpurun_out/bench.log ;;
    bench_c1|bench_c4|bench_c5|bench_ingest)
      w=${s#bench_}
      timeout -k 10 250 python bench.py --workload $w > gpurun_out/bench_$w.log 2>&1
      ok_or_stop $? $s; tail -1 gpurun_out/bench_$w.log | cut -c1-400 ;;
    bench_shuffled)
      timeout -k 10 300 python bench.py --order shuffled --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/bench_shuffled.log 2>&1
      ok_or_stop $? bench_shuffled; tail -1 gpurun_out/bench_shuffled.log | cut -c1-600 ;;
    prof_serial)
      timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --pipeline 0 --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/prof_serial.log 2>&1
      ok_or_stop $? prof_serial; find gpurun_out/prof_serial -name '*stats*' | head ;;
    prof_shuffled)
      timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_shuffled -o run --output-format csv -- python3 bench.py --order shuffled --steps 5 --warmup 1 --pipeline 0 --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/prof_shuffled.log 2>&1
      ok_or_stop $? prof_shuffled; find gpurun_out/prof_shuffled -name '*stats*' | head ;;
    prof)
      timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
      ok_or_stop $? prof; find gpurun_out/prof -name '*stats*' | head ;;
  esac
done
