#!/bin/bash
# One GPU-box session that regenerates the round's measurement artifacts under gpurun_out/:
# GPU tests, smoke, the bench lines (C2 default, C2 shuffled, C3 at G = 1, C1, C4, C5, ingest),
# rocprofv3 kernel stats of the pipelined, the serial and the shuffled C2 step, the K1 HBM PMC passes,
# and two-rank rehearsals of the N>1 path on one GPU (gloo; correctness checks of bench.py --gpus 2
# and of the C3 digest, not measurements).
# Every GPU step has its own time limit; a crash or timeout stops the script.
# usage: tools/refresh_profiles.sh <run label, e.g. r02_v3>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LABEL=${1:-builder run}
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc"
  if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
# PART=1: tests, smoke and the bench lines; PART=2: profiles, PMC and rehearsals; unset: both
if [ "${PART:-1}" = 1 ]; then
if [ -z "$SKIP_TESTS" ]; then
  step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
  tail -1 gpurun_out/gpu_tests.log
  step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 250 python bench.py
step bench_shuffled 250 python bench.py --order shuffled --cpu-sample 0
step bench_c3 400 python bench.py --workload c3 --steps 5 --warmup 1
step bench_c1 250 python bench.py --workload c1
step bench_c4 250 python bench.py --workload c4
step bench_c5 250 python bench.py --workload c5
step bench_ingest 250 python bench.py --workload ingest
fi
[ "${PART:-2}" = 2 ] || exit 0
step prof 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0
step prof_serial 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --pipeline 0
step prof_shuffled 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_shuffled -o run --output-format csv -- python3 bench.py --order shuffled --steps 5 --warmup 2 --cpu-sample 0 --pipeline 0
rm -rf gpurun_out/pmc
step pmc 300 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt
python3 tools/pmc_latest.py gpurun_out/pmc k_span_join 99999986 gpurun_out/pmc_latest.json "$LABEL" > /dev/null
step gloo2 300 env ZK_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2
tail -1 gpurun_out/gloo2.log
step gloo2_c3 400 env ZK_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --workload c3 --steps 2 --warmup 1
tail -1 gpurun_out/gloo2_c3.log | cut -c1-300
tail -1 gpurun_out/bench.log
