#!/bin/bash
# Round 6 GPU check: selected GPU test files (PYTESTS), then bench lines (LINES: c2 c5 ingest gloo2
# gloo2c5 shuffled c4). Every GPU step has its own limit; the chain stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06_check}
mkdir -p $OUT
export TMPDIR=/tmp
stop() { echo "[$1] exit $2"; exit $2; }
if [ -n "${PYTESTS:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout 300 --timeout-method thread $PYTESTS \
    > $OUT/tests.txt 2>&1
  rc=$?; tail -15 $OUT/tests.txt; [ $rc -ne 0 ] && stop tests $rc
fi
for l in ${LINES:-}; do
  case $l in
    c2) timeout -k 10 200 python bench.py --cpu-sample 0 > $OUT/c2.json 2>$OUT/c2.err || stop c2 $? ;;
    c2full) timeout -k 10 300 python bench.py > $OUT/c2full.json 2>$OUT/c2full.err || stop c2full $? ;;
    c5) timeout -k 10 200 python bench.py --workload c5 --cpu-sample 0 --steps 5 > $OUT/c5.json 2>$OUT/c5.err || stop c5 $? ;;
    c4) timeout -k 10 200 python bench.py --workload c4 --cpu-sample 0 > $OUT/c4.json 2>$OUT/c4.err || stop c4 $? ;;
    ingest) timeout -k 10 300 python bench.py --workload ingest > $OUT/ingest.json 2>$OUT/ingest.err || stop ingest $? ;;
    shuffled) timeout -k 10 300 python bench.py --order shuffled --cpu-sample 0 > $OUT/shuffled.json 2>$OUT/shuffled.err || stop shuffled $? ;;
    gloo2) ZK_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
             --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --records 200000000 --steps 3 --warmup 1 \
             > $OUT/gloo2.json 2>$OUT/gloo2.err || stop gloo2 $? ;;
    gloo2c5) ZK_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
             --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --workload c5 --records 100000000 --steps 3 \
             --warmup 1 > $OUT/gloo2c5.json 2>$OUT/gloo2c5.err || stop gloo2c5 $? ;;
  esac
  echo "[$l] ok"; tail -c 700 $OUT/$l.json; echo
done
