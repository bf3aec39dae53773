#!/bin/bash
# scratch GPU session used during tuning (rewritten per experiment)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kv.py tests/test_realtime.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kv_tests.log 2>&1; rc=$?; tail -2 gpurun_out/kv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cur -o run --output-format csv -- python3 bench.py --workload c4 --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/prof_cur.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --workload c4 > gpurun_out/bench_c4.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c4.log | cut -c 1-400
