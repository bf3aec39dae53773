#!/bin/bash
# P3 static stride + prefetch (ts1) vs work counter (ts0): order tests, then clustering kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
ZKAGG_LIB=$PWD/zipkin_amd/libzkagg_ts1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_order.py tests/test_gpu_sharded.py > gpurun_out/ts_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/ts_tests.log; exit 1; }
tail -2 gpurun_out/ts_tests.log
bash tools/diag/cl_ab.sh ts1 ts0 ts1 ts0
