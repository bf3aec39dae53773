#!/bin/bash
# K2x (static XCD stride + chunk table): parity tests, then kernel A/B (clustered C2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sharded.py > gpurun_out/k2x_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/k2x_tests.log; exit 1; }
tail -2 gpurun_out/k2x_tests.log
CL_SCRIPT=tools/diag/k1_run.py bash tools/diag/cl_ab.sh cur xk0 xg2 cur xk0
