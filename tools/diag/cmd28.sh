#!/bin/bash
# clustering P1/P2 shapes: U=4 x 2 or 3 workgroups per CU vs U=8 x 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
ZKAGG_LIB=$PWD/zipkin_amd/libzkagg_u4g2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_order.py > gpurun_out/u4_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/u4_tests.log; exit 1; }
tail -2 gpurun_out/u4_tests.log
bash tools/diag/cl_ab.sh cur u4g2 u4g3 cur u4g2
