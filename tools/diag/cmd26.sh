#!/bin/bash
# C4 partition: static-stride prefetching scatter (pxs) vs the claimed-chunk scatter (pxc)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
ZKAGG_LIB=$PWD/zipkin_amd/libzkagg${TEST_VARIANT:-}.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_kv.py tests/test_gpu_sketch_shards.py tests/test_launch.py > gpurun_out/pxs_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/pxs_tests.log; exit 1; }
tail -2 gpurun_out/pxs_tests.log
bash tools/c4_ab.sh ${C4_VARIANTS:-cur pxc}
