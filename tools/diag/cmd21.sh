#!/bin/bash
# K2x cursor padding A/B (clustered C2 kernels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
CL_SCRIPT=tools/diag/k1_run.py bash tools/diag/cl_ab.sh cur xp16 xp32 xg1 xk0 xp32
