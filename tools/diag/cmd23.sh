#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
CL_SCRIPT=tools/diag/k1_run.py bash tools/diag/cl_ab.sh xk0 xr1 xk0 xr1
