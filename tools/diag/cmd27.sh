#!/bin/bash
# C4 candidate-pass diagnostics: kd1 = no set probes/inserts, kd2 = + no estimates (results wrong)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
bash tools/c4_ab.sh ${C4_VARIANTS:-cur kd1 kd2}
