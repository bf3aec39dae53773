#!/bin/bash
# HBM bytes (FETCH_SIZE x2 gfx950 correction, WRITE_SIZE) per kernel of the shuffled C2 step and the C4
# step: two --pmc passes each (tools/pmc.sh), into gpurun_out/pmc_shuffled and gpurun_out/pmc_c4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/pmc gpurun_out/pmc_shuffled gpurun_out/pmc_c4
BENCH_ARGS="--order shuffled --pipeline 0" timeout -k 10 700 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
mv gpurun_out/pmc gpurun_out/pmc_shuffled
BENCH_ARGS="--workload c4" timeout -k 10 700 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
mv gpurun_out/pmc gpurun_out/pmc_c4
echo done
