#!/bin/bash
# One GPU session: the whole -m gpu suite, smoke, the default bench (C2) and its rocprof kernel
# stats, plus optional extra steps ($EXTRA: a command run last). Every GPU step has its own limit
# and the steps are chained: the first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05}
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o c2 --output-format csv -- python3 bench.py --pipeline 0 --steps 20 --cpu-sample 0 > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
if [ -n "$EXTRA" ]; then bash -c "$EXTRA" || exit 1; fi
echo "round check done"
