#!/bin/bash
# scratch GPU session used during tuning (rewritten per experiment)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/par_tests.log 2>&1; rc=$?; tail -2 gpurun_out/par_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab.sh cur prev
