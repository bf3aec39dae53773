cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ingest.py tests/test_gpu_reference_vectors.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ing_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ing_tests.log; [ $rc -eq 0 ] || exit $rc
ZK_STAMP_VARIANTS=ingstamps ZK_TIME_VARIANTS=cur,ingprev,cur,ingprev timeout -k 10 500 python tools/diag/ing_stamps.py
