cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ingest.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ing_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ing_tests.log; [ $rc -le 1 ] || exit $rc
bash tools/ing_ab.sh ingold ingnew || exit 1
bash tools/diag/cl_ab.sh cur cdiag1 cdiag2 cwg512 cwg256
