# round-4 session 21: the group join on rich anomalous spans (new test)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_order.py -m gpu -x -q --timeout 200 --timeout-method thread -k "rich or group_join" > gpurun_out/s21_tests.log 2>&1; rc=$?
tail -15 gpurun_out/s21_tests.log
exit $rc
