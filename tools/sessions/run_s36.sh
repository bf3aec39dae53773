# round-4 session 36: ingest decode with LDS budgets per wave of 10/13/16/20 (cur)/26/32 KiB
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ingest.py tests/test_gpu_reference_vectors.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s36_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s36_tests.log)"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 timeout -k 10 900 bash tools/ing_ab.sh cur ib10240 ib13312 ib16384 ib26624 ib32768 2>&1 | tee gpurun_out/s36_ab.txt
