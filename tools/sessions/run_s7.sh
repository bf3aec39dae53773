# round-4 session 7: K1 phase 6 with both records of a thread in lock step (ZK_K1_PAIRJOIN) -- parity + A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s7_tests.log 2>&1; rc=$?
tail -3 gpurun_out/s7_tests.log
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=3 timeout -k 10 600 bash tools/ab.sh cur pj0 2>&1 | tee gpurun_out/ab_k1_pairjoin.txt
