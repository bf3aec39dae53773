# round-4 session 19: ingest -- the wave copies the round's fragments into LDS one fragment at a time (coalesced) -- tests + A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ingest.py tests/test_gpu_reference_vectors.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s19_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s19_tests.log)"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 timeout -k 10 600 bash tools/ing_ab.sh cur ingold 2>&1 | tee gpurun_out/s19_ab.txt
