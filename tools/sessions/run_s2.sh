# round-4 session 2: GPU tests, K1 A/B (guided ranges vs static ranges vs round 3), C4 query, gloo C3 rehearsal
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--pipeline 0" AB_ROUNDS=3 timeout -k 10 400 bash tools/ab.sh cur g0 r03 2>&1 | tee gpurun_out/ab2.txt || exit 1
AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh cur g0 2>&1 | tee gpurun_out/ab2_pipelined.txt || exit 1
ZK_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 2 > gpurun_out/gloo2_c3.log 2>&1 || { tail -20 gpurun_out/gloo2_c3.log; exit 1; }
tail -1 gpurun_out/gloo2_c3.log | cut -c1-400
