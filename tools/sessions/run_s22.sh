# round-4 session 22: default pipeline depth 3 -- C2 default line, shuffled line, N=2 gloo rehearsal of the C3 default
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/s22_bench.log 2>&1 || { tail -5 gpurun_out/s22_bench.log; exit 1; }
tail -1 gpurun_out/s22_bench.log | cut -c1-400
timeout -k 10 300 python bench.py --order shuffled --cpu-sample 0 > gpurun_out/s22_shuffled.log 2>&1 || { tail -5 gpurun_out/s22_shuffled.log; exit 1; }
tail -1 gpurun_out/s22_shuffled.log | cut -c1-300
timeout -k 10 400 env ZK_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/s22_gloo2.log 2>&1 || { tail -5 gpurun_out/s22_gloo2.log; exit 1; }
tail -1 gpurun_out/s22_gloo2.log | cut -c1-300
