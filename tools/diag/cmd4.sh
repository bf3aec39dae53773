cd $GRAFT_REPO_ROOT
ZK_BENCH_DEBUG=1 timeout -k 10 200 python -u bench.py --order shuffled --cpu-sample 0 --steps 4 > gpurun_out/bs1.log 2>&1; echo "pipelined rc $?"
grep -v amdgpu.ids gpurun_out/bs1.log | cut -c1-2500 | tail -5
ZK_BENCH_DEBUG=1 timeout -k 10 200 python -u bench.py --cpu-sample 0 --steps 4 > gpurun_out/bc1.log 2>&1; echo "clustered pipelined rc $?"
grep debug gpurun_out/bc1.log | cut -c1-600
