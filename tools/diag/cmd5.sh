cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --order shuffled --cpu-sample 0 --steps 10 > gpurun_out/bs1.log 2>&1; echo "pipelined rc $?"
grep -v amdgpu.ids gpurun_out/bs1.log | tail -2 | cut -c1-3000
timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_shuf2 -o run --output-format csv -- python3 bench.py --order shuffled --steps 5 --warmup 1 --pipeline 0 --cpu-sample 0 > gpurun_out/prof_shuf2.log 2>&1; echo "prof rc $?"
