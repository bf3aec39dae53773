cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t6.log 2>&1; echo "tests rc $?"
tail -3 gpurun_out/t6.log
timeout -k 10 200 python -u bench.py --order shuffled --cpu-sample 0 --steps 10 > gpurun_out/bs6.log 2>&1; echo "shuffled rc $?"
timeout -k 10 200 python -u bench.py --cpu-sample 0 --steps 20 > gpurun_out/bc6.log 2>&1; echo "clustered rc $?"
timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6 -o run --output-format csv -- python3 bench.py --order shuffled --steps 5 --warmup 1 --pipeline 0 --cpu-sample 0 > gpurun_out/prof6.log 2>&1; echo "prof rc $?"
