cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for b1 in 8 6 10 11; do
  ZK_CL_B1=$b1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/clsplit_$b1 -o run --output-format csv -- python3 bench.py --order shuffled --steps 3 --warmup 1 --pipeline 0 --cpu-sample 0 > gpurun_out/clsplit_$b1.log 2>&1 || exit 1
  echo "b1=$b1 done"
done
