# round-4 session 28: K1 time vs batch size on one box (fixed per-launch cost)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for n in 25000000 50000000 100000000 200000000; do
    timeout -k 10 200 python bench.py --pipeline 0 --steps 10 --cpu-sample 0 --records $n > gpurun_out/s28_$n.log 2>&1 || { tail -3 gpurun_out/s28_$n.log; exit 1; }
    python -c "import json; j=json.loads(open('gpurun_out/s28_$n.log').read().strip().splitlines()[-1]); r=j['roofline']; print($n, round(j['ms_per_step'],4), round(r['avg_launch_ms'],4), round(r['frac'],3))"
  done
done
