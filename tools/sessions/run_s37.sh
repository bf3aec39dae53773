# round-4 session 37: shuffled C2, pipeline 3 (default) vs 0, interleaved on one box
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for p in 3 0; do
    timeout -k 10 150 python bench.py --order shuffled --cpu-sample 0 --pipeline $p > gpurun_out/s37_p$p.log 2>&1 || { tail -5 gpurun_out/s37_p$p.log; exit 1; }
    python3 -c "
import json; j = json.loads(open('gpurun_out/s37_p$p.log').read().strip().splitlines()[-1])
print('pipeline $p step %.4f ms join %.4f' % (j['ms_per_step'], j['roofline']['avg_launch_ms']))"
  done
done
