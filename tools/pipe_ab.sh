cd "${GRAFT_REPO_ROOT}"
for r in 1 2 3; do for p in ${PIPES:-1 2 3}; do
  timeout -k 10 120 python bench.py --cpu-sample 0 --steps 40 --pipeline $p > gpurun_out/pipe_$p.log 2>&1 || exit 1
  python -c "import json;j=json.loads(open('gpurun_out/pipe_$p.log').read().strip().splitlines()[-1]);print('pipeline $p', round(j['ms_per_step'],4), round(j['roofline']['avg_launch_ms'],4))"
done; done
