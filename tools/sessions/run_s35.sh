# round-4 session 35: shuffled C2 with the digit split 9 + 8 (ZK_CL_B1=9) vs the default 8 + 9
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for b in 8 9; do
    ZK_CL_B1=$b timeout -k 10 150 python bench.py --order shuffled --cpu-sample 0 --steps 40 --pipeline 0 > gpurun_out/s35_b$b.log 2>&1 || { tail -5 gpurun_out/s35_b$b.log; exit 1; }
    python3 -c "
import json; j = json.loads(open('gpurun_out/s35_b$b.log').read().strip().splitlines()[-1])
print('b1=$b step %.4f ms join %.4f parity %s' % (j['ms_per_step'], j['roofline']['avg_launch_ms'], j['parity']['shuffled_vs_clustered']['result']))"
  done
done
ZK_CL_B1=9 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/s35_prof -o run --output-format csv -- python3 bench.py --order shuffled --steps 10 --warmup 2 --cpu-sample 0 --pipeline 0 > gpurun_out/s35_prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/s35_prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_cl" in r["Name"] or "group_join" in r["Name"] or "span_join" in r["Name"]:
        print("b1=9", r["Name"][:48], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4))
PY
