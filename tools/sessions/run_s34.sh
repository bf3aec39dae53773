# round-4 session 34: P0 double-buffered, P2 prep in parallel, P2h 4 chunks per workgroup (cur) vs HEAD (base); order+parity tests first
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s34_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/s34_tests.log)"
[ $rc -eq 0 ] || exit $rc
for v in cur base; do
  if [ $v = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
  ZKAGG_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/s34_$v -o run --output-format csv -- python3 bench.py --order shuffled --steps 10 --warmup 2 --cpu-sample 0 --pipeline 0 > gpurun_out/s34_$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for v in ("cur", "base"):
    f = glob.glob(f"gpurun_out/s34_{v}/**/run_kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "k_cl" in r["Name"] or "group_join" in r["Name"]:
            print(v, r["Name"][:48], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4))
PY
