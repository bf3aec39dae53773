cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in cur ingabl1 ingabl2 ingabl3; do
  if [ $v = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$v.so; fi
  ZKAGG_LIB=$L timeout -k 10 150 python -u tools/diag/ing_abl.py >> gpurun_out/ing_abl11.txt 2>&1 || { echo "ing $v failed"; tail -5 gpurun_out/ing_abl11.txt; exit 1; }
done
cat gpurun_out/ing_abl11.txt | grep -v amdgpu.ids
AB_ROUNDS=2 AB_TIMEOUT=200 BENCH_ARGS="--order shuffled --pipeline 0 --steps 6" timeout -k 10 900 bash tools/ab.sh cur p3s2k p3s2kg3 scu4 clall > gpurun_out/ab_cl11.txt 2>&1; echo "ab rc $?"
cat gpurun_out/ab_cl11.txt
