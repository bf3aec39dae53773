# round-4 session 8: serial-step K1 A/B: lock-step phase 6 (cur) vs per-record (pj0), 5 WGs/CU + hash factor 4 (w5), hash factor 4 (hf4)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_ROUNDS=3 BENCH_ARGS="--pipeline 0" timeout -k 10 900 bash tools/ab.sh cur pj0 w5 hf4 2>&1 | tee gpurun_out/ab_k1_s8.txt
