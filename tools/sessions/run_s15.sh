# round-4 session 15: phase stamps of the group join (shuffled C2) and of K1 (clustered C2), same build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag/gj_stamps.py > gpurun_out/s15_gj_stamps.json 2> gpurun_out/s15_gj_stamps.err || { tail -5 gpurun_out/s15_gj_stamps.err; exit 1; }
cat gpurun_out/s15_gj_stamps.json
timeout -k 10 300 python tools/k1_stamps.py > gpurun_out/s15_k1_stamps.json 2> gpurun_out/s15_k1_stamps.err || { tail -5 gpurun_out/s15_k1_stamps.err; exit 1; }
cat gpurun_out/s15_k1_stamps.json
