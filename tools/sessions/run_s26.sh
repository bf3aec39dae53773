# round-4 session 26: group join phase stamps after the load spreading
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag/gj_stamps.py > gpurun_out/s26_gj_stamps.json 2> gpurun_out/s26_gj_stamps.err || { tail -5 gpurun_out/s26_gj_stamps.err; exit 1; }
cat gpurun_out/s26_gj_stamps.json
