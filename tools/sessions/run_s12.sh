# round-4 session 12: group join at WG 512 gives wrong links on a 470k-record batch -- which counters differ
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in libzkagg.so libzkagg_gj256.so libzkagg_gj1024.so; do
  for b in 8 9; do
    echo "== $L B1=$b"
    ZKAGG_LIB=$PWD/zipkin_amd/$L ZK_CL_B1=$b timeout -k 10 120 python tools/diag/gj_debug.py 20000 || exit 1
  done
done
