#!/bin/bash
# Library x schedule A/B: LIBS (space-separated variant names, "cur" = libzkagg.so) crossed with
# VARIANTS (';'-separated bench argument strings), three rounds interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -r -a VS <<< "${VARIANTS:---pipeline 0;--pipeline 1}"
for r in 1 2 3; do
  for lib in ${LIBS:-cur}; do
    if [ "$lib" = cur ]; then L=$PWD/zipkin_amd/libzkagg.so; else L=$PWD/zipkin_amd/libzkagg_$lib.so; fi
    for v in "${VS[@]}"; do
      ZKAGG_LIB=$L timeout -k 10 120 python bench.py --cpu-sample 0 --steps 40 $v > gpurun_out/lib_ab.log 2>&1 || { echo "[$lib $v] failed"; tail -5 gpurun_out/lib_ab.log; exit 1; }
      python - "$lib $v" gpurun_out/lib_ab.log <<'PY'
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = j["roofline"]
d = j.get("detail", {})
print(f"{sys.argv[1]:36s} step {j['ms_per_step']:.4f} ms  K1 timed {r['avg_launch_ms']:.4f} (frac {r['frac']:.3f})"
      f"  K1 isolated {r.get('isolated_avg_launch_ms') or 0:.4f}  reduce {d.get('reduce_avg_ms', 0):.4f}")
PY
    done
  done
done
