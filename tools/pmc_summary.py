#!/usr/bin/env python3
"""Average PMC counters per kernel over all pmc passes in gpurun_out/pmc (rocprofv3 csv)."""
import csv, glob, sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", r.get("Kernel-Name", ""))[:60]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "tg_" in k:
        continue
    print(k)
    for c, vs in sorted(cs.items()):
        print(f"   {c:28s} {sum(vs)/len(vs):16.4g}  (n={len(vs)})")
