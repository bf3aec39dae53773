#!/usr/bin/env python3
"""Per-launch HBM bytes of K1 from rocprofv3 --pmc passes -> profiles/pmc_latest.json.

Reads every *counter_collection.csv under the given directory (default gpurun_out/pmc), averages
FETCH_SIZE and WRITE_SIZE (KiB) over the launches of the K1 kernel and applies the gfx950
correction of /opt/skills/guides/MI355X_MICROARCH.md ("HBM"): FETCH_SIZE reports half the bytes of
a wide coalesced streaming read, so it is doubled; WRITE_SIZE is taken as is.
bench.py puts `hbm_bytes_per_launch` into roofline.traffic when `records` matches its workload.
"""
import csv
import glob
import json
import sys
from pathlib import Path

KERNEL = sys.argv[2] if len(sys.argv) > 2 else "k_span_join"
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
records = int(sys.argv[3]) if len(sys.argv) > 3 else 99999986

vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
name = None
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
        if KERNEL not in k or "spill" in k:
            continue
        name = k
        c = r["Counter_Name"]
        if c in vals:
            vals[c].append(float(r["Counter_Value"]))
if not vals["FETCH_SIZE"] or not vals["WRITE_SIZE"]:
    sys.exit(f"no FETCH_SIZE/WRITE_SIZE rows for {KERNEL} under {root}")
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"]) * 1024.0
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"]) * 1024.0
out = {
    "kernel": name,
    "records": records,
    "fetch_size_bytes_raw": fetch,
    "fetch_bytes_corrected": 2.0 * fetch,
    "write_bytes": write,
    "hbm_bytes_per_launch": 2.0 * fetch + write,
    "algorithmic_bytes_per_launch": 48 * records,
    "launches_averaged": {k: len(v) for k, v in vals.items()},
    "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); WRITE_SIZE as is",
    "run": sys.argv[5] if len(sys.argv) > 5 else "builder run",
}
dst = Path(sys.argv[4]) if len(sys.argv) > 4 else Path("profiles/pmc_latest.json")
dst.write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out))
