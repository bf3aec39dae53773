#!/usr/bin/env python3
"""Timeline of the last timed steps from a rocprofv3 --kernel-trace CSV: every dispatch's start/end
relative to the first K1 of the window, its stream, and the idle time between K1 launches.

  python tools/timeline.py gpurun_out/tl/<...>_kernel_trace.csv [--last 4]
"""
import argparse
import csv
import glob
import re


def short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1][:28]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last", type=int, default=4, help="K1 launches to show (from the end)")
    a = ap.parse_args()
    path = a.path
    if "*" in path:
        path = sorted(glob.glob(path))[0]
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                   r.get("Stream_Id") or r.get("Queue_Id", "?")))
    ev.sort()
    k1 = [i for i, e in enumerate(ev) if e[2].startswith("k_span_join_stream")]
    if len(k1) < a.last + 1:
        raise SystemExit(f"only {len(k1)} K1 launches")
    first = k1[-a.last - 1]
    t0 = ev[first][0]
    print(f"{'kernel':28s} {'stream':>6s} {'start_us':>9s} {'end_us':>9s} {'dur_us':>8s}")
    for s, e, n, q in ev[first:]:
        print(f"{n:28s} {q:>6s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}")
    starts = [ev[i][0] for i in k1[-a.last - 1:]]
    ends = [ev[i][1] for i in k1[-a.last - 1:]]
    gaps = [(starts[i + 1] - ends[i]) / 1e3 for i in range(len(starts) - 1)]
    period = [(starts[i + 1] - starts[i]) / 1e3 for i in range(len(starts) - 1)]
    print("K1 start-to-start us:", " ".join(f"{p:.1f}" for p in period))
    print("K1 end-to-next-start gap us:", " ".join(f"{g:.1f}" for g in gaps))


if __name__ == "__main__":
    main()
