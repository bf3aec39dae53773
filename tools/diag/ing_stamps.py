#!/usr/bin/env python3
"""Diagnostic: per-phase cycle shares of the LDS ingest decoder (k_ing_decode_lds) from the
-DZK_ING_STAMPS build (ZK_VARIANT, default "ingstamps"), on the bench's ingest workload, and the
decode time of each library named in ZK_TIME_VARIANTS (comma-separated; "cur" = libzkagg.so).
Only the SHARES mean anything for the stamps build (its waits forbid overlaps)."""
import ctypes as C
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent
PHASES = ["round setup", "copy-in", "snappy", "thrift walk", "resolve+publish", "round sync"]


def run_one(lib, stamps):
    os.environ["ZKAGG_LIB"] = str(lib)
    sys.path.insert(0, str(ROOT))
    import numpy as np
    import torch

    import bench
    from zipkin_amd import _abi, tracegen_host
    from zipkin_amd.ingest import DeviceSpanDecoder

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    base = tracegen_host(1, 9000, max_depth=6, num_services=500)
    blobs = bench._thrift_fragments(base, 500)
    reps = max(1, 20_000_000 // len(blobs))
    n = len(blobs) * reps
    lens = np.array([len(b) for b in blobs], np.int64)
    buf = torch.from_numpy(np.frombuffer(b"".join(blobs), np.uint8).copy()).to(dev).repeat(reps)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(np.tile(lens, reps))
    off = torch.from_numpy(offs).to(dev)
    dec = DeviceSpanDecoder(4096)
    cols, _ = dec.decode_device(buf, off, n)
    torch.cuda.synchronize()
    out = {"lib": Path(lib).name, "fragments": n}
    if stamps:
        dbg = C.CDLL(str(_abi.LIB_PATH)).zk_debug_ing_stamps
        dbg.argtypes = [C.c_void_p, C.c_int]
        raw = (C.c_ulonglong * 8)()
        dbg(raw, 1)
        dec.decode_device(buf, off, n, out=cols)
        torch.cuda.synchronize()
        dbg(raw, 1)
        tot = sum(raw[i] for i in range(len(PHASES)))
        out["shares"] = {PHASES[i]: round(raw[i] / tot, 4) for i in range(len(PHASES))}
    else:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(5):
            dec.decode_device(buf, off, n, out=cols)
        ev1.record()
        torch.cuda.synchronize()
        out["ms_per_decode"] = round(ev0.elapsed_time(ev1) / 5, 3)
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 2:
        run_one(sys.argv[1], sys.argv[2] == "1")
        return
    libs = [(v, True) for v in os.environ.get("ZK_STAMP_VARIANTS", "ingstamps").split(",") if v]
    libs += [(v, False) for v in os.environ.get("ZK_TIME_VARIANTS", "cur").split(",") if v]
    for v, st in libs:
        lib = ROOT / "zipkin_amd" / ("libzkagg.so" if v == "cur" else f"libzkagg_{v}.so")
        subprocess.run([sys.executable, __file__, str(lib), "1" if st else "0"], check=True, timeout=300)


if __name__ == "__main__":
    main()
