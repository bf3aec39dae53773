#!/usr/bin/env python3
"""Diagnostic: device decode time with and without the span indexer's items on the bench's ingest
workload (2e7 fragments), for the library in ZKAGG_LIB (A/B of -DZK_ING_ITEMS_DIAG builds: timing
only, their items are wrong)."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch

    import bench
    from zipkin_amd import tracegen_host
    from zipkin_amd.ingest import DeviceSpanDecoder

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    base = tracegen_host(2, 9000, max_depth=6, num_services=500)
    blobs = bench._thrift_fragments(base, 500)
    reps = max(1, 20_000_000 // len(blobs))
    n = len(blobs) * reps
    lens = np.array([len(b) for b in blobs], np.int64)
    buf = torch.from_numpy(np.frombuffer(b"".join(blobs), np.uint8).copy()).to(dev).repeat(reps)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(np.tile(lens, reps))
    off = torch.from_numpy(offs).to(dev)
    dec = DeviceSpanDecoder(4096)
    out = {"lib": Path(os.environ.get("ZKAGG_LIB", "libzkagg.so")).name, "fragments": n}
    for items in (False, True):
        cols = None
        for _ in range(2):
            r = dec.decode_device(buf, off, n, out=cols, items=items, item_cap=2 * n)
            cols = r[0]
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(5):
            dec.decode_device(buf, off, n, out=cols, items=items, item_cap=2 * n)
        ev1.record()
        torch.cuda.synchronize()
        out["items" if items else "records"] = round(ev0.elapsed_time(ev1) / 5, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
