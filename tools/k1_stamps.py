#!/usr/bin/env python3
"""Diagnostic: per-phase cycle shares of K1 (k_span_join_stream) from the -DZK_STAMPS build.

Run on the GPU box:  python tools/k1_stamps.py [records]
Reads the s_memtime sums the stamps build accumulates per phase (summed over waves). Only the
SHARES mean anything: the stamps' own waits forbid overlaps the product kernel has.
"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
variant = os.environ.get("ZK_VARIANT", "stamps")
os.environ["ZKAGG_LIB"] = str(ROOT / "zipkin_amd" / f"libzkagg_{variant}.so")
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from zipkin_amd import DepsContext, DeviceColumns, tracegen_params  # noqa: E402
from zipkin_amd import _abi  # noqa: E402

PHASES = ["boundaries", "scan+issue loads", "stage", "hash insert", "merge", "validate/join/emit",
          "prefix+write links", "loop end", "barrier waits"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    S = 500
    L = _abi.lib()
    dbg = C.CDLL(str(_abi.LIB_PATH)).zk_debug_stamps
    dbg.argtypes = [C.c_void_p, C.c_int]
    ctx = DepsContext(S, device=0, timing=True)
    cols = DeviceColumns(n, device="cuda:0")
    p = tracegen_params(2, n // 15 + 1000, target_records=n, max_depth=6, num_services=S)
    nrec, _ = ctx.tracegen_device(p, cols)
    buf = (C.c_ulonglong * 16)()
    for it in range(3):
        ctx.reset()
        ctx.accumulate(cols, clustered=True, verify=False)
        ctx.sync()
        if it == 0:
            dbg(buf, 1)  # warm-up: discard
    dbg(buf, 1)
    tm = ctx.timing()
    tot = sum(buf[i] for i in range(9))
    out = {"records": nrec, "join_ms_last": tm["join_ms"],
           "shares": {PHASES[i]: round(buf[i] / tot, 4) for i in range(9)},
           "raw": [int(buf[i]) for i in range(9)]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
