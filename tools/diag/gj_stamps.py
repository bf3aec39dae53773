#!/usr/bin/env python3
"""Diagnostic: per-phase cycle shares of the group join (k_group_join) from the -DZK_STAMPS build,
on the shuffled C2 batch. Run on the GPU box: python tools/diag/gj_stamps.py [records]
Only the SHARES mean anything (the stamps' own waits forbid overlaps the product kernel has)."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent
os.environ["ZKAGG_LIB"] = str(ROOT / "zipkin_amd" / f"libzkagg_{os.environ.get('ZK_VARIANT', 'stamps')}.so")
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from zipkin_amd import DepsContext, DeviceColumns, _abi, tracegen_params  # noqa: E402

PHASES = ["cut next batch", "stage (waits for the columns)", "hash insert", "merge", "validate/join/emit",
          "append links", "loop (load issue)", "-", "barrier waits"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    S = 500
    dbg = C.CDLL(str(_abi.LIB_PATH)).zk_debug_stamps
    dbg.argtypes = [C.c_void_p, C.c_int]
    ctx = DepsContext(S, device=0, timing=True)
    cols = DeviceColumns(n, device="cuda:0")
    nrec, _ = ctx.tracegen_device(tracegen_params(2, n // 15 + 1000, target_records=n, max_depth=6, num_services=S),
                                  cols)
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    perm = torch.randperm(nrec, device="cuda", generator=g)
    sc = DeviceColumns(nrec, device="cuda:0")
    for k in ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags"):
        torch.index_select(getattr(cols, k)[:nrec], 0, perm, out=getattr(sc, k))
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 16)()
    for it in range(3):
        ctx.reset()
        ctx.accumulate(sc, clustered=False, verify=False)
        ctx.sync()
        if it == 0:
            dbg(buf, 1)
    dbg(buf, 1)
    tot = sum(buf[i] for i in range(9))
    print(json.dumps({"records": nrec, "join_ms_last": ctx.timing()["join_ms"],
                      "shares": {PHASES[i]: round(buf[i] / tot, 4) for i in range(9)},
                      "raw": [int(buf[i]) for i in range(9)]}, indent=1))


if __name__ == "__main__":
    main()
