"""Diagnostic: a reused ctx (caller-owned table, torch stream, timing) over many steps vs a fresh ctx."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from zipkin_amd import DepsContext, DeviceColumns, tracegen_params  # noqa: E402
from zipkin_amd._abi import table_words  # noqa: E402

COLS = ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags")


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    order = sys.argv[2] if len(sys.argv) > 2 else "clustered"
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    S = 500
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    table = torch.zeros(table_words(S), dtype=torch.int64, device=dev)
    ctx = DepsContext(S, device=0, stream=stream.cuda_stream, timing=True, table_ptr=table.data_ptr(),
                      table_bytes=table.numel() * 8)
    p = tracegen_params(2, N // 15 + 1000, target_records=N, max_depth=6, num_services=S)
    cols = DeviceColumns(N, device="cuda:0")
    n, ntr = ctx.tracegen_device(p, cols)
    clustered = cols
    if order == "shuffled":
        g = torch.Generator(device=dev)
        g.manual_seed(1002)
        perm = torch.randperm(n, device=dev, generator=g)
        sc = DeviceColumns(n, device="cuda:0")
        for k in COLS:
            torch.index_select(getattr(cols, k)[:n], 0, perm, out=getattr(sc, k))
        cols = sc
    with DepsContext(S, device=0) as f:
        f.accumulate(clustered, clustered=True, verify=True, n=n)
        ref = f.finalize()
        rst = f.stats()
    print("fresh stats", rst, flush=True)
    for step in range(6):
        ctx.reset()
        ctx.accumulate(cols, clustered=(order == "clustered"), verify=False)
        got = ctx.finalize()
        st = ctx.stats()
        bad = [k for k in ("m0", "m1", "m2", "m3", "m4") if not np.array_equal(getattr(got, k), getattr(ref, k))]
        bads = {k: (st[k], rst[k]) for k in rst if st[k] != rst[k] and k != "spilled_traces"}
        print(f"step {step}: arrays differ {bad}, stats differ {bads}, m0 cells {int((got.m0 != ref.m0).sum())}",
              flush=True)


if __name__ == "__main__":
    main()
