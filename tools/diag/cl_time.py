"""Diagnostic: time the clustering pass of a shuffled C2 batch (1e8 records, 500 services) for the
library named by ZKAGG_LIB (A/B of clustering variants; no parity check -- diagnostic builds may
be wrong on purpose). Prints one line: variant, clustering ms per batch, K1 ms, step ms.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from zipkin_amd import DepsContext, DeviceColumns, tracegen_params  # noqa: E402

COLS = ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags")


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    with DepsContext(500, device=0, stream=stream.cuda_stream) as g:
        p = tracegen_params(2, int(N / 15) + 1000, target_records=N, max_depth=6, num_services=500)
        cols = DeviceColumns(N, device="cuda:0")
        n, _ = g.tracegen_device(p, cols)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    perm = torch.randperm(n, device=dev, generator=gen)
    sc = DeviceColumns(n, device="cuda:0")
    for k in COLS:
        torch.index_select(getattr(cols, k)[:n], 0, perm, out=getattr(sc, k))
    torch.cuda.synchronize()
    del perm, cols
    with DepsContext(500, device=0, stream=stream.cuda_stream, timing=True) as c:
        c.accumulate(sc, clustered=False, verify=False, n=n)  # warm: allocations
        torch.cuda.synchronize()
        t0 = c.timing()
        w0 = time.perf_counter()
        for _ in range(steps):
            c.reset()
            c.accumulate(sc, clustered=False, verify=False, n=n)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - w0) / steps * 1e3
        t1 = c.timing()
    cl = (t1["cluster_ms_total"] - t0["cluster_ms_total"]) / steps
    k1 = (t1["join_ms_total"] - t0["join_ms_total"]) / max(1, t1["join_calls"] - t0["join_calls"])
    name = os.path.basename(os.environ.get("ZKAGG_LIB", "libzkagg.so"))
    print(f"{name:28s} n {n} cluster {cl:.3f} ms  K1 {k1:.3f} ms  step {wall:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
