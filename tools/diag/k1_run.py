"""Diagnostic: run the clustered C2 accumulate (1e8 records, 500 services) `steps` times with the
library named by ZKAGG_LIB -- a short, K1-dominated workload for profilers (PC sampling,
counters). Prints K1's average launch time."""
import os
import sys

import torch

sys.path.insert(0, ".")
from zipkin_amd import DepsContext, DeviceColumns, tracegen_params  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream(device=torch.device("cuda", 0))
    torch.cuda.set_stream(stream)
    with DepsContext(500, device=0, stream=stream.cuda_stream, timing=True) as c:
        p = tracegen_params(2, n // 15 + 1000, target_records=n, max_depth=6, num_services=500)
        cols = DeviceColumns(n, device="cuda:0")
        nrec, _ = c.tracegen_device(p, cols)
        c.accumulate(cols, clustered=True, verify=False, n=nrec)
        torch.cuda.synchronize()
        t0 = c.timing()
        for _ in range(steps):
            c.reset()
            c.accumulate(cols, clustered=True, verify=False, n=nrec)
        torch.cuda.synchronize()
        t1 = c.timing()
    k1 = (t1["join_ms_total"] - t0["join_ms_total"]) / max(1, t1["join_calls"] - t0["join_calls"])
    print(f"{os.path.basename(os.environ.get('ZKAGG_LIB', 'libzkagg.so'))} records {nrec} K1 {k1:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
