"""Diagnostic: ZipkinAggregateJob over one 1e8-record TraceGen batch in HBM cut into K row batches
(the test_gpu_jobs case), run R times, for a rocprofv3 kernel trace of the job's timeline.

python tools/diag/job_trace.py [K] [R]
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from zipkin_amd import DepsContext, DeviceColumns, tracegen_params  # noqa: E402
from zipkin_amd.aggregates import Dictionary, ZipkinAggregateJob  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    S, N = 500, 100_000_000
    p = tracegen_params(2, N // 15 + 1000, target_records=N, max_depth=6, num_services=S)
    cols = DeviceColumns(N)
    with DepsContext(S) as g:
        n, _ = g.tracegen_device(p, cols)
    torch.cuda.synchronize()
    names = Dictionary([f"service-{i}" for i in range(S)])
    cuts = sorted(np.random.default_rng(2).choice(np.arange(1, n), K - 1, replace=False).tolist())
    bounds = [0, *[c + (c & 1) for c in cuts], n]

    def view(a, b):
        v = DeviceColumns.__new__(DeviceColumns)
        for k in ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags"):
            setattr(v, k, getattr(cols, k)[a:b])
        v.n = v.capacity = b - a
        return v

    parts = [view(a, b) for a, b in zip(bounds[:-1], bounds[1:])]
    job = ZipkinAggregateJob(names, clock=lambda: 10**15, order="rows", verify=False)
    job.run(parts, S)
    acc, enq = [], []
    for _ in range(R):
        t0 = time.perf_counter()
        ctx = job.accumulate_all(parts, S)
        t1 = time.perf_counter()
        ctx.sync()
        t2 = time.perf_counter()
        enq.append(t1 - t0)
        acc.append(t2 - t0)
    print(f"{K} batches: accumulate (enqueue {np.median(enq) * 1e3:.3f} ms) to sync {np.median(acc) * 1e3:.3f} ms",
          flush=True)
    job.close()


if __name__ == "__main__":
    main()
