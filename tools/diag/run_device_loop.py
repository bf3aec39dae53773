#!/usr/bin/env python3
"""Diagnostic: StoredSpanJob.run_device over the test_gpu_jobs input (1e7 TraceGen fragments in 40
row batches, in HBM), `reps` runs with or without the indexer items -- a short program to run under
`rocprofv3 --kernel-trace --stats`, whose per-kernel totals divided by `reps` are one run's.
usage: run_device_loop.py [indexer 0|1] [reps]"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from tests.bulkfrag import batches, encode
    from zipkin_amd import tracegen_host
    from zipkin_amd.aggregates import StoredSpanJob

    indexer = bool(int(sys.argv[1])) if len(sys.argv) > 1 else True
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    S = 500
    cols = tracegen_host(17, 1_000_000, target_records=10_000_000, max_depth=6, num_services=S)
    buf, off, _ = encode(cols)
    cuts = np.sort(np.random.default_rng(17).choice(np.arange(1, len(cols)), 39, replace=False)).tolist()
    dev = [(torch.from_numpy(b).cuda(), torch.from_numpy(o.view(np.int64)).cuda(), len(o) - 1)
           for b, o in batches(buf, off, cuts)]
    torch.cuda.synchronize()
    job = StoredSpanJob(clock=lambda: 10**15, max_services=S)
    job.run_device(dev, indexer=indexer)  # warm
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        job.run_device(dev, indexer=indexer)
        ts.append((time.perf_counter() - t0) * 1e3)
        print(f"run_device(indexer={indexer}): {ts[-1]:.2f} ms  phases {job.phase_ms}", flush=True)
    print(f"median {np.median(ts):.2f} ms, {len(cols) / np.median(ts) * 1e3:.3e} fragments/s", flush=True)
    job.close()


if __name__ == "__main__":
    main()
