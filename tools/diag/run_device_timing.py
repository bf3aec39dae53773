#!/usr/bin/env python3
"""Diagnostic: where StoredSpanJob.run_device's time goes on HBM-resident stored fragments (the
test_gpu_jobs input: 1e7 TraceGen fragments cut into 40 row batches). Prints the whole run and a
per-phase split (decoder / context creation, per-batch decode and accumulate, finalize)."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from tests.bulkfrag import batches, encode
    from zipkin_amd import DepsContext, tracegen_host
    from zipkin_amd.aggregates import StoredSpanJob
    from zipkin_amd.ingest import DeviceSpanDecoder

    S = 500
    n_target = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    cols = tracegen_host(17, n_target // 10, target_records=n_target, max_depth=6, num_services=S)
    buf, off, _ = encode(cols)
    cuts = np.sort(np.random.default_rng(17).choice(np.arange(1, len(cols)), 39, replace=False)).tolist()
    dev = [(torch.from_numpy(b).cuda(), torch.from_numpy(o.view(np.int64)).cuda(), len(o) - 1)
           for b, o in batches(buf, off, cuts)]
    torch.cuda.synchronize()
    job = StoredSpanJob(clock=lambda: 10**15, max_services=S)
    job.run_device(dev[:1])
    for indexer in (False, True, False, True):
        for _ in range(2):
            t0 = time.perf_counter()
            job.run_device(dev, indexer=indexer)
            print(f"run_device(indexer={indexer}): {len(cols)} fragments, {len(dev)} batches: "
                  f"{(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)

    # with an Aggregates store (as tests/test_gpu_jobs.py): the run, then the store call alone
    from zipkin_amd.aggregates import GpuAggregates

    for indexer in (False, True):
        store = GpuAggregates("cassandra")
        j2 = StoredSpanJob(aggregates=store, top_k=5, clock=lambda: 10**15, max_services=S)
        j2.run_device(dev[:1], indexer=indexer)
        t0 = time.perf_counter()
        deps = j2.run_device(dev, indexer=indexer)
        t1 = time.perf_counter()
        store.storeDependencies(deps)
        t2 = time.perf_counter()
        n_links = len(deps.links)
        t3 = time.perf_counter()
        print(f"run_device(indexer={indexer}) with a store: {(t1 - t0) * 1e3:.1f} ms; storeDependencies again "
              f"{(t2 - t1) * 1e3:.1f} ms; len(links) {(t3 - t2) * 1e3:.1f} ms ({n_links} links)", flush=True)
        j2.close()

    # the phases, by hand, on one stream (as run_device)
    stream = torch.cuda.Stream()
    t = {}

    def tick(k, t0):
        torch.cuda.synchronize()
        t[k] = t.get(k, 0.0) + time.perf_counter() - t0

    t0 = time.perf_counter()
    dec = DeviceSpanDecoder(4096, stream=stream.cuda_stream)
    tick("decoder create", t0)
    t0 = time.perf_counter()
    ctx = DepsContext(S, stream=stream.cuda_stream)
    tick("context create", t0)
    out = None
    for b, o, n in dev:
        if out is not None and out.capacity < n:
            out = None
        t0 = time.perf_counter()
        out, _ = dec.decode_device(b, o, n, out=out)
        tick("decode (40 batches)", t0)
        t0 = time.perf_counter()
        ctx.accumulate(out, clustered=True, continues=True)
        tick("accumulate (40 batches)", t0)
    t0 = time.perf_counter()
    ctx.finalize()
    tick("finalize", t0)
    # the same batches again through the warm decoder: per-batch decode times, without and with items,
    # and the two sketches' accumulates of the items
    from zipkin_amd.kv import KvSketch

    kvs = KvSketch(S, stream=stream.cuda_stream, width=4096)
    anns = KvSketch(S, stream=stream.cuda_stream, width=4096)
    for items in (False, True):
        per, sk = [], []
        for b, o, n in dev:
            if out.capacity < n:
                out = None
            t0 = time.perf_counter()
            if items:
                out, _, (ks, kh), (as_, ah) = dec.decode_device(b, o, n, out=out, items=True)
            else:
                out, _ = dec.decode_device(b, o, n, out=out)
            torch.cuda.synchronize()
            per.append((time.perf_counter() - t0) * 1e3)
            if items:
                t0 = time.perf_counter()
                kvs.accumulate(ks, kh)
                anns.accumulate(as_, ah)
                torch.cuda.synchronize()
                sk.append((time.perf_counter() - t0) * 1e3)
        per = np.array(per)
        print(f"  warm decoder (items={items}), per batch: median {np.median(per):.3f} ms, min {per.min():.3f}, "
              f"max {per.max():.3f}, sum {per.sum():.2f} ms", flush=True)
        if sk:
            sk = np.array(sk)
            print(f"  two sketch accumulates per batch: median {np.median(sk):.3f} ms, sum {sk.sum():.2f} ms", flush=True)
    kvs.close()
    anns.close()
    ctx.close()
    dec.close()
    for k, v in t.items():
        print(f"  {k:26s} {v * 1e3:8.2f} ms", flush=True)


if __name__ == "__main__":
    main()
