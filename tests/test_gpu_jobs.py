"""The job drivers on the path the bench measures (ZipkinAggregateJob.scala:20-45 fed as
StorageRecordReader.scala:49-54 reads rows): stored fragments in row order, cut into batches at
arbitrary points, streamed through StoredSpanJob (host decode of batch k+1 overlapping batch k on the
device, ZK_BATCH_TRACE_CLUSTERED | ZK_BATCH_CONTINUES), and ZipkinAggregateJob over device-resident
row-order batches. Bar: the stored Dependencies record bit-exact (m0 exact, m1..m4 identical fp64)
against the oracle over the decoded records; the measured job throughput is printed."""
import time

import numpy as np
import pytest

from oracle import oracle
from tests.bulkfrag import batches, encode, service_name
from zipkin_amd import DeviceColumns, tracegen_host
from zipkin_amd.aggregates import Dictionary, GpuAggregates, StoredSpanJob, ZipkinAggregateJob

pytestmark = pytest.mark.gpu


def _by_name(deps):
    return {(l.parent.name, l.child.name): tuple(l.duration_moments) for l in deps.links}


def _oracle_by_name(cols, S):
    ref = oracle.aggregate(cols, S, threads=16).moments()
    return {(service_name(p), service_name(c)): tuple(m) for (p, c), m in ref.items()}


def test_stored_span_job_streams_ten_million_fragments(gpu):
    S = 500
    cols = tracegen_host(17, 1_000_000, target_records=10_000_000, max_depth=6, num_services=S)
    assert len(cols) >= 9_900_000
    buf, off, exp = encode(cols)
    rng = np.random.default_rng(17)
    cuts = np.sort(rng.choice(np.arange(1, len(cols)), 39, replace=False)).tolist()  # 40 batches
    parts = batches(buf, off, cuts)
    want = _oracle_by_name(exp, S)
    store = GpuAggregates("cassandra")
    job = StoredSpanJob(aggregates=store, top_k=5, clock=lambda: 10**15)
    job.run(parts[:1])  # warm: buffers, kernels
    t0 = time.perf_counter()
    deps = job.run(parts)
    dt = time.perf_counter() - t0
    print(f"\nStoredSpanJob: {len(cols)} fragments ({len(buf) / 1e9:.2f} GB) in {len(parts)} batches: "
          f"{dt:.3f} s, {len(cols) / dt:.3e} fragments/s (host decode overlapped with the device job)")
    assert job.rejected == 0 and job.stats["records"] == len(cols)
    assert job.stats["not_clustered"] == 0
    assert _by_name(deps) == want
    stored = store.getDependencies(0, 10**15)
    assert {(l.parent.name, l.child.name) for l in stored.links} == set(want)
    # the annotation producers saw every fragment's indexer items
    assert all(v == ["custom.event"] for v in job.top_annotations.values())
    assert all(v == ["http.uri"] for v in job.top_kv.values())

    # the same 40 batches already in HBM, through the device decoder: with the indexer items (the
    # default) and dependencies only
    import torch

    dev = [(torch.from_numpy(b).cuda(), torch.from_numpy(o.view(np.int64)).cuda(), len(o) - 1) for b, o in parts]
    torch.cuda.synchronize()
    # the oracle's 250k-entry result dict is the test's, not the job's: kept out of the collector's
    # full passes while the job is timed
    import gc

    gc.collect()
    gc.freeze()
    for indexer in (True, False):
        if not indexer:
            # the previous iteration's records, released outside the timed region: comparing them
            # (_by_name) materialised ~250k DependencyLink objects each, whose teardown is the test's
            del ddeps, again
        dstore = GpuAggregates("cassandra")
        djob = StoredSpanJob(aggregates=dstore, top_k=5, clock=lambda: 10**15, max_services=S)
        djob.run_device(dev[:1], indexer=indexer)  # warm
        t0 = time.perf_counter()
        ddeps = djob.run_device(dev, indexer=indexer)
        ddt = time.perf_counter() - t0
        what = "decode with indexer items + accumulate + 2 sketches" if indexer else "decode + accumulate"
        job_ms = sum(v for k, v in djob.phase_ms.items() if k != "store")
        print(f"StoredSpanJob.run_device(indexer={indexer}): the same {len(cols)} fragments in HBM, {len(dev)} "
              f"batches: {ddt * 1e3:.1f} ms, {len(cols) / ddt:.3e} fragments/s ({what} + finalize + the "
              f"Aggregates store's puts); the job without the store's puts: {job_ms:.1f} ms, "
              f"{len(cols) / (job_ms * 1e-3):.3e} fragments/s")
        assert djob.rejected == 0 and djob.stats["records"] == len(cols)
        assert _by_name(ddeps) == want
        if indexer:  # the device decoder's items give run()'s top lists, stored the same way
            assert djob.top_kv == job.top_kv and djob.top_annotations == job.top_annotations
            for svc in job.top_kv:
                assert dstore.getTopKeyValueAnnotations(svc) == store.getTopKeyValueAnnotations(svc)
                assert dstore.getTopAnnotations(svc) == store.getTopAnnotations(svc)
        # a second run of the same job reuses its device objects (reset, not rebuilt): same result
        t0 = time.perf_counter()
        again = djob.run_device(dev, indexer=indexer)
        adt = time.perf_counter() - t0
        print("  phases (ms):", {k: round(v, 2) for k, v in djob.phase_ms.items()})
        print(f"  ... run again: {adt * 1e3:.1f} ms, {len(cols) / adt:.3e} fragments/s")
        assert _by_name(again) == want and djob.stats["records"] == len(cols)
        djob.close()
    gc.unfreeze()


def test_stored_span_job_on_the_device_decoder(gpu):
    import torch

    S = 97
    cols = tracegen_host(18, 100_000, target_records=1_000_000, max_depth=6, num_services=S)
    buf, off, exp = encode(cols)
    cuts = np.sort(np.random.default_rng(18).choice(np.arange(1, len(cols)), 7, replace=False)).tolist()
    dev = [(torch.from_numpy(b).cuda(), torch.from_numpy(o.view(np.int64)).cuda(), len(o) - 1)
           for b, o in batches(buf, off, cuts)]
    job = StoredSpanJob(clock=lambda: 10**15, top_k=5)
    deps = job.run_device(dev)
    assert job.rejected == 0 and job.stats["records"] == len(cols)
    assert _by_name(deps) == _oracle_by_name(exp, S)
    hjob = StoredSpanJob(clock=lambda: 10**15, top_k=5)
    hjob.run(batches(buf, off, cuts))
    assert job.top_kv == hjob.top_kv and job.top_annotations == hjob.top_annotations
    assert len(job.top_kv) == S


def test_run_device_top_lists_equal_run_on_rich_spans(gpu):
    """run_device's indexer items on spans with several binary annotations, distinct non-core
    values and hosts other than the span's service: the same top lists as the host-decode run()."""
    import torch

    from tests.richgen import gen_traces
    from tests.test_ingest import encode_all

    spans = gen_traces(207, 3000, max_depth=5, anomalies=0.0)
    by_trace: dict = {}
    for sp in spans:
        by_trace.setdefault(sp.trace_id, []).append(sp)
    traces = list(by_trace.values())
    host_batches, dev = [], []
    for i in range(0, len(traces), 400):
        blobs = encode_all([sp for t in traces[i:i + 400] for sp in t])
        offs = np.zeros(len(blobs) + 1, np.int64)
        offs[1:] = np.cumsum([len(b) for b in blobs])
        host_batches.append(blobs)
        dev.append((torch.from_numpy(np.frombuffer(b"".join(blobs), np.uint8).copy()).cuda(),
                    torch.from_numpy(offs).cuda(), len(blobs)))
    hjob = StoredSpanJob(clock=lambda: 10**15, top_k=8, strict=False)
    hdeps = hjob.run(host_batches)
    djob = StoredSpanJob(clock=lambda: 10**15, top_k=8, strict=False)
    ddeps = djob.run_device(dev)
    assert _by_name(ddeps) == _by_name(hdeps)
    assert djob.top_kv == hjob.top_kv and djob.top_annotations == hjob.top_annotations
    assert sum(len(v) for v in djob.top_kv.values()) > 20


def test_aggregate_job_on_device_row_batches(gpu):
    """ZipkinAggregateJob over one 1e8-record TraceGen batch in HBM cut into 4 row-order batches at
    arbitrary points: bit-exact against the oracle, and the job time per 1e8 records (accumulates +
    one finalize to host + the Dependencies record) printed next to the bench's C2 step."""
    import torch

    from zipkin_amd import DepsContext, tracegen_params

    S, N = 500, 100_000_000
    p = tracegen_params(2, N // 15 + 1000, target_records=N, max_depth=6, num_services=S)
    cols = DeviceColumns(N)
    with DepsContext(S) as g:
        n, _ = g.tracegen_device(p, cols)
    torch.cuda.synchronize()
    names = Dictionary([service_name(i) for i in range(S)])
    cuts = sorted(np.random.default_rng(2).choice(np.arange(1, n), 3, replace=False).tolist())
    bounds = [0, *[c + (c & 1) for c in cuts], n]  # even offsets keep the 16-B column alignment

    def view(a, b):
        v = DeviceColumns.__new__(DeviceColumns)
        for k in ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags"):
            setattr(v, k, getattr(cols, k)[a:b])
        v.n = v.capacity = b - a
        return v

    parts = [view(a, b) for a, b in zip(bounds[:-1], bounds[1:])]
    job = ZipkinAggregateJob(names, clock=lambda: 10**15, order="rows", verify=False)
    job.run(parts, S)  # warm
    times, acc_t, fin_t = [], [], []
    for _ in range(5):
        t0 = time.perf_counter()
        ctx = job.accumulate_all(parts, S)
        ctx.sync()
        t1 = time.perf_counter()
        table = ctx.finalize()
        t2 = time.perf_counter()
        deps = job._publish(table)
        t3 = time.perf_counter()
        times.append(t3 - t0)
        acc_t.append(t1 - t0)
        fin_t.append(t2 - t1)
    ms = sorted(times)[2] * 1e3
    print(f"\nZipkinAggregateJob: {n} device records in 4 row batches: {ms:.3f} ms per run (median of 5: "
          f"accumulates {sorted(acc_t)[2] * 1e3:.3f} ms, finalize to host {sorted(fin_t)[2] * 1e3:.3f} ms, "
          f"record {ms - (sorted(acc_t)[2] + sorted(fin_t)[2]) * 1e3:.3f} ms), {n / ms * 1e3:.3e} spans/s")
    # a longer job: the same four batches twice more (the multiset of records, three times)
    t0 = time.perf_counter()
    job.run(parts * 3, S)
    ms3 = (time.perf_counter() - t0) * 1e3
    print(f"ZipkinAggregateJob: {3 * n} device records in 12 row batches: {ms3:.3f} ms, "
          f"{ms3 / 3:.3f} ms per 1e8-record third, {3 * n / ms3 * 1e3:.3e} spans/s")
    host = cols.to_host(n)
    assert _by_name(deps) == _oracle_by_name(host, S)
    job.close()


def test_default_job_takes_batches_in_any_order(gpu):
    """ZipkinAggregateJob's defaults (order="any", verify=True) accept what the reference's groupBy
    traceId accepts (ZipkinAggregateJob.scala:21-22,28-33): each batch's fragments in any order. A
    trace that recurs in a later batch fails the job instead of being joined in two halves."""
    from zipkin_amd import ZkError, _abi

    S = 61
    cols = tracegen_host(41, 20_000, max_depth=6, num_services=S)
    names = Dictionary([service_name(i) for i in range(S)])
    # three batches of whole traces (by traceId), each shuffled
    part = (cols.trace_id % np.uint64(3)).astype(np.int64)
    rng = np.random.default_rng(41)
    parts = []
    for k in range(3):
        idx = np.flatnonzero(part == k)
        parts.append(cols.take(rng.permutation(idx)))
    job = ZipkinAggregateJob(names, clock=lambda: 10**15)
    deps = job.run(parts, S)
    assert _by_name(deps) == _oracle_by_name(cols, S)
    assert job.stats["not_clustered"] == 0
    # a trace cut across two batches: detected, not mis-joined
    idx = rng.permutation(len(cols))
    halves = [cols.take(np.sort(idx[: len(cols) // 2])), cols.take(np.sort(idx[len(cols) // 2:]))]
    with pytest.raises(ZkError) as e:
        job.run(halves, S)
    assert e.value.status == _abi.ZK_ERR_NOT_CLUSTERED
    job.close()


def test_run_device_waits_for_the_callers_stream(gpu):
    """StoredSpanJob.run_device reads tensors the caller's current stream is still writing: the
    job's stream is ordered after it (no torch.cuda.synchronize() by the caller)."""
    import torch

    S = 97
    cols = tracegen_host(43, 50_000, target_records=400_000, max_depth=6, num_services=S)
    buf, off, exp = encode(cols)
    cuts = np.sort(np.random.default_rng(43).choice(np.arange(1, len(cols)), 3, replace=False)).tolist()
    host = batches(buf, off, cuts)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        # the caller's stream: busy first, then the non_blocking uploads from pinned memory
        x = torch.randn(2048, 2048, device="cuda")
        for _ in range(8):
            x = (x @ x) * (1.0 / 2048)
        dev = [(torch.from_numpy(b).pin_memory().cuda(non_blocking=True),
                torch.from_numpy(o.view(np.int64)).pin_memory().cuda(non_blocking=True), len(o) - 1)
               for b, o in host]
        job = StoredSpanJob(clock=lambda: 10**15, max_services=S)
        deps = job.run_device(dev)
    assert job.rejected == 0 and job.stats["records"] == len(cols)
    assert _by_name(deps) == _oracle_by_name(exp, S)
