"""The C ABI's input-ownership rule (include/zkagg.h): HOST column pointers are borrowed for the
duration of the call only. A caller that reuses its page-locked batch buffer the moment
zk_deps_accumulate (or zk_kv_accumulate / zk_rt_accumulate) returns -- what a JNI host with one
direct ByteBuffer per column does, GpuDependenciesJob.scala -- must still get exactly the records it
passed: the values the drop-in receives are immutable (Aggregates.scala:26-37 takes plain Scala
values). Each test queues a few ms of unrelated work on the ctx stream first, so that the staging
copies would run well after the call returned if the call did not wait for them, then overwrites
the pinned buffers at once and compares against the oracle."""
import numpy as np
import pytest

from oracle import oracle
from tests.test_gpu_parity import COLS, assert_parity
from zipkin_amd import DepsContext, SpanColumns, tracegen_host

pytestmark = pytest.mark.gpu


def _busy(stream):
    """~ms of device work queued on `stream` ahead of the library's copies."""
    import torch

    with torch.cuda.stream(stream):
        x = torch.randn(2048, 2048, device="cuda")
        for _ in range(12):
            x = (x @ x) * (1.0 / 2048)
    return x


def _pinned_like(cols: SpanColumns, cap: int) -> SpanColumns:
    import torch

    out = []
    for k in COLS:
        a = getattr(cols, k)
        t = torch.empty(cap * a.dtype.itemsize, dtype=torch.uint8, pin_memory=True)
        out.append(t.numpy().view(a.dtype))
    return SpanColumns(*out)


def _fill(dst: SpanColumns, src: SpanColumns) -> SpanColumns:
    n = len(src)
    for k in COLS:
        getattr(dst, k)[:n] = getattr(src, k)
    return SpanColumns(*[getattr(dst, k)[:n] for k in COLS])  # views of the pinned buffers


def test_pinned_host_batch_reused_right_after_accumulate(gpu):
    import torch

    S = 97
    a = tracegen_host(31, 4000, max_depth=6, num_services=S)
    b = tracegen_host(32, 4000, max_depth=6, num_services=S)
    b.trace_id ^= np.uint64(1 << 63)  # disjoint traces
    cap = max(len(a), len(b))
    pin = _pinned_like(a, cap)
    stream = torch.cuda.Stream()
    with DepsContext(S, stream=stream.cuda_stream) as ctx:
        keep = _busy(stream)
        ctx.accumulate(_fill(pin, a), clustered=True, verify=True)
        # the caller's next batch goes into the same pinned buffers at once
        ctx.accumulate(_fill(pin, b), clustered=True, verify=True)
        for k in COLS:  # and then garbage, before the device has necessarily finished
            getattr(pin, k)[:] = np.frombuffer(np.random.default_rng(1).bytes(getattr(pin, k).nbytes),
                                               dtype=getattr(pin, k).dtype)
        got = ctx.finalize()
        st = ctx.stats()
        del keep
    ref = oracle.aggregate(SpanColumns.concat([a, b]), S, threads=8)
    assert_parity(got, st, ref)


def test_pinned_sketch_inputs_reused_right_after_accumulate(gpu):
    """zk_kv_accumulate with host keys: the same rule."""
    import torch

    from oracle.kv import KvOracle
    from zipkin_amd.kv import KvSketch

    S, n = 16, 200_000
    rng = np.random.default_rng(5)
    svc = rng.integers(0, S, n).astype(np.uint32)
    keys = (rng.zipf(1.3, n) % 5000).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    psvc = torch.empty(n, dtype=torch.int32, pin_memory=True).numpy().view(np.uint32)
    pkey = torch.empty(n, dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
    stream = torch.cuda.Stream()
    with KvSketch(S, width=1024, seed=3, stream=stream.cuda_stream) as sk:
        keep = _busy(stream)
        psvc[:] = svc
        pkey[:] = keys
        sk.accumulate(psvc, pkey)
        psvc[:] = 0
        pkey[:] = 1
        got_keys, got_est, got_cnt = sk.topk_all(8)
        del keep
    o = KvOracle(S, width=1024, seed=3)
    o.accumulate(svc, keys)
    want_keys, want_est, want_cnt = o.topk_all(8)
    assert np.array_equal(got_cnt, want_cnt)
    for s in range(S):
        assert list(got_keys[s][: got_cnt[s]]) == list(want_keys[s][: want_cnt[s]])
        assert list(got_est[s][: got_cnt[s]]) == list(want_est[s][: want_cnt[s]])
