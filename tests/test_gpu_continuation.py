"""Traces cut at batch edges (ZK_BATCH_CONTINUES), through the C ABI on the GPU.

The reference job has no batch boundary: every fragment of a trace meets its siblings in the
(id, traceId) and (parentId, traceId) shuffles whatever file or split it came from
(ZipkinAggregateJob.scala:20-33). A streaming reader of row-per-trace storage
(StorageRecordReader.scala:49-54) cuts batches wherever its buffer fills, so a trace can straddle
two or more batches. With ZK_BATCH_CONTINUES the library holds the batch's last trace back and joins
it with the next batch's leading fragments of the same traceId; the result must equal the oracle's
over the whole stream, bit for bit, and the clustering check must not fire."""
import numpy as np
import pytest

from oracle import oracle
from tests.test_gpu_parity import assert_parity, cols_from_rows, star_trace
from zipkin_amd import DepsContext, DeviceColumns, SpanColumns, ZkError, _abi, tracegen_host

pytestmark = pytest.mark.gpu


def cut(cols, points):
    bounds = [0, *sorted(points), len(cols)]
    return [cols.take(slice(a, b)) for a, b in zip(bounds[:-1], bounds[1:])]


def run_stream(parts, S, device=False, verify=True, last_continues=False, **kw):
    with DepsContext(S, **kw) as ctx:
        for i, p in enumerate(parts):
            b = DeviceColumns.from_host(p) if device else p
            cont = last_continues or i + 1 < len(parts)
            ctx.accumulate(b, clustered=True, verify=verify, continues=cont)
        return ctx.finalize(), ctx.stats()


@pytest.mark.parametrize("batches", [2, 3, 5])
@pytest.mark.parametrize("device", [False, True])
def test_traces_cut_at_batch_edges_equal_the_oracle(gpu, batches, device):
    S = 97
    cols = tracegen_host(61 + batches, 20_000, max_depth=6, num_services=S)
    ref = oracle.aggregate(cols, S)
    rng = np.random.default_rng(batches)
    pts = rng.choice(np.arange(1, len(cols)), batches - 1, replace=False)
    # cuts at random positions: most land inside a trace (and at odd and even offsets, so the
    # leading run's end is both)
    got, st = run_stream(cut(cols, pts), S, device=device)
    assert_parity(got, st, ref)
    assert st["not_clustered"] == 0


def test_one_trace_over_five_batches(gpu):
    """A 20k-record trace spread over five batches (three of them inside it entirely), between
    ordinary traces; cut points at odd and even offsets."""
    S = 9
    rows = []
    for t in range(50):
        rows += star_trace(100 + t, 1 + t % 6, svc_root=t % S, nsvc=S)
    big0 = len(rows)
    rows += star_trace(7777, 10_000, nsvc=S)
    big1 = len(rows)
    for t in range(50):
        rows += star_trace(900 + t, 1 + t % 5, svc_root=t % S, nsvc=S)
    cols = cols_from_rows(rows)
    ref = oracle.aggregate(cols, S)
    pts = [big0 + 3, big0 + 4_001, big0 + 9_000, big0 + 15_555, big1 - 2]
    for device in (False, True):
        got, st = run_stream(cut(cols, pts), S, device=device)
        assert_parity(got, st, ref)
        assert st["not_clustered"] == 0


def test_held_trace_is_flushed_by_finalize_and_by_a_plain_batch(gpu):
    S = 13
    cols = tracegen_host(71, 3_000, max_depth=5, num_services=S)
    ref = oracle.aggregate(cols, S)
    mid = len(cols) // 2 + 1
    # the last batch also says "continues": finalize aggregates the held trace
    got, st = run_stream(cut(cols, [mid]), S, last_continues=True)
    assert_parity(got, st, ref)
    # an empty batch without the flag flushes it too
    with DepsContext(S) as ctx:
        ctx.accumulate(cols.take(slice(0, mid)), clustered=True, continues=True)
        ctx.accumulate(cols.take(slice(mid, len(cols))), clustered=True, continues=True)
        ctx.accumulate(SpanColumns.empty(0), clustered=True)
        st = ctx.stats()
        assert st["records"] == len(cols)
        assert_parity(ctx.finalize(), ctx.stats(), ref)


def test_without_the_flag_a_cut_trace_is_detected(gpu):
    rows = star_trace(5, 40, nsvc=5)
    parts = cut(cols_from_rows(rows), [17])
    with DepsContext(5) as ctx:
        for p in parts:
            ctx.accumulate(p, clustered=True, verify=True)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_NOT_CLUSTERED
    got, st = run_stream(parts, 5)
    assert_parity(got, st, oracle.aggregate(cols_from_rows(rows), 5))


def test_continues_needs_clustered_batches(gpu):
    cols = cols_from_rows(star_trace(3, 4, nsvc=5))
    with DepsContext(5) as ctx:
        with pytest.raises(ZkError) as e:
            ctx.accumulate(cols, clustered=False, continues=True)
        assert e.value.status == _abi.ZK_ERR_INVALID_ARG


def test_held_trace_longer_than_max_trace_is_too_large(gpu):
    """max_trace_records bounds a held trace like any other: finalize reports it, the other traces
    of the stream are aggregated."""
    S = 7
    rows = star_trace(1, 30, nsvc=S) + star_trace(2, 800, nsvc=S) + star_trace(3, 30, nsvc=S)
    cols = cols_from_rows(rows)
    a, b = 61, 61 + 1601  # trace 2 (1601 records) spans three batches
    parts = cut(cols, [a + 500, a + 1100, b + 10])
    with DepsContext(S, max_trace_records=1000) as ctx:
        for p in parts[:-1]:
            ctx.accumulate(p, clustered=True, continues=True)
        ctx.accumulate(parts[-1], clustered=True)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_TRACE_TOO_LARGE
        assert ctx.stats()["trace_too_large"] == 1


@pytest.mark.parametrize("verify", [False, True])
def test_held_trace_then_a_batch_in_any_order(gpu, verify):
    """A batch without ZK_BATCH_TRACE_CLUSTERED after a CONTINUES batch ends the held trace
    (zkagg.h): the held fragments are aggregated as one trace, and the unclustered batch as a whole
    -- its fragments of the same traceId form a trace of their own, even when the batch happens to
    start with them (> 2^18 records, so without verification the group join takes it)."""
    S = 61
    cols = tracegen_host(93, 16_000, max_depth=6, num_services=S)
    tid = cols.trace_id
    starts = np.flatnonzero(np.r_[True, tid[1:] != tid[:-1]])
    t0, t1 = starts[200], starts[201]  # trace 200 is cut in the middle
    assert t1 - t0 >= 4
    mid = (t0 + t1) // 2
    held = cols.take(slice(0, mid))
    rest_of_t = cols.take(slice(mid, t1))
    tail = cols.take(slice(t1, len(cols)))
    tail = tail.take(np.random.default_rng(93).permutation(len(tail)))
    second = SpanColumns.concat([rest_of_t, tail])  # starts with the held trace's other fragments
    assert len(second) > 2 ** 18
    # expected: the two parts of trace 200 as two independent traces (its second part renamed)
    renamed = rest_of_t.take(np.arange(len(rest_of_t)))
    renamed.trace_id[:] = np.uint64(0xFEEDFACECAFE0001)
    ref = oracle.aggregate(SpanColumns.concat([held, renamed, tail]), S)
    for device in (False, True):
        with DepsContext(S) as ctx:
            a = DeviceColumns.from_host(held) if device else held
            b = DeviceColumns.from_host(second) if device else second
            ctx.accumulate(a, clustered=True, verify=verify, continues=True)
            ctx.accumulate(b, clustered=False, verify=verify)
            if verify:
                # trace 200 now arrived over two accumulate calls: the check reports it
                with pytest.raises(ZkError) as e:
                    ctx.finalize()
                assert e.value.status == _abi.ZK_ERR_NOT_CLUSTERED
                assert ctx.stats()["not_clustered"] == 1
                continue
            got, st = ctx.finalize(), ctx.stats()
        assert_parity(got, st, ref)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_random_streams_equal_the_oracle(gpu, seed):
    """The device-side held-trace state machine under random streams: TraceGen traces with long star
    traces (600-3000 records, longer than K1's 512-record window) mixed in, cut at random points
    (inside traces, at trace boundaries, 1-record batches, a batch inside one trace), empty CONTINUES
    batches between them, host and device pointers and ZK_BATCH_VERIFY_TRACES chosen per batch. Each
    stream equals the oracle over the whole stream, bit for bit, with no clustering report."""
    rng = np.random.default_rng(seed)
    S = 41
    base = tracegen_host(1000 + seed, 3_000, max_depth=5, num_services=S)
    tid = base.trace_id
    starts = np.flatnonzero(np.r_[True, tid[1:] != tid[:-1]])
    bounds = list(starts) + [len(base)]
    pieces, big_at = [], set(rng.choice(len(starts), 6, replace=False).tolist())
    for t in range(len(starts)):
        pieces.append(base.take(slice(bounds[t], bounds[t + 1])))
        if t in big_at:
            n_children = int(rng.integers(300, 1500))
            pieces.append(cols_from_rows(star_trace(0xB16000 + 97 * t + seed, n_children, svc_root=t % S, nsvc=S)))
    cols = SpanColumns.concat(pieces)
    n = len(cols)
    ref = oracle.aggregate(cols, S)
    tid = cols.trace_id
    tstarts = np.flatnonzero(np.r_[True, tid[1:] != tid[:-1]])
    cuts = set(rng.choice(np.arange(1, n), 25, replace=False).tolist())  # mostly inside traces
    cuts |= set(rng.choice(tstarts[1:], 8, replace=False).tolist())  # at trace boundaries
    c0 = int(rng.integers(1, n - 2))
    cuts |= {c0, c0 + 1}  # a one-record batch
    parts = cut(cols, sorted(cuts))
    with DepsContext(S) as ctx:
        for i, p in enumerate(parts):
            dev = bool(rng.integers(0, 2))
            b = DeviceColumns.from_host(p) if dev else p
            ctx.accumulate(b, clustered=True, verify=bool(rng.integers(0, 2)), continues=i + 1 < len(parts))
            if rng.random() < 0.15:
                ctx.accumulate(SpanColumns.empty(0), clustered=True, continues=True)
        got, st = ctx.finalize(), ctx.stats()
    assert_parity(got, st, ref)
    assert st["not_clustered"] == 0
    assert st["records"] == n


@pytest.mark.parametrize("only", [False, True])
@pytest.mark.parametrize("device", [False, True])
def test_continued_stream_feeds_a_bound_sketch_like_one_batch(gpu, only, device):
    """The carry path with a realtime sketch bound (zk_rt_bind, ZK_RT_WITH_DEPS and ZK_RT_ONLY): the
    held trace's merged spans reach the sketch through the spill kernel (K1 cannot append to the item
    lists there), so a stream cut inside traces must leave the HLL registers, the histogram bins
    and the drop counts exactly as one uncut batch does -- and, with the dependency join, the table
    equal to the oracle."""
    from zipkin_amd.realtime import RtSketch

    S = 61
    cols = tracegen_host(67, 15_000, max_depth=6, num_services=S)
    rng = np.random.default_rng(67)
    parts = cut(cols, rng.choice(np.arange(1, len(cols)), 4, replace=False))

    def run(batches):
        with DepsContext(S, strict=False) as ctx, RtSketch(S) as rt:
            rt.bind(ctx, only=only)
            for i, p in enumerate(batches):
                b = DeviceColumns.from_host(p) if device else p
                ctx.accumulate(b, clustered=True, verify=True, continues=i + 1 < len(batches))
            got = None if only else ctx.finalize()
            st = ctx.stats()
            ctx.sync()
            regs, hist = rt.read()
            return got, st, regs.copy(), hist.copy(), rt.dropped()

    one = run([cols])
    many = run(parts)
    assert np.array_equal(one[2], many[2]), "HLL registers differ"
    assert np.array_equal(one[3], many[3]), "histogram bins differ"
    assert one[4] == many[4]
    assert one[2].any() and one[3].any()
    if not only:
        assert_parity(many[0], many[1], oracle.aggregate(cols, S))
