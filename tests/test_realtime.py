"""Realtime span sketches: per-service distinct traces (HyperLogLog) and duration quantiles.

CPU: the oracle (oracle/realtime.py) -- bin layout, register fields against plain-int arithmetic,
the item definition against the span-level restatement of the reference semantics
(oracle/spans.py: mergeSpan / isValid / serviceName / duration), and the sketch contracts against
exact answers. GPU: the HIP path bit-exact against the oracle (registers, bins, estimates,
quantile bins), fed from merged spans and from span fragments through the bound K1 pass.
"""
import math
import random

import numpy as np
import pytest

from oracle.kv import mix64
from oracle.realtime import (
    SALT,
    RtOracle,
    bin_bounds,
    bins_of,
    exact_distinct,
    exact_quantile,
    hll_estimate,
    hll_fields,
    merged_span_items,
    nbins,
)
from oracle.spans import span_to_record
from tests.richgen import gen_traces
from zipkin_amd import SpanColumns, _abi

COLS = ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags")


def to_columns(spans, ids):
    recs = [span_to_record(s, ids) for s in spans]
    cols = SpanColumns.empty(len(recs))
    for k in COLS:
        getattr(cols, k)[:] = [r[k] for r in recs]
    return cols


# ------------------------------------------------------------------------------ CPU: the oracle
@pytest.mark.parametrize("m", [2, 4, 7, 8])
def test_bins_partition_the_duration_range(m):
    rng = np.random.default_rng(m)
    d = np.concatenate([np.arange(0, 5000), rng.integers(0, 1 << 40, 20000), [(1 << 40) - 1]]).astype(np.uint64)
    b = bins_of(d, m)
    assert b.max() < nbins(m)
    for x, bb in zip(d[::37], b[::37]):
        lo, hi = bin_bounds(int(bb), m)
        assert lo <= int(x) <= hi
        assert hi - lo <= lo >> m  # relative width <= 2^-m
    # consecutive bins tile the integers
    prev = -1
    for bb in range(nbins(m)):
        lo, hi = bin_bounds(bb, m)
        assert lo == prev + 1
        prev = hi
    assert prev == (1 << 40) - 1


def test_hll_fields_match_integer_arithmetic():
    tids = np.array([0, 1, 2, 12345, 2**63, 2**64 - 1] + list(range(100, 200)), dtype=np.uint64)
    for p, seed in ((4, 0), (14, 99), (16, 7)):
        idx, rho = hll_fields(tids, p, seed)
        for t, i, r in zip(tids, idx, rho):
            h = mix64(int(t) ^ seed ^ SALT)
            w = (h << p) & (2**64 - 1)
            assert i == h >> (64 - p)
            assert r == ((64 - w.bit_length() + 1) if w else 64 - p + 1)


def test_hll_estimate_error_bound():
    rng = np.random.default_rng(3)
    p = 12
    sigma = 1.04 / math.sqrt(1 << p)
    for true in (10, 1000, 30000, 200000):
        tids = rng.integers(0, 2**63, true, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
        o = RtOracle(1, p=p, seed=5)
        o.accumulate_merged(np.zeros(true, np.uint32), tids, np.zeros(true, np.int64))
        est = o.distinct()[0]
        assert abs(est - true) <= 4 * sigma * true + 2, (true, est)


def test_quantile_bin_contains_exact_nearest_rank():
    rng = np.random.default_rng(4)
    d = rng.lognormal(9, 1.5, 50000).astype(np.int64)
    o = RtOracle(1, p=4, m=7)
    o.accumulate_merged(np.zeros(len(d), np.uint32), np.arange(len(d), dtype=np.uint64), d)
    qs = [0.0, 0.01, 0.5, 0.9, 0.99, 0.999, 1.0]
    bins, n = o.quantile_bins(0, qs)
    assert n == len(d)
    for q, (lo, hi) in zip(qs, bins):
        x = exact_quantile(d, q)
        assert lo <= x <= hi
        assert abs((lo + hi) / 2 - x) <= x * 2.0 ** -8 + 0.5


def test_items_equal_span_level_semantics():
    """merged_span_items restates Span.mergeSpan/isValid/serviceName/duration on columns."""
    from oracle.spans import Span

    spans = gen_traces(11, 300, max_depth=5, anomalies=0.3)
    ids: dict = {}
    cols = to_columns(spans, ids)
    svc, tid, dur, dropped = merged_span_items(cols, len(ids))
    assert dropped == 0
    merged = {}
    for s in spans:  # reduce(mergeSpan) in input order
        k = (s.id, s.trace_id)
        merged[k] = merged[k].merge_span(s) if k in merged else s
    want = sorted(
        (ids[m.service_name], m.trace_id & (2**64 - 1), m.duration)
        for m in merged.values()
        if m.is_valid and m.service_name is not None and m.duration is not None
    )
    got = sorted(zip(svc.tolist(), tid.tolist(), dur.tolist()))
    assert got == want


@pytest.mark.parametrize("threads", [1, 5])
def test_c_port_equals_the_numpy_oracle(threads):
    """oracle/zk_rt_port.c (C5's large-prefix checker and CPU baseline) against RtOracle over
    merged_span_items: rich spans with anomalies (clustered by traceId) and a TraceGen batch."""
    from oracle.realtime import rt_port
    from zipkin_amd import tracegen_host

    spans = gen_traces(12, 400, max_depth=5, anomalies=0.4)
    ids: dict = {}
    rich = to_columns(spans, ids)
    rich = rich.take(np.argsort(rich.trace_id, kind="stable"))
    for cols, S, p, m in ((rich, len(ids), 10, 5), (tracegen_host(9, 5000, max_depth=6, num_services=57), 57, 14, 7)):
        o = RtOracle(S, p=p, m=m, seed=3)
        svc, tid, dur, dropped = merged_span_items(cols, S)
        o.accumulate_merged(svc, tid, dur)
        r = rt_port(cols, S, p=p, m=m, seed=3, threads=threads)
        assert np.array_equal(r.regs, o.regs) and np.array_equal(r.hist, o.hist)
        assert r.dropped_duration == dropped and r.dropped_service == 0
        assert np.array_equal(r.distinct(), o.distinct())


def test_rt_handle_rejects_bad_config_without_device():
    import ctypes as C

    L = _abi.lib()
    cfg = _abi.zk_rt_config()
    h = C.c_void_p()
    for S, p, m in ((0, 0, 0), (5000, 0, 0), (10, 3, 0), (10, 17, 0), (10, 0, 9), (10, 0, 1)):
        cfg.num_services, cfg.hll_p, cfg.sub_bits = S, p, m
        assert L.zk_rt_create(C.byref(cfg), C.byref(h)) == _abi.ZK_ERR_INVALID_ARG
    assert L.zk_rt_reset(None) == _abi.ZK_ERR_INVALID_ARG
    assert L.zk_rt_bind(None, None, 0) == _abi.ZK_ERR_INVALID_ARG


# ------------------------------------------------------------------------------ GPU: the product
def _assert_same(rt, o):
    regs, hist = rt.read()
    assert np.array_equal(regs, o.regs)
    assert np.array_equal(hist.astype(np.uint64), o.hist)
    est = rt.distinct_traces()
    assert np.array_equal(est, o.distinct())
    for s in range(min(o.S, 6)):
        assert rt.quantiles(s, (0.0, 0.5, 0.99, 1.0)) == o.quantile_bins(s, (0.0, 0.5, 0.99, 1.0))


@pytest.mark.gpu
@pytest.mark.parametrize("S,n,p,m", [(1, 1, 4, 2), (3, 1000, 8, 7), (57, 100_000, 14, 7), (500, 300_000, 12, 6),
                                     (2000, 150_000, 16, 8)])
def test_gpu_merged_input_bit_exact(gpu, S, n, p, m):
    from zipkin_amd.realtime import RtSketch

    rng = np.random.default_rng(n)
    svc = rng.integers(0, S, n, dtype=np.uint32)
    tid = rng.integers(0, n // 3 + 2, n).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    dur = rng.lognormal(8, 2, n).astype(np.int64)
    rt = RtSketch(S, hll_p=p, sub_bits=m, seed=17)
    o = RtOracle(S, p=p, m=m, seed=17)
    half = n // 2
    for a, b in ((0, half), (half, n)):  # two batches: order-independent merge
        rt.accumulate_merged(svc[a:b], tid[a:b], dur[a:b])
        o.accumulate_merged(svc[a:b], tid[a:b], dur[a:b])
    _assert_same(rt, o)
    assert rt.dropped() == (0, 0)


@pytest.mark.gpu
def test_gpu_merged_input_drops_out_of_range(gpu):
    from zipkin_amd.realtime import RtSketch

    rt = RtSketch(4, hll_p=6)
    o = RtOracle(4, p=6)
    svc = np.array([0, 1, 9, 2, 3], np.uint32)
    tid = np.arange(5, dtype=np.uint64)
    dur = np.array([5, -1, 7, 1 << 40, 9], np.int64)
    rt.accumulate_merged(svc, tid, dur)
    o.accumulate_merged(svc, tid, dur)
    assert rt.dropped() == (1, 2) == (o.dropped_service, o.dropped_duration)
    _assert_same(rt, o)


def _bound_run(cols, S, only, batches=None, **kw):
    from zipkin_amd import DepsContext
    from zipkin_amd.realtime import RtSketch

    ctx = DepsContext(S, device=0, strict=False)
    rt = RtSketch(S, **kw)
    rt.bind(ctx, only=only)
    for b in (batches or [cols]):
        ctx.accumulate(b)
    table = None if only else ctx.finalize()
    st = ctx.stats()
    return rt, ctx, table, st


@pytest.mark.gpu
@pytest.mark.parametrize("only", [True, False])
@pytest.mark.parametrize("seed,traces,depth,S", [(1, 5000, 7, 57), (3, 20000, 6, 500)])
def test_gpu_fragments_through_k1_bit_exact(gpu, only, seed, traces, depth, S):
    from oracle import oracle
    from tests.test_gpu_parity import assert_parity
    from zipkin_amd import tracegen_host

    cols = tracegen_host(seed, traces, max_depth=depth, num_services=S)
    rt, ctx, table, st = _bound_run(cols, S, only, hll_p=14, seed=3)
    o = RtOracle(S, p=14, seed=3)
    svc, tid, dur, dropped = merged_span_items(cols, S)
    o.accumulate_merged(svc, tid, dur)
    _assert_same(rt, o)
    assert rt.dropped()[1] == dropped
    ref = oracle.aggregate(cols, S)
    for k in ("records", "merged_spans", "valid_spans", "invalid_spans"):
        assert st[k] == ref.stats[k], k
    if not only:
        assert_parity(table, st, ref)  # the fused pass leaves the dependency path exact


@pytest.mark.gpu
@pytest.mark.parametrize("anomalies,shuffle", [(0.0, False), (0.4, True)])
def test_gpu_rich_spans_and_batches(gpu, anomalies, shuffle):
    spans = gen_traces(41, 500, max_depth=5, anomalies=anomalies)
    if shuffle:
        rng = random.Random(5)
        by = {}
        for s in spans:
            by.setdefault(s.trace_id, []).append(s)
        spans = []
        for ss in by.values():
            rng.shuffle(ss)
            spans += ss
    ids: dict = {}
    cols = to_columns(spans, ids)
    S = len(ids)
    starts = np.flatnonzero(np.r_[True, cols.trace_id[1:] != cols.trace_id[:-1]])
    cut = int(starts[len(starts) // 2])
    parts = [cols.take(slice(0, cut)), cols.take(slice(cut, len(cols)))]
    rt, *_ = _bound_run(cols, S, True, batches=parts, hll_p=10)
    o = RtOracle(S, p=10)
    o.accumulate_merged(*merged_span_items(cols, S)[:3])
    _assert_same(rt, o)


@pytest.mark.gpu
def test_gpu_giant_traces_spill_items(gpu):
    from tests.test_gpu_parity import cols_from_rows, star_trace

    rows = []
    for i, k in enumerate((300, 1500, 5000)):
        rows += star_trace(500 + i, k, svc_root=i % 7)
    cols = cols_from_rows(rows)
    rt, ctx, table, st = _bound_run(cols, 7, False, hll_p=8)
    assert st["spilled_traces"] >= 2
    o = RtOracle(7, p=8)
    o.accumulate_merged(*merged_span_items(cols, 7)[:3])
    _assert_same(rt, o)


@pytest.mark.gpu
def test_gpu_c5_shape_error_bounds(gpu):
    """Distinct traces within 4 sigma and quantile bins holding the exact p50/p99 (C5 shape)."""
    from zipkin_amd import tracegen_host

    S = 500
    cols = tracegen_host(9, 200_000, max_depth=6, num_services=S)
    rt, *_ = _bound_run(cols, S, True)
    svc, tid, dur, _ = merged_span_items(cols, S)
    exact = exact_distinct(svc, tid, S)
    est = rt.distinct_traces()
    sigma = 1.04 / math.sqrt(rt.registers)
    assert np.all(np.abs(est - exact) <= 4 * sigma * exact + 3)
    for s in range(0, S, 50):
        ds = dur[svc == s]
        if len(ds) == 0:
            continue
        (b50, b99), n = rt.quantiles(s, (0.5, 0.99))
        assert n == len(ds)
        for q, (lo, hi) in ((0.5, b50), (0.99, b99)):
            x = exact_quantile(ds, q)
            assert lo <= x <= hi



def test_tdigest_over_histogram_bounds():
    """The t-digest (delta = 200) of a log-normal duration sample: p50 and p99 within the t-digest's
    rank bound of the exact distribution, weights summing to N, centroid count O(delta)."""
    from oracle.realtime import tdigest, tdigest_quantile

    rng = np.random.default_rng(5)
    for n in (50, 5_000, 400_000):
        d = rng.lognormal(9, 1.5, n).astype(np.int64)
        o = RtOracle(1, p=4, m=7)
        o.accumulate_merged(np.zeros(n, np.uint32), np.arange(n, dtype=np.uint64), d)
        cent, vmin, vmax, N = tdigest(o.hist[0], 7, 200.0)
        assert N == n and abs(sum(w for _, w in cent) - n) < 1e-6
        assert len(cent) <= 400
        ds = np.sort(d)
        for q in (0.5, 0.99):
            est = tdigest_quantile(cent, vmin, vmax, N, q)
            assert d.min() <= est <= d.max()
            # the t-digest's accuracy is a rank bound: the estimate's rank is within the quantile
            # span of a k1 centroid there (pi sqrt(q (1 - q)) / delta, doubled) plus the histogram
            # bin (2^-7 relative: a few ranks), plus 2 / n
            rank = np.searchsorted(ds, est, side="right") / n
            assert abs(rank - q) <= 2 * math.pi * math.sqrt(q * (1 - q)) / 200 + 2 / n + 0.002, (n, q, rank)


@pytest.mark.gpu
def test_gpu_tdigest_equals_oracle(gpu):
    """zk_rt_tdigest on the device sketch == the oracle's digest of the same histogram (centroids
    and estimates bit for bit), and within the t-digest's rank bound at C5 shape."""
    from oracle.realtime import tdigest, tdigest_quantile
    from zipkin_amd import tracegen_host

    S = 500
    cols = tracegen_host(9, 200_000, max_depth=6, num_services=S)
    rt, *_ = _bound_run(cols, S, True)
    _, hist = rt.read()
    svc, tid, dur, _ = merged_span_items(cols, S)
    for s in range(0, S, 50):
        mean, weight, est, n = rt.tdigest(s, 200.0, (0.5, 0.99))
        cent, vmin, vmax, N = tdigest(hist[s], rt.m, 200.0)
        assert n == N and len(cent) == len(mean)
        assert np.array_equal(mean, np.array([c[0] for c in cent])) and np.array_equal(weight, np.array([c[1] for c in cent]))
        for q, e in zip((0.5, 0.99), est):
            assert e == tdigest_quantile(cent, vmin, vmax, N, q)
            ds = np.sort(dur[svc == s])
            if len(ds) >= 1000:
                rank = np.searchsorted(ds, e, side="right") / len(ds)
                assert abs(rank - q) <= 2 * math.pi * math.sqrt(q * (1 - q)) / 200 + 2 / len(ds) + 0.002, (s, q, rank)
