"""Parity of the HIP dependency path (libzkagg, through the C ABI) with the CPU oracle.

Bar: link counts (m0) AND m1..m4 bit-identical to the oracle's exactly-rounded Moments (the
oracle is within 1e-9 of the reference's Algebird fold, tests/test_oracle_cross.py), and every
device counter equal to the oracle's."""
import numpy as np
import pytest

from oracle import oracle
from oracle.moments import algebird_fold, moments_close
from oracle.spans import aggregate_job, span_to_record
from tests.richgen import gen_traces
from zipkin_amd import DepsContext, DeviceColumns, SpanColumns, ZkError, _abi, tracegen_host, tracegen_params

pytestmark = pytest.mark.gpu

COLS = ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags")
SERVER = _abi.ZK_F_HAS_ANNOTATIONS | _abi.ZK_F_SVC_SERVER | (1 << _abi.ZK_F_SR_SHIFT) | (1 << _abi.ZK_F_SS_SHIFT)
CLIENT = _abi.ZK_F_HAS_ANNOTATIONS | _abi.ZK_F_SVC_CLIENT | (1 << _abi.ZK_F_CS_SHIFT) | (1 << _abi.ZK_F_CR_SHIFT)


def run_gpu(cols, S, batches=None, device_cols=False, clustered=True, **kw):
    """The clustered fast path (K1 straight on the input) with the exact clustering check on;
    tests/test_gpu_order.py covers unclustered batches."""
    with DepsContext(S, **kw) as ctx:
        parts = batches or [cols]
        for p in parts:
            ctx.accumulate(DeviceColumns.from_host(p) if device_cols else p, clustered=clustered)
        got = ctx.finalize()
        return got, ctx.stats()


def assert_parity(got, st, ref):
    m0, ms = ref.dense()
    assert np.array_equal(got.m0, m0), "m0 (link counts) differ"
    for a, b, name in zip((got.m1, got.m2, got.m3, got.m4), ms, ("m1", "m2", "m3", "m4")):
        bad = np.flatnonzero(a != b)
        assert bad.size == 0, f"{name} differs in {bad.size} cells, first {bad[:3]}: {a[bad[:3]]} vs {b[bad[:3]]}"
    assert np.array_equal(got.present, (m0 > 0).astype(np.uint8))
    for k, v in ref.stats.items():
        if k == "spilled_traces":  # a GPU scheduling detail (tile overflow), not a job quantity
            continue
        assert st[k] == v, f"stat {k}: gpu {st[k]} != oracle {v}"


def star_trace(tid, n_children, svc_root=0, nsvc=7, t0=1_000_000, fragments=2):
    """root + n_children direct calls, each as client+server fragments (or server only)."""
    rows = [(tid, tid ^ 0xABCDEF, 0, t0, t0 + 10_000_000, svc_root, SERVER)]
    for i in range(n_children):
        sid = (tid * 1_000_003 + i * 7919 + 1) & (2**64 - 1)
        svc = 1 + (i % (nsvc - 1))
        cs = t0 + 10 + i
        rows.append((tid, sid, tid ^ 0xABCDEF, cs + 5, cs + 100 + (i % 97), svc, SERVER | 1))
        if fragments == 2:
            rows.append((tid, sid, tid ^ 0xABCDEF, cs, cs + 200 + (i % 89), svc, CLIENT | 1))
    return rows


def cols_from_rows(rows):
    c = SpanColumns.empty(len(rows))
    if rows:
        arr = list(zip(*rows))
        for k, v in zip(COLS, arr):
            getattr(c, k)[:] = np.array(v, dtype=np.uint64 if k in ("trace_id", "span_id", "parent_id") else getattr(c, k).dtype)
    return c


# ---------------------------------------------------------------------------------------------
def test_tracegen_device_equals_host(gpu):
    import torch

    for seed, T, depth, S, rank, world in [(1, 3000, 7, 57, 0, 1), (2, 5000, 6, 500, 2, 4)]:
        host = tracegen_host(seed, T, max_depth=depth, num_services=S, rank=rank, world=world)
        p = tracegen_params(seed, T, max_depth=depth, num_services=S, rank=rank, world=world)
        with DepsContext(S) as ctx:
            dev = DeviceColumns(len(host) + 1000)
            n, ntr = ctx.tracegen_device(p, dev)
            torch.cuda.synchronize()
        assert (n, ntr) == (len(host), T)
        back = dev.to_host()
        for k in COLS:
            assert np.array_equal(getattr(back, k), getattr(host, k)), k


@pytest.mark.parametrize(
    "seed,traces,depth,S",
    [(1, 10000, 7, 57), (2, 3000, 7, 20), (3, 20000, 6, 500), (4, 200000, 6, 500), (5, 50000, 3, 1),
     (6, 30000, 6, 1000), (7, 20000, 6, 1500)],
)
def test_parity_tracegen(gpu, seed, traces, depth, S):
    cols = tracegen_host(seed, traces, max_depth=depth, num_services=S)
    got, st = run_gpu(cols, S)
    assert_parity(got, st, oracle.aggregate(cols, S))
    assert st["records"] == len(cols)


def test_device_pointers_and_batches_agree(gpu):
    S = 57
    cols = tracegen_host(21, 20000, max_depth=7, num_services=S)
    ref = oracle.aggregate(cols, S)
    got, st = run_gpu(cols, S, device_cols=True)
    assert_parity(got, st, ref)
    # split into trace-complete batches at arbitrary trace boundaries: the monoid makes it exact
    starts = np.flatnonzero(np.r_[True, cols.trace_id[1:] != cols.trace_id[:-1]])
    cuts = sorted(np.random.default_rng(0).choice(starts[1:], 5, replace=False))
    bounds = [0, *cuts, len(cols)]
    parts = [cols.take(slice(a, b)) for a, b in zip(bounds[:-1], bounds[1:])]
    got2, st2 = run_gpu(cols, S, batches=parts)
    assert_parity(got2, st2, ref)


def test_repeatable_bit_identical(gpu):
    cols = tracegen_host(8, 30000, max_depth=7, num_services=100)
    a, _ = run_gpu(cols, 100)
    b, _ = run_gpu(cols, 100)
    for k in ("m0", "m1", "m2", "m3", "m4"):
        assert np.array_equal(getattr(a, k), getattr(b, k))


@pytest.mark.parametrize("sizes", [[1023, 1024, 1025], [2047, 2048, 2049, 2050], [3000, 10, 5000, 1], [50000, 3, 70000]])
def test_giant_traces_spill_path(gpu, sizes):
    rows = []
    rng = np.random.default_rng(sum(sizes))
    for i, n_children in enumerate(sizes):
        rows += star_trace(1000 + i, (n_children - 1) // 2, svc_root=i % 7)
        # interleave ordinary traces so giant ones straddle many tiles
        small = tracegen_host(int(rng.integers(1, 1e6)), 20, max_depth=4, num_services=7)
        rows += list(zip(*[getattr(small, k).tolist() for k in COLS]))
    cols = cols_from_rows(rows)
    got, st = run_gpu(cols, 7)
    ref = oracle.aggregate(cols, 7)
    assert_parity(got, st, ref)
    assert st["spilled_traces"] >= sum(1 for s in sizes if s > 2048)


def test_random_trace_lengths_tile_boundaries(gpu):
    rng = np.random.default_rng(123)
    rows = []
    tid = 1
    while len(rows) < 200_000:
        n = int(rng.choice([1, 2, 3, 50, 700, 1500, 2100, 4000]))
        frag = 2 if rng.random() < 0.8 else 1
        rows += star_trace(tid, max(0, (n - 1) // frag), svc_root=int(rng.integers(0, 9)), nsvc=9, fragments=frag)
        tid += 1
    cols = cols_from_rows(rows)
    got, st = run_gpu(cols, 9)
    assert_parity(got, st, oracle.aggregate(cols, 9))


@pytest.mark.parametrize("seed,anomalies,shuffle_within", [(31, 0.0, False), (32, 0.4, False), (33, 0.4, True)])
def test_rich_span_parity_with_reference_semantics(gpu, seed, anomalies, shuffle_within):
    spans = gen_traces(seed, 400, max_depth=5, anomalies=anomalies)
    if shuffle_within:  # storage order inside a trace is arbitrary; traces stay clustered
        rng = np.random.default_rng(seed)
        by = {}
        for s in spans:
            by.setdefault(s.trace_id, []).append(s)
        spans = []
        for tid, ss in by.items():
            rng.shuffle(ss)
            spans += ss
    ids: dict = {}
    recs = [span_to_record(s, ids) for s in spans]
    cols = SpanColumns.empty(len(recs))
    for k in COLS:
        getattr(cols, k)[:] = [r[k] for r in recs]
    names = {v: k for k, v in ids.items()}
    S = len(ids)
    got, st = run_gpu(cols, S, strict=False)
    ref = aggregate_job(spans, strict=False)
    assert st["no_service"] == ref.no_service and st["ambiguous"] == 0
    gl = {(names[p], names[c]): m for p, c, m in got.links()}
    want = ref.exact()
    assert set(gl) == set(want)
    for k, m in want.items():
        assert tuple(gl[k]) == tuple(m), k
        assert moments_close(algebird_fold(float(d) for d in ref.durations[k]), type(m)(*gl[k])), k


def test_strict_no_service_is_an_error_lenient_counts(gpu):
    rows = [(7, 70, 0, 1, 9, 0, SERVER), (7, 71, 70, 2, 4, 0, _abi.ZK_F_HAS_ANNOTATIONS | 1 | (1 << 12) | (1 << 14))]
    cols = cols_from_rows(rows)
    with DepsContext(3, strict=True) as ctx:
        ctx.accumulate(cols)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_NO_SERVICE
    got, st = run_gpu(cols, 3, strict=False)
    assert st["no_service"] == 1 and got.present.sum() == 0


def test_service_and_duration_range_errors(gpu):
    bad_svc = cols_from_rows([(1, 10, 0, 1, 9, 5, SERVER), (1, 11, 10, 2, 4, 1, SERVER | 1)])
    with DepsContext(3) as ctx:
        ctx.accumulate(bad_svc)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_SERVICE_RANGE
    long_span = cols_from_rows([(2, 20, 0, 1, 2**41, 0, SERVER), (2, 21, 20, 5, 5 + 2**40, 1, SERVER | 1),
                                (2, 22, 20, 5, 5 + 2**40 - 1, 2, SERVER | 1)])
    with DepsContext(3) as ctx:
        ctx.accumulate(long_span)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_DURATION_RANGE
        st = ctx.stats()
    assert st["duration_range"] == 1
    # the largest supported duration (2^40 - 1 us) is still exact
    got, _ = run_gpu(cols_from_rows([(2, 20, 0, 1, 2**41, 0, SERVER), (2, 22, 20, 5, 5 + 2**40 - 1, 2, SERVER | 1)]), 3)
    assert got.m0[0 * 3 + 2] == 1 and got.m1[2] == float(2**40 - 1)


def test_empty_single_and_unclustered(gpu):
    got, st = run_gpu(SpanColumns.empty(0), 5)
    assert got.present.sum() == 0 and st["records"] == 0
    got, st = run_gpu(cols_from_rows([(1, 1, 0, 5, 9, 0, SERVER)]), 5)
    assert got.present.sum() == 0 and st["merged_spans"] == 1
    # without the clustered promise the batch goes through the device clustering pass
    got, st = run_gpu(cols_from_rows([(1, 1, 0, 5, 9, 0, SERVER)]), 5, clustered=False)
    assert got.present.sum() == 0 and st["merged_spans"] == 1


M32 = 0xFFFFFFFF


def sid_key(sid):
    """A 32-bit fold of a span id (low word ^ high word * golden ratio)."""
    return ((sid & M32) ^ (((sid >> 32) * 0x9E3779B1) & M32)) & M32


def colliding(sid, hi):
    """A different span id with high word `hi` and the same 32-bit key as `sid`."""
    lo = ((sid & M32) ^ (((sid >> 32) * 0x9E3779B1) & M32) ^ ((hi * 0x9E3779B1) & M32)) & M32
    out = (hi << 32) | lo
    assert out != sid and sid_key(out) == sid_key(sid)
    return out


def collision_trace(tid, rng, nsvc=9):
    """A trace whose span ids agree in a 32-bit fold: sibling spans A and B, a grandchild under B,
    and a child whose absent parent folds like the root. Any key or hash narrower than the full
    64-bit span id would merge or join them wrongly."""
    t0 = 1_000_000 + tid
    root = int(rng.integers(1, 2**63))
    a = int(rng.integers(1, 2**63))
    b = colliding(a, int(rng.integers(1, 2**31)))
    c = int(rng.integers(1, 2**63))
    ghost = colliding(root, int(rng.integers(1, 2**31)))  # never stored
    d = int(rng.integers(1, 2**63))
    sv = lambda: int(rng.integers(0, nsvc))
    rows = [(tid, root, 0, t0, t0 + 900, sv(), SERVER)]
    for sid, par, dt in ((a, root, 10), (b, root, 20), (c, b, 30), (d, ghost, 40)):
        s1 = sv()
        rows.append((tid, sid, par, t0 + dt + 5, t0 + dt + 50, s1, SERVER | 1))
        rows.append((tid, sid, par, t0 + dt, t0 + dt + 60 + (tid % 7), s1, CLIENT | 1))
    order = rng.permutation(len(rows))
    return [rows[i] for i in order]


def test_span_id_key_collisions_are_exact(gpu):
    rng = np.random.default_rng(77)
    rows = []
    for t in range(3000):
        if t % 10 == 3:
            rows += collision_trace(10_000 + t, rng)
        else:
            rows += star_trace(10_000 + t, int(rng.integers(0, 40)), svc_root=int(rng.integers(0, 9)), nsvc=9)
    cols = cols_from_rows(rows)
    got, st = run_gpu(cols, 9)
    assert_parity(got, st, oracle.aggregate(cols, 9))


def test_trace_too_large(gpu):
    cols = cols_from_rows(star_trace(5, 4000))
    with DepsContext(7, max_trace_records=5000) as ctx:
        ctx.accumulate(cols)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_TRACE_TOO_LARGE


def test_large_device_generated_batch(gpu):
    """1e7 device-generated records (the bench's generator) against the oracle on the same data."""
    S = 500
    p = tracegen_params(2, 600_000, target_records=10_000_000, max_depth=6, num_services=S)
    with DepsContext(S) as ctx:
        dev = DeviceColumns(10_000_000)
        n, ntr = ctx.tracegen_device(p, dev)
        ctx.accumulate(dev)
        got = ctx.finalize()
        st = ctx.stats()
    host = dev.to_host()
    assert len(host) == n and n > 9_000_000
    assert_parity(got, st, oracle.aggregate(host, S))


def test_full_size_c2_batch(gpu):
    """The bench's own C2 batch (BASELINE configs[1]: 1e8 records, 500 services, seed 2, maxDepth 6,
    generated on the device exactly as bench.py does) against the oracle at full size."""
    import os

    S = 500
    p = tracegen_params(2, int(1e8 / 15) + 1000, target_records=100_000_000, max_depth=6, num_services=S)
    with DepsContext(S) as ctx:
        dev = DeviceColumns(100_000_000)
        n, ntr = ctx.tracegen_device(p, dev)
        ctx.accumulate(dev, clustered=True, verify=True)
        got = ctx.finalize()
        st = ctx.stats()
    host = dev.to_host()
    del dev
    assert n == len(host) and n > 99_000_000
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    assert_parity(got, st, oracle.aggregate(host, S, threads=threads))
    assert st["not_clustered"] == 0
