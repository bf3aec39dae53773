"""Order-agnostic input and the clustering check, through the C ABI on the GPU.

The reference accepts fragments in any order: Scalding shuffles by (id, traceId) before the merge
and by (parentId, traceId) before the join (ZipkinAggregateJob.scala:21-22,28-33). Batches without
the clustered promise go through the device clustering pass and must give the oracle's result for
every permutation (the oracle makes no clustering assumption). With ZK_BATCH_VERIFY_TRACES a trace
split into non-adjacent runs -- inside a batch or across two accumulate calls -- is an error, never
a silent mis-join."""
import numpy as np
import pytest

from oracle import oracle
from tests.test_gpu_parity import assert_parity, cols_from_rows, star_trace
from zipkin_amd import DepsContext, DeviceColumns, SpanColumns, ZkError, _abi, tracegen_host

pytestmark = pytest.mark.gpu


def run(batches, S, trace_pass=False, **acc):
    """verify (default True) keeps the clustering pass's P3 + K1; verify=False on batches of more
    than 2^18 records takes the group join (k_group_join) and its fallback, unless trace_pass
    (zk_config.trace_pass) forces P3 + K1."""
    with DepsContext(S, trace_pass=trace_pass) as ctx:
        for b in batches:
            ctx.accumulate(b, **acc)
        return ctx.finalize(), ctx.stats()


@pytest.mark.parametrize("verify", [True, False])
@pytest.mark.parametrize("seed,traces,S", [(51, 20_000, 57), (52, 100_000, 500)])
def test_any_permutation_equals_the_oracle(gpu, seed, traces, S, verify):
    cols = tracegen_host(seed, traces, max_depth=6, num_services=S)
    ref = oracle.aggregate(cols, S)
    perm = np.random.default_rng(seed).permutation(len(cols))
    shuffled = cols.take(perm)
    for batch in (shuffled, DeviceColumns.from_host(shuffled)):
        got, st = run([batch], S, verify=verify)
        assert_parity(got, st, ref)
        assert st["not_clustered"] == 0


def test_reversed_and_interleaved_traces(gpu):
    rows = []
    for t in range(300):
        rows += star_trace(5000 + t, t % 40, svc_root=t % 7, nsvc=7)
    cols = cols_from_rows(rows)
    ref = oracle.aggregate(cols, 7)
    for order in (np.arange(len(cols))[::-1], np.argsort(np.arange(len(cols)) % 3, kind="stable")):
        got, st = run([cols.take(order.copy())], 7)
        assert_parity(got, st, ref)


def test_trace_complete_batches_in_any_order(gpu):
    S = 57
    cols = tracegen_host(53, 20_000, max_depth=7, num_services=S)
    ref = oracle.aggregate(cols, S)
    tids = np.unique(cols.trace_id)
    groups = np.random.default_rng(3).integers(0, 4, len(tids))
    which = groups[np.searchsorted(tids, cols.trace_id)]
    parts = [cols.take(np.flatnonzero(which == g)[::-1].copy()) for g in range(4)]
    got, st = run(parts, S)
    assert_parity(got, st, ref)


def two_interleaved_traces():
    a, b = star_trace(1, 3, svc_root=0, nsvc=5), star_trace(2, 3, svc_root=1, nsvc=5)
    return cols_from_rows(a[:3] + b + a[3:])  # trace 1 | trace 2 | trace 1 again


def test_broken_promise_is_detected(gpu):
    cols = two_interleaved_traces()
    with DepsContext(5) as ctx:
        ctx.accumulate(cols, clustered=True, verify=True)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_NOT_CLUSTERED
        assert ctx.stats()["not_clustered"] == 1
    # without the promise the same batch is clustered on the device and exact
    got, st = run([cols], 5)
    assert_parity(got, st, oracle.aggregate(cols, 5))


def test_trace_split_over_two_batches_is_detected(gpu):
    rows = star_trace(9, 6, nsvc=5)
    first, second = cols_from_rows(rows[:5]), cols_from_rows(rows[5:])
    for clustered in (True, False):
        with DepsContext(5) as ctx:
            ctx.accumulate(first, clustered=clustered)
            ctx.accumulate(second, clustered=clustered)
            with pytest.raises(ZkError) as e:
                ctx.finalize()
            assert e.value.status == _abi.ZK_ERR_NOT_CLUSTERED
            # reset clears the set: the whole trace in one batch is fine
            ctx.reset()
            ctx.accumulate(cols_from_rows(rows), clustered=clustered)
            ctx.finalize()


def test_trace_id_zero_and_all_ones(gpu):
    rows = star_trace(0, 4, nsvc=5) + star_trace(2**64 - 1, 4, nsvc=5)
    cols = cols_from_rows(rows)
    got, st = run([cols], 5)
    assert_parity(got, st, oracle.aggregate(cols, 5))
    split0 = cols_from_rows(rows[:2] + rows[-3:] + rows[2:-3])  # trace 0 split around the other
    with DepsContext(5) as ctx:
        ctx.accumulate(split0, clustered=True)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_NOT_CLUSTERED


def test_verify_set_grows_over_many_batches(gpu):
    """The device traceId set is resized (rehash) as batches arrive; no false alarms."""
    S = 57
    cols = tracegen_host(54, 60_000, max_depth=7, num_services=S)
    starts = np.flatnonzero(np.r_[True, cols.trace_id[1:] != cols.trace_id[:-1]])
    cuts = list(starts[:: max(1, len(starts) // 40)][1:]) + [len(cols)]
    parts, lo = [], 0
    for hi in cuts:
        parts.append(cols.take(slice(lo, hi)))
        lo = hi
    got, st = run(parts, S, clustered=True, verify=True)
    assert_parity(got, st, oracle.aggregate(cols, S))
    assert st["not_clustered"] == 0


def test_empty_batches(gpu):
    got, st = run([SpanColumns.empty(0), SpanColumns.empty(0)], 5)
    assert got.present.sum() == 0 and st["records"] == 0


# ---- the hand-written clustering pass (zk_cluster.hip): every plan shape and its edge cases ----
M64 = (1 << 64) - 1
PART_SALT = 0xC2B2AE3D27D4EB4F  # zk_cluster.hip kPartSalt


def unmix64(z):
    """Inverse of zk_mix64 (zk_tracegen.h): lets a test pick a traceId's partition hash."""
    z = (z ^ (z >> 31) ^ (z >> 62)) & M64
    z = (z * 0x319642B2D24D8EC3) & M64
    z = (z ^ (z >> 27) ^ (z >> 54)) & M64
    z = (z * 0x96DE1B173F119089) & M64
    return (z ^ (z >> 30) ^ (z >> 60)) & M64


@pytest.mark.parametrize("verify", [True, False])
@pytest.mark.parametrize("traces,depth", [(150, 4), (1_500, 5), (6_000, 5), (40_000, 6)])
def test_plan_shapes(gpu, traces, depth, verify):
    """P3 alone (<= 4096 records), P1 + P3 (<= 2048 x 256 records), and P1 + P2 + P3, host and
    device pointers; without verification the largest shape takes the group join."""
    S = 97
    cols = tracegen_host(55 + traces, traces, max_depth=depth, num_services=S)
    ref = oracle.aggregate(cols, S)
    perm = np.random.default_rng(traces).permutation(len(cols))
    for batch in (cols.take(perm), DeviceColumns.from_host(cols.take(perm))):
        got, st = run([batch], S, verify=verify)
        assert_parity(got, st, ref)
        assert st["not_clustered"] == 0


def test_giant_trace_in_a_shuffled_batch(gpu):
    """One trace of 60k records among ordinary ones: its sub-bucket is done in rounds, and K1's
    spill kernel then joins it (longer than a window)."""
    S = 7
    rows = star_trace(777, 30_000, nsvc=S)
    for t in range(2_000):
        rows += star_trace(10_000 + t, 1 + t % 9, svc_root=t % S, nsvc=S)
    cols = cols_from_rows(rows)
    ref = oracle.aggregate(cols, S)
    got, st = run([cols.take(np.random.default_rng(5).permutation(len(cols)))], S)
    assert_parity(got, st, ref)
    assert st["spilled_traces"] >= 1


def test_singleton_traces_and_extreme_trace_ids(gpu):
    """300k single-span traces (as many distinct traceIds as records), plus traces 0 and 2^64-1
    (the trace table's empty-key marker takes its own slot) with many records."""
    S = 11
    rng = np.random.default_rng(8)
    n = 300_000
    c = SpanColumns.empty(n)
    c.trace_id[:] = rng.integers(2, 2**64 - 2, n, dtype=np.uint64)
    c.span_id[:] = rng.integers(1, 2**63, n, dtype=np.uint64)
    c.first_ts[:] = 1_000
    c.last_ts[:] = 1_000 + rng.integers(0, 5000, n)
    c.service_id[:] = rng.integers(0, S, n, dtype=np.uint32)
    from tests.test_gpu_parity import SERVER

    c.flags[:] = SERVER
    extra = cols_from_rows(star_trace(0, 3000, nsvc=S) + star_trace(M64, 2500, nsvc=S))
    cols = SpanColumns.concat([c, extra])
    ref = oracle.aggregate(cols, S)
    got, st = run([cols.take(rng.permutation(len(cols)))], S)
    assert_parity(got, st, ref)


def test_every_trace_in_one_sub_bucket(gpu):
    """Adversarial traceIds: all share the top 24 bits of the partition hash, so every first- and
    second-level digit is the same and one sub-bucket holds the whole batch (many rounds of the
    trace table, with restarts when a round's hash range overfills it)."""
    S = 13
    rows = []
    for t in range(12_000):
        tid = unmix64(((0xABCDEF << 40) | (t * 2654435761 & ((1 << 40) - 1))) & M64) ^ PART_SALT
        rows += star_trace(tid, 1 + t % 5, svc_root=t % S, nsvc=S)
    cols = cols_from_rows(rows)
    assert len(cols) > 65_536  # the partition runs (P1 + P2), not P3 alone
    ref = oracle.aggregate(cols, S)
    got, st = run([cols.take(np.random.default_rng(9).permutation(len(cols)))], S)
    assert_parity(got, st, ref)


TRACE_SALT = 0x165667B19E3779F9  # zk_cluster.hip kTraceSalt


def test_trace_hash_collisions_fail_with_capacity(gpu):
    """Crafted traceIds whose trace hash shares bits 40..63 (the bits the trace pass splits its
    rounds on) overfill the LDS table at every doubling: the pass gives the sub-bucket up after a
    bounded number of restarts and finalize reports ZK_ERR_CAPACITY, instead of sweeping 2^24 rounds.
    Honest traceIds of the same batch shape are exact."""
    S = 5
    n = 4096  # P3 alone: one sub-bucket of 4096 singleton traces, more than the table's 2048 slots
    c = SpanColumns.empty(n)
    c.trace_id[:] = [unmix64(t + 1) ^ TRACE_SALT for t in range(n)]  # trace hash = t + 1 < 2^40
    c.span_id[:] = np.arange(1, n + 1, dtype=np.uint64)
    c.first_ts[:] = 1_000
    c.last_ts[:] = 2_000
    from tests.test_gpu_parity import SERVER

    c.flags[:] = SERVER
    with DepsContext(S) as ctx:
        ctx.accumulate(c.take(np.random.default_rng(3).permutation(n)), verify=False)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_CAPACITY
    c.trace_id[:] = np.random.default_rng(4).integers(1, 2**63, n, dtype=np.uint64)
    got, st = run([c], S)
    assert_parity(got, st, oracle.aggregate(c, S))


@pytest.mark.parametrize("verify", [True, False])
def test_shuffled_c2_shape_at_scale(gpu, verify):
    """2e7 device-generated TraceGen records (the bench's shape), shuffled on the device: the result
    equals the clustered batch's bit for bit (m0..m4 and every counter); verify=False: through the
    group join."""
    import torch

    from zipkin_amd import tracegen_params

    S, N = 500, 20_000_000
    with DepsContext(S) as g:
        cols = DeviceColumns(N)
        n, _ = g.tracegen_device(tracegen_params(2, N // 15 + 1000, target_records=N, max_depth=6, num_services=S),
                                 cols)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(11)
    perm = torch.randperm(n, device="cuda", generator=gen)
    sc = DeviceColumns(n)
    for k in ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags"):
        torch.index_select(getattr(cols, k)[:n], 0, perm, out=getattr(sc, k))
    torch.cuda.synchronize()  # the contexts below run on their own streams
    with DepsContext(S) as a:
        a.accumulate(cols, clustered=True, verify=True, n=n)
        ra, sa = a.finalize(), a.stats()
    with DepsContext(S) as b:
        b.accumulate(sc, clustered=False, verify=verify)
        rb, sb = b.finalize(), b.stats()
    for k in ("m0", "m1", "m2", "m3", "m4", "present"):
        assert np.array_equal(getattr(ra, k), getattr(rb, k)), k
    for k in sa:
        if k != "spilled_traces":
            assert sa[k] == sb[k], k


def test_group_join_fallback(gpu):
    """The group join's fallback: a 60k-record trace (spilled by K1), a 3k-record trace, and 900
    crafted traces sharing their partition-hash digits (one ~4.5k-record sub-bucket) are longer than
    the group join's LDS capacity; P3 clusters just those sub-buckets and K1 appends their links to
    the group join's lists. Everything else (~300k records) is joined by the group join."""
    S = 11
    rows = star_trace(777, 30_000, nsvc=S) + star_trace(778, 1_500, nsvc=S)
    for t in range(900):
        tid = unmix64(((0x5A5A5A << 40) | (t * 2654435761 & ((1 << 40) - 1))) & M64) ^ PART_SALT
        rows += star_trace(tid, 1 + t % 4, svc_root=t % S, nsvc=S)
    for t in range(30_000):
        rows += star_trace(100_000 + t, t % 9, svc_root=t % S, nsvc=S, fragments=1 + t % 2)
    cols = cols_from_rows(rows)
    assert len(cols) > 2 ** 18
    ref = oracle.aggregate(cols, S)
    shuffled = cols.take(np.random.default_rng(12).permutation(len(cols)))
    for batch in (shuffled, DeviceColumns.from_host(shuffled)):
        got, st = run([batch], S, verify=False)
        assert_parity(got, st, ref)
        assert st["spilled_traces"] >= 1


def test_group_join_equals_the_trace_path(gpu):
    """The same shuffled batch through the group join and through P3 + K1 (zk_config.trace_pass):
    identical tables and counters."""
    S = 200
    cols = tracegen_host(61, 60_000, max_depth=6, num_services=S)
    shuffled = cols.take(np.random.default_rng(61).permutation(len(cols)))
    got, st = run([shuffled], S, verify=False)
    ref, sr = run([shuffled], S, verify=False, trace_pass=True)
    for k in ("m0", "m1", "m2", "m3", "m4", "present"):
        assert np.array_equal(getattr(got, k), getattr(ref, k)), k
    for k in st:
        if k != "spilled_traces":
            assert st[k] == sr[k], k


def test_group_join_rich_spans_with_anomalies(gpu):
    """Rich spans with the injected anomalies of tests/richgen.py (missing and invalid parents,
    duplicated core annotations, disagreeing fragments, client-only and nameless services), in 40
    copies with distinct traceIds (> 2^18 records), shuffled: the group join equals the oracle and
    the P3 + K1 path, every counter included."""
    from tests.richgen import gen_traces
    from tests.test_gpu_parity import COLS
    from oracle.spans import span_to_record

    spans = gen_traces(34, 600, max_depth=5, anomalies=0.4)
    ids: dict = {}
    recs = [span_to_record(s, ids) for s in spans]
    one = SpanColumns.empty(len(recs))
    for k in COLS:
        getattr(one, k)[:] = [r[k] for r in recs]
    copies = []
    for c in range(40):
        x = one.take(np.arange(len(one)))
        x.trace_id[:] = x.trace_id ^ np.uint64((c * 0x9E3779B97F4A7C15) & (2**64 - 1))
        copies.append(x)
    cols = SpanColumns.concat(copies)
    assert len(cols) > 2 ** 18
    S = len(ids)
    ref = oracle.aggregate(cols, S)
    shuffled = cols.take(np.random.default_rng(34).permutation(len(cols)))
    with DepsContext(S, strict=False) as ctx:
        ctx.accumulate(shuffled, verify=False)
        got, st = ctx.finalize(), ctx.stats()
    assert_parity(got, st, ref)
    with DepsContext(S, strict=False, trace_pass=True) as ctx:
        ctx.accumulate(shuffled, verify=False)
        got2, st2 = ctx.finalize(), ctx.stats()
    for k in ("m0", "m1", "m2", "m3", "m4", "present"):
        assert np.array_equal(getattr(got, k), getattr(got2, k)), k
    assert {k: v for k, v in st.items() if k != "spilled_traces"} == {k: v for k, v in st2.items() if k != "spilled_traces"}


def test_group_join_over_several_trace_complete_batches(gpu):
    """Two shuffled trace-complete batches of > 2^18 records each through the group join (its
    long-sub-bucket list, fallback cursor and per-CU link lists restart per batch): the oracle's
    result for the union."""
    S = 61
    cols = tracegen_host(81, 50_000, max_depth=6, num_services=S)
    tids = np.unique(cols.trace_id)
    which = np.random.default_rng(81).integers(0, 2, len(tids))[np.searchsorted(tids, cols.trace_id)]
    parts = []
    for g in range(2):
        idx = np.flatnonzero(which == g)
        parts.append(cols.take(idx[np.random.default_rng(g).permutation(len(idx))]))
    assert all(len(p) > 2 ** 18 for p in parts)
    got, st = run(parts, S, verify=False)
    assert_parity(got, st, oracle.aggregate(cols, S))


def test_group_join_respects_max_trace_records(gpu):
    """max_trace_records below the group join's LDS tile: a 1500-record trace in a shuffled batch
    of > 2^18 records without verification is too large exactly as on the clustered path (the
    library then takes P3 + K1, which enforces the bound)."""
    S = 31
    rows = star_trace(4242, 749, nsvc=S)  # 1 + 2 x 749 = 1499 records
    cols = SpanColumns.concat([cols_from_rows(rows), tracegen_host(83, 12_000, max_depth=6, num_services=S)])
    assert len(cols) > 2 ** 18
    shuffled = cols.take(np.random.default_rng(83).permutation(len(cols)))
    for batch, clustered in ((shuffled, False), (cols, True)):
        with DepsContext(S, max_trace_records=1000) as ctx:
            ctx.accumulate(batch, clustered=clustered, verify=False)
            with pytest.raises(ZkError) as e:
                ctx.finalize()
            assert e.value.status == _abi.ZK_ERR_TRACE_TOO_LARGE
            assert ctx.stats()["trace_too_large"] == 1
