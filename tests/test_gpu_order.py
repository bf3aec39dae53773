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


def run(batches, S, **acc):
    with DepsContext(S) as ctx:
        for b in batches:
            ctx.accumulate(b, **acc)
        return ctx.finalize(), ctx.stats()


@pytest.mark.parametrize("seed,traces,S", [(51, 20_000, 57), (52, 100_000, 500)])
def test_any_permutation_equals_the_oracle(gpu, seed, traces, S):
    cols = tracegen_host(seed, traces, max_depth=6, num_services=S)
    ref = oracle.aggregate(cols, S)
    perm = np.random.default_rng(seed).permutation(len(cols))
    shuffled = cols.take(perm)
    for batch in (shuffled, DeviceColumns.from_host(shuffled)):
        got, st = run([batch], S)  # default: clustering pass + verification
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
