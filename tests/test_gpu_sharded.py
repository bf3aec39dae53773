"""The N>1 product path on one GPU: traceId-hash shards -> one DepsContext per shard over a
caller-owned table -> zk_deps_partial (counters folded into the tail) -> SUM of the tables ->
zk_deps_note_merged -> finalize.

The SUM is a torch add of the int64 tables: exactly what RCCL's SUM all-reduce computes on every
rank, so this is the merge of ZipkinAggregateJob.scala:39-43 (`.group.sum` and the final `.sum`
across reducers) with the collective replaced by its arithmetic. Bar: m0..m4 and every counter
bit-identical to the oracle over the union and to the 1-shard run; the device limb layout decodes
(zipkin_amd/table.py) to the oracle's exact power sums."""
import numpy as np
import pytest

from oracle import oracle
from tests.test_gpu_parity import SERVER, assert_parity, cols_from_rows
from zipkin_amd import DepsContext, ZkError, _abi, table, tracegen_host
from zipkin_amd.shards import device_view, split

pytestmark = pytest.mark.gpu


class Shard:
    def __init__(self, S, **kw):
        import torch

        self.table = torch.zeros(_abi.table_words(S), dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        self.ctx = DepsContext(S, table_ptr=self.table.data_ptr(), table_bytes=self.table.numel() * 8, **kw)

    def close(self):
        self.ctx.close()


def run_sharded(cols, S, world, **kw):
    """-> (finalized table and stats of every rank, the summed int64 table)."""
    import torch

    parts = split(cols, world)
    shards = [Shard(S, **kw) for _ in range(world)]
    try:
        views = []
        for sh, p in zip(shards, parts):
            sh.ctx.accumulate(p, clustered=True, verify=True)
            ptr, nbytes = sh.ctx.partial()  # the exchange form: 12 limbs of 56 bits per cell + tail
            assert nbytes == _abi.xchg_words(S) * 8
            views.append(device_view(ptr, nbytes, torch.int64))
        for sh in shards:
            sh.ctx.sync()
        # the exchange form packs the accumulator exactly (zipkin_amd/table.py pack is the host view)
        assert np.array_equal(views[0].cpu().numpy(), table.pack(shards[0].table.cpu().numpy(), S))
        total = torch.stack(views).sum(0)  # the all-reduce's SUM
        outs = []
        for sh, v in zip(shards, views):  # every rank holds the same merged buffer after the all-reduce
            v.copy_(total)
            torch.cuda.synchronize()
            sh.ctx.note_merged(0)
            try:
                outs.append((sh.ctx.finalize(), sh.ctx.stats(), None))
            except ZkError as e:
                outs.append((None, sh.ctx.stats(), e.status))
        # the merged accumulator (unpacked on every rank) is the host unpack of the summed exchange form
        merged = shards[0].table.cpu().numpy()
        assert np.array_equal(merged, table.unpack(total.cpu().numpy(), S))
        return outs, merged
    finally:
        for sh in shards:
            sh.close()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_sharded_tables_sum_to_the_oracle(gpu, world):
    S = 500
    cols = tracegen_host(41, 60_000, max_depth=6, num_services=S)
    ref = oracle.aggregate(cols, S)
    outs, total = run_sharded(cols, S, world)
    for got, st, status in outs:
        assert status is None
        assert_parity(got, st, ref)
        assert st["records"] == len(cols) and st["not_clustered"] == 0
    # the device layout decodes to the oracle's exact power sums (table.py is the host view)
    dec = table.decode(total, S)
    want = {}
    for c in ref.present_cells():
        want[(int(c) // S, int(c) % S)] = ref.power_sums(int(c))
    assert dec == want
    tail = table.tail_stats(total, S)
    for k, v in ref.stats.items():
        if k != "spilled_traces":
            assert tail[k] == v, k


def test_sharded_equals_one_shard_bit_for_bit(gpu):
    S = 57
    cols = tracegen_host(42, 30_000, max_depth=7, num_services=S)
    one, t1 = run_sharded(cols, S, 1)
    eight, t8 = run_sharded(cols, S, 8)
    # limbs hold sums of 32-bit chunks, so their split depends on how links were grouped; the
    # values they encode (the exact power sums) do not
    assert table.decode(t1, S) == table.decode(t8, S)
    for k in ("m0", "m1", "m2", "m3", "m4", "present"):
        assert np.array_equal(getattr(one[0][0], k), getattr(eight[0][0], k)), k


def test_strict_error_is_decided_from_the_merged_counters(gpu):
    """A no-service pair on ONE shard fails finalize on EVERY rank (reference: the whole job fails
    on None.get, ZipkinAggregateJob.scala:36-37), so no rank runs ahead into the next collective."""
    S = 9
    good = tracegen_host(43, 2000, max_depth=4, num_services=S)
    bad = cols_from_rows([(7, 70, 0, 1, 9, 0, SERVER),
                          (7, 71, 70, 2, 4, 0, _abi.ZK_F_HAS_ANNOTATIONS | 1 | (1 << 12) | (1 << 14))])
    from zipkin_amd.columns import SpanColumns

    cols = SpanColumns.concat([good, bad])
    outs, _ = run_sharded(cols, S, 4, strict=True)
    assert [s for _, _, s in outs] == [_abi.ZK_ERR_NO_SERVICE] * 4
    assert all(st["no_service"] == 1 for _, st, _ in outs)
    outs, _ = run_sharded(cols, S, 4, strict=False)
    assert all(s is None for _, _, s in outs)
    ref = oracle.aggregate(cols, S)
    for got, st, _ in outs:
        assert_parity(got, st, ref)


def test_accumulate_after_merge_uses_local_counters_again(gpu):
    S = 20
    a = tracegen_host(44, 1000, max_depth=5, num_services=S)
    sh = Shard(S)
    try:
        sh.ctx.accumulate(a)
        sh.ctx.partial()
        sh.ctx.sync()
        sh.ctx.note_merged(0)
        assert sh.ctx.stats()["records"] == len(a)
        sh.ctx.reset()
        sh.ctx.accumulate(a)
        got = sh.ctx.finalize()
        assert_parity(got, sh.ctx.stats(), oracle.aggregate(a, S))
    finally:
        sh.close()


def test_note_merged_requires_partial(gpu):
    """zk_deps_note_merged trusts the table's counter tail, which only zk_deps_partial fills: without
    it (or after a later accumulate) the call is refused instead of dropping every error counter."""
    S = 20
    a = tracegen_host(45, 500, max_depth=5, num_services=S)
    sh = Shard(S)
    try:
        sh.ctx.accumulate(a)
        with pytest.raises(ZkError) as e:
            sh.ctx.note_merged(0)
        assert e.value.status == _abi.ZK_ERR_INVALID_ARG
        sh.ctx.partial()
        sh.ctx.accumulate(a.take(np.arange(0)))  # an empty batch changes nothing
        sh.ctx.note_merged(0)
        sh.ctx.reset()  # reset forgets the fold
        sh.ctx.accumulate(a)
        with pytest.raises(ZkError):
            sh.ctx.note_merged(len(a))
    finally:
        sh.close()


def test_accumulate_into_merged_table_keeps_the_job_counters(gpu):
    """A batch accumulated into a merged table: finalize reports the merged job plus the batch, and
    the table's values are the union's (the ctx's counters restart from the merged tail)."""
    S = 20
    a = tracegen_host(46, 800, max_depth=5, num_services=S)
    b = tracegen_host(47, 600, max_depth=5, num_services=S)
    from zipkin_amd.columns import SpanColumns

    sh = Shard(S)
    try:
        sh.ctx.accumulate(a)
        sh.ctx.partial()
        sh.ctx.sync()
        sh.ctx.note_merged(0)
        sh.ctx.accumulate(b)
        got = sh.ctx.finalize()
        st = sh.ctx.stats()
        assert st["records"] == len(a) + len(b)
        assert_parity(got, st, oracle.aggregate(SpanColumns.concat([a, b]), S))
        # this ctx now holds the whole job: a second exchange would add it once per rank
        with pytest.raises(ZkError) as e:
            sh.ctx.partial()
        assert e.value.status == _abi.ZK_ERR_INVALID_ARG
        sh.ctx.reset()  # a reset starts a fresh shard that may be exchanged again
        sh.ctx.accumulate(b)
        sh.ctx.partial()
    finally:
        sh.close()


def test_held_trace_dropped_on_one_shard_fails_every_rank(gpu):
    """A held trace (ZK_BATCH_CONTINUES) that outgrows max_trace_records on ONE shard is counted on
    the device, so zk_deps_partial carries it in the exchange tail and every rank's finalize returns
    ZK_ERR_TRACE_TOO_LARGE (zkagg.h: every rank reaches the same status)."""
    import torch

    from tests.test_gpu_continuation import cut

    S = 7
    from tests.test_gpu_parity import star_trace

    big = cols_from_rows(star_trace(1, 30, nsvc=S) + star_trace(2, 800, nsvc=S) + star_trace(3, 30, nsvc=S))
    parts = cut(big, [561, 1161, 1672])
    other = tracegen_host(48, 500, max_depth=5, num_services=S)
    shards = [Shard(S, max_trace_records=1000) for _ in range(2)]
    try:
        for p in parts[:-1]:
            shards[0].ctx.accumulate(p, clustered=True, continues=True)
        shards[0].ctx.accumulate(parts[-1], clustered=True)
        shards[1].ctx.accumulate(other, clustered=True, verify=True)
        views = []
        for sh in shards:
            ptr, nbytes = sh.ctx.partial()
            views.append(device_view(ptr, nbytes, torch.int64))
        for sh in shards:
            sh.ctx.sync()
        total = torch.stack(views).sum(0)
        for sh, v in zip(shards, views):
            v.copy_(total)
            torch.cuda.synchronize()
            sh.ctx.note_merged(0)
            with pytest.raises(ZkError) as e:
                sh.ctx.finalize()
            assert e.value.status == _abi.ZK_ERR_TRACE_TOO_LARGE
            assert sh.ctx.stats()["trace_too_large"] == 1
    finally:
        for sh in shards:
            sh.close()


def test_global_trace_set_on_eight_device_shards_equals_the_oracle(gpu):
    """configs[2]'s sharding at a size the oracle checks in seconds: ONE global TraceGen set whose
    traceIds do not depend on the world size (zk_tracegen_device with global_ids), 8 shards each
    generated on the device and accumulated in its own ctx, the exchange buffers summed as RCCL's
    SUM all-reduce would; every rank's table is bit-exact against the oracle over the whole set
    (generated on the host at world 1)."""
    import torch

    from zipkin_amd import DeviceColumns, tracegen_params

    S, G, N = 500, 8, 2_000_000
    whole = tracegen_host(7, N // 15 + 1000, target_records=N, max_depth=6, num_services=S, global_ids=True)
    ref = oracle.aggregate(whole, S)
    shards = [Shard(S) for _ in range(G)]
    try:
        views, n_all = [], 0
        for r, sh in enumerate(shards):
            p = tracegen_params(7, N // 15 + 1000, target_records=N, max_depth=6, num_services=S, rank=r, world=G,
                                global_ids=True)
            cols = DeviceColumns(N // G * 2 + 10_000)
            n, _ = sh.ctx.tracegen_device(p, cols)
            n_all += n
            sh.ctx.accumulate(cols, clustered=True, verify=True, n=n)
            ptr, nbytes = sh.ctx.partial()
            views.append(device_view(ptr, nbytes, torch.int64))
            sh._cols = cols
        assert n_all == len(whole)
        for sh in shards:
            sh.ctx.sync()
        total = torch.stack(views).sum(0)
        for sh, v in zip(shards, views):
            v.copy_(total)
            torch.cuda.synchronize()
            sh.ctx.note_merged(0)
            assert_parity(sh.ctx.finalize(), sh.ctx.stats(), ref)
    finally:
        for sh in shards:
            sh.close()


def test_aborted_rank_fails_every_rank_after_the_exchange(gpu):
    """zk_deps_abort (a rank that failed on the host before the exchange, GpuDependenciesJob.guarded):
    its exchange buffer is a zero table whose tail carries one abort mark, the SUM delivers the mark
    to every rank, and every rank's finalize returns ZK_ERR_RANK_FAILED; the merged records count
    excludes the mark. A reset clears it."""
    import torch

    S, world = 97, 4
    cols = tracegen_host(44, 6000, max_depth=6, num_services=S)
    parts = split(cols, world)
    shards = [Shard(S) for _ in range(world)]
    try:
        views = []
        for r, (sh, p) in enumerate(zip(shards, parts)):
            sh.ctx.accumulate(p, clustered=True, verify=True)
            if r == 2:
                sh.ctx.abort()
            ptr, nbytes = sh.ctx.partial()
            views.append(device_view(ptr, nbytes, torch.int64))
        for sh in shards:
            sh.ctx.sync()
        aborted = views[2].cpu().numpy()
        assert not aborted[:-16].any() and aborted[-16] == 1 << 48 and not aborted[-15:].any()
        total = torch.stack(views).sum(0)
        for r, (sh, v) in enumerate(zip(shards, views)):
            v.copy_(total)
            torch.cuda.synchronize()
            sh.ctx.note_merged(0)
            with pytest.raises(ZkError) as e:
                sh.ctx.finalize()
            assert e.value.status == _abi.ZK_ERR_RANK_FAILED
            st = sh.ctx.stats()
            assert st["records"] == sum(len(p) for i, p in enumerate(parts) if i != 2)
        # the next job on the same contexts is clean again
        for sh in shards:
            sh.ctx.reset()
        outs, _ = run_sharded(cols, S, 2)
        ref = oracle.aggregate(cols, S)
        for got, st, status in outs:
            assert status is None
            assert_parity(got, st, ref)
    finally:
        for sh in shards:
            sh.close()
