"""The realtime link store (include/zksketch.h zk_rl_*) on the GPU, through the C ABI: every join row
(parent service, child service, child duration, traceId) K1 and the spill kernel emit, queried by
server service, must equal the oracle's rows (oracle/realtime.py joined_links: the job's join before
its group.sum, ZipkinAggregateJob.scala:25-37) exactly -- clustered and shuffled batches, traces
through the spill kernel, traces cut across batches (ZK_BATCH_CONTINUES), several batches in one
window -- while the dependency table stays equal to the dependency oracle. Then GpuRealtimeAggregates
(the RealtimeAggregates trait, RealtimeAggregates.scala:26-38) on the device against the same rows."""
import numpy as np
import pytest

from oracle import oracle
from oracle.realtime import joined_links, server_links
from tests.bulkfrag import service_name
from tests.test_gpu_parity import assert_parity, cols_from_rows, star_trace
from zipkin_amd import DepsContext, DeviceColumns, SpanColumns, ZkError, _abi, tracegen_host
from zipkin_amd.realtime import RealtimeLinks, RtSketch

pytestmark = pytest.mark.gpu


def check_all_servers(rl, cols, S):
    links = joined_links(cols, S)
    n, dropped = rl.count()
    assert (n, dropped) == (len(links[0]), 0)
    for s in range(S):
        got = rl.server_links(s)
        want = server_links(links, s)
        for g, w, name in zip(got, want, ("parent", "duration", "traceId")):
            assert np.array_equal(g.astype(np.int64 if name != "traceId" else np.uint64),
                                  w.astype(np.int64 if name != "traceId" else np.uint64)), f"server {s}: {name}"


@pytest.mark.parametrize("clustered", [True, False])
def test_join_rows_equal_the_oracle(gpu, clustered):
    S = 61
    cols = tracegen_host(71, 20_000, max_depth=6, num_services=S)
    if not clustered:
        cols = cols.take(np.random.default_rng(71).permutation(len(cols)))
    with DepsContext(S) as ctx, RealtimeLinks(S) as rl:
        rl.bind(ctx)
        ctx.accumulate(cols, clustered=clustered, verify=clustered)
        got = ctx.finalize()
        st = ctx.stats()
        check_all_servers(rl, cols, S)
    assert_parity(got, st, oracle.aggregate(cols, S))


def test_spilled_and_continued_traces(gpu):
    """Rows from the spill kernel (a 12k-record trace) and from held traces joined across batch
    edges, over several batches of one window (the window grows past its first allocation)."""
    S = 9
    rows = []
    for t in range(40):
        rows += star_trace(100 + t, 1 + t % 6, svc_root=t % S, nsvc=S)
    rows += star_trace(7777, 6_000, nsvc=S)  # 12k records: longer than a K1 window -> spill kernel
    for t in range(40):
        rows += star_trace(900 + t, 1 + t % 5, svc_root=t % S, nsvc=S)
    big = cols_from_rows(rows)
    tg = tracegen_host(72, 6000, max_depth=6, num_services=S)
    cols = SpanColumns.concat([big, tg])
    cuts = sorted(np.random.default_rng(72).choice(np.arange(1, len(cols)), 5, replace=False).tolist())
    bounds = [0, *cuts, len(cols)]
    with DepsContext(S) as ctx, RealtimeLinks(S) as rl:
        rl.bind(ctx)
        for i, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
            part = cols.take(slice(a, b))
            ctx.accumulate(DeviceColumns.from_host(part) if i % 2 else part, clustered=True, verify=True,
                           continues=i + 2 < len(bounds))
        got = ctx.finalize()
        st = ctx.stats()
        assert st["spilled_traces"] >= 1
        check_all_servers(rl, cols, S)
        rl.reset()
        assert rl.count() == (0, 0)
    assert_parity(got, st, oracle.aggregate(cols, S))


def test_binding_rules(gpu):
    S = 5
    with DepsContext(S) as ctx, RealtimeLinks(S) as rl, RtSketch(S) as rt, RealtimeLinks(S + 1) as other:
        rt.bind(ctx)  # ZK_RT_WITH_DEPS
        with pytest.raises(ZkError) as e:
            rl.bind(ctx)
        assert e.value.status == _abi.ZK_ERR_UNSUPPORTED
        rt.unbind()
        with pytest.raises(ZkError):
            other.bind(ctx)  # num_services differ
        rl.bind(ctx)
        with pytest.raises(ZkError):
            rl.server_links(S)  # no such server
        rl.unbind()


def test_gpu_realtime_aggregates_answers_the_trait(gpu):
    from zipkin_amd.aggregates import Dictionary, GpuRealtimeAggregates

    S = 31
    names = Dictionary([service_name(i) for i in range(S)])
    a = tracegen_host(73, 5000, max_depth=6, num_services=S)
    b = tracegen_host(74, 5000, max_depth=6, num_services=S)
    hour = 3_600_000_000
    store = GpuRealtimeAggregates(names)
    store.accumulate(a.take(np.random.default_rng(1).permutation(len(a))), 10 * hour + 5)
    store.accumulate(b, 11 * hour, clustered=True)
    for cols, t in ((a, 10 * hour), (b, 11 * hour + 17)):
        p, c, d, tid = joined_links(cols, S)
        for server in (0, 3, 17):
            sel = c == server
            want_d, want_t = {}, {}
            for pi, di, ti in zip(p[sel].tolist(), d[sel].tolist(), tid[sel].tolist()):
                want_d.setdefault(names.name(pi), []).append(di)
                want_t.setdefault(names.name(pi), set()).add(ti - (1 << 64) if ti >= 1 << 63 else ti)
            assert store.getSpanDurations(t, names.name(server), "") == {k: sorted(v) for k, v in want_d.items()}
            assert store.getServiceNamesToTraceIds(t, names.name(server), "") == {k: sorted(v) for k, v in want_t.items()}
    assert store.getSpanDurations(12 * hour, names.name(0), "") == {}
    store.close()
