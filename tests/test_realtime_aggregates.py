"""RealtimeAggregates (zipkin-common/.../storage/RealtimeAggregates.scala:26-38) on CPU: the join-row
restatement the realtime link store is checked against (oracle/realtime.py joined_links), pinned to
the dependency oracle (oracle/zk_oracle.c): the rows aggregated per (parent, child) give exactly the
oracle's link counts and duration sums -- and the GpuRealtimeAggregates twin's mapping of those rows
to the trait's answers (client service -> every duration / every distinct trace id, windows by
time stamp, unknown names and windows empty), run over the oracle's rows."""
import numpy as np
import pytest

from oracle import oracle
from oracle.realtime import joined_links, server_links
from tests.bulkfrag import service_name
from zipkin_amd import SpanColumns, tracegen_host
from zipkin_amd.aggregates import Dictionary, GpuRealtimeAggregates, NullRealtimeAggregates


class OracleWindow:
    """A GpuRealtimeAggregates window over the oracle's join rows (the device's is _DeviceLinkWindow)."""

    def __init__(self, S):
        self.S = S
        self.parts = []
        self.closed = False

    def add(self, cols, clustered):
        self.parts.append(cols)

    def server_links(self, server):
        return server_links(joined_links(SpanColumns.concat(self.parts), self.S), server)

    def close(self):
        self.closed = True


def test_join_rows_sum_to_the_dependency_oracle():
    S = 57
    cols = tracegen_host(5, 3000, max_depth=6, num_services=S)
    p, c, d, t = joined_links(cols, S)
    ref = oracle.aggregate(cols, S)
    m0, ms = ref.dense()
    cnt = np.zeros(S * S, np.int64)
    np.add.at(cnt, p * S + c, 1)
    assert np.array_equal(cnt, m0.astype(np.int64))
    assert len(p) == ref.stats["joined_links"]
    s1 = np.zeros(S * S)
    np.add.at(s1, p * S + c, d.astype(float))
    mean = np.divide(s1, cnt, out=np.zeros_like(s1), where=cnt > 0)
    assert np.allclose(mean, ms[0], rtol=1e-12)
    # every row's trace id is one of the batch's, and each child's service is the server side
    assert np.isin(t, cols.trace_id).all()


def _expected(cols, S, names, server):
    p, c, d, t = joined_links(cols, S)
    durs, tids = {}, {}
    for pi, ci, di, ti in zip(p.tolist(), c.tolist(), d.tolist(), t.tolist()):
        if ci != server:
            continue
        durs.setdefault(names.name(pi), []).append(di)
        tids.setdefault(names.name(pi), set()).add(ti - (1 << 64) if ti >= 1 << 63 else ti)
    return {k: sorted(v) for k, v in durs.items()}, {k: sorted(v) for k, v in tids.items()}


def test_twin_maps_join_rows_to_the_trait():
    S = 23
    names = Dictionary([service_name(i) for i in range(S)])
    a = tracegen_host(7, 1500, max_depth=6, num_services=S)
    b = tracegen_host(8, 1500, max_depth=6, num_services=S)
    b.trace_id |= np.uint64(1 << 63)  # negative Longs on the JVM side
    hour = 3_600_000_000
    store = GpuRealtimeAggregates(names, window_factory=OracleWindow)
    store.accumulate(a, 5 * hour + 10)
    store.accumulate(b, 6 * hour + 10)
    for server in range(S):
        want_d, want_t = _expected(a, S, names, server)
        assert store.getSpanDurations(5 * hour + 999, names.name(server), "") == want_d
        assert store.getServiceNamesToTraceIds(5 * hour, names.name(server), "any rpc") == want_t
        want_d, want_t = _expected(b, S, names, server)
        assert store.getSpanDurations(6 * hour, names.name(server), "") == want_d
        assert store.getServiceNamesToTraceIds(7 * hour - 1, names.name(server), "") == want_t
    assert any(v and min(v) < 0 for v in store.getServiceNamesToTraceIds(6 * hour, names.name(1), "").values())
    # unknown window / server: empty maps, like NullRealtimeAggregates
    assert store.getSpanDurations(4 * hour, names.name(1), "") == {}
    assert store.getServiceNamesToTraceIds(5 * hour, "no-such-service", "") == {}
    null = NullRealtimeAggregates()
    assert null.getSpanDurations(0, "x", "") == {} and null.getServiceNamesToTraceIds(0, "x", "") == {}
    store.close()


def test_twin_keeps_the_last_windows():
    S = 7
    names = Dictionary([service_name(i) for i in range(S)])
    cols = tracegen_host(9, 200, max_depth=5, num_services=S)
    store = GpuRealtimeAggregates(names, window_us=1000, keep=3, window_factory=OracleWindow)
    made = []
    store._factory = lambda s: made.append(OracleWindow(s)) or made[-1]
    for w in range(5):
        store.accumulate(cols, w * 1000 + 1)
    assert sorted(store._windows) == [2, 3, 4]
    assert [m.closed for m in made] == [True, True, False, False, False]
    assert store.getSpanDurations(1500, names.name(1), "") == {}
    assert store.getSpanDurations(4500, names.name(1), "") == _expected(cols, S, names, 1)[0]
    with pytest.raises(ValueError):
        GpuRealtimeAggregates(names, window_us=0)
