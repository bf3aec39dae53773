"""The shared TraceGen restatement (zk_tracegen.h) on the host: shape, determinism, sharding."""
import numpy as np

from zipkin_amd import tracegen_host
from zipkin_amd.columns import trace_shard


def test_deterministic_and_clustered():
    a = tracegen_host(seed=11, num_traces=500, max_depth=7, num_services=57)
    b = tracegen_host(seed=11, num_traces=500, max_depth=7, num_services=57)
    for k in ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags"):
        assert np.array_equal(getattr(a, k), getattr(b, k))
    # every trace is one contiguous run of records
    change = np.flatnonzero(np.diff(a.trace_id.view(np.int64)) != 0)
    assert len(change) + 1 == len(np.unique(a.trace_id)) == 500


def test_tracegen_shape_matches_survey():
    # SURVEY A.4 (sim of TraceGen.scala): maxDepth 7 -> ~35.9 records, ~18.5 logical spans per trace
    c = tracegen_host(seed=1, num_traces=10000, max_depth=7, num_services=57)
    rpt = len(c) / 10000
    assert 30 < rpt < 42
    spans = len(np.unique(np.stack([c.trace_id, c.span_id], 1), axis=0))
    assert 1.85 < len(c) / spans < 2.0  # ~1.95 fragments per logical span
    roots = int(((c.flags & 1) == 0).sum())
    assert roots == 10000
    # client fragments carry cs/cr, server fragments sr/ss; durations are non-negative
    assert (c.last_ts >= c.first_ts).all()
    assert set(np.unique(c.flags)) <= {0b1010 | (1 << 12) | (1 << 14), 0b1011 | (1 << 12) | (1 << 14),
                                        0b0111 | (1 << 8) | (1 << 10)}


def test_target_records_cuts_on_trace_boundary():
    full = tracegen_host(seed=3, num_traces=1000, max_depth=6, num_services=100)
    cut = tracegen_host(seed=3, num_traces=1000, max_depth=6, num_services=100, target_records=len(full) // 2)
    assert 0 < len(cut) <= len(full) // 2
    assert np.array_equal(cut.trace_id, full.trace_id[: len(cut)])
    assert len(cut) == len(full) or full.trace_id[len(cut)] != full.trace_id[len(cut) - 1]


def test_shards_are_disjoint_and_owned():
    world = 4
    ids = []
    for r in range(world):
        c = tracegen_host(seed=9, num_traces=200, max_depth=4, num_services=50, rank=r, world=world)
        u = np.unique(c.trace_id)
        assert all(trace_shard(int(t), world) == r for t in u[:50])
        ids.append(u)
    allids = np.concatenate(ids)
    assert len(np.unique(allids)) == len(allids)


def _rows(c):
    return np.stack([c.trace_id, c.span_id, c.parent_id, c.first_ts.view(np.uint64), c.last_ts.view(np.uint64),
                     c.service_id.astype(np.uint64), c.flags.astype(np.uint64)], 1)


def test_global_set_is_the_same_for_every_world():
    """global_ids (configs[2]): one trace set, cut at the same record target for every world size;
    shard r of world G holds exactly the set's traces whose zk_trace_shard(traceId, G) == r, each
    trace whole and trace-clustered, and the shards together are the G = 1 set."""
    kw = dict(max_depth=6, num_services=100, target_records=40_000, global_ids=True)
    one = tracegen_host(seed=7, num_traces=5_000, **kw)
    assert 0 < len(one) <= 40_000
    ref = _rows(one)
    ref = ref[np.lexsort(ref.T[::-1])]
    for world in (2, 3, 4, 8):
        parts = [tracegen_host(seed=7, num_traces=5_000, rank=r, world=world, **kw) for r in range(world)]
        for r, p in enumerate(parts):
            u = np.unique(p.trace_id)
            assert all(trace_shard(int(t), world) == r for t in u[:50])
            change = np.flatnonzero(np.diff(p.trace_id.view(np.int64)) != 0)
            assert len(change) + 1 == len(u)  # every trace one contiguous run
        got = np.concatenate([_rows(p) for p in parts])
        got = got[np.lexsort(got.T[::-1])]
        assert np.array_equal(got, ref)
    # at world 1 the global set is the per-shard set (the same traceIds): C2 and C3 agree at G = 1
    assert np.array_equal(tracegen_host(seed=7, num_traces=5_000, max_depth=6, num_services=100,
                                        target_records=40_000).trace_id, one.trace_id)
