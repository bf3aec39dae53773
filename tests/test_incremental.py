"""Watermark-incremental runs (zipkin_amd/incremental.py; AnormAggregator.scala:32-121 driver logic).

CPU tests drive IncrementalAggregator with the oracle's job (oracle/oracle.py) in place of the
device job; the GPU test runs the device job and checks each stored record against the oracle on
exactly the traces that were new."""
import numpy as np
import pytest

from oracle import oracle
from zipkin_amd import tracegen_host
from zipkin_amd.aggregates import Dependencies, DependencyLink, Dictionary, GpuAggregates, Moments, Service
from zipkin_amd.incremental import IncrementalAggregator, trace_created

S = 20
NAMES = [f"svc{i}" for i in range(S)]


class OracleJob:
    """ZipkinAggregateJob.run with the CPU restatement (test infrastructure)."""

    def __init__(self, services):
        self.services = services
        self.runs = []

    def run(self, batch, num_services=None):
        self.runs.append(len(batch))
        ref = oracle.aggregate(batch, num_services or S)
        m0, (m1, m2, m3, m4) = ref.dense()
        links = tuple(
            DependencyLink(Service(self.services.name(int(c) // S)), Service(self.services.name(int(c) % S)),
                           Moments(int(m0[c]), float(m1[c]), float(m2[c]), float(m3[c]), float(m4[c])))
            for c in np.flatnonzero(m0))
        return Dependencies(0, 1, links) if links else None


def _created(cols, base):
    """created_ts per record: trace k (in batch order) was created at base + 10 k (+ up to 3 us
    jitter per fragment, so the trace's created time is the max over its fragments)."""
    start = np.ones(len(cols), bool)
    start[1:] = cols.trace_id[1:] != cols.trace_id[:-1]
    k = np.cumsum(start) - 1
    rng = np.random.default_rng(base)
    return base + 10 * k + rng.integers(0, 4, len(cols))


def _by_key(deps):
    return {(l.parent.name, l.child.name): l.duration_moments for l in deps.links}


def _expect(cols, mask, services):
    return _by_key(OracleJob(services).run(cols.take(np.flatnonzero(mask)), S))


def test_trace_created_is_max_over_fragments():
    cols = tracegen_host(seed=3, num_traces=50, max_depth=4, num_services=S)
    ts = _created(cols, 1000)
    got = trace_created(cols, ts)
    for t in np.unique(cols.trace_id):
        m = cols.trace_id == t
        assert np.all(got[m] == ts[m].max())
    with pytest.raises(ValueError):
        trace_created(cols, ts[:-1])


def test_watermark_empty_then_max_end():
    agg = GpuAggregates("anorm", services=Dictionary(NAMES))
    assert agg.watermark() == 0  # IFNULL(MAX(END_TS), 0)
    agg.storeDependencies(Dependencies(5, 70, ()))
    agg.storeDependencies(Dependencies(80, 90, ()))
    agg.storeDependencies(Dependencies(1, 40, ()))
    assert agg.watermark() == 90


@pytest.mark.parametrize("mode", ["anorm", "cassandra"])
def test_incremental_runs_aggregate_each_trace_once(mode):
    services = Dictionary(NAMES)
    agg = GpuAggregates(mode, services=services)
    job = OracleJob(services)
    inc = IncrementalAggregator(agg, job=job)
    a = tracegen_host(seed=11, num_traces=300, max_depth=5, num_services=S)
    ts_a = _created(a, 10_000)

    # run 1: everything is new
    rec1 = inc.apply(a, ts_a, num_services=S)
    tc = trace_created(a, ts_a)
    assert rec1.start_time == tc.min() and rec1.end_time == tc.max()
    # the first step is created_ts > minTime (AnormAggregator.scala:46-47,79): the earliest trace is skipped
    assert _by_key(rec1) == _expect(a, tc > tc.min(), services)
    assert agg.watermark() == tc.max() and agg.count() == 1

    # run 2: the same traces again plus newer ones: only the newer ones are aggregated
    b = tracegen_host(seed=12, num_traces=200, max_depth=5, num_services=S)
    ts_b = _created(b, int(tc.max()) + 1)
    both = type(a).concat([a, b])
    ts_both = np.concatenate([ts_a, ts_b])
    rec2 = inc.apply(both, ts_both, num_services=S)
    tcb = trace_created(both, ts_both)
    new = (tcb > tc.max()) & (tcb > trace_created(b, ts_b).min())
    assert inc.last_selected == int(new.sum()) and 0 < int(new.sum()) < len(b)
    assert _by_key(rec2) == _expect(both, new, services)
    # Cassandra keys records by day and clobbers the row (CassandraAggregates.scala:111-116): both
    # runs fall on day 0, so the second record replaces the first; Anorm keeps both rows
    rows = 2 if mode == "anorm" else 1
    assert rec2.start_time == trace_created(b, ts_b).min() and agg.count() == rows

    # run 3: nothing new -> nothing stored ("already up-to-date")
    assert inc.apply(both, ts_both, num_services=S) is None
    assert agg.count() == rows and job.runs == [int((tc > tc.min()).sum()), int(new.sum())]


def test_incremental_trace_straddling_the_watermark_is_new_as_a_whole():
    services = Dictionary(NAMES)
    agg = GpuAggregates("anorm", services=services)
    inc = IncrementalAggregator(agg, job=OracleJob(services))
    agg.storeDependencies(Dependencies(0, 500, ()))
    cols = tracegen_host(seed=5, num_traces=40, max_depth=4, num_services=S)
    ts = np.full(len(cols), 100, np.int64)
    first = cols.trace_id == cols.trace_id[0]
    ts[np.flatnonzero(first)[-1]] = 600  # one late fragment: the whole first trace is new
    inc.apply(cols, ts, num_services=S)
    assert inc.last_selected == int(first.sum())


@pytest.mark.gpu
def test_incremental_device_job_matches_oracle():
    """Runs until up to date: every record covers exactly the traces created in (previous
    watermark, its end] (the step boundary rule), with the device job's links equal to the
    oracle's, and every trace is aggregated exactly once."""
    services = Dictionary(NAMES)
    agg = GpuAggregates("anorm", services=services)
    inc = IncrementalAggregator(agg)  # device ZipkinAggregateJob
    a = tracegen_host(seed=21, num_traces=2000, max_depth=6, num_services=S)
    ts_a = _created(a, 50_000)
    b = tracegen_host(seed=22, num_traces=1500, max_depth=6, num_services=S)
    ts_b = _created(b, int(trace_created(a, ts_a).max()) + 1)
    seen = np.zeros(len(a) + len(b), np.int64)
    skipped = np.zeros(len(a) + len(b), bool)
    for cols, ts in ((a, ts_a), (type(a).concat([a, b]), np.concatenate([ts_a, ts_b]))):
        tc = trace_created(cols, ts)
        while True:
            wm = agg.watermark()
            rec = inc.apply(cols, ts, num_services=S)
            if rec is None:
                break
            new = tc > wm
            lo, hi = int(tc[new].min()), int(tc[new].max())
            step = (hi - lo) // max(int(new.sum()) // 10000, 1)
            sel = new & (tc <= rec.end_time)
            if step != 0:  # first step: created_ts > minTime (a zero step keeps them, see incremental.py)
                sel &= tc > lo
            assert inc.last_selected == int(sel.sum()) and rec.start_time == lo
            assert _by_key(rec) == _expect(cols, sel, services)
            seen[: len(cols)] += sel
            if step != 0:
                skipped[: len(cols)] |= new & (tc == lo)
        assert agg.watermark() == tc.max()
    # every trace exactly once, except those created exactly at a run's minTime, which the
    # reference never aggregates
    assert (seen[~skipped] == 1).all() and (seen[skipped] == 0).all() and skipped.any()


def test_run_without_links_still_advances_the_watermark():
    """AnormAggregator folds from Monoid.zero and stores whenever new spans exist (:41-56), so a
    run whose new traces join nothing still moves the watermark and is not selected again."""
    services = Dictionary(NAMES)
    agg = GpuAggregates("anorm", services=services)
    job = OracleJob(services)
    inc = IncrementalAggregator(agg, job=job)
    roots = tracegen_host(seed=13, num_traces=50, max_depth=1, num_services=S)  # root spans only
    ts = _created(roots, 1000)
    rec = inc.apply(roots, ts, num_services=S)
    assert rec is not None and rec.links == () and agg.count() == 1
    assert agg.watermark() == trace_created(roots, ts).max()
    assert inc.apply(roots, ts, num_services=S) is None and job.runs == [len(roots) - 1]  # all but the first


def test_record_ends_at_the_last_step_boundary():
    """More than 10000 new records: steps = count / 10000, the record ends on the last boundary of
    Range.Long(min, max + 1, stepSize) and later traces wait for the next run (:35-39)."""
    services = Dictionary(NAMES)
    agg = GpuAggregates("anorm", services=services)
    job = OracleJob(services)
    inc = IncrementalAggregator(agg, job=job)
    cols = tracegen_host(seed=14, num_traces=1500, max_depth=5, num_services=S)
    starts = np.r_[True, cols.trace_id[1:] != cols.trace_id[:-1]]
    k = np.cumsum(starts) - 1  # trace index per record
    ts = (1000 + 7 * k).astype(np.int64)  # one created time per trace, 7 us apart
    tc = trace_created(cols, ts)
    rec = inc.apply(cols, ts, num_services=S)
    lo, hi, count = int(tc.min()), int(tc.max()), len(cols)
    steps = max(count // 10000, 1)
    step = (hi - lo) // steps
    end = lo + ((hi - lo) // step) * step
    assert count > 10000 and (rec.start_time, rec.end_time) == (lo, end)
    assert inc.last_selected == int(((tc <= end) & (tc > lo)).sum())
    rest = inc.apply(cols, ts, num_services=S)  # the traces after the boundary (but its first)
    after = tc > end
    lo2 = tc[after].min()
    # one created instant left: stepSize 0 (the reference's Range throws), those traces are kept
    expect = after if (tc[after] == lo2).all() else after & (tc > lo2)
    assert rest is None or inc.last_selected == int(expect.sum())
