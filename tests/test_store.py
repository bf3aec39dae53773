"""The Aggregates store surface (include/zkstore.h via zipkin_amd.aggregates), on CPU.

Pinned by the reference's own tests and fixtures:
  * AnormAggregatesTest.scala:30-58   store/get round trip and the six window cases
  * DependenciesTest.scala:28-81      Service case-sensitivity, DependencyLink.plus assert, monoid
  * aggregates.sql (zipkin-tracegen/src/testdata)   150 stored links round-trip exactly
  * CassandraAggregatesTest.scala:57-123            top annotation store / get / clobber
Moments arithmetic (zk_moments_plus, C++) is checked bit for bit against the oracle's restatement
of algebird 0.8.1 MomentsGroup.plus (oracle/moments.py).
"""
import json
import random
import threading
from collections import Counter
from pathlib import Path

import numpy as np
import pytest

from oracle.moments import Moments as OMoments
from oracle.moments import algebird_plus
from oracle.spans import Dependencies as ODeps
from oracle.spans import DependencyLink as OLink
from zipkin_amd import ZkError, _abi
from zipkin_amd.aggregates import (
    Dependencies,
    DependencyLink,
    Dictionary,
    GpuAggregates,
    Moments,
    NullAggregates,
    Service,
    links_from_table,
)

GOLD = Path(__file__).resolve().parent / "golden"
KATS = json.loads((GOLD / "reference_kats.json").read_text())
NOW = 1_421_053_208_373_000  # a pinned Time.now (us)


def link(p, c, m):
    return DependencyLink(Service(p), Service(c), m)


def _same_bits(a, b):
    return a.m0 == b.m0 and all(np.float64(x).tobytes() == np.float64(y).tobytes()
                                for x, y in zip(a[1:], b[1:]))


# ---- Moments ---------------------------------------------------------------------------------
def test_moments_plus_bitwise_equals_algebird_restatement():
    rng = random.Random(7)
    vals = [Moments.of(v) for v in (2, 4, 1, 3, 10, 18, 1000, 0, 5000)]
    for _ in range(300):
        a = vals[rng.randrange(len(vals))]
        b = vals[rng.randrange(len(vals))]
        got = a.plus(b)
        exp = algebird_plus(OMoments(*a), OMoments(*b))
        assert _same_bits(got, exp), (a, b, got, exp)
        vals.append(got)


def test_moments_plus_is_symmetric_and_has_zero():
    a = Moments.of(3).plus(Moments.of(11)).plus(Moments.of(2))
    b = Moments.of(7).plus(Moments.of(9))
    assert _same_bits(a.plus(b), b.plus(a))
    assert a.plus(Moments.zero()) == a
    assert Moments.zero().plus(Moments.zero()) == Moments.zero()


def test_moments_kats_from_dependencies_test():
    # DependenciesTest.scala:43-50: Moments(2) + Moments(4)
    m = Moments.of(2).plus(Moments.of(4))
    assert tuple(m) == (2, 3.0, 2.0, 0.0, 2.0)


# ---- DependencyLink / Dependencies (DependenciesTest.scala) ----------------------------------
def test_services_compare_case_sensitively():
    assert Service("foo") == Service("foo")
    assert Service("foo") != Service("bar")
    assert Service("foo") != Service("Foo") and Service("foo") != Service("FOO")


def test_dependency_link_plus_asserts_on_mismatched_keys():
    d1 = link("tfe", "mobileweb", Moments.of(2))
    d2 = link("tfe", "mobileweb", Moments.of(4))
    d3 = link("Gizmoduck", "tflock", Moments.of(4))
    assert d1.plus(d2) == link("tfe", "mobileweb", Moments.of(2).plus(Moments.of(4)))
    with pytest.raises(AssertionError):
        d1.plus(d3)


def test_dependencies_monoid_kat():
    k = KATS["dependencies_monoid"]

    def deps(d):
        return Dependencies(d["start_s"] * 1_000_000, d["end_s"] * 1_000_000,
                            tuple(link(p, c, Moments.of(v)) for p, c, v in d["links"]))

    d1, d2 = deps(k["deps1"]), deps(k["deps2"])
    assert d1.plus(Dependencies.zero()) == d1
    r = d1.plus(d2)
    assert r.start_time == k["expected_start_s"] * 1_000_000 and r.end_time == k["expected_end_s"] * 1_000_000
    exp = Counter()
    for p, c, vs in k["expected_links"]:
        m = Moments.zero()
        for v in vs:
            m = m.plus(Moments.of(v))
        exp[link(p, c, m)] += 1
    assert Counter(r.links) == exp


# ---- storeDependencies / getDependencies -----------------------------------------------------
def test_anorm_window_cases():
    k = KATS["anorm_window"]
    agg = GpuAggregates("anorm", clock=lambda: NOW)
    st = k["stored"]
    dep = Dependencies(st["start_us"], st["end_us"], tuple(link(p, c, Moments.of(v)) for p, c, v in st["links"]))
    agg.storeDependencies(dep)
    for q in k["queries"]:
        end = NOW if q["end_us"] == "now" else q["end_us"]
        got = agg.getDependencies(q["start_us"], end)
        assert (got.links == dep.links) if q["hit"] else (got.links == ()), q["what"]
        assert got.start_time == q["start_us"] and got.end_time == (NOW if end is None else end)


def test_anorm_defaults_and_newest_first():
    agg = GpuAggregates("anorm", clock=lambda: NOW)
    old = Dependencies(NOW - 3 * 3600_000_000, NOW - 2 * 3600_000_000, (link("a", "b", Moments.of(1)),))
    new = Dependencies(NOW - 3600_000_000, NOW - 1, (link("c", "d", Moments.of(2)),))
    ancient = Dependencies(NOW - 3 * 86_400_000_000, NOW - 2 * 86_400_000_000, (link("e", "f", Moments.of(3)),))
    for d in (old, new, ancient):
        agg.storeDependencies(d)
    got = agg.getDependencies(None)  # start = now - 1 day, end = now
    assert got.links == new.links + old.links
    assert got.start_time == NOW - 86_400_000_000 and got.end_time == NOW
    # ORDER BY dlid DESC: the last stored row first
    assert agg.getDependencies(0, None).links == ancient.links + new.links + old.links
    assert agg.count() == 3


def test_aggregates_sql_fixture_round_trips_exactly():
    fx = json.loads((GOLD / "aggregates_sql.json").read_text())
    row = fx["dependencies"][0]
    links = tuple(link(l["parent"], l["child"], Moments(l["m0"], l["m1"], l["m2"], l["m3"], l["m4"]))
                  for l in fx["links"])
    assert len(links) == 150
    for mode in ("anorm", "cassandra", "hbase"):
        agg = GpuAggregates(mode, clock=lambda: NOW)
        agg.storeDependencies(Dependencies(row["start_ts"], row["end_ts"], links))
        # hbase: the scan starts at MaxValue - start ms and runs to the end without an end bound
        got = agg.getDependencies(0, None if mode == "hbase" else row["end_ts"])
        assert got.start_time == (0 if mode == "anorm" else row["start_ts"])
        assert Counter(got.links) == Counter(links)
        assert all(_same_bits(a.duration_moments, b.duration_moments)
                   for a, b in zip(sorted(got.links, key=str), sorted(links, key=str)))


def _random_records(seed, n, start_of):
    rng = random.Random(seed)
    names = ["tfe", "mobileweb", "Gizmoduck", "tflock", "cassie"]
    records = []
    for r in range(n):
        ls = {}
        for _ in range(rng.randrange(1, 6)):
            p, c = rng.sample(names, 2)
            m = Moments.zero()
            for _ in range(rng.randrange(1, 5)):
                m = m.plus(Moments.of(rng.randrange(1, 100_000)))
            ls[(p, c)] = m
        records.append(Dependencies(start_of(r), start_of(r) + 3600_000_000,
                                    tuple(link(p, c, m) for (p, c), m in ls.items())))
    return records


def _oracle_sum(records):
    """The oracle's restatement of Dependencies.plus, reduceLeft over the records in order."""
    acc = None
    for d in records:
        od = ODeps(d.start_time, d.end_time,
                   tuple(OLink(l.parent.name, l.child.name, OMoments(*l.duration_moments)) for l in d.links))
        acc = od if acc is None else acc.plus(od)
    return acc


def _assert_sum(got, records):
    acc = _oracle_sum(records)
    assert (got.start_time, got.end_time) == (acc.start_time, acc.end_time)
    exp = {(l.parent, l.child): l.moments for l in acc.links}
    assert len(got.links) == len(exp)
    for l in got.links:
        assert _same_bits(l.duration_moments, exp[(l.parent.name, l.child.name)])


DAY = 86_400_000_000


def test_cassandra_rows_clobber_per_day_and_every_row_is_summed():
    """CassandraAggregates.scala:111-136: row key = start floored to the day, store() = removeRow +
    insert, so a second record of the same day replaces the first (CassandraAggregatesTest.scala
    :101-112 only checks that the store does not throw). getDependencies keeps a column unless its
    NAME -- the index 0 -- exceeds a bound in us (:58-61): any non-negative window returns every
    row, Monoid-summed in row order."""
    agg = GpuAggregates("cassandra", clock=lambda: NOW)
    records = _random_records(3, 6, lambda r: r * DAY + 7)
    for d in records:
        agg.storeDependencies(d)
    replaced = _random_records(4, 1, lambda r: 2 * DAY + 99)[0]  # same day as records[2]
    agg.storeDependencies(replaced)
    assert agg.count() == 6
    kept = records[:2] + [replaced] + records[3:]
    for window in ((0, 1), (5 * DAY, 6 * DAY), (None, None), (0, None), (10**15, 10**15 + 1)):
        _assert_sum(agg.getDependencies(*window), kept)
    assert agg.getDependencies(-1, None) == Dependencies.zero()  # 0 > -1: the column is filtered
    assert agg.getDependencies(0, -5) == Dependencies.zero()
    assert GpuAggregates("cassandra").getDependencies(0, 1) == Dependencies.zero()


def test_hbase_reverse_ms_keys_and_reversed_scan():
    """HBaseAggregates.scala:39-60: row key Long.MaxValue - start ms; getDependencies scans
    [MaxValue - start ms, MaxValue - end ms), i.e. records with end ms < start <= start ms, newest
    first. HBaseAggregatesSpec.scala:44-48: deps stored at 2 s come back from
    getDependencies(Some(100 s)) unchanged."""
    spec = Dependencies(2_000_000, 1_000_000_000, (link("HBase.Client", "HBase.RegionServer", Moments.of(1)),
                                                     link("HBase.RegionServer", "HBase.Master", Moments.of(2))))
    agg = GpuAggregates("hbase", clock=lambda: NOW)
    agg.storeDependencies(spec)
    assert agg.getDependencies(100_000_000) == spec
    records = _random_records(5, 6, lambda r: (r + 1) * 3600_000_000)
    agg = GpuAggregates("hbase", clock=lambda: NOW)
    for d in records:
        agg.storeDependencies(d)
    h = 3600_000_000
    # start bound 3.5 h, no end: records starting at <= 3.5 h, newest first
    _assert_sum(agg.getDependencies(3 * h + h // 2), records[:3][::-1])
    # start 5 h, end 2 h: (2 h, 5 h] -> records at 3, 4, 5 h, newest first
    _assert_sum(agg.getDependencies(5 * h, 2 * h), records[2:5][::-1])
    # the usual start < end window scans nothing
    assert agg.getDependencies(0, 10 * h) == Dependencies.zero()
    # start and end in the same millisecond: startRow == stopRow is HBase's get-scan (inclusive
    # stop row): exactly the record stored at that key, and nothing when no record is there
    _assert_sum(agg.getDependencies(4 * h, 4 * h + 999), [records[3]])
    assert agg.getDependencies(4 * h + 1000, 4 * h + 1000) == Dependencies.zero()
    # no start: from key 0 = every record, newest first
    _assert_sum(agg.getDependencies(None), records[::-1])
    # a second record of the same millisecond replaces the first
    again = _random_records(6, 1, lambda r: h + 250)[0]  # 1 h + 0.25 ms -> the same ms as records[0]
    agg.storeDependencies(again)
    assert agg.count() == 6
    _assert_sum(agg.getDependencies(h), [again])


def test_get_dependencies_capacity_error_is_reported():
    import ctypes as C

    L = _abi.lib()
    h = C.c_void_p()
    assert L.zk_store_create(0, C.byref(h)) == _abi.ZK_OK
    arr = (_abi.zk_dep_link * 2)()
    arr[0] = _abi.zk_dep_link(0, 1, _abi.zk_moments(1, 1.0, 0, 0, 0))
    arr[1] = _abi.zk_dep_link(1, 2, _abi.zk_moments(1, 2.0, 0, 0, 0))
    assert L.zk_store_put_dependencies(h, 0, 10, arr, 2) == _abi.ZK_OK
    n = C.c_uint64()
    s, e = C.c_int64(0), C.c_int64(10)
    assert L.zk_store_get_dependencies(h, C.byref(s), C.byref(e), 0, None, 0, C.byref(n), None, None) == 0
    assert n.value == 2
    out = (_abi.zk_dep_link * 1)()
    assert L.zk_store_get_dependencies(h, C.byref(s), C.byref(e), 0, out, 1, C.byref(n), None, None) == \
        _abi.ZK_ERR_CAPACITY
    assert b"capacity" in L.zk_store_last_error(h)
    assert L.zk_store_create(7, C.byref(h)) == _abi.ZK_ERR_INVALID_ARG
    assert L.zk_store_destroy(None) == _abi.ZK_ERR_INVALID_ARG


def test_concurrent_stores_are_serialised():
    agg = GpuAggregates("anorm", services=Dictionary(["a", "b"]), clock=lambda: NOW)

    def worker(i):
        for j in range(50):
            agg.storeDependencies(Dependencies(i * 1000 + j, i * 1000 + j + 1, (link("a", "b", Moments.of(j)),)))

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert agg.count() == 400
    assert len(agg.getDependencies(0, 10**9).links) == 400


# ---- top annotations (CassandraAggregatesTest.scala:57-123) ----------------------------------
def test_top_annotations_store_get_and_clobber():
    agg = GpuAggregates("cassandra")
    assert agg.getTopAnnotations("mockingbird") == []
    agg.storeTopAnnotations("mockingbird", ["finagle.retry", "finagle.timeout", "annotation1"])
    agg.storeTopKeyValueAnnotations("mockingbird", ["hi", "there"])
    assert agg.getTopAnnotations("mockingbird") == ["finagle.retry", "finagle.timeout", "annotation1"]
    assert agg.getTopKeyValueAnnotations("mockingbird") == ["hi", "there"]
    agg.storeTopAnnotations("mockingbird", ["a", "b"])  # clobber: removeRow then insert
    assert agg.getTopAnnotations("mockingbird") == ["a", "b"]
    assert agg.getTopKeyValueAnnotations("mockingbird") == ["hi", "there"]
    assert agg.getTopKeyValueAnnotations("other") == []
    agg.storeTopKeyValueAnnotations("mockingbird", [])
    assert agg.getTopKeyValueAnnotations("mockingbird") == []


def test_null_aggregates():
    n = NullAggregates()
    assert n.getDependencies(None) == Dependencies.zero()
    n.storeDependencies(Dependencies(0, 1, ()))
    assert n.getTopAnnotations("x") == [] and n.getTopKeyValueAnnotations("x") == []


# ---- the job's output record -----------------------------------------------------------------
def test_links_from_table_compacts_present_cells():
    from zipkin_amd.context import LinkTable

    S = 3
    names = Dictionary(["web", "api", "db"])
    m0 = np.zeros(9, np.uint64)
    ms = [np.zeros(9) for _ in range(4)]
    pr = np.zeros(9, np.uint8)
    for c, v in ((1, 5.0), (5, 7.5), (6, 1.0)):
        m0[c] = 2
        ms[0][c] = v
        pr[c] = 1
    got = links_from_table(LinkTable(S, m0, *ms, pr), names)
    assert [(l.parent.name, l.child.name, l.duration_moments.m0, l.duration_moments.m1) for l in got] == [
        ("web", "api", 2, 5.0), ("api", "db", 2, 7.5), ("db", "web", 2, 1.0)]


@pytest.mark.gpu
def test_gpu_job_stores_the_record_the_oracle_predicts(gpu):
    from oracle import oracle
    from zipkin_amd import tracegen_host
    from zipkin_amd.aggregates import ZipkinAggregateJob

    S = 57
    names = Dictionary([f"svc{i}" for i in range(S)])
    cols = tracegen_host(seed=5, num_traces=3000, max_depth=7, num_services=S)
    agg = GpuAggregates("anorm", services=names, clock=lambda: NOW)
    deps = ZipkinAggregateJob(names, aggregates=agg, clock=lambda: NOW).run(cols, S)
    ref = oracle.aggregate(cols, S).moments()
    assert deps is not None and deps.start_time == 0 and deps.end_time == NOW
    got = {(names.get(l.parent.name), names.get(l.child.name)): l.duration_moments for l in deps.links}
    assert set(got) == set(ref)
    for k, m in ref.items():
        assert tuple(got[k]) == tuple(m)
    back = agg.getDependencies(0, NOW)
    assert back.links == deps.links


@pytest.mark.gpu
def test_gpu_job_with_no_links_writes_nothing(gpu):
    from zipkin_amd import SpanColumns
    from zipkin_amd.aggregates import ZipkinAggregateJob

    names = Dictionary(["a", "b"])
    agg = GpuAggregates("anorm", services=names, clock=lambda: NOW)
    assert ZipkinAggregateJob(names, aggregates=agg).run(SpanColumns.empty(0), 2) is None
    assert agg.count() == 0


# ---- the Dependencies record on the wire (Cassandra column value) ------------------------------
def _fixture_deps():
    fx = json.loads((GOLD / "aggregates_sql.json").read_text())
    row = fx["dependencies"][0]
    links = tuple(link(l["parent"], l["child"], Moments(l["m0"], l["m1"], l["m2"], l["m3"], l["m4"]))
                  for l in fx["links"])
    return Dependencies(row["start_ts"], row["end_ts"], links)


def test_dependencies_thrift_is_byte_exact_and_round_trips():
    from tests import thriftenc as T
    from zipkin_amd.aggregates import dependencies_from_thrift, dependencies_to_thrift

    deps = _fixture_deps()
    raw = dependencies_to_thrift(deps)
    want = T.dependencies(deps.start_time, deps.end_time,
                          [(l.parent.name, l.child.name, tuple(l.duration_moments)) for l in deps.links])
    assert raw == want
    back = dependencies_from_thrift(raw)
    assert (back.start_time, back.end_time) == (deps.start_time, deps.end_time)
    assert back.links == deps.links  # same order, names and Moments
    assert all(_same_bits(a.duration_moments, b.duration_moments) for a, b in zip(back.links, deps.links))


def test_dependencies_thrift_edge_cases():
    from tests import thriftenc as T
    from zipkin_amd.aggregates import cassandra_row_key, dependencies_from_thrift, dependencies_to_thrift

    # empty record (the monoid zero's times), case-sensitive and empty names, extreme Moments
    zero = Dependencies(_abi.ZK_TIME_TOP, -2**63, ())
    assert dependencies_from_thrift(dependencies_to_thrift(zero)) == zero
    odd = Dependencies(5, 7, (link("", "a", Moments(1, -0.0, float("inf"), 1e-308, 5e-324)),
                              link("A", "a", Moments(2**62, 1.5, 2.5, -3.5, 4.5))))
    back = dependencies_from_thrift(dependencies_to_thrift(odd))
    assert [(l.parent.name, l.child.name) for l in back.links] == [("", "a"), ("A", "a")]
    assert all(_same_bits(a.duration_moments, b.duration_moments) for a, b in zip(back.links, odd.links))
    # fields a newer writer might add are skipped; absent fields keep thrift defaults
    raw = T.dependencies(1, 2, [("p", "c", (3, 1.0, 2.0, 3.0, 4.0))])
    extra = T._fh(T.T_STRING, 9) + T._str("future") + b"\0"
    got = dependencies_from_thrift(raw[:-1] + extra)
    assert got.links == (link("p", "c", Moments(3, 1.0, 2.0, 3.0, 4.0)),)
    assert dependencies_from_thrift(b"\0") == Dependencies(0, 0, ())
    for bad in (raw[:-3], raw[:20], b"\x0f\x00\x03\x0c\x7f\xff\xff\xff"):
        with pytest.raises(ZkError) as e:
            dependencies_from_thrift(bad)
        assert e.value.status == _abi.ZK_ERR_INVALID_SPAN
    # row key: startTime.floor(1.day)
    day = 86_400_000_000
    assert cassandra_row_key(0) == 0
    assert cassandra_row_key(NOW) == NOW // day * day
    assert cassandra_row_key(3 * day - 1) == 2 * day


def test_anorm_top_annotations_are_stubs():
    """AnormAggregates.scala:111-137: store* do nothing, get* return Seq.empty."""
    agg = GpuAggregates("anorm")
    agg.storeTopAnnotations("mockingbird", ["a"])
    agg.storeTopKeyValueAnnotations("mockingbird", ["k"])
    assert agg.getTopAnnotations("mockingbird") == [] and agg.getTopKeyValueAnnotations("mockingbird") == []


def test_hbase_top_annotations_one_family():
    """HBaseAggregates.scala:62-110: both store* write the top-annotation family (the newest list
    wins), getTopKeyValueAnnotations scans the key-value family and finds nothing, and
    getTopAnnotations' open-ended scan falls through to the next service id holding a list."""
    agg = GpuAggregates("hbase", services=Dictionary(["s0", "s1", "s2"]))
    agg.storeTopAnnotations("s1", ["a", "b"])
    assert agg.getTopAnnotations("s1") == ["a", "b"]
    assert agg.getTopKeyValueAnnotations("s1") == []
    agg.storeTopKeyValueAnnotations("s1", ["k1"])  # lands in the annotation family, newest
    assert agg.getTopAnnotations("s1") == ["k1"]
    assert agg.getTopAnnotations("s0") == ["k1"]  # no row for s0: the scan reaches s1's row
    assert agg.getTopAnnotations("s2") == []
