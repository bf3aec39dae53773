"""Pin the CPU oracle to the reference's own tests and data (tests/golden/*.json).

Each case reads like the reference test it comes from (file:line in the fixture)."""
import json
import math
from pathlib import Path

import pytest

from oracle.moments import Moments, algebird_fold, algebird_plus, exact_moments, moments_close
from oracle.spans import (
    Annotation,
    Dependencies,
    DependencyLink,
    Endpoint,
    NoServiceNameError,
    Span,
    aggregate_job,
    merge_dependency_links,
    thrift_annotation,
    thrift_endpoint,
    thrift_span,
)

GOLD = Path(__file__).resolve().parent / "golden"
KATS = json.loads((GOLD / "reference_kats.json").read_text())


def _ann(a):
    ts, value, host = a[0], a[1], (a[2] if len(a) > 2 else None)
    return Annotation(ts, value, Endpoint(*host) if host else None)


def _span(d):
    return Span(d["trace_id"], d["name"], d["id"], d["parent_id"], tuple(_ann(a) for a in d["annotations"]), (), d["debug"])


def test_merge_two_span_parts():  # SpanTest.scala:59-68
    k = KATS["span_merge"]
    assert _span(k["span1"]).merge_span(_span(k["span2"])) == _span(k["expected"])


def test_merge_unknown_name():  # SpanTest.scala:70-76
    a, b = (Span(1, n, 2, None) for n in KATS["span_merge_unknown"]["names"])
    assert a.merge_span(b).name == "get" and b.merge_span(a).name == "get"


def test_first_last_duration_and_service_names():  # SpanTest.scala:47-51,78-93
    k = KATS["first_last_duration"]
    anns = tuple(_ann(a) for a in k["annotations"])
    s = Span(12345, "methodcall", 666, None, anns)
    assert s.first_annotation == anns[k["first"]]
    assert s.last_annotation == anns[k["last"]]
    assert s.duration == k["duration"]
    assert sorted(s.service_names) == k["service_names"]  # lower-cased
    assert s.service_name is None  # no core annotation carries a host


def test_no_annotations_no_duration():  # SpanTest.scala:95-98
    assert Span(1, "n", 2, None).duration is None


def test_validate_span():  # SpanTest.scala:100-113
    k = KATS["validate"]
    assert Span(1, "i", 123, None, tuple(Annotation(t, v) for t, v in k["valid"])).is_valid
    assert not Span(1, "i", 123, None, tuple(Annotation(t, v) for t, v in k["invalid"])).is_valid


def test_not_client_side():  # SpanTest.scala:86-89
    s = Span(1, "n", 2, None, tuple(Annotation(t, v) for t, v in KATS["not_client_side"]["annotations"]))
    assert not s.is_client_side()


def test_dependency_link_plus_and_assert():  # DependenciesTest.scala:42-54
    links = [DependencyLink(p, c, Moments.of(v)) for p, c, v in KATS["dependency_link_plus"]["links"]]
    d1, d2, d3 = links
    assert d1.plus(d2) == DependencyLink("tfe", "mobileweb", algebird_plus(d1.moments, d2.moments))
    with pytest.raises(AssertionError):
        d1.plus(d3)


def test_dependencies_monoid():  # DependenciesTest.scala:57-81
    k = KATS["dependencies_monoid"]

    def deps(d):
        return Dependencies(d["start_s"] * 10**6, d["end_s"] * 10**6,
                            tuple(DependencyLink(p, c, Moments.of(v)) for p, c, v in d["links"]))

    deps1, deps2 = deps(k["deps1"]), deps(k["deps2"])
    assert deps1.plus(Dependencies.zero()) == Dependencies(deps1.start_time, deps1.end_time, deps1.links)
    r = deps1.plus(deps2)
    assert r.start_time == k["expected_start_s"] * 10**6 and r.end_time == k["expected_end_s"] * 10**6
    got = sorted((l.parent, l.child, l.moments) for l in r.links)
    want = sorted((p, c, algebird_fold(vs)) for p, c, vs in k["expected_links"])
    assert got == want
    assert sorted(merge_dependency_links(list(deps1.links) + list(deps2.links)), key=lambda l: (l.parent, l.child)) == \
        sorted(r.links, key=lambda l: (l.parent, l.child))


def test_services_case_sensitive():  # DependenciesTest.scala:28-40
    k = KATS["services_case_sensitive"]
    assert all(a == b for a, b in k["equal"]) and all(a != b for a, b in k["different"])


def test_thrift_ingest_validation():  # thrift.scala:36-45,64-75,99-121; ThriftConversionsTest.scala:55-81
    for v in KATS["thrift_unknown_service"]["input"]:
        assert thrift_endpoint(1, 2, v).service_name == KATS["thrift_unknown_service"]["expected"]
    with pytest.raises(ValueError):
        thrift_annotation(0, "cs")
    with pytest.raises(ValueError):
        thrift_annotation(5, "")
    with pytest.raises(Exception):
        thrift_span(1, None, 2, None)
    s = thrift_span(1, "n", 2, None, None, None)
    assert s.annotations == () and s.binary_annotations == ()


def test_moments_kats_exact_and_fold():
    cases = json.loads((GOLD / "moments_kats.json").read_text())["cases"]
    for c in cases:
        vs = c["values"]
        assert list(exact_moments(vs)) == c["exact"]
        assert list(algebird_fold(float(v) for v in vs)) == c["algebird_fold"]
        assert moments_close(Moments(*c["exact"]), Moments(*c["algebird_fold"]))
    # the DependenciesTest pair and the {1,2,3,4,10} case are exactly representable
    assert list(exact_moments([2, 4])) == [2, 3.0, 2.0, 0.0, 2.0]
    assert list(exact_moments([1, 2, 3, 4, 10])) == [5, 4.0, 50.0, 180.0, 1394.0]


def test_moment_accessors_match_reference_js():
    """Accessors of oracle Moments == the reference's own momentAnnotations.js run by node."""
    d = json.loads((GOLD / "moment_accessors.json").read_text())
    for m, ref in zip(d["inputs"], d["outputs"]):
        mm = Moments(m["m0"], m["m1"], m["m2"], m["m3"], m["m4"])
        assert mm.count == ref["count"] and mm.mean == ref["mean"]
        assert math.isclose(mm.variance, ref["variance"], rel_tol=1e-15)
        assert math.isclose(mm.stddev, ref["stddev"], rel_tol=1e-15)
        if m["m2"] > 0:
            assert math.isclose(mm.skewness, ref["skewness"], rel_tol=1e-12)
            assert math.isclose(mm.kurtosis, ref["kurtosis"], rel_tol=1e-12, abs_tol=1e-12)
        else:
            assert ref["skewness"] is None and ref["kurtosis"] is None  # NaN in JSON


def test_aggregates_sql_fixture_is_consistent():
    """The 150 stored links of aggregates.sql are valid Moments (count >= 1, m2, m4 >= 0)."""
    d = json.loads((GOLD / "aggregates_sql.json").read_text())
    assert len(d["links"]) == 150 and d["dependencies"][0]["start_ts"] == 0
    for l in d["links"]:
        assert l["m0"] >= 1 and l["m2"] >= 0 and l["m4"] >= 0
        if l["m0"] == 1:
            assert l["m2"] == 0 and l["m3"] == 0 and l["m4"] == 0


@pytest.mark.parametrize("name", sorted(json.loads((GOLD / "job_kats.json").read_text())["cases"]))
def test_job_kats(name):
    case = json.loads((GOLD / "job_kats.json").read_text())["cases"][name]
    spans = [
        Span(s["trace_id"], s["name"], s["id"], s["parent_id"],
             tuple(Annotation(t, v, Endpoint(1, 2, h) if h else None) for t, v, h in s["annotations"]))
        for s in case["spans"]
    ]
    r = aggregate_job(spans, strict=False)
    got = [{"parent": k[0], "child": k[1], "durations": v, "exact": list(exact_moments(v))}
           for k, v in sorted(r.durations.items())]
    assert got == case["links"] and r.no_service == case["no_service"]
    if case["no_service"]:
        with pytest.raises(NoServiceNameError):  # the reference job fails on None.get
            aggregate_job(spans, strict=True)
