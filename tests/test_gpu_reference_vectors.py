"""Every reference-held vector of the dependency path, routed through the HIP path.

The job itself has no tests and no runnable build in the reference, so these
are the strongest pins available: the hand-built job KATs (tests/golden/job_kats.json, whose
expected links the CPU restatement reproduces in tests/test_oracle_kats.py), the SpanTest KATs
(zipkin-common/src/test/scala/com/twitter/zipkin/common/SpanTest.scala:59-113, via
tests/golden/reference_kats.json) and the reference's base64 thrift Span fixtures
(ScribeSpanReceiverTest.scala:37, ScribeFilterSpec.scala:36, tests/golden/thrift_spans.json).
Each goes through the device twice: as 48-B records (span_to_record, the ingest contract) and as
stored fragment bytes (thrift + Snappy) decoded by the DEVICE decoder straight into the join."""
import base64
import json
from pathlib import Path

import pytest

from oracle.moments import exact_moments
from oracle.spans import Annotation, Endpoint, Span, span_to_record
from tests import thriftenc as T
from zipkin_amd import DepsContext, SpanColumns, ZkError, _abi
from zipkin_amd.columns import COLUMNS

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).resolve().parent / "golden"
JOB = json.loads((GOLD / "job_kats.json").read_text())["cases"]
KATS = json.loads((GOLD / "reference_kats.json").read_text())
THRIFT = json.loads((GOLD / "thrift_spans.json").read_text())


def kat_spans(case):
    return [Span(s["trace_id"], s["name"], s["id"], s["parent_id"],
                 tuple(Annotation(t, v, Endpoint(1, 2, h) if h else None) for t, v, h in s["annotations"]))
            for s in case["spans"]]


def records(spans):
    ids: dict = {}
    recs = [span_to_record(s, ids) for s in spans]
    cols = SpanColumns.empty(len(recs))
    for k, _ in COLUMNS:
        getattr(cols, k)[:] = [r[k] for r in recs]
    return cols, {v: k for k, v in ids.items()}


def device_decoded(spans):
    """thrift + Snappy bytes of every fragment -> device decoder -> device columns + names."""
    from zipkin_amd.ingest import DeviceSpanDecoder

    dd = DeviceSpanDecoder(64)
    cols, rej = dd.decode([T.snappy(T.span(s)) for s in spans])
    assert rej == 0
    return cols, dd.service_names()


def job_links(cols, names, *, strict=False, device_cols=False):
    S = max(1, len(names))
    with DepsContext(S, strict=strict) as ctx:
        ctx.accumulate(cols, clustered=False)
        got = ctx.finalize()
        st = ctx.stats()
    out = [{"parent": names[p], "child": names[c], "exact": list(m)} for p, c, m in got.links()]
    return sorted(out, key=lambda d: (d["parent"], d["child"])), st


def expected(case):
    return sorted(({"parent": l["parent"], "child": l["child"], "exact": l["exact"]} for l in case["links"]),
                  key=lambda d: (d["parent"], d["child"]))


@pytest.mark.parametrize("name", sorted(JOB))
@pytest.mark.parametrize("path", ["records", "device_decoder"])
def test_job_kats_through_the_device(gpu, name, path):
    case = JOB[name]
    spans = kat_spans(case)
    cols, names = records(spans) if path == "records" else device_decoded(spans)
    if path == "records":
        names = [names[i] for i in range(len(names))]
    got, st = job_links(cols, names)
    assert got == expected(case), name
    assert st["no_service"] == case["no_service"] and st["ambiguous"] == 0
    # the durations behind each link are exact: m1 of a single observation is the duration itself
    for l in case["links"]:
        assert list(exact_moments(l["durations"])) == l["exact"]
    if case["no_service"] and spans:  # the reference job fails on None.get (ZipkinAggregateJob.scala:36-37)
        with pytest.raises(ZkError) as e:
            job_links(cols, names, strict=True)
        assert e.value.status == _abi.ZK_ERR_NO_SERVICE


def _host(svc):
    return Endpoint(1, 2, svc)


def _root(tid):
    return Span(tid, "root", 1, None, (Annotation(1, "sr", _host("root")), Annotation(100, "ss", _host("root"))))


def test_spantest_validate_kat_through_the_device(gpu):
    """SpanTest.scala:100-113: a span with cs twice is invalid, so it never joins its parent; the
    valid span of the same KAT joins with duration last - first = 4 - 1."""
    k = KATS["validate"]
    for anns, want in ((k["valid"], [("root", "child", [1, 3.0, 0.0, 0.0, 0.0])]), (k["invalid"], [])):
        child = Span(7, "i", 123, 1, tuple(Annotation(t, v, _host("child")) for t, v in anns))
        for path in ("records", "device_decoder"):
            spans = [_root(7), child]
            cols, names = records(spans) if path == "records" else device_decoded(spans)
            names = [names[i] for i in range(len(names))]
            got, st = job_links(cols, names)
            assert [(g["parent"], g["child"], g["exact"]) for g in got] == want
            assert st["invalid_spans"] == (0 if want else 1)


def test_spantest_merge_and_duration_kats_through_the_device(gpu):
    """SpanTest.scala:59-68 (two parts of span 666 merge into one span) and :78-93 (first = ts 1,
    last = ts 3, duration 2): the KAT's parts, with a core annotation added at the KAT's own
    timestamps so the merged span has a service and joins a parent."""
    m = KATS["span_merge"]
    s1, s2 = m["span1"], m["span2"]
    p1 = Span(s1["trace_id"], s1["name"], s1["id"], 1,
              tuple(Annotation(a[0], "cs", _host("svc")) for a in s1["annotations"]))
    p2 = Span(s2["trace_id"], s2["name"], s2["id"], 1,
              tuple(Annotation(a[0], "cr", _host("svc")) for a in s2["annotations"]))
    spans = [_root(s1["trace_id"]), p1, p2]
    for path in ("records", "device_decoder"):
        cols, names = records(spans) if path == "records" else device_decoded(spans)
        names = [names[i] for i in range(len(names))]
        got, st = job_links(cols, names)
        assert st["merged_spans"] == 2 and st["records"] == 3  # root + the merged span 666
        assert [(g["parent"], g["child"], g["exact"][:2]) for g in got] == [("root", "svc", [1, 1.0])]
    f = KATS["first_last_duration"]
    child = Span(12345, "methodcall", 666, 1,
                 tuple(Annotation(a[0], ("sr", "cs", "ss")[i], _host("svc")) for i, a in enumerate(f["annotations"])))
    for path in ("records", "device_decoder"):
        spans = [_root(12345), child]
        cols, names = records(spans) if path == "records" else device_decoded(spans)
        names = [names[i] for i in range(len(names))]
        got, _ = job_links(cols, names)
        assert got[0]["exact"][1] == float(f["duration"])


@pytest.mark.parametrize("key", ["with_debug", "without_debug"])
def test_reference_thrift_fixtures_through_the_device(gpu, key):
    """The reference's own stored Span bytes -> device decoder -> the fixture's record -> join."""
    from zipkin_amd.ingest import DeviceSpanDecoder

    raw = base64.b64decode(THRIFT[key])
    dd = DeviceSpanDecoder(8)
    for blob, snappy in ((raw, False), (T.snappy(raw), True)):
        cols, rej = dd.decode([blob], snappy=snappy)
        assert rej == 0 and cols.n == 1
        host = cols.to_host()
        for k, v in THRIFT["record"].items():
            assert int(getattr(host, k)[0]) == v, k
        with DepsContext(max(1, dd.num_services)) as ctx:
            ctx.accumulate(cols, clustered=False)
            got = ctx.finalize()
            st = ctx.stats()
        assert got.present.sum() == 0 and st["merged_spans"] == 1 and st["valid_spans"] == 1
