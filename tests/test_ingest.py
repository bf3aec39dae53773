"""Span ingest decoder (include/zkingest.h): stored fragment bytes -> columnar records + indexer items.

Pinned three ways: the reference's own base64 thrift fixtures (tests/golden/thrift_spans.json), an
independent Snappy implementation (pyarrow's libsnappy) for the codec, and the span-level oracle
(oracle/spans.py span_to_record / thrift_* validation) for every decoded field. Host-only: runs
without a GPU. The GPU test at the end feeds decoded bytes through the HIP job."""
import base64
import json
import random
from collections import Counter
from pathlib import Path

import numpy as np
import pytest

from oracle.spans import (CORE_ANNOTATIONS, UNKNOWN_SERVICE_NAME, Annotation, BinaryAnnotation, Endpoint, Span,
                          aggregate_job, span_to_record)
from tests import thriftenc as T
from tests.richgen import gen_traces
from zipkin_amd import ZkError, _abi
from zipkin_amd.ingest import SpanDecoder, hash_string, snappy_uncompress

COLS = ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags")
GOLDEN = json.loads((Path(__file__).parent / "golden" / "thrift_spans.json").read_text())


def records(cols):
    return [{k: int(getattr(cols, k)[i]) for k in COLS} for i in range(len(cols))]


def expected_records(spans):
    ids: dict = {}
    return [span_to_record(s, ids) for s in spans], ids


def encode_all(spans, snappy=True):
    return [T.snappy(T.span(s)) if snappy else T.span(s) for s in spans]


def expected_items(spans):
    """The span indexer (CassieSpanStore.scala:214-242) restated: only spans with annotations;
    one key-value item per binary annotation with a host; per distinct non-core annotation value
    the min annotation (Annotation.scala:36-38 truncated compare, first of equals), if it has a host."""
    kv, ann = [], []
    for s in spans:
        if not s.annotations:
            continue
        for b in s.binary_annotations:
            if b.host is not None:
                kv.append((b.host.service_name, b.key))
        groups: dict = {}
        for a in s.annotations:
            if a.value in CORE_ANNOTATIONS:
                continue
            m = groups.get(a.value)
            if m is None:
                groups[a.value] = a
            else:
                d = (m.timestamp - a.timestamp) & 0xFFFFFFFF
                if d >= 2**31:
                    d -= 2**32
                if d > 0:
                    groups[a.value] = a
        for a in groups.values():
            if a.host is not None:
                ann.append((a.host.service_name, a.value))
    return Counter(kv), Counter(ann)


# ---- the reference's fixtures -------------------------------------------------------------------
def test_encoder_is_byte_exact_with_reference_fixtures():
    g = GOLDEN["span"]
    s = Span(g["trace_id"], g["name"], g["id"], g["parent_id"], tuple(Annotation(t, v) for t, v in g["annotations"]))
    assert T.span(s) == base64.b64decode(GOLDEN["with_debug"])
    assert T.span(s, write_debug=False) == base64.b64decode(GOLDEN["without_debug"])


@pytest.mark.parametrize("key", ["with_debug", "without_debug"])
def test_decode_reference_fixtures(key):
    raw = base64.b64decode(GOLDEN[key])
    for snappy, blob in ((False, raw), (True, T.snappy(raw))):
        dec = SpanDecoder()
        cols, rej = dec.decode([blob], snappy=snappy)
        assert rej == 0 and records(cols) == [GOLDEN["record"]]
        assert dec.num_services == 0  # the annotation has no host


# ---- Snappy --------------------------------------------------------------------------------------
@pytest.mark.parametrize("kind", ["empty", "tiny", "random", "repetitive", "long_literal", "big"])
def test_snappy_against_libsnappy(kind):
    rnd = random.Random(7)
    data = {
        "empty": b"",
        "tiny": b"a",
        "random": bytes(rnd.getrandbits(8) for _ in range(5000)),
        "repetitive": b"".join(rnd.choice([b"zipkin", b"span", b"sr", b"ss", b"\x00" * 9]) for _ in range(20000)),
        "long_literal": bytes(rnd.getrandbits(8) for _ in range(70000)) + b"x" * 70000,
        "big": b"".join(T.span(s) for s in gen_traces(3, 300)),
    }[kind]
    assert snappy_uncompress(T.snappy(data)) == data


def test_snappy_hand_vectors():
    # varint length 5, literal tag (len-1)<<2, then a copy-1 (len 4, offset 1) of the last byte
    assert snappy_uncompress(b"\x05\x00a" + bytes([((4 - 4) << 2) | 1, 1])) == b"aaaaa"
    assert snappy_uncompress(b"\x03\x08abc") == b"abc"
    # copy-2 and copy-4 with offset 3, length 6 (overlapping copy)
    assert snappy_uncompress(b"\x09\x08abc" + bytes([(5 << 2) | 2, 3, 0])) == b"abcabcabc"
    assert snappy_uncompress(b"\x09\x08abc" + bytes([(5 << 2) | 3, 3, 0, 0, 0])) == b"abcabcabc"
    # literal length in one extra byte (tag 60)
    assert snappy_uncompress(bytes([100, 60 << 2, 99]) + b"q" * 100) == b"q" * 100


@pytest.mark.parametrize("bad", [b"", b"\x05", b"\x05\x10ab", b"\x05\x00a" + bytes([1, 2]), b"\x03\x00a" + bytes([1, 0]),
                                 b"\x80\x80\x80\x80\x80\x01", b"\x02\x08abc"])
def test_snappy_corrupt_is_an_error(bad):
    with pytest.raises(ZkError) as e:
        snappy_uncompress(bad)
    assert e.value.status == _abi.ZK_ERR_INVALID_SPAN


# ---- record parity with the span oracle ----------------------------------------------------------
@pytest.mark.parametrize("seed,anomalies,snappy", [(11, 0.0, True), (12, 0.4, True), (13, 0.4, False)])
def test_records_equal_span_oracle(seed, anomalies, snappy):
    spans = gen_traces(seed, 250, max_depth=5, anomalies=anomalies)
    want, ids = expected_records(spans)
    dec = SpanDecoder()
    cols, rej = dec.decode(encode_all(spans, snappy), snappy=snappy)
    assert rej == 0
    assert records(cols) == want
    assert dec.service_names() == list(ids)  # ids in order of first appearance


def test_decoder_keeps_its_dictionary_across_batches():
    spans = gen_traces(21, 120, anomalies=0.2)
    want, ids = expected_records(spans)
    dec = SpanDecoder()
    got = []
    for lo in range(0, len(spans), 37):
        cols, _ = dec.decode(encode_all(spans[lo:lo + 37]))
        got += records(cols)
    assert got == want and dec.service_names() == list(ids)
    assert dec.service_id(list(ids)[3]) == 3
    assert dec.service_id("a-new-service") == len(ids)


def test_edge_spans_decode_like_the_oracle():
    e1, e2 = Endpoint(1, 80, "alpha"), Endpoint(2, 81, "Alpha")  # names are case-sensitive
    spans = [
        Span(1, "", 10, None),                                                 # no annotations at all
        Span(1, "x", 11, 10, (Annotation(5, "cs", e1), Annotation(9, "cr", e1))),
        Span(1, "x", 11, 10, (Annotation(6, "sr", e2), Annotation(8, "ss", e2))),
        Span(-1, "x", -2, -3, (Annotation(2**62, "sr", None), Annotation(3, "cs", e1))),  # negative ids, host-less sr
        Span(2, "x", 20, None, tuple(Annotation(t, "sr", e1) for t in (7, 3, 9, 1))),     # 4 x sr saturates at 2
        Span(3, "x", 30, 30, (Annotation(4, "custom", e2), Annotation(1, "ss", None))),   # self-parent, no service
    ]
    want, ids = expected_records(spans)
    dec = SpanDecoder()
    cols, rej = dec.decode(encode_all(spans))
    assert rej == 0 and records(cols) == want and dec.service_names() == list(ids) == ["alpha", "Alpha"]


def test_missing_or_empty_service_name_is_unknown():
    # thrift.scala:36-43: a null or "" service_name becomes Endpoint.UnknownServiceName
    a = T._fh(T.T_I64, 1) + T._i64(5) + T._fh(T.T_STRING, 2) + T._str("sr")
    no_name = a + T._fh(T.T_STRUCT, 3) + T.endpoint(Endpoint(1, 2, ""), service_name=None) + b"\0"
    empty = a + T._fh(T.T_STRUCT, 3) + T.endpoint(Endpoint(1, 2, "")) + b"\0"
    for ann in (no_name, empty):
        body = T._fh(T.T_I64, 1) + T._i64(1) + T._fh(T.T_STRING, 3) + T._str("n") + T._fh(T.T_I64, 4) + T._i64(2)
        body += T._fh(T.T_LIST, 6) + bytes([T.T_STRUCT]) + (1).to_bytes(4, "big") + ann + b"\0"
        dec = SpanDecoder()
        cols, _ = dec.decode([T.snappy(body)])
        assert dec.service_names() == [UNKNOWN_SERVICE_NAME] and int(cols.service_id[0]) == 0
        assert int(cols.flags[0]) & _abi.ZK_F_SVC_SERVER


def test_unknown_fields_and_types_are_skipped():
    s = Span(9, "n", 8, 7, (Annotation(3, "sr", Endpoint(1, 2, "svc"), duration=44), Annotation(4, "ss", None)),
             (BinaryAnnotation("k", b"\x00\x01", "BYTES", Endpoint(1, 2, "svc")),))
    body = T.span(s)[:-1]
    # extra fields a newer writer could add: a map, a set of strings, a nested struct, a double
    extra = T._fh(13, 20) + bytes([T.T_STRING, T.T_I32]) + (2).to_bytes(4, "big")
    extra += T._str("a") + (1).to_bytes(4, "big") + T._str("b") + (2).to_bytes(4, "big")
    extra += T._fh(14, 21) + bytes([T.T_STRING]) + (1).to_bytes(4, "big") + T._str("zz")
    extra += T._fh(T.T_STRUCT, 22) + T._fh(4, 1) + b"\x40" + b"\0" * 7 + b"\0"
    extra += T._fh(4, 23) + b"\x3f\xf0" + b"\0" * 6
    want, _ = expected_records([s])
    cols, rej = SpanDecoder().decode([T.snappy(body + extra + b"\0")])
    assert rej == 0 and records(cols) == want


# ---- validation (thrift.scala) -------------------------------------------------------------------
def bad_spans():
    e = Endpoint(1, 2, "svc")
    ok = Span(5, "n", 50, None, (Annotation(10, "sr", e), Annotation(20, "ss", e)))
    return ok, [
        ("No name set in Span", T.span(ok, name=None)),
        ("Annotation must have a timestamp", T.span(Span(5, "n", 51, 50, (Annotation(0, "sr", e),)))),
        ("Annotation must have a timestamp", T.span(Span(5, "n", 52, 50, (Annotation(-7, "cs", e),)))),
        ("Annotation must have a value", T.span(Span(5, "n", 53, 50, (Annotation(3, "", e),)))),
        ("undecodable thrift span", T.span(ok)[:-9]),
    ]


def test_strict_rejects_like_the_reference():
    ok, bads = bad_spans()
    for why, blob in bads:
        dec = SpanDecoder()
        with pytest.raises(ZkError) as ex:
            dec.decode([T.snappy(T.span(ok)), T.snappy(blob)])
        assert ex.value.status == _abi.ZK_ERR_INVALID_SPAN and why in ex.value.message and "span 1" in ex.value.message


def test_lenient_skips_and_counts():
    ok, bads = bad_spans()
    blobs = [T.snappy(T.span(ok))] + [T.snappy(b) for _, b in bads] + [b"\x7f\x00garbage", T.snappy(T.span(ok))]
    want, _ = expected_records([ok, ok])
    cols, rej = SpanDecoder().decode(blobs, strict=False)
    assert rej == len(bads) + 1 and records(cols) == want


def test_fuzzed_bytes_never_crash():
    spans = gen_traces(5, 40)
    raw = [T.span(s) for s in spans]
    rnd = random.Random(99)
    blobs = []
    for r in raw:
        b = bytearray(r)
        for _ in range(rnd.randint(1, 6)):
            b[rnd.randrange(len(b))] = rnd.getrandbits(8)
        blobs.append(bytes(b[: rnd.randrange(1, len(b) + 1)] if rnd.random() < 0.3 else b))
    for snappy in (False, True):
        dec = SpanDecoder()
        cols, rej = dec.decode([T.snappy(b) if snappy else b for b in blobs], strict=False)
        assert len(cols) + rej == len(blobs)


@pytest.mark.parametrize("header", [b"\xff\xff\xff\xff\x0f", b"\x80\x80\x80\x10", b"\x81\x80\x80\x08\x00"])
def test_hostile_snappy_length_is_rejected_before_allocating(header):
    """A header announcing gigabytes (or more than the format can expand the payload to) is
    undecodable, without the decoder allocating it (zkingest.h ZK_INGEST_MAX_FRAGMENT)."""
    from zipkin_amd.ingest import snappy_uncompress

    blob = header + b"\x00a"
    with pytest.raises(ZkError) as e:
        snappy_uncompress(blob)
    assert e.value.status == _abi.ZK_ERR_INVALID_SPAN
    cols, rej = SpanDecoder().decode([blob, T.snappy(T.span(gen_traces(1, 1)[0]))], strict=False)
    assert rej == 1 and len(cols) == 1
    with pytest.raises(ZkError) as e:
        SpanDecoder().decode([blob], strict=True)
    assert e.value.status == _abi.ZK_ERR_INVALID_SPAN


def test_snappy_expansion_bound_admits_real_maximum():
    """The densest legal block (runs of 64-byte copies) still decodes under the expansion bound."""
    data = b"z" * 200_000
    assert snappy_roundtrip(data) == data


def snappy_roundtrip(data):
    from zipkin_amd.ingest import snappy_uncompress

    return snappy_uncompress(T.snappy(data))


def test_empty_batch_and_bad_arguments():
    cols, rej = SpanDecoder().decode([])
    assert len(cols) == 0 and rej == 0
    L = _abi.lib()
    assert L.zk_ingest_create(None) == _abi.ZK_ERR_INVALID_ARG
    dec = SpanDecoder()
    with pytest.raises(ZkError):
        dec.service_name(0)


# ---- indexer items -------------------------------------------------------------------------------
@pytest.mark.parametrize("seed", [41, 42])
def test_items_equal_the_indexer(seed):
    spans = gen_traces(seed, 150, anomalies=0.3)
    # add annotation groups whose min needs the truncated (timestamp diff).toInt compare
    e = Endpoint(3, 4, "lorem")
    spans.append(Span(77, "n", 1, None, (Annotation(2**32 + 10, "tick", None), Annotation(5, "tick", e),
                                          Annotation(7, "tock", e), Annotation(7, "tock", None),
                                          Annotation(9, "sr", e))))
    spans.append(Span(77, "n", 2, 1, (), (BinaryAnnotation("k", b"v", "String", e),)))  # no annotations: no items
    kv_want, ann_want = expected_items(spans)
    dec = SpanDecoder()
    cols, rej, (kv_s, kv_k), (an_s, an_v) = dec.decode(encode_all(spans), items=True)
    assert rej == 0
    names = dec.service_names()
    assert Counter((names[s], dec.string(int(h))) for s, h in zip(kv_s, kv_k)) == kv_want
    assert Counter((names[s], dec.string(int(h))) for s, h in zip(an_s, an_v)) == ann_want
    assert all(int(h) == hash_string(dec.string(int(h))) for h in kv_k[:50])


def test_items_capacity_error_still_writes_records():
    spans = gen_traces(43, 30)
    dec = SpanDecoder()
    with pytest.raises(ZkError) as ex:
        dec.decode(encode_all(spans), items=True, item_cap=3)
    assert ex.value.status == _abi.ZK_ERR_CAPACITY


def test_hash_string_is_stable():
    # FNV-1a 64 then the splitmix64 finalizer: fixed values (a change breaks persisted sketches)
    def ref(b: bytes) -> int:
        h = 0xCBF29CE484222325
        for x in b:
            h = ((h ^ x) * 0x100000001B3) & (2**64 - 1)
        h = ((h ^ (h >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        h = ((h ^ (h >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        return h ^ (h >> 31)

    for s in ["", "a", "http.uri", "Unknown service name", "ünïcode"]:
        assert hash_string(s) == ref(s.encode())


# ---- stored bytes -> dependencies on the GPU -----------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("seed,anomalies", [(51, 0.0), (52, 0.4)])
def test_stored_bytes_to_dependencies(gpu, seed, anomalies):
    from zipkin_amd import DepsContext

    spans = gen_traces(seed, 300, max_depth=5, anomalies=anomalies)
    dec = SpanDecoder()
    cols, rej = dec.decode(encode_all(spans))
    assert rej == 0
    names = dec.service_names()
    with DepsContext(len(names), strict=False) as ctx:
        ctx.accumulate(cols)
        got = ctx.finalize()
    ref = aggregate_job(spans, strict=False)
    gl = {(names[p], names[c]): tuple(m) for p, c, m in got.links()}
    want = {k: tuple(m) for k, m in ref.exact().items()}
    assert gl == want


@pytest.mark.gpu
def test_stored_span_job_end_to_end(gpu):
    """Stored bytes -> decoder -> device job + top-annotation sketches -> Aggregates store, against
    the span oracle (dependencies) and the count-min restatement fed the indexer items (tops)."""
    from oracle.kv import KvOracle
    from zipkin_amd.aggregates import GpuAggregates, StoredSpanJob

    spans = gen_traces(61, 400, max_depth=5, anomalies=0.3)
    by_trace: dict = {}
    for sp in spans:
        by_trace.setdefault(sp.trace_id, []).append(sp)
    traces = list(by_trace.values())
    batches = [encode_all([sp for t in traces[i:i + 90] for sp in t]) for i in range(0, len(traces), 90)]
    store = GpuAggregates("cassandra")  # per-service top lists (Anorm's are stubs)
    job = StoredSpanJob(strict=False, aggregates=store, top_k=5, clock=lambda: 10**15)
    deps = job.run(batches)
    ref = aggregate_job(spans, strict=False)
    got = {(l.parent.name, l.child.name): tuple(l.duration_moments) for l in deps.links}
    assert got == {k: tuple(m) for k, m in ref.exact().items()}
    assert job.stats["records"] == len(spans) and job.rejected == 0
    stored = store.getDependencies(0, 10**15)
    assert {(l.parent.name, l.child.name) for l in stored.links} == set(got)

    names = job.services
    S = len(names)
    strings = {}
    kvo, ano = KvOracle(S), KvOracle(S)
    kv_s, kv_k, an_s, an_v = [], [], [], []
    for sp in spans:  # the indexer items, in decode order (ids from the job's dictionary)
        if not sp.annotations:
            continue
        for b in sp.binary_annotations:
            if b.host is not None:
                kv_s.append(names.get(b.host.service_name))
                kv_k.append(hash_string(b.key))
                strings[kv_k[-1]] = b.key
        seen = {}
        for a in sp.annotations:
            if a.value in CORE_ANNOTATIONS:
                continue
            m = seen.get(a.value)
            if m is None or (((m.timestamp - a.timestamp) & 0xFFFFFFFF) ^ 0x80000000) - 0x80000000 > 0:
                seen[a.value] = a
        for a in seen.values():
            if a.host is not None:
                an_s.append(names.get(a.host.service_name))
                an_v.append(hash_string(a.value))
                strings[an_v[-1]] = a.value
    kvo.accumulate(np.array(kv_s, np.uint32), np.array(kv_k, np.uint64))
    ano.accumulate(np.array(an_s, np.uint32), np.array(an_v, np.uint64))
    for o, tops, getter in ((kvo, job.top_kv, store.getTopKeyValueAnnotations),
                            (ano, job.top_annotations, store.getTopAnnotations)):
        keys, _, cnt = o.topk_all(5)
        want = {names.name(s): [strings[int(h)] for h in keys[s][: cnt[s]]] for s in range(S) if cnt[s]}
        assert tops == want
        for svc, lst in want.items():
            assert getter(svc) == lst


# ---- the device decoder (zk_ingest_dev) against the host decoder ---------------------------------
def _named(cols, names):
    recs = records(cols)
    for r in recs:
        r["service"] = names[r.pop("service_id")] if r["flags"] & (_abi.ZK_F_SVC_SERVER | _abi.ZK_F_SVC_CLIENT) else None
    return recs


def _fuzz(blobs, seed):
    rnd = random.Random(seed)
    out = []
    for r in blobs:
        b = bytearray(r)
        for _ in range(rnd.randint(0, 4)):
            b[rnd.randrange(len(b))] = rnd.getrandbits(8)
        out.append(bytes(b[: rnd.randrange(1, len(b) + 1)] if rnd.random() < 0.2 else b))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("seed,anomalies,snappy,strict", [(71, 0.0, True, True), (72, 0.4, True, False),
                                                          (73, 0.4, False, False)])
def test_device_decoder_equals_host_decoder(gpu, seed, anomalies, snappy, strict):
    from zipkin_amd.ingest import DeviceSpanDecoder

    spans = gen_traces(seed, 300, max_depth=5, anomalies=anomalies)
    ok, bads = bad_spans()
    blobs = [T.span(s) for s in spans] + ([] if strict else [b for _, b in bads] + [T.span(ok)])
    blobs = [T.snappy(b) for b in blobs] if snappy else blobs
    hd = SpanDecoder()
    hcols, hrej = hd.decode(blobs, snappy=snappy, strict=strict)
    dd = DeviceSpanDecoder(64)
    dcols, drej = dd.decode(blobs, snappy=snappy, strict=strict)
    assert drej == hrej
    assert _named(dcols.to_host(), dd.service_names()) == _named(hcols, hd.service_names())
    assert sorted(dd.service_names()) == sorted(hd.service_names())


@pytest.mark.gpu
@pytest.mark.parametrize("snappy", [True, False])
def test_device_decoder_large_fragments_take_the_global_path(gpu, snappy):
    """Waves of 64 fragments whose bytes exceed the LDS staging (16 KiB in / 24 KiB out) are
    deferred to the global-memory decoder: mixed batches give the same records either way."""
    import dataclasses

    from zipkin_amd.ingest import DeviceSpanDecoder

    rnd = random.Random(77)
    spans = gen_traces(77, 300, max_depth=5, anomalies=0.2)
    out = []
    for k, s in enumerate(spans):
        if k % 97 == 5 or k % 89 == 7 or 640 <= k < 704:  # giants, near-budget ones, a run of mid-size ones
            size = 24000 if k % 97 == 5 else 18000 if k % 89 == 7 else 700
            pad = BinaryAnnotation("blob", bytes(rnd.getrandbits(8) for _ in range(size)), "BYTES", None)
            s = dataclasses.replace(s, binary_annotations=s.binary_annotations + (pad,))
        out.append(s)
    blobs = encode_all(out, snappy)
    hd = SpanDecoder()
    hcols, hrej = hd.decode(blobs, snappy=snappy, strict=False)
    dd = DeviceSpanDecoder(64)
    dcols, drej = dd.decode(blobs, snappy=snappy, strict=False)
    assert drej == hrej
    assert _named(dcols.to_host(), dd.service_names()) == _named(hcols, hd.service_names())


@pytest.mark.gpu
@pytest.mark.parametrize("scratch", [1, 200, 30000])
def test_device_decoder_scratch_exhaustion_decodes_again(gpu, scratch):
    """The Snappy scratch (deferred fragments' Spans, names of new services) is bump-allocated from
    one counter; a decoder created with a tiny one runs out, grows it and decodes the fragments that
    missed out again: records and rejections equal the host decoder's, batch after batch."""
    import dataclasses

    from zipkin_amd.ingest import DeviceSpanDecoder

    rnd = random.Random(79)
    hd = SpanDecoder()
    dd = DeviceSpanDecoder(256, scratch_bytes=scratch)
    for batch in range(3):
        spans = gen_traces(790 + batch, 200, max_depth=4, anomalies=0.3)
        out = []
        for k, s in enumerate(spans):
            if k % 53 == 3:  # deferred to the global path: needs scratch for its whole Span
                pad = BinaryAnnotation("blob", bytes(rnd.getrandbits(8) for _ in range(22000)), "BYTES", None)
                s = dataclasses.replace(s, binary_annotations=s.binary_annotations + (pad,))
            out.append(s)
        blobs = encode_all(out, True)
        hcols, hrej = hd.decode(blobs, snappy=True, strict=False)
        dcols, drej = dd.decode(blobs, snappy=True, strict=False)
        assert drej == hrej
        assert _named(dcols.to_host(), dd.service_names()) == _named(hcols, hd.service_names())


@pytest.mark.gpu
def test_device_decoder_names_around_the_inline_prefix(gpu):
    """The LDS decoder resolves a known name from the dictionary slot's first 16 bytes, then the
    arena for the rest: names of 0-40 bytes, exactly 16 and 17, and names sharing a 16-byte
    prefix, over several batches (each name resolved from the dictionary after its first batch)."""
    import dataclasses

    from zipkin_amd.ingest import DeviceSpanDecoder

    base = ["", "a", "svc-15-bytes-xx", "svc-16-bytes-xxx", "svc-16-bytes-xxxy", "svc-16-bytes-xxxz",
            "prefix-sixteen--" + "A" * 16, "prefix-sixteen--" + "A" * 15 + "B", "n" * 40, "é-ünïcode-名前"]
    rnd = random.Random(81)
    hd = SpanDecoder()
    dd = DeviceSpanDecoder(64)
    for batch in range(4):
        spans = gen_traces(810 + batch, 150, max_depth=4)
        out = []
        for s in spans:
            nm = rnd.choice(base)
            anns = tuple(dataclasses.replace(x, host=Endpoint(x.host.ipv4, x.host.port, nm)) if x.host else x
                         for x in s.annotations)
            out.append(dataclasses.replace(s, annotations=anns))
        blobs = encode_all(out, True)
        hcols, hrej = hd.decode(blobs, snappy=True, strict=False)
        dcols, drej = dd.decode(blobs, snappy=True, strict=False)
        assert drej == hrej
        assert _named(dcols.to_host(), dd.service_names()) == _named(hcols, hd.service_names())


def _snappy_runs_then_literals(data: bytes) -> bytes:
    """A legal Snappy block no standard compressor writes: runs of one byte as a literal plus
    64-byte copies (offset 1), every other byte as its own 1-byte literal. After a long run the
    output is far ahead of the input, and the literal tail then eats into that lead, so in-place
    decompression must stop before it overwrites input it has not read."""
    out = bytearray()
    n = len(data)
    while True:  # varint length
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            break
    i = 0
    while i < len(data):
        j = i
        while j < len(data) and data[j] == data[i]:
            j += 1
        out += bytes([0, data[i]])  # 1-byte literal
        run = j - i - 1
        while run >= 4:
            ln = min(64, run)
            out += bytes([((ln - 1) << 2) | 2, 1, 0])  # copy-2, offset 1
            run -= ln
        for _ in range(run):
            out += bytes([0, data[i]])
        i = j
    return bytes(out)


@pytest.mark.gpu
def test_device_decoder_unsafe_in_place_streams(gpu):
    from zipkin_amd.ingest import DeviceSpanDecoder

    spans = gen_traces(78, 120, max_depth=4)
    raw = []
    for k, s in enumerate(spans):
        if k % 3 == 0:  # a long run early in the span, then hundreds of single-byte literals
            run = BinaryAnnotation("fill", b"a" * (3000 + 50 * (k % 7)), "BYTES", None)
            s = Span(s.trace_id, s.name, s.id, s.parent_id, s.annotations, (run,) + s.binary_annotations, s.debug)
        raw.append(T.span(s))
    blobs = [_snappy_runs_then_literals(b) for b in raw]
    assert all(snappy_uncompress(c) == b for c, b in zip(blobs, raw))
    hd = SpanDecoder()
    hcols, hrej = hd.decode(blobs)
    dd = DeviceSpanDecoder(64)
    dcols, drej = dd.decode(blobs)
    assert drej == hrej == 0
    assert _named(dcols.to_host(), dd.service_names()) == _named(hcols, hd.service_names())


@pytest.mark.gpu
def test_device_decoder_strict_errors_and_fuzz(gpu):
    from zipkin_amd.ingest import DeviceSpanDecoder

    ok, bads = bad_spans()
    for why, blob in bads:
        dd = DeviceSpanDecoder(16)
        with pytest.raises(ZkError) as ex:
            dd.decode([T.snappy(T.span(ok)), T.snappy(blob)])
        assert ex.value.status == _abi.ZK_ERR_INVALID_SPAN and "span 1" in ex.value.message
    spans = gen_traces(74, 80)
    raw = [T.span(s) for s in spans]
    for snappy in (False, True):
        blobs = _fuzz([T.snappy(b) for b in raw] if snappy else raw, 5 + snappy)
        hd, dd = SpanDecoder(), DeviceSpanDecoder(4096)
        hcols, hrej = hd.decode(blobs, snappy=snappy, strict=False)
        dcols, drej = dd.decode(blobs, snappy=snappy, strict=False)
        assert dcols.n + drej == len(blobs)
        assert drej == hrej
        assert _named(dcols.to_host(), dd.service_names()) == _named(hcols, hd.service_names())
    # reference fixtures
    for key in ("with_debug", "without_debug"):
        cols, rej = DeviceSpanDecoder(4).decode([T.snappy(base64.b64decode(GOLDEN[key]))])
        assert rej == 0 and records(cols.to_host()) == [GOLDEN["record"]]


@pytest.mark.gpu
def test_device_decoder_dictionary_across_batches_and_capacity(gpu):
    from zipkin_amd.ingest import DeviceSpanDecoder

    spans = gen_traces(75, 200, anomalies=0.2)
    want, ids = expected_records(spans)
    names = list(ids)
    dd = DeviceSpanDecoder(len(names))
    got = []
    for lo in range(0, len(spans), 53):
        cols, _ = dd.decode(encode_all(spans[lo:lo + 53]))
        got += _named(cols.to_host(), dd.service_names())
    for r in want:
        r["service"] = names[r.pop("service_id")] if r["flags"] & 12 else None
    assert got == want and sorted(dd.service_names()) == sorted(names)
    small = DeviceSpanDecoder(3)
    with pytest.raises(ZkError) as ex:
        small.decode(encode_all(spans))
    assert ex.value.status == _abi.ZK_ERR_SERVICE_RANGE


@pytest.mark.gpu
def test_device_decoded_bytes_to_dependencies(gpu):
    from zipkin_amd import DepsContext
    from zipkin_amd.ingest import DeviceSpanDecoder

    spans = gen_traces(76, 400, max_depth=5, anomalies=0.3)
    dd = DeviceSpanDecoder(128)
    cols, rej = dd.decode(encode_all(spans))
    assert rej == 0
    names = dd.service_names()
    with DepsContext(len(names), strict=False) as ctx:
        ctx.accumulate(cols)
        got = ctx.finalize()
    ref = aggregate_job(spans, strict=False)
    assert {(names[p], names[c]): tuple(m) for p, c, m in got.links()} == {k: tuple(m) for k, m in ref.exact().items()}


# ---- the host decoder's threads ------------------------------------------------------------------
def _decode_both(blobs, **kw):
    one, many = SpanDecoder(), SpanDecoder()
    out = []
    for dec, flag in ((one, True), (many, False)):
        try:
            out.append(("ok", dec.decode(blobs, one_thread=flag, **kw), dec.service_names()))
        except ZkError as e:
            out.append(("err", (e.status, e.message), dec.service_names()))
    return out


@pytest.mark.parametrize("strict", [False, True])
def test_threaded_decode_equals_one_thread(strict):
    """A batch large enough for several decode threads (contiguous ranges, then one ordered commit)
    gives the records, items (in order), service ids, rejected count and first error of a one-thread
    decode -- with bad and undecodable fragments spread over every range."""
    spans = gen_traces(61, 1200, max_depth=5, anomalies=0.3)
    blobs = encode_all(spans)
    assert len(blobs) >= 8 * 2048, len(blobs)
    ok, bads = bad_spans()
    rnd = random.Random(61)
    for k in range(24):  # lenient: skipped and counted; strict: the first one fails the batch
        at = rnd.randrange(len(blobs)) if k else len(blobs) // 2 + 3
        blobs.insert(at, T.snappy(bads[k % len(bads)][1]) if k % 3 else b"\x7f\x00garbage")
    a, b = _decode_both(blobs, strict=strict, items=True)
    assert a[0] == b[0] == ("err" if strict else "ok")
    assert a[2] == b[2]  # the dictionary, ids in order of first appearance
    if strict:
        assert a[1] == b[1]
        return
    (ca, ra, kva, ana), (cb, rb, kvb, anb) = a[1], b[1]
    assert ra == rb == 24
    assert records(ca) == records(cb)
    for x, y in zip(kva + ana, kvb + anb):
        assert np.array_equal(x, y)


def test_threaded_decode_bad_offsets_and_item_overflow():
    spans = gen_traces(62, 1000, max_depth=5)
    blobs = encode_all(spans)
    a, b = _decode_both(blobs, items=True, item_cap=5000)
    assert a[0] == b[0] == "err" and a[1] == b[1] and a[1][0] == _abi.ZK_ERR_CAPACITY and a[2] == b[2]
    buf = np.frombuffer(b"".join(blobs), dtype=np.uint8)
    offs = np.zeros(len(blobs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(x) for x in blobs])
    offs[len(blobs) * 3 // 4] = offs[len(blobs) * 3 // 4 + 1] + 1  # not ascending, in a later range
    a, b = _decode_both((buf, offs), strict=False)
    assert a[0] == b[0] == "err" and a[1] == b[1] and a[1][0] == _abi.ZK_ERR_INVALID_ARG and a[2] == b[2]
