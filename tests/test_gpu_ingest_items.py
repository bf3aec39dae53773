"""The device decoder's span-indexer items (zk_ingest_dev_spans_items) against the host decoder's
(zk_ingest_spans with items), which tests/test_ingest.py pins to the indexer restated from
CassieSpanStore.scala:214-242. Items come in no particular order within a batch on the device, so a
batch's items are compared as multisets of (service name, string), the strings read back through
each decoder's hash -> string map. Covered: the canonical layout (LDS fast path), the generic walk
(anomalous layouts, deferred giants in global memory), item hosts that are not the fragment's own
service (known and new names, "" and absent names -> "Unknown service name"), the truncated
timestamp compare of Annotation.compare, lenient rejections and fuzzed bytes, the scratch running
out mid-batch (the failed attempt's items are not emitted twice), the captured-string set and the
extra-name list filling up inside one batch, and the capacity error."""
import dataclasses
import random
from collections import Counter

import pytest

from oracle.spans import UNKNOWN_SERVICE_NAME, Annotation, BinaryAnnotation, Endpoint, Span
from tests import thriftenc as T
from tests.richgen import gen_traces
from tests.test_ingest import _fuzz, _named, encode_all, expected_items
from zipkin_amd import ZkError, _abi
from zipkin_amd.ingest import SpanDecoder, hash_string

pytestmark = pytest.mark.gpu


def _host_items(hd, blobs, snappy=True, strict=False):
    cols, rej, (ks, kh), (as_, ah) = hd.decode(blobs, snappy=snappy, strict=strict, items=True)
    names = hd.service_names()
    kv = Counter((names[int(s)], hd.string(int(h))) for s, h in zip(ks, kh))
    an = Counter((names[int(s)], hd.string(int(h))) for s, h in zip(as_, ah))
    return cols, rej, kv, an


def _dev_items(dd, blobs, snappy=True, strict=False, **kw):
    cols, rej, (ks, kh), (as_, ah) = dd.decode(blobs, snappy=snappy, strict=strict, items=True, **kw)
    names = dd.service_names()
    ks, kh, as_, ah = (t.cpu().numpy() for t in (ks, kh, as_, ah))
    for h in list(kh[:64]) + list(ah[:64]):  # the device hash is zk_hash_string of the kept string
        assert hash_string(dd.string(int(h)).encode("utf-8", "surrogateescape")) == int(h) & (2**64 - 1)
    kv = Counter((names[int(s)], dd.string(int(h))) for s, h in zip(ks, kh))
    an = Counter((names[int(s)], dd.string(int(h))) for s, h in zip(as_, ah))
    return cols, rej, kv, an


def _unknown_named(c):
    """expected_items with "" host names as the decoders read them (thrift.scala:36-43)"""
    out = Counter()
    for (n, v), k in c.items():
        out[(n or UNKNOWN_SERVICE_NAME, v)] += k
    return out


def _odd_spans():
    """Item hosts that differ from the span's own service, new and known; the truncated compare."""
    e, f = Endpoint(3, 4, "lorem"), Endpoint(5, 6, "only-an-item-host")
    blank, unk = Endpoint(7, 8, ""), Endpoint(9, 1, "Unknown service name")
    return [
        Span(77, "n", 1, None, (Annotation(2**32 + 10, "tick", None), Annotation(5, "tick", e),
                                Annotation(7, "tock", e), Annotation(7, "tock", None), Annotation(9, "sr", e))),
        Span(77, "n", 2, 1, (), (BinaryAnnotation("k", b"v", "String", e),)),  # no annotations: no items
        Span(78, "m", 3, None, (Annotation(10, "cs", e), Annotation(11, "x", f), Annotation(12, "cr", e)),
             (BinaryAnnotation("key-f", b"v", "String", f), BinaryAnnotation("key-b", b"v", "String", blank),
              BinaryAnnotation("key-u", b"v", "String", unk), BinaryAnnotation("key-none", b"v", "String", None))),
        Span(79, "m", 4, 3, (Annotation(20, "sr", blank), Annotation(21, "y", blank), Annotation(22, "ss", blank)),
             (BinaryAnnotation("", b"", "String", f),)),
        Span(80, "m", 5, None, (Annotation(30, "z", unk), Annotation(31, "z", f), Annotation(29, "z", e))),
    ]


@pytest.mark.parametrize("seed,anomalies,snappy", [(101, 0.0, True), (102, 0.4, True), (103, 0.4, False)])
def test_device_items_equal_host_items(gpu, seed, anomalies, snappy):
    from zipkin_amd.ingest import DeviceSpanDecoder

    spans = gen_traces(seed, 300, max_depth=5, anomalies=anomalies) + _odd_spans()
    blobs = encode_all(spans, snappy)
    hcols, hrej, hkv, han = _host_items(SpanDecoder(), blobs, snappy)
    dd = DeviceSpanDecoder(256)
    dcols, drej, dkv, dan = _dev_items(dd, blobs, snappy)
    assert drej == hrej == 0
    assert (dkv, dan) == (hkv, han)
    assert (hkv, han) == tuple(_unknown_named(c) for c in expected_items(spans))
    assert sum(dkv.values()) > 100 and sum(dan.values()) > 20
    # the same batch again: every string and name is known now (one probe per item)
    _, _, dkv2, dan2 = _dev_items(dd, blobs, snappy)
    assert (dkv2, dan2) == (hkv, han)


def test_device_items_lenient_and_fuzzed(gpu):
    from zipkin_amd.ingest import DeviceSpanDecoder

    spans = gen_traces(104, 300, max_depth=5, anomalies=0.4) + _odd_spans()
    blobs = _fuzz(encode_all(spans), 104)
    hcols, hrej, hkv, han = _host_items(SpanDecoder(), blobs)
    dd = DeviceSpanDecoder(512)
    dcols, drej, dkv, dan = _dev_items(dd, blobs)
    assert drej == hrej
    assert (dkv, dan) == (hkv, han)


@pytest.mark.parametrize("scratch", [1, 200, 30000])
def test_device_items_survive_scratch_exhaustion(gpu, scratch):
    """Deferred giants need scratch for their whole Span and new strings need it for their copy: a
    tiny scratch runs out mid-batch, the failed fragments are decoded again, and the items their
    first attempt appended are passed over (skip counts), so each item is emitted once."""
    from zipkin_amd.ingest import DeviceSpanDecoder

    rnd = random.Random(105)
    hd, dd = SpanDecoder(), DeviceSpanDecoder(512, scratch_bytes=scratch)
    for batch in range(3):
        spans = gen_traces(1050 + batch, 200, max_depth=4, anomalies=0.3) + _odd_spans()
        out = []
        for k, s in enumerate(spans):
            if k % 53 == 3:
                pad = BinaryAnnotation("blob%d" % k, bytes(rnd.getrandbits(8) for _ in range(22000)), "BYTES",
                                       Endpoint(1, 2, "giant-host-%d" % (k % 3)))
                s = dataclasses.replace(s, binary_annotations=s.binary_annotations + (pad,))
            out.append(s)
        blobs = encode_all(out, True)
        hcols, hrej, hkv, han = _host_items(hd, blobs)
        dcols, drej, dkv, dan = _dev_items(dd, blobs)
        assert drej == hrej
        assert (dkv, dan) == (hkv, han)
        assert _named(dcols.to_host(), dd.service_names()) == _named(hcols, hd.service_names())


def test_device_items_string_set_and_extra_list_fill_up(gpu):
    """70k distinct keys in one batch (the captured-string set starts at 2^16 slots) and 5000 item
    hosts that are not yet service names (the extra-name list starts at 4096): both fill up inside
    the batch, grow, and the fragments that missed out are decoded again."""
    from zipkin_amd.ingest import DeviceSpanDecoder

    e = Endpoint(1, 2, "svc")
    spans = []
    for k in range(70_000):
        host = Endpoint(3, 4, "item-host-%d" % k) if k < 5000 else e
        spans.append(Span(1000 + k // 7, "op", k + 1, None, (Annotation(10 + k, "sr", e), Annotation(20 + k, "ss", e)),
                          (BinaryAnnotation("key-%d" % k, b"v", "String", host),)))
    blobs = encode_all(spans, True)
    hcols, hrej, hkv, han = _host_items(SpanDecoder(), blobs)
    dd = DeviceSpanDecoder(8192)
    dcols, drej, dkv, dan = _dev_items(dd, blobs)
    assert drej == hrej == 0
    assert dkv == hkv and len(dkv) == 70_000
    assert dan == han
    assert dd.num_services == 5001


def test_device_items_capacity_error_still_writes_records(gpu):
    from zipkin_amd.ingest import DeviceSpanDecoder

    spans = gen_traces(106, 40)
    blobs = encode_all(spans)
    dd = DeviceSpanDecoder(64)
    import numpy as np
    import torch

    offs = np.zeros(len(blobs) + 1, np.int64)
    offs[1:] = np.cumsum([len(b) for b in blobs])
    buf = torch.from_numpy(np.frombuffer(b"".join(blobs), np.uint8).copy()).cuda()
    off = torch.from_numpy(offs).cuda()
    ks = torch.empty(3, dtype=torch.int32, device="cuda")
    kh = torch.empty(3, dtype=torch.int64, device="cuda")
    from zipkin_amd.columns import DeviceColumns

    cols = DeviceColumns(len(blobs))
    import ctypes as C

    it = _abi.zk_ingest_items(ks.data_ptr(), kh.data_ptr(), 3, 0, None, None, 0, 0)
    nout, nrej = C.c_uint64(), C.c_uint64()
    st = _abi.lib().zk_ingest_dev_spans_items(dd._h, buf.data_ptr(), off.data_ptr(), len(blobs),
                                             _abi.ZK_CODEC_SNAPPY_THRIFT, 0, C.byref(cols.abi(len(blobs))),
                                             C.byref(nout), C.byref(nrej), C.byref(it))
    assert st == _abi.ZK_ERR_CAPACITY
    assert it.kv_n == 3 and it.ann_n == 0 and nout.value == len(blobs)
    hcols, _ = SpanDecoder().decode(blobs)
    cols.n = nout.value
    assert _named(cols.to_host(), dd.service_names())[0]["trace_id"] == int(hcols.trace_id[0])
    with pytest.raises(ZkError):
        dd.string(12345)
