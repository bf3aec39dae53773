"""Several stored batches in one device decode (zk_ingest_dev_spans_multi) against the same
fragments joined into ONE batch (zk_ingest_dev_spans / _items, which tests/test_ingest.py and
tests/test_gpu_ingest_items.py pin to the host decoder): records equal and in the same order, the
rejected count equal, the items equal as multisets. Batches are separate allocations at unrelated
addresses, some empty; covered: the canonical LDS path, anomalous layouts and giants (the global
decoder), lenient rejections and fuzzed bytes, the strict error, and a single non-empty batch."""
import dataclasses
import random

import numpy as np
import pytest

from oracle.spans import BinaryAnnotation
from tests.richgen import gen_traces
from tests.test_gpu_ingest_items import _odd_spans
from tests.test_ingest import _fuzz, _named, encode_all
from zipkin_amd import ZkError

pytestmark = pytest.mark.gpu


def _device_batches(blobs, cuts, order_seed):
    """blobs cut at `cuts` into (buf, offsets, n) device tensors, allocated in a shuffled order"""
    import torch

    bounds = [0] + list(cuts) + [len(blobs)]
    parts = [blobs[a:b] for a, b in zip(bounds, bounds[1:])]
    slots = [None] * len(parts)
    order = list(range(len(parts)))
    random.Random(order_seed).shuffle(order)
    keep = []
    for k in order:
        p = parts[k]
        off = np.zeros(len(p) + 1, np.int64)
        if p:
            off[1:] = np.cumsum([len(b) for b in p])
        raw = np.frombuffer(b"".join(p) or b"\0", dtype=np.uint8).copy()
        keep.append(torch.empty(random.Random(k).randrange(1, 4096), dtype=torch.uint8, device="cuda"))  # spread
        slots[k] = (torch.from_numpy(raw).cuda(), torch.from_numpy(off).cuda(), len(p))
    torch.cuda.synchronize()
    return slots


def _items(dd, ks, kh, as_, ah):
    from collections import Counter

    names = dd.service_names()
    ks, kh, as_, ah = (t.cpu().numpy() for t in (ks, kh, as_, ah))
    kv = Counter((names[int(s)], dd.string(int(h))) for s, h in zip(ks, kh))
    an = Counter((names[int(s)], dd.string(int(h))) for s, h in zip(as_, ah))
    return kv, an


def _check(blobs, cuts, snappy=True, strict=False, seed=0):
    from zipkin_amd.ingest import DeviceSpanDecoder

    one = DeviceSpanDecoder(256)
    c1, r1, (ks1, kh1), (as1, ah1) = one.decode(blobs, snappy=snappy, strict=strict, items=True)
    many = DeviceSpanDecoder(256)
    batches = _device_batches(blobs, cuts, seed)
    c2, r2, (ks2, kh2), (as2, ah2) = many.decode_device_many(batches, snappy=snappy, strict=strict, items=True)
    assert r2 == r1
    assert c2.n == c1.n
    assert _named(c2.to_host(), many.service_names()) == _named(c1.to_host(), one.service_names())
    assert _items(many, ks2, kh2, as2, ah2) == _items(one, ks1, kh1, as1, ah1)
    # without items: the same records
    c3, r3 = DeviceSpanDecoder(256).decode_device_many(batches, snappy=snappy, strict=strict)
    assert r3 == r1 and c3.n == c1.n
    return c1.n, r1


@pytest.mark.parametrize("seed,anomalies,snappy", [(301, 0.0, True), (302, 0.4, True), (303, 0.4, False)])
def test_multi_batch_decode_equals_one_joined_batch(gpu, seed, anomalies, snappy):
    spans = gen_traces(seed, 400, max_depth=5, anomalies=anomalies) + _odd_spans()
    blobs = encode_all(spans, snappy)
    rnd = random.Random(seed)
    cuts = sorted(rnd.sample(range(1, len(blobs)), 11))
    cuts = cuts[:3] + [cuts[3]] * 3 + cuts[4:]  # two empty batches in the middle
    n, rej = _check(blobs, [0] + cuts + [len(blobs)], snappy=snappy, seed=seed)  # empty first / last too
    assert n > 0 and rej == 0


def test_multi_batch_decode_lenient_fuzzed_and_giants(gpu):
    rnd = random.Random(305)
    spans = gen_traces(305, 300, max_depth=5, anomalies=0.3)
    out = []
    for k, s in enumerate(spans):
        if k % 53 == 5:  # giants: deferred to the global-memory decoder
            pad = BinaryAnnotation("blob", bytes(rnd.getrandbits(8) for _ in range(20000)), "BYTES", None)
            s = dataclasses.replace(s, binary_annotations=s.binary_annotations + (pad,))
        out.append(s)
    blobs = _fuzz(encode_all(out), 306)
    cuts = sorted(rnd.sample(range(1, len(blobs)), 25))
    n, rej = _check(blobs, cuts, seed=306)
    assert rej > 0 and n > 0


def test_multi_batch_strict_error_and_single_batch(gpu):
    from zipkin_amd.ingest import DeviceSpanDecoder

    spans = gen_traces(307, 200, max_depth=4)
    blobs = encode_all(spans)
    # one non-empty batch among empty ones: that batch's own decode
    _check(blobs, [0, 0, len(blobs), len(blobs)], seed=307)
    bad = blobs[:150] + [b"\x05\x00garbage"] + blobs[150:]
    with pytest.raises(ZkError) as e:
        DeviceSpanDecoder(256).decode_device_many(_device_batches(bad, [40, 120, 170], 308), strict=True)
    assert "span 150" in str(e.value)
    # no batches at all, and only empty ones
    dd = DeviceSpanDecoder(256)
    c, r = dd.decode_device_many([])
    assert c.n == 0 and r == 0
    c, r = dd.decode_device_many(_device_batches([], [], 309))
    assert c.n == 0 and r == 0
