"""Stored span fragments in bulk (test infrastructure): TraceGen records -> Snappy(TBinaryProtocol
Span) bytes, vectorised with numpy so that 1e7 fragments take seconds.

Every fragment has the layout of bench.py's ingest workload and of tests/thriftenc.py's `span`
(zipkinCore.thrift:50-58 in field order, as Scrooge writes it): traceId, name "rpc", id, [parentId],
three annotations -- the record's first core annotation (sr or cs) at first_ts, "custom.event" at
the midpoint, the second (ss or cr) at last_ts, each with the host {127.0.0.1:9410, "svc-NNNN"} --
one binary annotation http.uri="/api/v1" (type STRING, same host) and debug = false. Service names
are fixed-width and a root span's name is 11 bytes longer than a child's ("rpc:root-spans" vs "rpc",
the size of the parentId field it lacks), so every fragment has one length: the batch is an
(n, L) byte matrix, a template with its fields written in as columns. The Snappy block is one literal (a valid stream any decoder reads: varint length,
tag 61 with a 2-byte length, the bytes).

encode(cols) also returns the records the reference's thrift conversion gives back for those bytes
(thrift.scala:64-121 as restated in oracle/spans.py): the TraceGen record with its flags
normalised to what the fragment carries (one of each of its two core annotations, HAS_ANNOTATIONS,
HAS_PARENT, the service side), and the service names, so parity is checked by name against the
oracle over those records."""
from __future__ import annotations

import struct

import numpy as np

from zipkin_amd import _abi
from zipkin_amd.columns import SpanColumns

NAME_DIGITS = 4


def service_name(i: int) -> str:
    return f"svc-{i:0{NAME_DIGITS}d}"


def _fh(t, i):
    return struct.pack(">bh", t, i)


def _st(b):
    return struct.pack(">i", len(b)) + b


def _template(parent: bool):
    """(bytes, {field: [offsets]}) of one fragment body with zeroed fields."""
    pos = {}
    out = bytearray()

    def mark(name, width, placeholder=None):
        pos.setdefault(name, []).append(len(out))
        out.extend(placeholder if placeholder is not None else bytes(width))

    name = b"svc-" + b"0" * NAME_DIGITS

    def ep(fid):
        out.extend(_fh(12, fid) + _fh(8, 1) + struct.pack(">i", 0x7F000001) + _fh(6, 2) + struct.pack(">h", 9410))
        out.extend(_fh(11, 3) + struct.pack(">i", len(name)) + b"svc-")
        mark("digits", NAME_DIGITS)
        out.extend(b"\0")

    def ann(ts_field, value_field):
        out.extend(_fh(10, 1))
        mark(ts_field, 8)
        out.extend(_fh(11, 2) + struct.pack(">i", 2 if value_field else 12))
        if value_field:
            mark(value_field, 2)
        else:
            out.extend(b"custom.event")
        ep(3)
        out.extend(b"\0")

    out.extend(_fh(10, 1))
    mark("trace_id", 8)
    out.extend(_fh(11, 3) + _st(b"rpc" if parent else b"rpc:root-spans") + _fh(10, 4))
    mark("span_id", 8)
    if parent:
        out.extend(_fh(10, 5))
        mark("parent_id", 8)
    out.extend(_fh(15, 6) + struct.pack(">bi", 12, 3))
    ann("first", "core0")
    ann("mid", None)
    ann("last", "core1")
    out.extend(_fh(15, 8) + struct.pack(">bi", 12, 1) + _fh(11, 1) + _st(b"http.uri") + _fh(11, 2) + _st(b"/api/v1"))
    out.extend(_fh(8, 3) + struct.pack(">i", 6))
    ep(4)
    out.extend(b"\0")
    out.extend(_fh(2, 9) + b"\0" + b"\0")
    return bytes(out), pos


def _snappy_literal_header(n: int) -> bytes:
    v = bytearray()
    x = n
    while True:
        b = x & 0x7F
        x >>= 7
        v.append(b | (0x80 if x else 0))
        if not x:
            break
    return bytes(v) + bytes([61 << 2]) + struct.pack("<H", n - 1)


def encode(cols: SpanColumns):
    """-> (buf uint8, offsets uint64[n + 1], the records those bytes decode to)."""
    n = len(cols)
    f = cols.flags.astype(np.uint32)
    has_parent = (f & _abi.ZK_F_HAS_PARENT) != 0
    server = (f & _abi.ZK_F_SVC_SERVER) != 0
    svc = cols.service_id.astype(np.int64)
    assert svc.max(initial=0) < 10 ** NAME_DIGITS
    digits = np.stack([(svc // 10 ** (NAME_DIGITS - 1 - k)) % 10 + ord("0") for k in range(NAME_DIGITS)], 1)
    digits = digits.astype(np.uint8)
    first = cols.first_ts.astype(np.int64)
    last = cols.last_ts.astype(np.int64)
    mid = first + (last - first) // 2

    def be64(a):
        return np.ascontiguousarray(a).astype(">u8").view(np.uint8).reshape(-1, 8)

    fields = {"trace_id": be64(cols.trace_id), "span_id": be64(cols.span_id), "parent_id": be64(cols.parent_id),
              "first": be64(first.view(np.uint64)), "mid": be64(mid.view(np.uint64)),
              "last": be64(last.view(np.uint64))}
    core0 = np.where(server[:, None], np.frombuffer(b"sr", np.uint8), np.frombuffer(b"cs", np.uint8))
    core1 = np.where(server[:, None], np.frombuffer(b"ss", np.uint8), np.frombuffer(b"cr", np.uint8))
    fields["core0"], fields["core1"] = core0.astype(np.uint8), core1.astype(np.uint8)
    tpl = {}
    for parent in (False, True):
        body, pos = _template(parent)
        hdr = _snappy_literal_header(len(body))
        tpl[parent] = (np.frombuffer(hdr + body, np.uint8), {k: [len(hdr) + o for o in v] for k, v in pos.items()})
    L = len(tpl[True][0])
    assert len(tpl[False][0]) == L
    mat = np.empty((n, L), np.uint8)
    mat[:] = tpl[False][0]
    diff = int(np.flatnonzero(tpl[False][0] != tpl[True][0]).max()) + 1  # the layouts agree after this
    mat[has_parent, :diff] = tpl[True][0][:diff]
    for name in set(tpl[False][1]) | set(tpl[True][1]):
        src = digits if name == "digits" else fields[name]
        a, b = tpl[False][1].get(name), tpl[True][1].get(name)
        if a == b:  # the same place in both layouts: every record at once
            for o in a:
                mat[:, o:o + src.shape[1]] = src
            continue
        for offs, rows in ((a, ~has_parent), (b, has_parent)):
            for o in offs or ():
                mat[rows, o:o + src.shape[1]] = src[rows]
    buf = mat.reshape(-1)
    offsets = np.arange(n + 1, dtype=np.uint64) * np.uint64(L)
    exp = cols.take(np.arange(n))
    ef = _abi.ZK_F_HAS_ANNOTATIONS | np.where(has_parent, _abi.ZK_F_HAS_PARENT, 0)
    ef = ef | np.where(server, _abi.ZK_F_SVC_SERVER | (1 << _abi.ZK_F_SR_SHIFT) | (1 << _abi.ZK_F_SS_SHIFT),
                       _abi.ZK_F_SVC_CLIENT | (1 << _abi.ZK_F_CS_SHIFT) | (1 << _abi.ZK_F_CR_SHIFT))
    exp.flags[:] = ef.astype(exp.flags.dtype)
    exp.parent_id[:] = np.where(has_parent, cols.parent_id, 0).astype(exp.parent_id.dtype)
    return buf, offsets, exp


def batches(buf, offsets, cuts):
    """The packed form cut at record indices `cuts` (sorted): [(buf, offsets)] per batch."""
    out = []
    bounds = [0, *cuts, len(offsets) - 1]
    for a, b in zip(bounds[:-1], bounds[1:]):
        lo, hi = int(offsets[a]), int(offsets[b])
        out.append((buf[lo:hi], (offsets[a:b + 1] - offsets[a]).astype(np.uint64)))
    return out
