"""TBinaryProtocol encoder for the zipkinCore.thrift Span (zipkin-thrift/.../zipkinCore.thrift:27-58),
written the way Scrooge's generated `Span.encode` writes it (fields in id order, optional fields only
when set, `debug` always since it has a default). Test infrastructure only: it produces the stored
fragment bytes the ingest decoder (include/zkingest.h) reads. Pinned byte-exact against the
reference's own base64 fixtures (tests/test_ingest.py)."""
from __future__ import annotations

import struct
from typing import Optional

from oracle.spans import Annotation, BinaryAnnotation, Endpoint, Span

T_STOP, T_BOOL, T_I16, T_I32, T_I64, T_STRING, T_STRUCT, T_LIST = 0, 2, 6, 8, 10, 11, 12, 15
ANNOTATION_TYPES = {"BOOL": 0, "BYTES": 1, "I16": 2, "I32": 3, "I64": 4, "DOUBLE": 5, "String": 6, "STRING": 6}


def _fh(t: int, fid: int) -> bytes:
    return struct.pack(">bh", t, fid)


def _str(s) -> bytes:
    b = s.encode() if isinstance(s, str) else bytes(s)
    return struct.pack(">i", len(b)) + b


def _i64(v: int) -> bytes:
    return struct.pack(">q", ((v + 2**63) % 2**64) - 2**63)


def endpoint(e: Endpoint, service_name: Optional[str] = "__from_e__") -> bytes:
    name = e.service_name if service_name == "__from_e__" else service_name
    out = _fh(T_I32, 1) + struct.pack(">i", ((e.ipv4 + 2**31) % 2**32) - 2**31)
    out += _fh(T_I16, 2) + struct.pack(">h", ((e.port + 2**15) % 2**16) - 2**15)
    if name is not None:
        out += _fh(T_STRING, 3) + _str(name)
    return out + bytes([T_STOP])


def annotation(a: Annotation, value: Optional[str] = "__from_a__") -> bytes:
    v = a.value if value == "__from_a__" else value
    out = _fh(T_I64, 1) + _i64(a.timestamp)
    if v is not None:
        out += _fh(T_STRING, 2) + _str(v)
    if a.host is not None:
        out += _fh(T_STRUCT, 3) + endpoint(a.host)
    if a.duration is not None:
        out += _fh(T_I32, 4) + struct.pack(">i", a.duration)
    return out + bytes([T_STOP])


def binary_annotation(b: BinaryAnnotation) -> bytes:
    out = _fh(T_STRING, 1) + _str(b.key) + _fh(T_STRING, 2) + _str(b.value)
    out += _fh(T_I32, 3) + struct.pack(">i", ANNOTATION_TYPES[b.annotation_type])
    if b.host is not None:
        out += _fh(T_STRUCT, 4) + endpoint(b.host)
    return out + bytes([T_STOP])


def span(s: Span, *, name: Optional[str] = "__from_s__", write_debug: bool = True,
         binary_annotations_field: bool = True) -> bytes:
    nm = s.name if name == "__from_s__" else name
    out = _fh(T_I64, 1) + _i64(s.trace_id)
    if nm is not None:
        out += _fh(T_STRING, 3) + _str(nm)
    out += _fh(T_I64, 4) + _i64(s.id)
    if s.parent_id is not None:
        out += _fh(T_I64, 5) + _i64(s.parent_id)
    out += _fh(T_LIST, 6) + struct.pack(">bi", T_STRUCT, len(s.annotations))
    out += b"".join(annotation(a) for a in s.annotations)
    if binary_annotations_field:
        out += _fh(T_LIST, 8) + struct.pack(">bi", T_STRUCT, len(s.binary_annotations))
        out += b"".join(binary_annotation(b) for b in s.binary_annotations)
    if write_debug:
        out += _fh(T_BOOL, 9) + bytes([1 if s.debug else 0])
    return out + bytes([T_STOP])


def dependencies(start_time: int, end_time: int, links) -> bytes:
    """thriftscala.Dependencies (zipkinDependencies.thrift:24-43); links = [(parent, child,
    (m0, m1, m2, m3, m4))]. Scrooge writes every field of these structs (none is optional)."""
    out = _fh(T_I64, 1) + _i64(start_time) + _fh(T_I64, 2) + _i64(end_time)
    out += _fh(T_LIST, 3) + struct.pack(">bi", T_STRUCT, len(links))
    for parent, child, m in links:
        out += _fh(T_STRING, 1) + _str(parent) + _fh(T_STRING, 2) + _str(child) + _fh(T_STRUCT, 3)
        out += _fh(T_I64, 1) + _i64(m[0])
        for fid, v in zip((2, 3, 4, 5), m[1:]):
            out += _fh(T_DOUBLE, fid) + struct.pack(">d", v)
        out += bytes([T_STOP, T_STOP])
    return out + bytes([T_STOP])


T_DOUBLE = 4


def snappy(data: bytes) -> bytes:
    """Raw Snappy block, as iq80 Snappy.compress writes it (SnappyCodec.scala:34-41); pyarrow's
    bundled libsnappy is an independent implementation of the same format."""
    import pyarrow as pa

    return pa.Codec("snappy").compress(data, asbytes=True)
