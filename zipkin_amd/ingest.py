"""SpanDecoder: stored span fragments (Snappy + TBinaryProtocol thrift Span) -> SpanColumns.

Binds include/zkingest.h. The decoder owns the service-name dictionary; its ids are the
service ids of the columnar records (zkagg.h), the dependency table and the sketches.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence

import numpy as np

from . import _abi
from .columns import SpanColumns


def hash_string(s: str | bytes) -> int:
    b = s.encode() if isinstance(s, str) else s
    return int(_abi.lib().zk_hash_string(b, len(b)))


class SpanDecoder:
    def __init__(self):
        self._L = _abi.lib()
        h = C.c_void_p()
        st = self._L.zk_ingest_create(C.byref(h))
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, _abi.status_str(st))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.zk_ingest_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st: int) -> None:
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, self._L.zk_ingest_last_error(self._h).decode() or _abi.status_str(st))

    def decode(self, blobs, *, snappy: bool = True, strict: bool = True, items: bool = False,
               item_cap: int | None = None, one_thread: bool = False):
        """Decode stored fragments: a sequence of bytes objects (one per fragment), or the packed
        form (buf uint8[total], offsets uint64[n + 1]) -- fragment i is buf[offsets[i]:offsets[i+1]].
        Returns (SpanColumns, rejected) or, with items=True, (SpanColumns, rejected,
        (kv_service, kv_key), (ann_service, ann_value)). one_thread: decode on the calling thread
        only (ZK_INGEST_ONE_THREAD; the default splits large batches over up to 16 threads, with the
        same results)."""
        if isinstance(blobs, tuple) and len(blobs) == 2 and isinstance(blobs[0], np.ndarray):
            buf = np.ascontiguousarray(blobs[0], dtype=np.uint8)
            offsets = np.ascontiguousarray(blobs[1], dtype=np.uint64)
            n = len(offsets) - 1
            if not len(buf):
                buf = np.zeros(1, np.uint8)
        else:
            n = len(blobs)
            offsets = np.zeros(n + 1, np.uint64)
            if n:
                offsets[1:] = np.cumsum([len(b) for b in blobs], dtype=np.uint64)
            buf = np.frombuffer(b"".join(blobs) or b"\0", dtype=np.uint8)
        cols = SpanColumns.empty(n)
        nout, nrej = C.c_uint64(), C.c_uint64()
        it = None
        arrs = None
        if items:
            cap = item_cap if item_cap is not None else max(16, 8 * n)
            arrs = (np.zeros(cap, np.uint32), np.zeros(cap, np.uint64), np.zeros(cap, np.uint32), np.zeros(cap, np.uint64))
            it = _abi.zk_ingest_items(arrs[0].ctypes.data, arrs[1].ctypes.data, cap, 0,
                                      arrs[2].ctypes.data, arrs[3].ctypes.data, cap, 0)
        codec = _abi.ZK_CODEC_SNAPPY_THRIFT if snappy else _abi.ZK_CODEC_THRIFT
        flags = (_abi.ZK_INGEST_STRICT if strict else 0) | (_abi.ZK_INGEST_ONE_THREAD if one_thread else 0)
        ab = cols.abi()
        self._check(self._L.zk_ingest_spans(self._h, buf.ctypes.data, offsets.ctypes.data, n, codec, flags,
                                            C.byref(ab), C.byref(nout), C.byref(nrej),
                                            C.byref(it) if it is not None else None))
        cols = cols.take(slice(0, nout.value))
        if not items:
            return cols, int(nrej.value)
        kv = (arrs[0][: it.kv_n].copy(), arrs[1][: it.kv_n].copy())
        ann = (arrs[2][: it.ann_n].copy(), arrs[3][: it.ann_n].copy())
        return cols, int(nrej.value), kv, ann

    @property
    def num_services(self) -> int:
        n = C.c_uint32()
        self._check(self._L.zk_ingest_num_services(self._h, C.byref(n)))
        return int(n.value)

    def service_id(self, name: str) -> int:
        b = name.encode()
        i = C.c_uint32()
        self._check(self._L.zk_ingest_service_id(self._h, b, len(b), C.byref(i)))
        return int(i.value)

    def service_name(self, i: int) -> str:
        ln = C.c_uint64()
        self._check(self._L.zk_ingest_service_name(self._h, i, None, 0, C.byref(ln)))
        buf = C.create_string_buffer(max(1, ln.value))
        self._check(self._L.zk_ingest_service_name(self._h, i, buf, ln.value, C.byref(ln)))
        return buf.raw[: ln.value].decode("utf-8", "surrogateescape")

    def service_names(self) -> List[str]:
        return [self.service_name(i) for i in range(self.num_services)]

    def string(self, h: int) -> str:
        ln = C.c_uint64()
        self._check(self._L.zk_ingest_string(self._h, h, None, 0, C.byref(ln)))
        buf = C.create_string_buffer(max(1, ln.value))
        self._check(self._L.zk_ingest_string(self._h, h, buf, ln.value, C.byref(ln)))
        return buf.raw[: ln.value].decode("utf-8", "surrogateescape")


def snappy_uncompress(data: bytes) -> bytes:
    L = _abi.lib()
    src = np.frombuffer(data or b"\0", dtype=np.uint8)
    n = C.c_uint64()
    st = L.zk_snappy_uncompress(src.ctypes.data, len(data), None, 0, C.byref(n))
    if st != _abi.ZK_OK:
        raise _abi.ZkError(st, _abi.status_str(st))
    out = np.zeros(max(1, n.value), np.uint8)
    st = L.zk_snappy_uncompress(src.ctypes.data, len(data), out.ctypes.data, n.value, C.byref(n))
    if st != _abi.ZK_OK:
        raise _abi.ZkError(st, _abi.status_str(st))
    return out[: n.value].tobytes()


class DeviceSpanDecoder:
    """zk_ingest_dev: stored fragments already in HBM -> device columns (one lane per fragment).

    `decode_device(buf, offsets, n)` takes torch tensors (uint8 bytes, int64 offsets[n+1]) on the
    device; `decode(blobs)` uploads a list of bytes objects first (tests, small batches)."""

    def __init__(self, max_services: int = 4096, *, device: int = 0, stream: int | None = None,
                 scratch_bytes: int = 0):
        self._L = _abi.lib()
        h = C.c_void_p()
        st = self._L.zk_ingest_dev_create(device, stream, max_services, C.byref(h))
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, _abi.status_str(st))
        self._h = h
        self.device = device
        if scratch_bytes:  # the Snappy scratch's first size (zk_ingest_dev_set_scratch); it grows on demand
            st = self._L.zk_ingest_dev_set_scratch(self._h, scratch_bytes)
            if st != _abi.ZK_OK:
                raise _abi.ZkError(st, _abi.status_str(st))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.zk_ingest_dev_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st: int) -> None:
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, self._L.zk_ingest_dev_last_error(self._h).decode() or _abi.status_str(st))

    def decode_device(self, buf, offsets, n: int, *, snappy: bool = True, strict: bool = True, out=None,
                      items: bool = False, item_cap: int | None = None):
        """-> (DeviceColumns with .n = records written, rejected), or with items=True
        (cols, rejected, (kv_service, kv_key), (ann_service, ann_value)): the span indexer's items as
        device tensors (int32 service ids of this decoder, int64 hashes = uint64 bit patterns), in no
        particular order within the batch (zk_ingest_dev_spans_items). item_cap: the items per kind
        to allow for (default 2n + 16; a batch with more is decoded again with 4x the room)."""
        L, h = self._L, self._h
        bp, op = buf.data_ptr(), offsets.data_ptr()

        def call(codec, flags, ab, nout, nrej, it):
            if it is None:
                return L.zk_ingest_dev_spans(h, bp, op, n, codec, flags, C.byref(ab), C.byref(nout), C.byref(nrej))
            return L.zk_ingest_dev_spans_items(h, bp, op, n, codec, flags, C.byref(ab), C.byref(nout), C.byref(nrej),
                                               C.byref(it))

        return self._run(call, n, snappy, strict, out, items, item_cap)

    def decode_device_many(self, batches, *, snappy: bool = True, strict: bool = True, out=None,
                           items: bool = False, item_cap: int | None = None):
        """Several HBM-resident batches [(buf, offsets, n), ...] in ONE decode
        (zk_ingest_dev_spans_multi): the results of decode_device over the batches joined in order,
        for one set of launches and one host round trip."""
        L, h = self._L, self._h
        nb = len(batches)
        n = sum(int(b[2]) for b in batches)
        bufs = (C.c_void_p * max(1, nb))(*[b[0].data_ptr() if int(b[2]) else None for b in batches])
        offs = (C.c_void_p * max(1, nb))(*[b[1].data_ptr() if int(b[2]) else None for b in batches])
        ns = (C.c_uint64 * max(1, nb))(*[int(b[2]) for b in batches])

        def call(codec, flags, ab, nout, nrej, it):
            return L.zk_ingest_dev_spans_multi(h, nb, bufs, offs, ns, codec, flags, C.byref(ab), C.byref(nout),
                                               C.byref(nrej), None if it is None else C.byref(it))

        return self._run(call, n, snappy, strict, out, items, item_cap)

    def _run(self, call, n, snappy, strict, out, items, item_cap):
        import torch

        from .columns import DeviceColumns

        dev = f"cuda:{self.device}"
        cols = out if out is not None else DeviceColumns(max(1, n), device=dev)
        nout, nrej = C.c_uint64(), C.c_uint64()
        ab = cols.abi(n)
        codec = _abi.ZK_CODEC_SNAPPY_THRIFT if snappy else _abi.ZK_CODEC_THRIFT
        flags = _abi.ZK_INGEST_STRICT if strict else 0
        if not items:
            self._check(call(codec, flags, ab, nout, nrej, None))
            cols.n = int(nout.value)
            return cols, int(nrej.value)
        cap = item_cap if item_cap is not None else 2 * n + 16
        while True:
            ks = torch.empty(cap, dtype=torch.int32, device=dev)
            kh = torch.empty(cap, dtype=torch.int64, device=dev)
            as_ = torch.empty(cap, dtype=torch.int32, device=dev)
            ah = torch.empty(cap, dtype=torch.int64, device=dev)
            it = _abi.zk_ingest_items(ks.data_ptr(), kh.data_ptr(), cap, 0, as_.data_ptr(), ah.data_ptr(), cap, 0)
            st = call(codec, flags, ab, nout, nrej, it)
            if st == _abi.ZK_ERR_CAPACITY and (it.kv_n == cap or it.ann_n == cap):
                cap *= 4  # more items than guessed: the batch again
                continue
            self._check(st)
            break
        cols.n = int(nout.value)
        return cols, int(nrej.value), (ks[: it.kv_n], kh[: it.kv_n]), (as_[: it.ann_n], ah[: it.ann_n])

    def string(self, h: int) -> str:
        """The key / value string behind a hash an items batch has seen (zk_ingest_dev_string);
        memoised (a hash keeps the string first captured for it)."""
        h = int(h) & 0xFFFFFFFFFFFFFFFF
        memo = self.__dict__.setdefault("_strings", {})
        if h in memo:
            return memo[h]
        ln = C.c_uint64()
        self._check(self._L.zk_ingest_dev_string(self._h, h, None, 0, C.byref(ln)))
        buf = C.create_string_buffer(max(1, ln.value))
        self._check(self._L.zk_ingest_dev_string(self._h, h, buf, ln.value, C.byref(ln)))
        v = buf.raw[: ln.value].decode("utf-8", "surrogateescape")
        memo[h] = v
        return v

    def decode(self, blobs: Sequence[bytes], *, snappy: bool = True, strict: bool = True, items: bool = False):
        import torch

        dev = f"cuda:{self.device}"
        offsets = np.zeros(len(blobs) + 1, np.int64)
        if blobs:
            offsets[1:] = np.cumsum([len(b) for b in blobs])
        raw = np.frombuffer(b"".join(blobs) or b"\0", dtype=np.uint8)
        buf = torch.from_numpy(raw.copy()).to(dev)
        off = torch.from_numpy(offsets).to(dev)
        return self.decode_device(buf, off, len(blobs), snappy=snappy, strict=strict, items=items)

    @property
    def num_services(self) -> int:
        n = C.c_uint32()
        self._check(self._L.zk_ingest_dev_num_services(self._h, C.byref(n)))
        return int(n.value)

    def service_name(self, i: int) -> str:
        """Memoised: a decoder's service ids never change."""
        memo = self.__dict__.setdefault("_names", {})
        if i in memo:
            return memo[i]
        ln = C.c_uint64()
        self._check(self._L.zk_ingest_dev_service_name(self._h, i, None, 0, C.byref(ln)))
        buf = C.create_string_buffer(max(1, ln.value))
        self._check(self._L.zk_ingest_dev_service_name(self._h, i, buf, ln.value, C.byref(ln)))
        v = buf.raw[: ln.value].decode("utf-8", "surrogateescape")
        memo[i] = v
        return v

    def service_names(self) -> List[str]:
        return [self.service_name(i) for i in range(self.num_services)]
