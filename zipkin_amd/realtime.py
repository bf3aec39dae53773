"""RtSketch: per-service distinct traces (HyperLogLog) and duration quantiles (include/zksketch.h).

The realtime aggregates the reference declares but never implements (RealtimeAggregates.scala:26-38,
QueryService.scala:416-430): fed either from already-merged spans (`accumulate_merged`) or, bound
to a DepsContext, from the same K1 pass over span fragments that feeds the dependency path
(`bind`). Host-side names map service ids back to names, as for the dependency table.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi


def _ptr(a) -> int:
    return a.data_ptr() if hasattr(a, "data_ptr") else a.ctypes.data


class RtSketch:
    def __init__(self, num_services: int, *, device: int = 0, stream: int | None = None, hll_p: int = 0,
                 sub_bits: int = 0, seed: int = 0):
        self._L = _abi.lib()
        cfg = _abi.zk_rt_config()
        cfg.num_services = num_services
        cfg.device = device
        cfg.stream = stream
        cfg.hll_p = hll_p
        cfg.sub_bits = sub_bits
        cfg.seed = seed
        h = C.c_void_p()
        st = self._L.zk_rt_create(C.byref(cfg), C.byref(h))
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, _abi.status_str(st))
        self._h = h
        self.num_services = num_services
        self.seed = seed
        r, b = C.c_uint32(), C.c_uint32()
        self._check(self._L.zk_rt_geometry(h, C.byref(r), C.byref(b)))
        self.registers, self.bins = r.value, b.value
        self.p = self.registers.bit_length() - 1
        self.m = sub_bits or 7
        self._bound = None

    def _check(self, st: int) -> None:
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, self._L.zk_rt_last_error(self._h).decode() or _abi.status_str(st))

    def close(self) -> None:
        if getattr(self, "_h", None):
            if self._bound is not None:
                self.unbind()
            self._L.zk_rt_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def reset(self) -> None:
        self._check(self._L.zk_rt_reset(self._h))

    def bind(self, ctx, only: bool = False) -> None:
        """Feed this sketch from every later ctx.accumulate (only=True: skip the dependency path)."""
        mode = _abi.ZK_RT_ONLY if only else _abi.ZK_RT_WITH_DEPS
        st = self._L.zk_rt_bind(ctx.handle, self._h, mode)
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, self._L.zk_last_error(ctx.handle).decode())
        self._bound = ctx

    def unbind(self) -> None:
        if self._bound is not None:
            self._L.zk_rt_bind(self._bound.handle, None, 0)
            self._bound = None

    def accumulate_merged(self, service_id, trace_id, duration) -> None:
        n = len(service_id)
        if hasattr(service_id, "data_ptr"):
            flags, s, t, d = _abi.ZK_BATCH_DEVICE_PTRS, service_id, trace_id, duration
        else:
            flags = 0
            s = np.ascontiguousarray(service_id, dtype=np.uint32)
            t = np.asarray(trace_id)
            t = np.ascontiguousarray(t.view(np.uint64) if t.dtype == np.int64 else t, dtype=np.uint64)
            d = np.ascontiguousarray(duration, dtype=np.int64)
        self._check(self._L.zk_rt_accumulate_merged(self._h, _ptr(s), _ptr(t), _ptr(d), n, flags))
        if flags:  # device batches the stream may still read (see DepsContext._hold)
            inflight = self.__dict__.setdefault("_inflight", [])
            inflight.append((s, t, d))
            if len(inflight) > 8:
                self._check(self._L.zk_rt_dropped(self._h, None, None))  # (synchronises the stream)
                inflight.clear()

    def distinct_traces(self) -> np.ndarray:
        out = np.zeros(self.num_services, np.float64)
        self._check(self._L.zk_rt_distinct_traces(self._h, out.ctypes.data))
        return out

    def quantiles(self, service: int, qs=(0.5, 0.99)):
        """([(lo, hi)] bin bounds holding each nearest-rank quantile, count)."""
        q = np.ascontiguousarray(qs, dtype=np.float64)
        lo = np.zeros(len(q), np.int64)
        hi = np.zeros(len(q), np.int64)
        cnt = C.c_uint64()
        self._check(self._L.zk_rt_quantiles(self._h, service, q.ctypes.data, len(q), lo.ctypes.data, hi.ctypes.data,
                                            C.byref(cnt)))
        return [(int(a), int(b)) for a, b in zip(lo, hi)], int(cnt.value)

    def quantiles_all(self, qs=(0.5, 0.99)):
        """(lo int64[S, nq], hi int64[S, nq], count uint64[S]) for every service at once
        (zk_rt_quantiles_all: one device pass and one copy)."""
        q = np.ascontiguousarray(qs, dtype=np.float64)
        S = self.num_services
        lo = np.zeros((S, len(q)), np.int64)
        hi = np.zeros((S, len(q)), np.int64)
        cnt = np.zeros(S, np.uint64)
        self._check(self._L.zk_rt_quantiles_all(self._h, q.ctypes.data, len(q), lo.ctypes.data, hi.ctypes.data,
                                                cnt.ctypes.data_as(_abi._U64P)))
        return lo, hi, cnt

    def tdigest(self, service: int, compression: float = 200.0, qs=(0.5, 0.99)):
        """(centroid means, centroid weights, t-digest estimates of qs, count) of one service's
        duration digest (zk_rt_tdigest: a merging t-digest over the exact histogram)."""
        q = np.ascontiguousarray(qs, dtype=np.float64)
        val = np.zeros(len(q), np.float64)
        n, cnt = C.c_uint32(), C.c_uint64()
        self._check(self._L.zk_rt_tdigest(self._h, service, compression, None, None, 0, C.byref(n), None, 0, None,
                                          None))
        mean = np.zeros(n.value, np.float64)
        weight = np.zeros(n.value, np.float64)
        self._check(self._L.zk_rt_tdigest(self._h, service, compression, mean.ctypes.data, weight.ctypes.data, n.value,
                                          C.byref(n), q.ctypes.data, len(q), val.ctypes.data, C.byref(cnt)))
        return mean, weight, val, int(cnt.value)

    def read(self):
        """(registers uint8[S, 2^p], histogram uint32[S, bins]) host copies."""
        regs = np.zeros((self.num_services, self.registers), np.uint8)
        hist = np.zeros((self.num_services, self.bins), np.uint32)
        self._check(self._L.zk_rt_read(self._h, regs.ctypes.data, hist.ctypes.data))
        return regs, hist

    def dropped(self) -> tuple[int, int]:
        a, b = C.c_uint64(), C.c_uint64()
        self._check(self._L.zk_rt_dropped(self._h, C.byref(a), C.byref(b)))
        return int(a.value), int(b.value)

    def partial(self):
        """(registers ptr, bytes, histogram ptr, bytes): device buffers for MAX / SUM all-reduce."""
        rp, rb, hp, hb = C.c_void_p(), C.c_uint64(), C.c_void_p(), C.c_uint64()
        self._check(self._L.zk_rt_partial(self._h, C.byref(rp), C.byref(rb), C.byref(hp), C.byref(hb)))
        return int(rp.value), int(rb.value), int(hp.value), int(hb.value)


class RealtimeLinks:
    """The realtime link store (zk_rl_*): every join row (parent service, child service, child
    duration, traceId) of the dependency path since the last reset, kept in HBM and queried by
    server (child) service -- the state behind RealtimeAggregates (GpuRealtimeAggregates below in
    zipkin_amd/aggregates.py). Bound to a DepsContext, K1 writes the rows beside its links."""

    def __init__(self, num_services: int, *, device: int = 0, stream: int | None = None):
        self._L = _abi.lib()
        cfg = _abi.zk_rl_config()
        cfg.num_services = num_services
        cfg.device = device
        cfg.stream = stream
        h = C.c_void_p()
        st = self._L.zk_rl_create(C.byref(cfg), C.byref(h))
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, _abi.status_str(st))
        self._h = h
        self.num_services = num_services
        self._bound = None

    def _check(self, st: int) -> None:
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, self._L.zk_rl_last_error(self._h).decode() or _abi.status_str(st))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.unbind()
            self._L.zk_rl_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def bind(self, ctx) -> None:
        st = self._L.zk_rl_bind(ctx.handle, self._h)
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, self._L.zk_last_error(ctx.handle).decode())
        self._bound = ctx

    def unbind(self) -> None:
        if self._bound is not None and getattr(self._bound, "_h", None):
            self._L.zk_rl_bind(self._bound.handle, None)
        self._bound = None

    def reset(self) -> None:
        self._check(self._L.zk_rl_reset(self._h))

    def count(self) -> tuple[int, int]:
        """(rows in the window, rows dropped past its capacity -- always 0)."""
        n, d = C.c_uint64(), C.c_uint64()
        self._check(self._L.zk_rl_count(self._h, C.byref(n), C.byref(d)))
        return int(n.value), int(d.value)

    def server_links(self, server: int):
        """(parent ids uint32, durations int64 us, traceIds uint64) of every row whose child service
        is `server`, ordered by (parent, duration, traceId)."""
        n = C.c_uint64()
        self._check(self._L.zk_rl_server_links(self._h, server, None, None, None, 0, C.byref(n)))
        m = int(n.value)
        par = np.zeros(max(1, m), np.uint32)
        dur = np.zeros(max(1, m), np.int64)
        tid = np.zeros(max(1, m), np.uint64)
        if m:
            self._check(self._L.zk_rl_server_links(self._h, server, par.ctypes.data, dur.ctypes.data, tid.ctypes.data,
                                                   m, C.byref(n)))
        return par[:m], dur[:m], tid[:m]
