"""KvSketch: per-service count-min + top-K of binary-annotation keys (include/zksketch.h).

Device half of Aggregates.getTopKeyValueAnnotations (Aggregates.scala:34): the host maps service
names and annotation keys to ids / 64-bit hashes, feeds (service id, key hash) items and asks for
the most popular key hashes of a service, best first.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi


def _ptr(a) -> int:
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data


class KvSketch:
    def __init__(self, num_services: int, *, device: int = 0, stream: int | None = None, width: int = 0,
                 depth: int = 0, candidates: int = 0, seed: int = 0, timing: bool = False):
        self._L = _abi.lib()
        cfg = _abi.zk_kv_config()
        cfg.reserved[0] = 1 if timing else 0  # ZK_KV_TIMING
        cfg.num_services = num_services
        cfg.device = device
        cfg.stream = stream
        cfg.width = width
        cfg.depth = depth
        cfg.candidates = candidates
        cfg.seed = seed
        h = C.c_void_p()
        st = self._L.zk_kv_create(C.byref(cfg), C.byref(h))
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, _abi.status_str(st))
        self._h = h
        self.num_services = num_services
        w, d, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
        self._check(self._L.zk_kv_geometry(h, C.byref(w), C.byref(d), C.byref(c)))
        self.width, self.depth, self.candidates = w.value, d.value, c.value
        self.seed = seed
        self._inflight: list = []  # device batches the stream may still read (see DepsContext._hold)

    def _drain(self) -> None:
        """Wait for the sketch's stream (zk_kv_totals synchronises it) and release held batches."""
        tot = np.zeros(self.num_services, np.uint64)
        self._check(self._L.zk_kv_totals(self._h, tot.ctypes.data))
        self._inflight = []

    def _check(self, st: int) -> None:
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, self._L.zk_kv_last_error(self._h).decode() or _abi.status_str(st))

    def phase_ms(self) -> dict:
        """Device ms of the last accumulate's phases (needs timing=True)."""
        out = (C.c_double * 4)()
        self._check(self._L.zk_kv_phase_ms(self._h, out))
        return dict(zip(("partition", "sketch", "candidates", "merge"), list(out)))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.zk_kv_destroy(self._h)  # (drains the stream)
            self._h = None
        self._inflight = []

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
        self._check(self._L.zk_kv_reset(self._h))

    def accumulate(self, service_id, key_hash) -> None:
        """One batch: numpy (host) arrays, or torch device tensors (uint32/int32, uint64/int64)."""
        n = len(service_id)
        if len(key_hash) != n:
            raise ValueError("service_id and key_hash differ in length")
        if hasattr(service_id, "data_ptr"):
            flags = _abi.ZK_BATCH_DEVICE_PTRS
            s, k = service_id, key_hash
        else:
            flags = 0
            s = np.ascontiguousarray(service_id, dtype=np.uint32)
            k = np.ascontiguousarray(np.asarray(key_hash).view(np.uint64) if np.asarray(key_hash).dtype == np.int64
                                     else key_hash, dtype=np.uint64)
        self._check(self._L.zk_kv_accumulate(self._h, _ptr(s), _ptr(k), n, flags))
        if flags:
            self._inflight.append((s, k))
            if len(self._inflight) > 8:
                self._drain()

    def topk_all(self, k: int):
        """(keys uint64[S, k], est uint32[S, k], count uint32[S]); row s best first."""
        S = self.num_services
        keys = np.zeros((S, k), np.uint64)
        est = np.zeros((S, k), np.uint32)
        cnt = np.zeros(S, np.uint32)
        self._check(self._L.zk_kv_topk_all(self._h, k, keys.ctypes.data, est.ctypes.data, cnt.ctypes.data))
        return keys, est, cnt

    def topk(self, service: int, k: int) -> list[tuple[int, int]]:
        """[(key_hash, estimate)] of one service, best first (getTopKeyValueAnnotations)."""
        keys = np.zeros(k, np.uint64)
        est = np.zeros(k, np.uint32)
        cnt = C.c_uint32()
        self._check(self._L.zk_kv_topk(self._h, service, k, keys.ctypes.data, est.ctypes.data, C.byref(cnt)))
        return [(int(keys[i]), int(est[i])) for i in range(cnt.value)]

    def estimate(self, service: int, keys) -> np.ndarray:
        q = np.ascontiguousarray(np.asarray(keys).view(np.uint64) if np.asarray(keys).dtype == np.int64 else keys,
                                 dtype=np.uint64)
        out = np.zeros(len(q), np.uint32)
        self._check(self._L.zk_kv_estimate(self._h, service, q.ctypes.data, len(q), out.ctypes.data))
        return out

    def totals(self) -> np.ndarray:
        out = np.zeros(self.num_services, np.uint64)
        self._check(self._L.zk_kv_totals(self._h, out.ctypes.data))
        return out

    # -- multi-GPU ---------------------------------------------------------------------------
    def partial(self):
        """(counters ptr, bytes, totals ptr, bytes): device buffers to SUM all-reduce."""
        cp, cb, tp, tb = C.c_void_p(), C.c_uint64(), C.c_void_p(), C.c_uint64()
        self._check(self._L.zk_kv_partial(self._h, C.byref(cp), C.byref(cb), C.byref(tp), C.byref(tb)))
        return int(cp.value), int(cb.value), int(tp.value), int(tb.value)

    def candidate_buffers(self):
        kp, ep, kb, eb = C.c_void_p(), C.c_void_p(), C.c_uint64(), C.c_uint64()
        self._check(self._L.zk_kv_candidates(self._h, C.byref(kp), C.byref(ep), C.byref(kb), C.byref(eb)))
        return int(kp.value), int(ep.value), int(kb.value), int(eb.value)

    def merge_candidates(self, keys, est, lists: int) -> None:
        """keys/est: device tensors [lists, S, candidates] gathered from all ranks."""
        self._check(self._L.zk_kv_merge_candidates(self._h, _ptr(keys), _ptr(est), lists))
