"""DepsContext: one device-resident zipkin-aggregate accumulator (a zk_ctx).

Mirrors the compute half of ZipkinAggregateJob.scala:20-43: `accumulate` takes span fragment
batches (in any order, like the reference's shuffles; `clustered=True` skips the device clustering
pass for batches whose traces are already contiguous), `finalize` produces the dense
(parent, child) -> Moments table that the job would turn into one Dependencies record.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _abi
from .columns import DeviceColumns, SpanColumns


_PINNED_POOL: dict = {}  # nbytes -> page-locked torch tensors no array uses any more
_PINNED_KEEP = 2


def _pinned_release(nbytes: int, tensor) -> None:
    free = _PINNED_POOL.setdefault(nbytes, [])
    if len(free) < _PINNED_KEEP:
        free.append(tensor)


def _host_buffer(nbytes: int) -> np.ndarray:
    """nbytes of host memory as a uint8 array: page-locked when a HIP device is visible to torch, else
    ordinary memory. A page-locked block goes back to a small pool when the last array viewing it
    is gone (weakref.finalize on the array), so a job that finalizes run after run neither allocates
    nor frees page-locked memory in the steady state (dropping a finalized table used to free its
    block: ~33 ms on MI355X hosts, measured in tests/test_gpu_jobs.py)."""
    try:
        import weakref

        import torch

        if torch.cuda.is_available():
            free = _PINNED_POOL.get(nbytes)
            t = free.pop() if free else torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            arr = t.numpy()
            weakref.finalize(arr, _pinned_release, nbytes, t)
            return arr
    except Exception:  # pragma: no cover - torch missing or without a device: pageable memory
        pass
    return np.empty(nbytes, np.uint8)


@dataclass
class LinkTable:
    """Dense S x S table: cell p*S + c is DependencyLink(parent=p, child=c)."""

    num_services: int
    m0: np.ndarray
    m1: np.ndarray
    m2: np.ndarray
    m3: np.ndarray
    m4: np.ndarray
    present: np.ndarray

    def links(self):
        """Yield (parent_id, child_id, (m0, m1, m2, m3, m4)) for every present cell."""
        S = self.num_services
        for c in np.flatnonzero(self.present):
            yield int(c // S), int(c % S), (
                int(self.m0[c]),
                float(self.m1[c]),
                float(self.m2[c]),
                float(self.m3[c]),
                float(self.m4[c]),
            )

    def as_dict(self) -> dict:
        return {(p, c): m for p, c, m in self.links()}


class DepsContext:
    def __init__(
        self,
        num_services: int,
        *,
        device: int = 0,
        stream: int | None = None,
        strict: bool = True,
        max_trace_records: int = 0,
        timing: bool = False,
        table_ptr: int = 0,
        table_bytes: int = 0,
        trace_pass: bool = False,
    ):
        self._L = _abi.lib()
        cfg = _abi.zk_config()
        cfg.num_services = num_services
        cfg.device = device
        cfg.stream = stream
        cfg.strict = 1 if strict else 0
        cfg.max_trace_records = max_trace_records
        cfg.timing = 1 if timing else 0
        cfg.table = table_ptr or None
        cfg.table_bytes = table_bytes
        cfg.trace_pass = 1 if trace_pass else 0  # the A/B against the group join (zkagg.h)
        h = C.c_void_p()
        st = self._L.zk_ctx_create(C.byref(cfg), C.byref(h))
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, _abi.status_str(st))
        self._h = h
        self.num_services = num_services
        # device batches accumulated since the last drain: their memory must outlive the ctx stream's
        # reads (zkagg.h), and a torch tensor dropped by the caller returns to torch's caching
        # allocator at once, where the next allocation may reuse it while the ctx stream still reads
        self._inflight: list = []

    # -- plumbing ---------------------------------------------------------------------------
    def _check(self, st: int) -> None:
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, self._L.zk_last_error(self._h).decode() or _abi.status_str(st))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.zk_ctx_destroy(self._h)  # (drains the stream)
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
    def handle(self) -> C.c_void_p:
        return self._h

    # -- dependency path --------------------------------------------------------------------
    def reset(self) -> None:
        self._check(self._L.zk_deps_reset(self._h))

    _MAX_INFLIGHT = 8  # device batches kept alive before a drain

    def _hold(self, cols) -> None:
        self._inflight.append(cols)
        if len(self._inflight) > self._MAX_INFLIGHT:
            self.sync()

    def accumulate(self, cols, *, clustered: bool = False, verify: bool = True, n: int | None = None,
                   continues: bool = False) -> None:
        """One batch of span fragments.

        clustered: the caller promises that every trace's fragments are adjacent (Cassandra
          row-per-trace reads); otherwise the device clusters the batch first (a hash partition by
          traceId, zk_cluster.hip).
        verify: check exactly, on the device, that no trace recurs after its run ended -- within the
          batch or across accumulate calls since the last reset (a split trace would be mis-joined);
          finalize then raises ZK_ERR_NOT_CLUSTERED. Costs one extra read of the traceId column.
        continues (needs clustered): the batch's last trace may continue in the next accumulate
          (ZK_BATCH_CONTINUES): its fragments are held back and joined with the next batch's leading
          fragments of the same traceId.
        """
        flags = _abi.ZK_BATCH_TRACE_CLUSTERED if clustered else 0
        if verify:
            flags |= _abi.ZK_BATCH_VERIFY_TRACES
        if continues:
            flags |= _abi.ZK_BATCH_CONTINUES
        if isinstance(cols, DeviceColumns):
            ab = cols.abi(n)
            flags |= _abi.ZK_BATCH_DEVICE_PTRS
            self._hold(cols)
        elif isinstance(cols, SpanColumns):
            ab = cols.abi()
        else:
            ab = cols  # a prepared zk_span_cols; flags from `clustered` / `verify`
        self._check(self._L.zk_deps_accumulate(self._h, C.byref(ab), flags))

    def finalize(self, out_device=None) -> LinkTable | None:
        """Finalize into host numpy arrays (default) or into caller device buffers.

        out_device: optional dict of torch tensors m0 (int64), m1..m4 (float64), present (uint8).
        """
        S = self.num_services
        cells = S * S
        t = _abi.zk_link_table()
        if out_device is not None:
            for k in ("m0", "m1", "m2", "m3", "m4", "present"):
                setattr(t, k, out_device[k].data_ptr())
            t.device_ptrs = 1
            self._check(self._L.zk_deps_finalize(self._h, C.byref(t)))  # (waits for the counters)
            self._inflight = []
            return None
        # (finalize writes every cell) into page-locked host memory when torch has it, laid out as
        # the library's staging block [m0 | m1 | m2 | m3 | m4 | present]: one device copy lands
        # directly (~2x the pageable rate for the 41 B per cell)
        buf = _host_buffer(cells * 41)
        m0 = buf[: cells * 8].view(np.uint64)
        ms = [buf[cells * 8 * (k + 1): cells * 8 * (k + 2)].view(np.float64) for k in range(4)]
        pr = buf[cells * 40: cells * 41]
        t.m0 = m0.ctypes.data
        t.m1, t.m2, t.m3, t.m4 = (a.ctypes.data for a in ms)
        t.present = pr.ctypes.data
        t.device_ptrs = 0
        self._check(self._L.zk_deps_finalize(self._h, C.byref(t)))  # (synchronous)
        self._inflight = []
        return LinkTable(S, m0, *ms, pr)

    def stats(self) -> dict:
        s = _abi.zk_stats()
        self._check(self._L.zk_ctx_stats(self._h, C.byref(s)))
        return s.as_dict()

    def timing(self) -> dict:
        t = _abi.zk_timing()
        self._check(self._L.zk_ctx_timing(self._h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in t._fields_ if k != "reserved"}

    def sync(self) -> None:
        self._check(self._L.zk_ctx_sync(self._h))
        self._inflight = []

    def partial(self) -> tuple[int, int]:
        """(device pointer, bytes) of the exact table + counter tail, counters folded in (enqueued
        on the ctx stream): the buffer a SUM all-reduce merges across shards."""
        p, b = C.c_void_p(), C.c_uint64()
        self._check(self._L.zk_deps_partial(self._h, C.byref(p), C.byref(b)))
        return int(p.value or 0), int(b.value)

    def abort(self) -> None:
        """zk_deps_abort: this rank failed on the host before the exchange; its next partial carries
        an abort mark, so after the all-reduce finalize raises ZK_ERR_RANK_FAILED on every rank."""
        self._check(self._L.zk_deps_abort(self._h))

    def note_merged(self, total_records: int) -> None:
        """The table now holds the merged job: finalize/stats use the merged counters."""
        self._check(self._L.zk_deps_note_merged(self._h, total_records))

    def tracegen_device(self, params: _abi.zk_tracegen_params, out: DeviceColumns) -> tuple[int, int]:
        nrec, ntr = C.c_uint64(), C.c_uint64()
        ab = out.abi(out.capacity)
        self._check(
            self._L.zk_tracegen_device(self._h, C.byref(params), C.byref(ab), out.capacity, C.byref(nrec), C.byref(ntr))
        )
        out.n = int(nrec.value)
        return int(nrec.value), int(ntr.value)
