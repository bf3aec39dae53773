"""Columnar span batches (48 B per stored span fragment) and the synthetic tracegen workload.

Column meaning is fixed by include/zkagg.h (zk_span_cols). Host batches are numpy arrays; device
batches are torch tensors on a HIP device (torch is only the allocator here).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _abi

COLUMNS = (
    ("trace_id", np.uint64),
    ("span_id", np.uint64),
    ("parent_id", np.uint64),
    ("first_ts", np.int64),
    ("last_ts", np.int64),
    ("service_id", np.uint32),
    ("flags", np.uint32),
)
BYTES_PER_RECORD = 48


@dataclass
class SpanColumns:
    trace_id: np.ndarray
    span_id: np.ndarray
    parent_id: np.ndarray
    first_ts: np.ndarray
    last_ts: np.ndarray
    service_id: np.ndarray
    flags: np.ndarray

    @staticmethod
    def empty(n: int) -> "SpanColumns":
        return SpanColumns(*[np.zeros(n, dtype=dt) for _, dt in COLUMNS])

    @staticmethod
    def concat(parts) -> "SpanColumns":
        parts = list(parts)
        if not parts:
            return SpanColumns.empty(0)
        return SpanColumns(*[np.concatenate([getattr(p, k) for p in parts]).astype(dt) for k, dt in COLUMNS])

    def __len__(self) -> int:
        return int(self.trace_id.shape[0])

    def take(self, idx) -> "SpanColumns":
        return SpanColumns(*[np.ascontiguousarray(getattr(self, k)[idx]) for k, _ in COLUMNS])

    def validate(self) -> None:
        n = len(self)
        for k, dt in COLUMNS:
            a = getattr(self, k)
            if a.dtype != dt or a.shape != (n,) or not a.flags["C_CONTIGUOUS"]:
                raise ValueError(f"column {k} must be contiguous {np.dtype(dt)}[{n}]")

    def abi(self) -> _abi.zk_span_cols:
        self.validate()
        return _abi.zk_span_cols(*[getattr(self, k).ctypes.data for k, _ in COLUMNS], len(self))


class DeviceColumns:
    """The same seven columns as torch tensors in HBM (u64 columns stored as int64)."""

    def __init__(self, n: int, device: str = "cuda", packed: bool = False):
        """packed: the seven columns back to back in ONE allocation (each column 256-B aligned), so
        that their bases are not all aligned alike (seven separate allocations start on the same
        large alignment, and the same record index of every column then lands on the same HBM
        channel); the ABI takes any 16-B aligned column pointers either way."""
        import torch

        self.n = n
        self.capacity = n
        if packed:
            offs, at = [], 0
            for _, dt in COLUMNS:
                offs.append(at)
                at += (n * np.dtype(dt).itemsize + 255) // 256 * 256
            self._block = torch.empty(max(at, 1), dtype=torch.uint8, device=device)
            for (k, dt), o in zip(COLUMNS, offs):
                w = np.dtype(dt).itemsize
                view = self._block[o:o + n * w].view(torch.int64 if w == 8 else torch.int32)
                setattr(self, k, view)
            return
        self.trace_id = torch.empty(n, dtype=torch.int64, device=device)
        self.span_id = torch.empty(n, dtype=torch.int64, device=device)
        self.parent_id = torch.empty(n, dtype=torch.int64, device=device)
        self.first_ts = torch.empty(n, dtype=torch.int64, device=device)
        self.last_ts = torch.empty(n, dtype=torch.int64, device=device)
        self.service_id = torch.empty(n, dtype=torch.int32, device=device)
        self.flags = torch.empty(n, dtype=torch.int32, device=device)

    def slice(self, a: int, b: int) -> "DeviceColumns":
        """Records [a, b) as a view of the same HBM (capacity b - a, n = b - a)."""
        v = DeviceColumns.__new__(DeviceColumns)
        for k, _ in COLUMNS:
            setattr(v, k, getattr(self, k)[a:b])
        v.n = v.capacity = b - a
        v._parent = self  # (keeps the storage alive)
        return v

    def abi(self, n: int | None = None) -> _abi.zk_span_cols:
        return _abi.zk_span_cols(
            *[getattr(self, k).data_ptr() for k, _ in COLUMNS], self.n if n is None else n
        )

    @staticmethod
    def from_host(cols: SpanColumns, device: str = "cuda") -> "DeviceColumns":
        import torch

        d = DeviceColumns(len(cols), device)
        for k, _ in COLUMNS:
            a = getattr(cols, k)
            t = torch.from_numpy(a.view(np.int64) if a.dtype.itemsize == 8 else a.view(np.int32))
            getattr(d, k).copy_(t)
        return d

    def to_host(self, n: int | None = None) -> SpanColumns:
        """The first n records (default: all) as host columns."""
        n = self.n if n is None else min(n, self.n)
        out = []
        for k, dt in COLUMNS:
            t = getattr(self, k)[:n].cpu().numpy()
            out.append(t.view(dt))
        return SpanColumns(*out)


def tracegen_params(
    seed: int,
    num_traces: int,
    *,
    target_records: int = 0,
    max_depth: int = 7,
    num_services: int = 57,
    base_ts: int = 1_421_053_208_373_000,
    rank: int = 0,
    world: int = 1,
    global_ids: bool = False,
) -> _abi.zk_tracegen_params:
    p = _abi.zk_tracegen_params()
    p.seed = seed
    p.num_traces = num_traces
    p.target_records = target_records
    p.max_depth = max_depth
    p.num_services = num_services
    p.base_ts = base_ts
    p.rank = rank
    p.world = world
    p.global_ids = 1 if global_ids else 0
    return p


def tracegen_host(seed: int, num_traces: int, **kw) -> SpanColumns:
    """Host (CPU) run of the shared TraceGen restatement (zk_tracegen.h)."""
    L = _abi.lib()
    p = tracegen_params(seed, num_traces, **kw)
    nrec, ntr = C.c_uint64(), C.c_uint64()
    st = L.zk_tracegen_host(C.byref(p), None, 0, C.byref(nrec), C.byref(ntr))
    if st != _abi.ZK_OK:
        raise _abi.ZkError(st, _abi.status_str(st))
    cols = SpanColumns.empty(nrec.value)
    ab = cols.abi()
    st = L.zk_tracegen_host(C.byref(p), C.byref(ab), nrec.value, C.byref(nrec), C.byref(ntr))
    if st != _abi.ZK_OK:
        raise _abi.ZkError(st, _abi.status_str(st))
    assert nrec.value == len(cols)
    return cols


def trace_shard(trace_id: int, world: int) -> int:
    return int(_abi.lib().zk_trace_shard(trace_id, world))
