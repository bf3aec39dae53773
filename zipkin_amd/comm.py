"""RCCL communicator of the library (include/zkcomm.h): the multi-GPU merges without torch.distributed.

This is the surface the JVM host binds (ZkNative.commCreate / depsAllreduce / ...): rank 0 makes a
unique id, every rank opens the communicator with it, and one call per state merges the ranks'
traceId-disjoint parts -- the dependency table by one int64 SUM all-reduce of its exchange form
(ZipkinAggregateJob.scala:39-43, the cross-reducer .group.sum / .sum), the realtime sketch by
MAX/SUM, the top-K sketch by an all-gather of the candidate lists plus SUM. The Python job drivers
and the bench use torch.distributed (zipkin_amd/shards.py) for the same arithmetic.
"""
from __future__ import annotations

import ctypes as C

from . import _abi

ID_BYTES = 128  # ZK_COMM_ID_BYTES


def unique_id() -> bytes:
    """ZK_COMM_ID_BYTES bytes for zk_comm_create (rank 0 makes it and ships it to the others)."""
    buf = (C.c_uint8 * ID_BYTES)()
    L = _abi.lib()
    st = L.zk_comm_unique_id(buf, ID_BYTES)
    if st != _abi.ZK_OK:
        raise _abi.ZkError(st, L.zk_comm_last_error(None).decode() or _abi.status_str(st))
    return bytes(buf)


class Comm:
    def __init__(self, uid: bytes, rank: int, world: int, device: int = 0):
        self._L = _abi.lib()
        if len(uid) < ID_BYTES:
            raise ValueError("unique id too short")
        src = (C.c_uint8 * ID_BYTES).from_buffer_copy(uid[:ID_BYTES])
        h = C.c_void_p()
        st = self._L.zk_comm_create(src, ID_BYTES, rank, world, device, C.byref(h))
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, self._L.zk_comm_last_error(None).decode() or _abi.status_str(st))
        self._h = h
        self.rank, self.world, self.device = rank, world, device

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.zk_comm_destroy(self._h)
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

    def allreduce_deps(self, ctx, total_records: int = 0) -> None:
        """zk_deps_allreduce: partial -> int64 SUM -> note_merged, on the ctx stream."""
        ctx._check(self._L.zk_deps_allreduce(ctx.handle, self._h, total_records))

    def allreduce_rt(self, rt) -> None:
        rt._check(self._L.zk_rt_allreduce(rt.handle, self._h))

    def allreduce_kv(self, kv) -> None:
        kv._check(self._L.zk_kv_allreduce(kv.handle, self._h))
