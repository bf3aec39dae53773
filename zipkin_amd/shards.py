"""Multi-GPU step of the dependency path: traceId-hash shards and one exact SUM all-reduce.

Both shuffle keys of the reference job contain traceId -- the merge key (id, traceId) at
ZipkinAggregateJob.scala:21 and the join key (parentId, traceId) at :30 -- so with
shard = mix64(traceId) % world (zk_trace_shard) every merge and every join is rank-local. The only
exchange is the reduce of the per-(parent, child) link table (`.group.sum`, :40): one SUM
all-reduce of the carry-free u64-limb accumulator (zipkin_amd/table.py), which is exact and
order-independent, so any world size gives bit-identical Moments. One process per GPU;
backend "nccl" (RCCL over xGMI) on the GPU box, "gloo" for the CPU tests.
"""
from __future__ import annotations

import numpy as np

from .columns import SpanColumns


def _mix64(z: np.ndarray) -> np.ndarray:
    """splitmix64 finalizer, vectorised (zk_mix64 in zk_tracegen.h; uint64 wrap-around)."""
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def shard_of(trace_ids: np.ndarray, world: int) -> np.ndarray:
    """Shard index of every traceId: zk_trace_shard = mix64(traceId) % world (the hash the device
    tracegen and ingest use; tests/test_multirank.py checks it against the library)."""
    tids = np.asarray(trace_ids, dtype=np.uint64)
    if world <= 1:
        return np.zeros(len(tids), np.uint32)
    return (_mix64(tids) % np.uint64(world)).astype(np.uint32)


def split(cols: SpanColumns, world: int) -> list[SpanColumns]:
    """Partition a trace-clustered batch into per-rank batches (order inside a shard is kept)."""
    s = shard_of(cols.trace_id, world)
    return [cols.take(np.flatnonzero(s == r)) for r in range(world)]


def allreduce_table(table, group=None) -> None:
    """In-place SUM of the exact accumulator's exchange form (int64 tensor, device or host: the
    buffer zk_deps_partial returns) across ranks.

    int64 two's-complement addition is bit-identical to the u64 limb addition the layout needs.
    """
    import torch.distributed as dist

    dist.all_reduce(table, op=dist.ReduceOp.SUM, group=group)


def allreduce_sketch(registers, histogram, group=None) -> None:
    """In-place merge of realtime sketches of disjoint shards (zk_rt_partial): HyperLogLog
    registers by element-wise MAX (uint8), duration histogram bins by SUM (int32 as the u32 bins:
    two's-complement addition is the same below 2^31 per bin and shard sum)."""
    import torch.distributed as dist

    dist.all_reduce(registers, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(histogram, op=dist.ReduceOp.SUM, group=group)


def allreduce_kv_counters(counters, totals, group=None) -> None:
    """In-place SUM of count-min counters and per-service totals (zk_kv_partial); the candidate
    lists are then all-gathered and re-estimated on every rank (zk_kv_merge_candidates)."""
    import torch.distributed as dist

    dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(totals, op=dist.ReduceOp.SUM, group=group)


_TYPESTR = {"uint8": "|u1", "int32": "<i4", "int64": "<i8"}


class _DeviceBuffer:
    """__cuda_array_interface__ (v3) of a library-owned device buffer, for torch.as_tensor."""

    def __init__(self, ptr: int, nbytes: int, dtype):
        name = str(dtype).replace("torch.", "")
        size = {"uint8": 1, "int32": 4, "int64": 8}[name]
        if nbytes % size:
            raise ValueError(f"{nbytes} bytes is not a whole number of {name}")
        self.__cuda_array_interface__ = {"shape": (nbytes // size,), "typestr": _TYPESTR[name],
                                         "data": (int(ptr), False), "version": 3, "strides": None}


def device_view(ptr: int, nbytes: int, dtype, device: int = 0):
    """Zero-copy torch tensor over a buffer the library owns (zk_rt_partial / zk_kv_partial /
    zk_kv_candidates), so that RCCL reduces the sketch state in place. The view does not keep
    the handle alive: use it only while the sketch is open."""
    import torch

    return torch.as_tensor(_DeviceBuffer(ptr, nbytes, dtype), device=torch.device("cuda", device))


def rt_views(rt, device: int = 0):
    """(registers uint8[S*2^p], histogram int32[S*bins]) device views of an RtSketch."""
    import torch

    rp, rb, hp, hb = rt.partial()
    return device_view(rp, rb, torch.uint8, device), device_view(hp, hb, torch.int32, device)


def kv_views(kv, device: int = 0):
    """(counters int32[S*depth*width], totals int64[S], candidate keys int64[S, C], candidate
    estimates int32[S, C]) device views of a KvSketch."""
    import torch

    cp, cb, tp, tb = kv.partial()
    kp, ep, kb, eb = kv.candidate_buffers()
    S, C = kv.num_services, kv.candidates
    return (device_view(cp, cb, torch.int32, device), device_view(tp, tb, torch.int64, device),
            device_view(kp, kb, torch.int64, device).view(S, C), device_view(ep, eb, torch.int32, device).view(S, C))


def merge_rt(rt, group=None, device: int = 0) -> None:
    """Job-wide realtime sketch on every rank: MAX/SUM all-reduce of this rank's RtSketch state
    (each rank fed a disjoint traceId shard). Call after the rank's accumulates; the library's
    stream is drained first, the collective runs on torch's current stream and is complete on
    return, so the sketch's queries read the merged state."""
    import torch

    torch.cuda.synchronize(device)
    regs, hist = rt_views(rt, device)
    allreduce_sketch(regs, hist, group)
    torch.cuda.current_stream(device).synchronize()


def merge_kv(kv, group=None, device: int = 0) -> None:
    """Job-wide key-value top-K on every rank (any item sharding): SUM all-reduce of the count-min
    counters and totals, all-gather of every rank's candidate lists, then zk_kv_merge_candidates
    re-estimates them against the merged counters, so every rank holds the same lists."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    torch.cuda.synchronize(device)
    counters, totals, keys, est = kv_views(kv, device)
    # the candidate lists are gathered before anything changes them: the merge overwrites them
    all_keys = torch.empty((world,) + tuple(keys.shape), dtype=keys.dtype, device=keys.device)
    all_est = torch.empty((world,) + tuple(est.shape), dtype=est.dtype, device=est.device)
    dist.all_gather_into_tensor(all_keys, keys.contiguous(), group=group)
    dist.all_gather_into_tensor(all_est, est.contiguous(), group=group)
    allreduce_kv_counters(counters, totals, group)
    torch.cuda.current_stream(device).synchronize()
    kv.merge_candidates(all_keys, all_est, world)
    torch.cuda.synchronize(device)


def allreduce_stats(stats: dict, device="cpu", group=None) -> dict:
    """Job-wide zk_stats: every counter is a sum over ranks."""
    import torch
    import torch.distributed as dist

    keys = sorted(stats)
    t = torch.tensor([int(stats[k]) for k in keys], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return {k: int(v) for k, v in zip(keys, t.tolist())}


class ShardedDeps:
    """One rank of the sharded job: a DepsContext whose exchange buffer is all-reduced.

    step(cols): reset -> accumulate this rank's shard -> zk_deps_partial (counters folded into the
    accumulator's tail, the accumulator packed into 56-bit limbs in the ctx's exchange buffer) -> ONE
    SUM all-reduce of THAT buffer (never of the accumulator itself: note_merged overwrites the
    accumulator from the exchange buffer) -> note_merged -> finalize. With
    world == 1 the all-reduce is skipped. Every rank ends with the same finalized table AND the
    same status: finalize decides errors from the job-wide counters, so a strict-mode failure on
    one shard fails every rank instead of leaving the others blocked in the next collective.
    """

    def __init__(self, num_services: int, *, device: int = 0, stream=None, timing: bool = False,
                 group=None):
        import torch
        import torch.distributed as dist

        from .context import DepsContext

        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.group = group
        self.device = device
        self.num_services = num_services
        dev = torch.device("cuda", device)
        # the library's kernels and the RCCL all-reduce must be ordered on ONE stream
        self.stream = torch.cuda.Stream(device=dev) if stream is None else stream
        self.ctx = DepsContext(num_services, device=device, stream=self.stream.cuda_stream, timing=timing)

    def step(self, cols, total_records: int | None = None, out_device=None, *, clustered: bool = False,
             verify: bool = True):
        import torch

        self.ctx.reset()
        self.ctx.accumulate(cols, clustered=clustered, verify=verify)
        if self.world > 1:
            # counters -> table tail, then the table's 56-bit-limb exchange form, on the ctx stream
            ptr, nbytes = self.ctx.partial()
            with torch.cuda.stream(self.stream):  # RCCL waits for the pack on this stream
                allreduce_table(device_view(ptr, nbytes, torch.int64, self.device), self.group)
            # 0: the library reads the merged record count from the all-reduced tail
            self.ctx.note_merged(total_records or 0)
        return self.ctx.finalize(out_device=out_device)
