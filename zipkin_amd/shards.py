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

from . import _abi
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
    """In-place SUM of the exact accumulator (int64 tensor, device or host) across ranks.

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


def allreduce_stats(stats: dict, device="cpu", group=None) -> dict:
    """Job-wide zk_stats: every counter is a sum over ranks."""
    import torch
    import torch.distributed as dist

    keys = sorted(stats)
    t = torch.tensor([int(stats[k]) for k in keys], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return {k: int(v) for k, v in zip(keys, t.tolist())}


class ShardedDeps:
    """One rank of the sharded job: a DepsContext over a caller-owned (all-reducible) table.

    step(cols): reset -> accumulate this rank's shard -> fold the counters into the table's tail
    (zk_deps_partial) -> ONE SUM all-reduce of limbs + counters -> note_merged -> finalize. With
    world == 1 the all-reduce is skipped. Every rank ends with the same finalized table AND the
    same status: finalize decides errors from the job-wide counters, so a strict-mode failure on
    one shard fails every rank instead of leaving the others blocked in the next collective.
    """

    def __init__(self, num_services: int, *, device: int = 0, stream=None, timing: bool = False,
                 group=None, ablate: int = 0):
        import torch
        import torch.distributed as dist

        from .context import DepsContext

        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.group = group
        self.num_services = num_services
        dev = torch.device("cuda", device)
        # the library's kernels and the RCCL all-reduce must be ordered on ONE stream
        self.stream = torch.cuda.Stream(device=dev) if stream is None else stream
        self.table = torch.zeros(_abi.table_words(num_services), dtype=torch.int64, device=dev)
        torch.cuda.current_stream(dev).synchronize()  # the zeroed table, before the library's stream
        self.ctx = DepsContext(num_services, device=device, stream=self.stream.cuda_stream, timing=timing,
                               table_ptr=self.table.data_ptr(), table_bytes=self.table.numel() * 8, ablate=ablate)

    def step(self, cols, total_records: int | None = None, out_device=None, *, clustered: bool = False,
             verify: bool = True):
        import torch

        self.ctx.reset()
        self.ctx.accumulate(cols, clustered=clustered, verify=verify)
        if self.world > 1:
            self.ctx.partial()  # counters -> table tail, on the ctx stream
            with torch.cuda.stream(self.stream):  # RCCL waits for the accumulate on this stream
                allreduce_table(self.table, self.group)
            # 0: the library reads the merged record count from the all-reduced tail
            self.ctx.note_merged(total_records or 0)
        return self.ctx.finalize(out_device=out_device)
