"""The N > 1 path on CPU: world_size-2 gloo processes, traceId-hash shards, exact SUM all-reduce.

What the multi-GPU step relies on (zipkin_amd/shards.py):
  * shard = mix64(traceId) % world puts every fragment of a trace on one rank, so merges
    (ZipkinAggregateJob.scala:21) and joins (:30) are rank-local;
  * the carry-free limb table of disjoint shards adds limb-wise to the table of the union, so one
    SUM all-reduce (RCCL on the GPU box, gloo here) gives the exact job-wide power sums.
Each rank aggregates its shard with the oracle (the GPU accumulator is covered by the gpu tests),
encodes the exact sums in the device limb layout, all-reduces through zipkin_amd.shards and checks
the decoded result against the oracle run over the union of all shards.
"""
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle.oracle import aggregate
from zipkin_amd import SpanColumns, table, tracegen_host
from zipkin_amd.shards import shard_of, split

S = 57
WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_sums(cols):
    r = aggregate(cols, S, threads=2)
    return {(int(c) // S, int(c) % S): r.power_sums(int(c)) for c in r.present_cells()}, r.stats


def _worker(rank, world, port, mode):
    import torch
    import torch.distributed as dist

    from zipkin_amd.shards import allreduce_stats, allreduce_table

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        if mode == "tracegen":
            # weak scaling as in bench.py: every rank generates its own shard
            shards = [tracegen_host(seed=5, num_traces=300, max_depth=6, num_services=S, rank=r, world=world)
                      for r in range(world)]
        else:
            # one global batch, partitioned by the ingest-side hash
            full = tracegen_host(seed=6, num_traces=600, max_depth=6, num_services=S)
            shards = split(full, world)
        mine = shards[rank]
        assert len(mine) > 0
        assert (shard_of(np.unique(mine.trace_id), world) == rank).all()

        sums, stats = _oracle_sums(mine)
        # the exchange form zk_deps_partial hands to the all-reduce (56-bit limbs), as the host packs it
        t = torch.from_numpy(table.pack(table.encode(sums, S), S))
        allreduce_table(t)
        got = table.decode(table.unpack(t.numpy(), S), S)
        assert got == table.decode_exchange(t.numpy(), S)
        gstats = allreduce_stats(stats)

        want, wstats = _oracle_sums(SpanColumns.concat(shards))
        assert got == want, "all-reduced limb table differs from the oracle over the union"
        for k in ("records", "merged_spans", "valid_spans", "child_spans", "joined_links", "missing_parent"):
            assert gstats[k] == wstats[k], k
    finally:
        dist.destroy_process_group()


def _sketch_worker(rank, world, port):
    import torch
    import torch.distributed as dist

    from oracle.kv import KvOracle, zipf_items
    from oracle.realtime import RtOracle, merged_span_items
    from zipkin_amd.shards import allreduce_kv_counters, allreduce_sketch

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        full = tracegen_host(seed=8, num_traces=800, max_depth=6, num_services=S)
        shards = split(full, world)
        # realtime sketch: per-shard state, merged by MAX / SUM, equals the sketch of the union
        mine = RtOracle(S, p=10, seed=3)
        mine.accumulate_merged(*merged_span_items(shards[rank], S)[:3])
        regs = torch.from_numpy(mine.regs.copy())
        hist = torch.from_numpy(mine.hist.astype(np.int32))
        allreduce_sketch(regs, hist)
        union = RtOracle(S, p=10, seed=3)
        union.accumulate_merged(*merged_span_items(full, S)[:3])
        assert np.array_equal(regs.numpy(), union.regs)
        assert np.array_equal(hist.numpy().astype(np.uint64), union.hist)
        # count-min counters of item shards add up to the counters of all items
        svc, keys = zipf_items(20_000, S, num_keys=3000, seed=1)
        part = np.arange(len(svc)) % world == rank
        kv = KvOracle(S, width=256, depth=4, candidates=16, seed=2)
        kv.accumulate(svc[part], keys[part])
        cm = torch.from_numpy(kv.cm.astype(np.int64))
        tot = torch.from_numpy(kv.totals.astype(np.int64))
        allreduce_kv_counters(cm, tot)
        allkv = KvOracle(S, width=256, depth=4, candidates=16, seed=2)
        allkv.accumulate(svc, keys)
        assert np.array_equal(cm.numpy().astype(np.uint64), allkv.cm)
        assert np.array_equal(tot.numpy().astype(np.uint64), allkv.totals)
    finally:
        dist.destroy_process_group()


def test_two_rank_sketch_merges_are_exact():
    mp.spawn(_sketch_worker, args=(WORLD, _free_port()), nprocs=WORLD, join=True)


@pytest.mark.parametrize("mode", ["tracegen", "split"])
def test_two_rank_allreduce_is_exact(mode):
    mp.spawn(_worker, args=(WORLD, _free_port(), mode), nprocs=WORLD, join=True)


def test_limb_encoding_roundtrip_and_linearity():
    rng = np.random.default_rng(0)
    d = rng.integers(0, 1 << 40, size=1000, dtype=np.uint64)
    a, b = d[:400], d[400:]

    def sums(x):
        v = [int(t) for t in x]
        return (len(v), sum(v), sum(t * t for t in v), sum(t ** 3 for t in v), sum(t ** 4 for t in v))

    ta = table.encode({(0, 1): sums(a)}, 2).view(np.uint64)
    tb = table.encode({(0, 1): sums(b)}, 2).view(np.uint64)
    tot = (ta + tb).view(np.int64)  # limb-wise u64 addition = the all-reduce
    assert table.decode(tot, 2) == {(0, 1): sums(d)}
    assert table.decode(table.encode({(1, 0): sums(d)}, 2), 2) == {(1, 0): sums(d)}


def test_split_partitions_whole_traces():
    full = tracegen_host(seed=7, num_traces=400, max_depth=5, num_services=S)
    parts = split(full, 4)
    assert sum(len(p) for p in parts) == len(full)
    seen = set()
    for r, p in enumerate(parts):
        u = set(np.unique(p.trace_id).tolist())
        assert not (u & seen)
        seen |= u
        # trace-clustered order survives the split
        change = np.flatnonzero(np.diff(p.trace_id.view(np.int64)) != 0)
        assert len(change) + 1 == len(u)


def test_exchange_form_bounds_and_linearity():
    """56-bit limbs: pack/unpack round trip at the largest sums the accumulator can hold (2^32 - 1
    records of d = 2^40 - 1), and the limb-wise SUM of 256 ranks' exchange buffers decodes to the sum
    of their sums without any limb passing 2^64."""
    n, d = (1 << 32) - 1, (1 << 40) - 1
    big = (n, n * d, n * d ** 2, n * d ** 3, n * d ** 4)
    x = table.encode_exchange({(0, 1): big}, 2)
    assert table.decode_exchange(x, 2) == {(0, 1): big}
    assert np.array_equal(table.unpack(table.pack(table.encode({(0, 1): big}, 2), 2), 2), table.encode({(0, 1): big}, 2))
    # the tightest limb is S2's top one (bits 56..111 of a value below 2^112: up to 2^56 - 1): 256
    # copies of the largest cell still sum without a carry out of any u64 limb, and decode exactly
    xc = table.encode_exchange_cell(*big)
    assert int(xc[4]) < 1 << 56 and int(xc[4]) > (1 << 55)  # S2's top limb really is near 2^56
    summed = [sum(int(v) for _ in range(256)) for v in xc]
    assert max(summed) < 1 << 64
    assert table.decode_exchange_cell(summed) == tuple(256 * v for v in big)
    # 256 ranks each holding 1/256 of the job: every limb of the sum stays below 2^64
    share = tuple(v // 256 for v in big)
    cell = table.encode_exchange_cell(*share).astype(object)
    assert all(int(v) * 256 < 1 << 64 for v in cell)
    rng = np.random.default_rng(3)
    parts = []
    for _ in range(4):
        ds = [int(v) for v in rng.integers(0, 1 << 40, 50, dtype=np.uint64)]
        parts.append((len(ds), sum(ds), sum(v * v for v in ds), sum(v ** 3 for v in ds), sum(v ** 4 for v in ds)))
    tot = sum(table.encode_exchange({(1, 0): p}, 2).view(np.uint64) for p in parts).view(np.int64)
    assert table.decode_exchange(tot, 2) == {(1, 0): tuple(sum(p[i] for p in parts) for i in range(5))}
