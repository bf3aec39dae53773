"""The N>1 sketch merges on one GPU (C4 and C5 of SURVEY.md §8): per-shard sketches, their device
state merged in place through zipkin_amd.shards' zero-copy views, queried after the merge.

C5 (RtSketch): each shard is a traceId-hash shard fed through K1 (bound, only=True); the merge is
an element-wise MAX of the HyperLogLog registers and a SUM of the duration bins -- what
shards.allreduce_sketch's RCCL MAX / SUM all-reduce computes on every rank, here as the same torch
reduction over the shards' views. Bar: every rank's registers, bins, distinct-trace estimates and
quantile bins bit-identical to ONE sketch over the whole batch and to the oracle.

C4 (KvSketch): disjoint (ragged, one empty) item shards; counters and totals SUMmed in place, every
shard's candidate lists gathered (as all_gather_into_tensor would) and zk_kv_merge_candidates run
on every rank. Bar: counters bit-identical to one sketch over all items, every rank's top-K
bit-identical to oracle.kv.KvOracle.merged over the per-shard oracles, and the count-min bound
against the exact counts. merge_rt / merge_kv themselves run through RCCL at world size 1
(idempotence); their N>1 collectives are covered by the gloo tests in test_multirank.py.
"""
import math

import numpy as np
import pytest

from oracle.kv import KvOracle, exact_counts, zipf_items
from oracle.realtime import RtOracle, merged_span_items
from zipkin_amd import shards as sh

pytestmark = pytest.mark.gpu


def _rt_shards(cols, S, world, **kw):
    from zipkin_amd import DepsContext
    from zipkin_amd.realtime import RtSketch

    out = []
    for part in sh.split(cols, world):
        ctx = DepsContext(S, device=0, strict=False)
        rt = RtSketch(S, **kw)
        rt.bind(ctx, only=True)
        if len(part):
            ctx.accumulate(part, clustered=True)
        out.append((ctx, rt))
    return out


def _assert_rt_equal(rt, ref, o):
    regs, hist = rt.read()
    r2, h2 = ref.read()
    assert np.array_equal(regs, r2) and np.array_equal(hist, h2)
    assert np.array_equal(regs, o.regs) and np.array_equal(hist.astype(np.uint64), o.hist)
    assert np.array_equal(rt.distinct_traces(), ref.distinct_traces())
    qs = (0.0, 0.5, 0.99, 1.0)
    lo, hi, cnt = rt.quantiles_all(qs)  # every service in one device pass
    for s in range(0, rt.num_services, max(1, rt.num_services // 8)):
        assert rt.quantiles(s, qs) == ref.quantiles(s, qs) == o.quantile_bins(s, qs)
        assert (list(zip(lo[s].tolist(), hi[s].tolist())), int(cnt[s])) == rt.quantiles(s, qs)


@pytest.mark.parametrize("world,seed,traces,S,p", [(2, 1, 4000, 57, 12), (4, 2, 20000, 500, 14), (3, 5, 50, 9, 6)])
def test_rt_shard_merge_bit_exact(gpu, world, seed, traces, S, p):
    import torch

    from zipkin_amd import tracegen_host

    cols = tracegen_host(seed, traces, max_depth=6, num_services=S)
    ref = _rt_shards(cols, S, 1, hll_p=p, seed=7)
    parts = _rt_shards(cols, S, world, hll_p=p, seed=7)
    torch.cuda.synchronize()
    views = [sh.rt_views(rt) for _, rt in parts]
    regs = torch.stack([v[0] for v in views]).amax(0)
    hist = torch.stack([v[1] for v in views]).sum(0, dtype=torch.int32)
    for r, h in views:  # every rank ends with the reduced state, written into the library's buffers
        r.copy_(regs)
        h.copy_(hist)
    torch.cuda.synchronize()
    o = RtOracle(S, p=p, seed=7)
    o.accumulate_merged(*merged_span_items(cols, S)[:3])
    for _, rt in parts:
        _assert_rt_equal(rt, ref[0][1], o)
    for ctx, rt in parts + ref:
        rt.close()
        ctx.close()


def _kv_shards(svc, keys, S, cuts, **kw):
    from zipkin_amd.kv import KvSketch

    gpu, ora = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        k = KvSketch(S, **kw)
        o = KvOracle(S, width=k.width, depth=k.depth, candidates=k.candidates, seed=kw.get("seed", 0))
        if b > a:
            k.accumulate(svc[a:b], keys[a:b])
            o.accumulate(svc[a:b], keys[a:b])
        gpu.append(k)
        ora.append(o)
    return gpu, ora


def _bound(N_s, width):
    return math.ceil(math.e / width * N_s)


@pytest.mark.parametrize("S,n,cuts,cand", [
    (57, 300_000, (0, 0.5, 1.0), 64),
    (500, 600_000, (0, 0.1, 0.1, 0.7, 1.0), 16),  # ragged, one empty shard
    (3, 2000, (0, 0.3, 1.0), 8),
])
def test_kv_shard_merge_bit_exact(gpu, S, n, cuts, cand):
    import torch

    svc, keys = zipf_items(n, S, num_keys=max(10, n // 5), seed=S + 3)
    idx = [int(round(c * n)) for c in cuts]
    world = len(idx) - 1
    (one,), _ = _kv_shards(svc, keys, S, [0, n], candidates=cand, seed=5)
    parts, oras = _kv_shards(svc, keys, S, idx, candidates=cand, seed=5)
    torch.cuda.synchronize()
    views = [sh.kv_views(k) for k in parts]
    all_keys = torch.stack([v[2] for v in views])  # [world, S, C]: gathered before any merge
    all_est = torch.stack([v[3] for v in views])
    counters = torch.stack([v[0] for v in views]).sum(0, dtype=torch.int32)
    totals = torch.stack([v[1] for v in views]).sum(0)
    for v in views:
        v[0].copy_(counters)
        v[1].copy_(totals)
    torch.cuda.synchronize()
    for k in parts:
        k.merge_candidates(all_keys, all_est, world)
    torch.cuda.synchronize()
    o = KvOracle.merged(oras)
    one_counters = sh.kv_views(one)[0]
    ok_, oe, oc = o.topk_all(cand)
    ex = exact_counts(svc, keys, S)
    for k in parts:
        assert torch.equal(sh.kv_views(k)[0], one_counters)  # count-min is linear: SUM is exact
        assert np.array_equal(k.totals(), one.totals())
        gk, ge, gc = k.topk_all(cand)
        assert np.array_equal(gc, oc) and np.array_equal(ge, oe) and np.array_equal(gk, ok_)
    # the merged lists against the exact counts: estimates within the count-min bound, and every
    # key truly above the 10th estimate + eps is reported
    gk, ge, gc = parts[0].topk_all(min(cand, 10))
    tot = parts[0].totals()
    for s in range(0, S, max(1, S // 10)):
        eps = _bound(int(tot[s]), parts[0].width)
        for key, est in zip(gk[s][: gc[s]], ge[s][: gc[s]]):
            t = ex[s].get(int(key), 0)
            assert t <= est <= t + eps
        if gc[s] == min(cand, 10):
            reported = set(int(x) for x in gk[s][: gc[s]])
            for key, t in ex[s].items():
                if t > int(ge[s][gc[s] - 1]) + eps:
                    assert int(key) in reported
    for k in parts + [one]:
        k.close()


@pytest.fixture(scope="module")
def rccl_world1(gpu):
    import os

    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        yield None
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield None
    dist.destroy_process_group()


def test_merge_helpers_through_rccl_are_idempotent(rccl_world1):
    """merge_rt / merge_kv through RCCL at world size 1: the views alias the library's buffers
    and the collective leaves a single rank's state (and therefore its answers) unchanged."""
    from zipkin_amd import tracegen_host

    S = 57
    cols = tracegen_host(3, 3000, max_depth=5, num_services=S)
    ((ctx, rt),) = _rt_shards(cols, S, 1, hll_p=10)
    regs0, hist0 = rt.read()
    d0 = rt.distinct_traces()
    sh.merge_rt(rt)
    regs1, hist1 = rt.read()
    assert np.array_equal(regs0, regs1) and np.array_equal(hist0, hist1)
    assert np.array_equal(d0, rt.distinct_traces())
    rt.close()
    ctx.close()

    svc, keys = zipf_items(100_000, S, num_keys=20_000, seed=2)
    (kv,), (o,) = _kv_shards(svc, keys, S, [0, len(svc)], candidates=32, seed=1)
    before = kv.topk_all(32)
    sh.merge_kv(kv)
    after = kv.topk_all(32)
    for x, y in zip(before, after):
        assert np.array_equal(x, y)
    ok_, oe, oc = o.topk_all(32)
    assert np.array_equal(after[0], ok_) and np.array_equal(after[1], oe)
    kv.close()
