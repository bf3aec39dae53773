"""Key-value popularity sketch (getTopKeyValueAnnotations, Aggregates.scala:34).

CPU: the oracle (oracle/kv.py) against exact counts -- never undercounts, the count-min error
bound, heavy hitters found. GPU: the HIP path (zk_kv_* through ctypes) bit-exact against the
oracle (same counters, same candidate lists), plus the bound against exact counts at C4 shape.
"""
import math

import numpy as np
import pytest

from oracle.kv import KvOracle, auto_width, exact_counts, mix64, zipf_items
from zipkin_amd import _abi


def _bound(N_s, width):
    return math.e / width * N_s


# ---------------------------------------------------------------------------- CPU: the oracle
def test_mix64_matches_python_int_path():
    xs = np.array([0, 1, 2, 0xFFFFFFFFFFFFFFFF, 0x123456789ABCDEF0], dtype=np.uint64)
    assert [int(v) for v in mix64(xs)] == [mix64(int(x)) for x in xs]
    assert mix64(0) == 0  # splitmix64 finalizer fixes 0


def test_auto_width_budget():
    assert auto_width(500) == 2048 and auto_width(1) == 4096 and auto_width(4096) == 256


def test_oracle_never_undercounts_and_meets_bound():
    S = 8
    svc, keys = zipf_items(200_000, S, num_keys=20_000, seed=1)
    o = KvOracle(S, width=256, depth=4, candidates=32, seed=7)
    o.accumulate(svc, keys)
    ex = exact_counts(svc, keys, S)
    for s in range(S):
        ks = np.array(list(ex[s].keys()), dtype=np.uint64)
        tr = np.array([ex[s][int(k)] for k in ks])
        est = o.estimate(s, ks).astype(np.int64)
        assert (est >= tr).all()
        over = est - tr
        # per key P[over > e/w N_s] <= e^-4: allow 3x that fraction
        assert (over > _bound(int(o.totals[s]), 256)).mean() <= 3 * math.exp(-4)


def test_oracle_topk_finds_heavy_hitters_across_batches():
    S = 4
    svc, keys = zipf_items(120_000, S, num_keys=5000, s=1.3, seed=2)
    o = KvOracle(S, width=1024, depth=4, candidates=16, seed=3)
    for b in range(0, len(svc), 40_000):
        o.accumulate(svc[b:b + 40_000], keys[b:b + 40_000])
    ex = exact_counts(svc, keys, S)
    for s in range(S):
        truth = sorted(ex[s].items(), key=lambda kv: (-kv[1], kv[0]))[:5]
        got = [k for k, _ in o.topk(s, 10)]
        for k, _ in truth:
            assert k in got


def test_oracle_shard_merge_equals_one_sketch_on_heavy_hitters():
    """KvOracle.merged (the restatement of the N>1 merge): summed counters equal one sketch over
    all items bit for bit, and the clear heavy hitters come out with the same estimates."""
    S = 5
    svc, keys = zipf_items(90_000, S, num_keys=4000, s=1.3, seed=6)
    one = KvOracle(S, width=1024, depth=4, candidates=32, seed=3)
    one.accumulate(svc, keys)
    parts = []
    for a, b in ((0, 20_000), (20_000, 20_000), (20_000, 90_000)):
        o = KvOracle(S, width=1024, depth=4, candidates=32, seed=3)
        o.accumulate(svc[a:b], keys[a:b])
        parts.append(o)
    m = KvOracle.merged(parts)
    assert np.array_equal(m.cm, one.cm) and np.array_equal(m.totals, one.totals)
    for s in range(S):
        assert m.topk(s, 5) == one.topk(s, 5)
        for k, e in m.topk(s, 32):  # every merged estimate is the one-sketch estimate
            assert int(one.estimate(s, [k])[0]) == e


def test_oracle_drops_out_of_range_services():
    o = KvOracle(3, width=64, depth=2, candidates=4)
    o.accumulate(np.array([0, 1, 3, 7], np.uint32), np.array([5, 5, 5, 5], np.uint64))
    assert o.dropped == 2 and int(o.totals.sum()) == 2


@pytest.mark.parametrize("S,n,width,seed", [(7, 20_000, 0, 1), (500, 400_000, 0, 2), (64, 100_000, 256, 3),
                                            (1, 5_000, 64, 4)])
def test_c_port_equals_the_oracle(S, n, width, seed):
    """oracle/zk_kv_port.c (the C4 line's checker on large prefixes and its CPU baseline) gives the
    numpy restatement's counters, totals, dropped count and top lists for one batch, bit for bit."""
    from oracle.kv import kv_port

    svc, keys = zipf_items(n, S, seed=seed)
    svc[::97] = S + 3  # out-of-range services are dropped and counted
    o = KvOracle(S, width=width, seed=5)
    o.accumulate(svc, keys)
    p = kv_port(svc, keys, S, o.width, o.depth, o.cand, seed=5, threads=4)
    assert np.array_equal(o.cm.astype(np.uint32), p.cm) and np.array_equal(o.totals, p.totals)
    assert o.dropped == p.dropped
    for x, y in zip(o.topk_all(o.cand), p.topk_all(o.cand)):
        assert np.array_equal(x, y)


def test_kv_handle_rejects_bad_config_without_device():
    import ctypes as C

    L = _abi.lib()
    cfg = _abi.zk_kv_config()
    h = C.c_void_p()
    cfg.num_services = 0
    assert L.zk_kv_create(C.byref(cfg), C.byref(h)) == _abi.ZK_ERR_INVALID_ARG
    cfg.num_services = 10
    cfg.width = 100  # not a power of two
    assert L.zk_kv_create(C.byref(cfg), C.byref(h)) == _abi.ZK_ERR_INVALID_ARG
    cfg.width = 4096
    cfg.depth = 8  # 32k counters: more than the 64 KB LDS budget
    assert L.zk_kv_create(C.byref(cfg), C.byref(h)) == _abi.ZK_ERR_INVALID_ARG
    assert L.zk_kv_reset(None) == _abi.ZK_ERR_INVALID_ARG


# ---------------------------------------------------------------------------- GPU: the product
def _pair(S, **kw):
    from zipkin_amd.kv import KvSketch

    k = KvSketch(S, **kw)
    o = KvOracle(S, width=k.width, depth=k.depth, candidates=k.candidates, seed=kw.get("seed", 0))
    return k, o


def _assert_same(k, o, kk):
    gk, ge, gc = k.topk_all(kk)
    ok_, oe, oc = o.topk_all(kk)
    assert np.array_equal(gc, oc)
    assert np.array_equal(ge, oe)
    assert np.array_equal(gk, ok_)
    assert np.array_equal(k.totals(), o.totals)


@pytest.mark.gpu
@pytest.mark.parametrize("S,n,width,depth,cand", [
    (1, 1, 64, 1, 1),
    (3, 1000, 64, 2, 8),
    (57, 50_000, 0, 4, 64),
    (7, 200_000, 0, 4, 64),  # >= kKvSmallPerService keys per service: the counters through LDS (the others: global)
    (500, 300_000, 0, 4, 16),
    (1022, 200_000, 0, 2, 32),  # largest S whose line-scatter carry fits the LDS
    (1024, 200_000, 0, 2, 32),  # one past it: item-by-item scatter (the line kernel would not launch)
    (2000, 200_000, 0, 3, 256),
    (3, 300_000, 0, 4, 256),  # the LDS path at the largest candidate list: blocks of more survivors than
    (2, 400_000, 256, 4, 200),  # the sort buffer takes are inserted in steps with compactions between
])
def test_gpu_topk_bit_exact_vs_oracle(gpu, S, n, width, depth, cand):
    k, o = _pair(S, width=width, depth=depth, candidates=cand, seed=11)
    svc, keys = zipf_items(n, S, num_keys=max(10, n // 5), seed=S)
    k.accumulate(svc, keys)
    o.accumulate(svc, keys)
    _assert_same(k, o, min(cand, 10))
    _assert_same(k, o, cand)
    # point estimates equal the oracle's counters
    for s in range(min(S, 4)):
        q = keys[:200]
        assert np.array_equal(k.estimate(s, q), o.estimate(s, q).astype(np.uint32))


@pytest.mark.gpu
def test_gpu_multi_batch_and_units_spanning_services(gpu):
    # one service with > 1 unit (64k keys per unit) next to tiny and empty ones
    S = 6
    rng = np.random.default_rng(5)
    svc = np.concatenate([np.full(150_000, 2, np.uint32), rng.integers(0, S, 3000, dtype=np.uint32)])
    _, keys = zipf_items(len(svc), 1, num_keys=30_000, seed=9)
    k, o = _pair(S, width=512, depth=4, candidates=32, seed=1)
    for b in (0, 50_000, 120_000):
        e = {0: 50_000, 50_000: 120_000, 120_000: len(svc)}[b]
        k.accumulate(svc[b:e], keys[b:e])
        o.accumulate(svc[b:e], keys[b:e])
        _assert_same(k, o, 32)
    k.reset()
    o2 = KvOracle(S, width=512, depth=4, candidates=32, seed=1)
    _assert_same(k, o2, 32)


@pytest.mark.gpu
def test_gpu_sentinel_key_and_ties(gpu):
    S = 2
    keys = np.array([0xFFFFFFFFFFFFFFFF] * 5 + [0] * 5 + [7] * 3 + [8] * 3, np.uint64)
    svc = np.zeros(len(keys), np.uint32)
    k, o = _pair(S, width=4096, depth=4, candidates=4)
    k.accumulate(svc, keys)
    o.accumulate(svc, keys)
    _assert_same(k, o, 4)
    top = k.topk(0, 4)
    assert top[0] == (0, 5) and top[1] == (0xFFFFFFFFFFFFFFFF, 5)  # ties: smaller key first
    assert k.topk(1, 4) == []


@pytest.mark.gpu
def test_gpu_service_range_is_an_error(gpu):
    from zipkin_amd import ZkError

    k, _ = _pair(4, width=64, depth=1, candidates=2)
    k.accumulate(np.array([0, 9], np.uint32), np.array([1, 2], np.uint64))
    with pytest.raises(ZkError) as e:
        k.topk_all(2)
    assert e.value.status == _abi.ZK_ERR_SERVICE_RANGE


@pytest.mark.gpu
def test_gpu_device_pointers_and_c4_bound(gpu):
    import torch

    S = 500
    n = 2_000_000
    svc, keys = zipf_items(n, S, seed=4)
    k, o = _pair(S, seed=4)
    k.accumulate(torch.from_numpy(svc.view(np.int32)).cuda(), torch.from_numpy(keys.view(np.int64)).cuda())
    o.accumulate(svc, keys)
    _assert_same(k, o, 10)
    ex = exact_counts(svc, keys, S)
    tot = k.totals()
    gk, ge, gc = k.topk_all(10)
    for s in range(0, S, 25):
        truth = sorted(ex[s].items(), key=lambda kv: (-kv[1], kv[0]))
        eps = _bound(int(tot[s]), k.width)
        for key, est in zip(gk[s][: gc[s]], ge[s][: gc[s]]):
            t = ex[s].get(int(key), 0)
            assert t <= est <= t + eps
        # every key truly above the 10th estimate + eps is reported
        for key, t in truth:
            if t > int(ge[s][gc[s] - 1]) + eps:
                assert int(key) in set(int(x) for x in gk[s])
