"""The CPU baseline (oracle/zk_cpu_port.c, bench.py's cpu_baseline leg) equals the oracle bit for
bit: exact power sums and every counter, clustered and any-order modes, any thread count."""
import numpy as np
import pytest

from oracle import oracle
from tests.test_gpu_parity import cols_from_rows, star_trace
from zipkin_amd import tracegen_host


def same(a, b):
    assert np.array_equal(a.cells, b.cells)
    assert a.stats == b.stats


@pytest.mark.parametrize("seed,traces,depth,S", [(1, 3000, 7, 57), (2, 20000, 6, 500), (3, 5000, 3, 1)])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_port_equals_oracle(seed, traces, depth, S, threads):
    cols = tracegen_host(seed, traces, max_depth=depth, num_services=S)
    ref = oracle.aggregate(cols, S, threads=4)
    same(oracle.aggregate_port(cols, S, threads=threads, clustered=True), ref)
    shuffled = cols.take(np.random.default_rng(seed).permutation(len(cols)))
    same(oracle.aggregate_port(shuffled, S, threads=threads, clustered=False), ref)


def test_port_edge_traces():
    rows = []
    for t, n in enumerate([0, 1, 2, 700, 3000, 5]):
        rows += star_trace(100 + t, n, svc_root=t % 5, nsvc=5, fragments=1 + t % 2)
    # a span with many duplicate fragments (saturating core counts) and an invalid parent
    rows += [(9, 90, 0, 1, 50, 0, 0x2 | 0x8 | (1 << 12) | (1 << 14))] * 3
    rows += [(9, 91, 90, 2, 9, 1, 0x2 | 0x8 | 1 | (1 << 12) | (1 << 14))]
    cols = cols_from_rows(rows)
    ref = oracle.aggregate(cols, 5)
    for threads in (1, 2, 7):
        same(oracle.aggregate_port(cols, 5, threads=threads, clustered=True), ref)
        same(oracle.aggregate_port(cols, 5, threads=threads, clustered=False), ref)
    empty = cols_from_rows([])
    same(oracle.aggregate_port(empty, 5, threads=4), oracle.aggregate(empty, 5))
