"""The library's own RCCL communicator (include/zkcomm.h) -- the multi-GPU step a JVM host calls
through JNI -- at world size 1 on the GPU box (one GPU per rank; RCCL refuses two ranks on one
device). At world 1 each collective is the identity, so every merge must leave the result
bit-exact: the dependency table against the oracle, the sketches against their state before the
merge. The N>1 arithmetic of the same merges is covered on one GPU by test_gpu_sharded.py and
test_gpu_sketch_shards.py, and over gloo by test_multirank.py."""
import numpy as np
import pytest

from oracle import oracle
from tests.test_gpu_parity import assert_parity
from zipkin_amd import DepsContext, ZkError, _abi, tracegen_host
from zipkin_amd.comm import Comm, unique_id

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm(gpu):
    with Comm(unique_id(), 0, 1, device=0) as c:
        yield c


def test_deps_allreduce_at_world_one_is_exact(comm):
    S = 500
    cols = tracegen_host(31, 40_000, max_depth=6, num_services=S)
    ref = oracle.aggregate(cols, S)
    with DepsContext(S) as ctx:
        ctx.accumulate(cols, clustered=True, verify=True)
        comm.allreduce_deps(ctx)  # partial -> RCCL int64 SUM -> note_merged (total read from the tail)
        assert_parity(ctx.finalize(), ctx.stats(), ref)
        ctx.reset()  # a fresh job on the same ctx and communicator, total given by the caller
        ctx.accumulate(cols, clustered=True)
        comm.allreduce_deps(ctx, total_records=len(cols))
        assert_parity(ctx.finalize(), ctx.stats(), ref)


def test_deps_allreduce_carries_the_error_counters(comm):
    """The strict-mode failure travels in the exchange tail, so finalize fails after the merge."""
    from tests.test_gpu_parity import SERVER, cols_from_rows

    bad = cols_from_rows([(7, 70, 0, 1, 9, 0, SERVER),
                          (7, 71, 70, 2, 4, 0, _abi.ZK_F_HAS_ANNOTATIONS | 1 | (1 << 12) | (1 << 14))])
    with DepsContext(3, strict=True) as ctx:
        ctx.accumulate(bad, clustered=True)
        comm.allreduce_deps(ctx)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_NO_SERVICE


def test_sketch_allreduce_at_world_one_is_identity(comm):
    from oracle.kv import zipf_items
    from zipkin_amd.kv import KvSketch
    from zipkin_amd.realtime import RtSketch

    S = 57
    cols = tracegen_host(32, 8_000, max_depth=6, num_services=S)
    with DepsContext(S, strict=False) as ctx, RtSketch(S) as rt:
        rt.bind(ctx, only=True)
        ctx.accumulate(cols, clustered=True)
        regs, hist = rt.read()
        est = rt.distinct_traces()
        comm.allreduce_rt(rt)
        r2, h2 = rt.read()
        assert np.array_equal(regs, r2) and np.array_equal(hist, h2)
        assert np.array_equal(est, rt.distinct_traces())
        rt.unbind()
    svc, keys = zipf_items(200_000, S, 5000, seed=3)
    with KvSketch(S) as kv:
        kv.accumulate(svc, keys)
        before = kv.topk_all(10)
        tot = kv.totals()
        comm.allreduce_kv(kv)
        after = kv.topk_all(10)
        for a, b in zip(before, after):
            assert np.array_equal(a, b)
        assert np.array_equal(tot, kv.totals())


def test_aborted_rank_through_the_communicator(comm):
    """zk_deps_abort + zk_deps_allreduce (the JVM job's failure path): finalize fails with
    ZK_ERR_RANK_FAILED instead of a rank waiting in the collective; reset clears the mark."""
    S = 57
    cols = tracegen_host(33, 3_000, max_depth=6, num_services=S)
    with DepsContext(S) as ctx:
        ctx.accumulate(cols, clustered=True)
        ctx.abort()
        comm.allreduce_deps(ctx)
        with pytest.raises(ZkError) as e:
            ctx.finalize()
        assert e.value.status == _abi.ZK_ERR_RANK_FAILED
        ctx.reset()
        ctx.accumulate(cols, clustered=True)
        comm.allreduce_deps(ctx)
        assert_parity(ctx.finalize(), ctx.stats(), oracle.aggregate(cols, S))


def test_comm_create_error_text(gpu):
    """A failed zk_comm_create reports RCCL's reason through zk_comm_last_error(NULL)."""
    from zipkin_amd import _abi as A

    L = A.lib()
    import ctypes as C

    h = C.c_void_p()
    st = L.zk_comm_create((C.c_uint8 * 128)(), 128, 0, 1, 99, C.byref(h))  # no device 99
    assert st == A.ZK_ERR_NO_DEVICE and not h.value
    assert b"device" in L.zk_comm_last_error(None)
