// zk_cluster.hip — order-agnostic input and the trace-clustering check.
//
// The reference job accepts span fragments in any order: Scalding shuffles them by key before
// every reduce (groupBy((id, traceId)) at ZipkinAggregateJob.scala:21-22, the (parentId, traceId)
// join key at :28-33). K1 instead merges and joins inside a trace segment, so it needs every
// fragment of a trace to be adjacent. Two device pieces bridge that:
//
//  * clustering pass (batches without ZK_BATCH_TRACE_CLUSTERED): a radix sort of the 64-bit
//    traceIds carrying the record index (rocprim, stable), then one gather of the seven columns
//    into ctx-owned, 16-byte-aligned scratch columns. The full 64-bit key is sorted: clustering
//    on any narrower hash would interleave two traces whose hashes collide.
//  * trace set (ZK_BATCH_VERIFY_TRACES): every trace segment start inserts its traceId into an
//    open-addressing set of all traceIds accumulated since the last reset. A traceId found again
//    means a trace split into two non-adjacent runs, or spread over two accumulate calls -- both
//    would be mis-joined silently -- and is counted in ST_NOT_CLUSTERED (finalize then returns
//    ZK_ERR_NOT_CLUSTERED). Exact: the set stores whole traceIds, so it has no false positives.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "zk_cluster.h"
#include "zk_launch.h"
#include "zk_tracegen.h"

namespace zk {
namespace {

constexpr uint64_t kSetSalt = 0x6A09E667F3BCC909ull;

__device__ __forceinline__ uint64_t set_slot(uint64_t tid, uint64_t mask) { return zk_mix64(tid ^ kSetSalt) & mask; }

// insert `tid` (!= 0); returns true if it was already present
__device__ __forceinline__ bool set_insert(unsigned long long* set, uint64_t mask, uint64_t tid) {
    uint64_t s = set_slot(tid, mask);
    for (;;) {
        const unsigned long long old = atomicCAS(&set[s], 0ull, (unsigned long long)tid);
        if (old == 0ull) return false;
        if (old == tid) return true;
        s = (s + 1) & mask;
    }
}

__global__ __launch_bounds__(256) void k_gather_cols(SpanColsDev in, const uint32_t* __restrict__ idx,
                                                     SpanColsMut out) {
    const uint64_t n = in.n;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t j = idx[i];
        out.span_id[i] = in.span_id[j];
        out.parent_id[i] = in.parent_id[j];
        out.first_ts[i] = in.first_ts[j];
        out.last_ts[i] = in.last_ts[j];
        out.service_id[i] = in.service_id[j];
        out.flags[i] = in.flags[j];
    }
}

// One lane per record: a record whose traceId differs from its predecessor's starts a segment.
// set[slots] counts segments of the traceId 0 (the empty-slot marker cannot be stored).
__global__ __launch_bounds__(256) void k_trace_set_insert(const uint64_t* __restrict__ tid, uint64_t n,
                                                          unsigned long long* __restrict__ set, uint64_t slots,
                                                          unsigned long long* __restrict__ dup) {
    uint32_t found = 0;
    const uint64_t mask = slots - 1;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = tid[i];
        if (i > 0 && tid[i - 1] == t) continue;
        if (t == 0ull) {
            if (atomicAdd(&set[slots], 1ull) > 0ull) ++found;
        } else if (set_insert(set, mask, t)) {
            ++found;
        }
    }
    if (found) atomicAdd(dup, (unsigned long long)found);
}

__global__ __launch_bounds__(256) void k_trace_set_rehash(const unsigned long long* __restrict__ old, uint64_t old_slots,
                                                          unsigned long long* __restrict__ set, uint64_t slots) {
    const uint64_t mask = slots - 1;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= old_slots; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long v = old[i];
        if (i == old_slots)
            set[slots] = v;  // the traceId-0 counter
        else if (v)
            set_insert(set, mask, v);
    }
}

// stats shards -> the 16 totals in the table's tail (zk_deps_partial)
__global__ __launch_bounds__(256) void k_stats_fold(const unsigned long long* __restrict__ shards, int nshards,
                                                    unsigned long long* __restrict__ out) {
    __shared__ unsigned long long s[256];
    const int t = threadIdx.x, stat = t & (ST_N - 1), part = t / ST_N;  // 16 partial sums per stat
    unsigned long long v = 0;
    for (int sh = part; sh < nshards; sh += 256 / ST_N) v += shards[(uint64_t)sh * ST_N + stat];
    s[t] = v;
    __syncthreads();
    if (t < ST_N) {
        unsigned long long tot = 0;
        for (int p = 0; p < 256 / ST_N; ++p) tot += s[p * ST_N + t];
        out[t] = tot;
    }
}

unsigned grid_for(uint64_t n) {
    const uint64_t g = (n + 255) / 256;
    return (unsigned)(g < 8192 ? (g ? g : 1) : 8192);
}

}  // namespace

hipError_t cluster_temp_bytes(uint64_t n, size_t* bytes) {
    size_t b = 0;
    const hipError_t e = rocprim::radix_sort_pairs(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                   rocprim::counting_iterator<uint32_t>(0u), (uint32_t*)nullptr,
                                                   (uint32_t)n, 0u, 64u, (hipStream_t)0);
    *bytes = b;
    return e;
}

hipError_t launch_cluster(const SpanColsDev& in, const SpanColsMut& out, uint32_t* idx, void* temp, size_t temp_bytes,
                          hipStream_t s) {
    if (in.n == 0) return hipSuccess;
    size_t b = temp_bytes;
    // sorted traceIds land directly in the output traceId column
    hipError_t e = rocprim::radix_sort_pairs(temp, b, in.trace_id, out.trace_id, rocprim::counting_iterator<uint32_t>(0u),
                                             idx, (uint32_t)in.n, 0u, 64u, s);
    if (e != hipSuccess) return e;
    return launch_checked("k_gather_cols", k_gather_cols, dim3(grid_for(in.n)), dim3(256), 0, s, in, idx, out);
}

hipError_t launch_trace_set_insert(const uint64_t* trace_id, uint64_t n, uint64_t* set, uint64_t slots,
                                   unsigned long long* dup, hipStream_t s) {
    if (n == 0) return hipSuccess;
    return launch_checked("k_trace_set_insert", k_trace_set_insert, dim3(grid_for(n)), dim3(256), 0, s, trace_id, n,
                          (unsigned long long*)set, slots, dup);
}

hipError_t launch_trace_set_rehash(const uint64_t* old, uint64_t old_slots, uint64_t* set, uint64_t slots,
                                   hipStream_t s) {
    return launch_checked("k_trace_set_rehash", k_trace_set_rehash, dim3(grid_for(old_slots + 1)), dim3(256), 0, s,
                          (const unsigned long long*)old, old_slots, (unsigned long long*)set, slots);
}

hipError_t launch_stats_fold(const unsigned long long* shards, unsigned long long* out, hipStream_t s) {
    return launch_checked("k_stats_fold", k_stats_fold, dim3(1), dim3(256), 0, s, shards, (int)kStatShards, out);
}

}  // namespace zk
