// zk_kv.hip — count-min sketch + top-K candidates of binary-annotation keys per service.
//
// Behind Aggregates.getTopKeyValueAnnotations(serviceName) (zipkin-common/.../storage/
// Aggregates.scala:34; the Cassandra store keeps "the most popular keys" per service,
// CassandraAggregates.scala:86-88,104-108). No reference computes it any more (its producer was
// removed, CHANGELOG:7-8); the key definition follows the span indexer: one item per binary
// annotation, service = the annotation host's service name (CassieSpanStore.scala:235-241).
//
// Per batch, after the partition by service (zk_partition.hip):
//   sketch      one workgroup per unit (<= 64k keys of one service): count-min rows in LDS
//               (depth x width u32), flushed with one atomic per non-zero counter;
//   candidates  same units, after every unit's counts are in: estimate every key with the final
//               counters (min over rows) and keep the unit's top `cand` distinct keys by
//               (estimate desc, key asc) in an LDS hash set with a rising threshold;
//   merge       one workgroup per service: previous candidates and the units' lists, all
//               re-estimated with the current counters, -> the service's top `cand`.
// The result is deterministic: it equals "top `cand` by current estimate among (previous
// candidates U this batch's distinct keys)", which oracle/kv.py restates.
#include "zk_sketch_internal.h"

namespace zk {
namespace {

constexpr int kKvWG = 256;
constexpr uint32_t kSetCap = 2048;  // LDS hash-set slots (load <= 0.5)
constexpr uint32_t kSortCap = 1024; // compaction sort buffer
constexpr uint32_t kRound = 2 * kKvWG;
constexpr uint64_t kEmptyKey = ~0ull;

__device__ __forceinline__ bool beats(uint32_t e1, uint64_t k1, uint32_t e2, uint64_t k2) {
    return e1 > e2 || (e1 == e2 && k1 < k2);
}

__device__ __forceinline__ uint32_t row_index(uint64_t key, uint64_t seed, uint32_t wbits) {
    return (uint32_t)(sk_mix64(key ^ seed) >> (64 - wbits));
}

__device__ __forceinline__ uint32_t estimate(const uint32_t* cm, const KvArgs& a, uint64_t key) {
    uint32_t e = 0xFFFFFFFFu;
    for (uint32_t r = 0; r < a.depth; ++r) e = min(e, cm[r * a.width + row_index(key, a.seeds[r], a.wbits)]);
    return e;
}

// Distinct (key, estimate) set keeping the best `keep` entries (estimate desc, key asc).
struct TopSet {
    uint64_t hk[kSetCap];
    uint32_t he[kSetCap];
    uint64_t sk[kSortCap];
    uint32_t se[kSortCap];
    uint32_t count, gcount;
    uint32_t has_thr, thr_est;
    uint64_t thr_key;
    uint32_t special, special_est;  // the key equal to the empty sentinel
};

__device__ void ts_init(TopSet& t) {
    for (uint32_t x = threadIdx.x; x < kSetCap; x += kKvWG) t.hk[x] = kEmptyKey;
    if (threadIdx.x == 0) {
        t.count = 0;
        t.has_thr = 0;
        t.special = 0;
    }
    __syncthreads();
}

__device__ __forceinline__ void ts_insert(TopSet& t, uint64_t key, uint32_t est) {
    if (key == kEmptyKey) {
        if (atomicCAS(&t.special, 0u, 1u) == 0u) {
            t.special_est = est;
            atomicAdd(&t.count, 1u);
        }
        return;
    }
    uint32_t slot = (uint32_t)sk_mix64(key ^ 0x2545F4914F6CDD1Dull) & (kSetCap - 1);
    for (;;) {
        const unsigned long long old =
            atomicCAS((unsigned long long*)&t.hk[slot], (unsigned long long)kEmptyKey, (unsigned long long)key);
        if (old == kEmptyKey) {
            t.he[slot] = est;
            atomicAdd(&t.count, 1u);
            return;
        }
        if (old == key) return;
        slot = (slot + 1) & (kSetCap - 1);
    }
}

__device__ __forceinline__ void ts_offer(TopSet& t, uint64_t key, uint32_t est) {
    if (est == 0u) return;
    if (t.has_thr && !beats(est, key, t.thr_est, t.thr_key)) return;
    ts_insert(t, key, est);
}

// gather + sort (best first) into sk/se; returns the number of entries. Clears the set.
__device__ uint32_t ts_sort(TopSet& t) {
    if (threadIdx.x == 0) t.gcount = 0;
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < kSetCap; x += kKvWG) {
        const uint64_t k = t.hk[x];
        if (k != kEmptyKey) {
            const uint32_t p = atomicAdd(&t.gcount, 1u);
            t.sk[p] = k;
            t.se[p] = t.he[x];
        }
        t.hk[x] = kEmptyKey;
    }
    __syncthreads();
    if (threadIdx.x == 0 && t.special) {
        const uint32_t p = t.gcount++;
        t.sk[p] = kEmptyKey;
        t.se[p] = t.special_est;
    }
    __syncthreads();
    const uint32_t n = t.gcount;
    for (uint32_t x = n + threadIdx.x; x < kSortCap; x += kKvWG) {
        t.sk[x] = kEmptyKey;
        t.se[x] = 0u;  // padding never beats a real entry (real estimates are >= 1)
    }
    __syncthreads();
    for (uint32_t k = 2; k <= kSortCap; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t x = threadIdx.x; x < kSortCap; x += kKvWG) {
                const uint32_t y = x ^ j;
                if (y > x) {
                    const bool best_first = (x & k) == 0;
                    const uint32_t ex = t.se[x], ey = t.se[y];
                    const uint64_t kx = t.sk[x], ky = t.sk[y];
                    const bool sw = best_first ? beats(ey, ky, ex, kx) : beats(ex, kx, ey, ky);
                    if (sw) {
                        t.se[x] = ey;
                        t.se[y] = ex;
                        t.sk[x] = ky;
                        t.sk[y] = kx;
                    }
                }
            }
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) {
        t.count = 0;
        t.special = 0;
    }
    __syncthreads();
    return n;
}

// keep the best `keep`, raise the threshold when the kept set is full
__device__ void ts_compact(TopSet& t, uint32_t keep) {
    const uint32_t n = ts_sort(t);
    const uint32_t m = n < keep ? n : keep;
    if (threadIdx.x == 0 && m == keep && keep > 0) {
        t.has_thr = 1;
        t.thr_est = t.se[m - 1];
        t.thr_key = t.sk[m - 1];
    }
    for (uint32_t x = threadIdx.x; x < m; x += kKvWG) ts_insert(t, t.sk[x], t.se[x]);
    __syncthreads();
}

__device__ __forceinline__ uint32_t find_service(const uint32_t* __restrict__ unit_base, uint32_t S, uint32_t u) {
    // largest s with unit_base[s] <= u (services without units share their successor's base)
    uint32_t lo = 0, hi = S;  // invariant: unit_base[lo] <= u < unit_base[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (unit_base[mid] <= u)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kKvWG) void k_kv_sketch(KvArgs a) {
    extern __shared__ uint32_t cm[];
    const uint32_t u = blockIdx.x;
    if (u >= a.unit_base[a.S]) return;
    const uint32_t s = find_service(a.unit_base, a.S, u);
    const uint64_t lo = a.seg[s] + (uint64_t)(u - a.unit_base[s]) * a.unit_items;
    const uint64_t end = a.seg[s + 1];
    const uint64_t hi = lo + a.unit_items < end ? lo + a.unit_items : end;
    const uint32_t cells = a.depth * a.width;
    for (uint32_t x = threadIdx.x; x < cells; x += kKvWG) cm[x] = 0u;
    __syncthreads();
    constexpr int U = 4;
    for (uint64_t b = lo; b < hi; b += (uint64_t)kKvWG * U) {
        uint64_t k[U];
#pragma unroll
        for (int e = 0; e < U; ++e) {
            const uint64_t i = b + (uint64_t)e * kKvWG + threadIdx.x;
            k[e] = a.keys[i < hi ? i : lo];
        }
#pragma unroll
        for (int e = 0; e < U; ++e) {
            if (b + (uint64_t)e * kKvWG + threadIdx.x < hi)
                for (uint32_t r = 0; r < a.depth; ++r)
                    atomicAdd(&cm[r * a.width + row_index(k[e], a.seeds[r], a.wbits)], 1u);
        }
    }
    __syncthreads();
    uint32_t* g = a.cm + (uint64_t)s * cells;
    for (uint32_t x = threadIdx.x; x < cells; x += kKvWG) {
        const uint32_t v = cm[x];
        if (v) atomicAdd(&g[x], v);
    }
    if (threadIdx.x == 0) atomicAdd((unsigned long long*)&a.totals[s], (unsigned long long)(hi - lo));
}

__device__ void load_cm(uint32_t* cm, const KvArgs& a, uint32_t s) {
    const uint32_t cells = a.depth * a.width;
    const uint32_t* g = a.cm + (uint64_t)s * cells;
    for (uint32_t x = threadIdx.x; x < cells; x += kKvWG) cm[x] = g[x];
}

__global__ __launch_bounds__(kKvWG) void k_kv_candidates(KvArgs a) {
    extern __shared__ uint32_t cm[];
    __shared__ TopSet t;
    const uint32_t u = blockIdx.x;
    if (u >= a.unit_base[a.S]) return;
    const uint32_t s = find_service(a.unit_base, a.S, u);
    const uint64_t lo = a.seg[s] + (uint64_t)(u - a.unit_base[s]) * a.unit_items;
    const uint64_t end = a.seg[s + 1];
    const uint64_t hi = lo + a.unit_items < end ? lo + a.unit_items : end;
    load_cm(cm, a, s);
    ts_init(t);  // contains the barrier that publishes cm
    for (uint64_t b = lo; b < hi; b += kRound) {
        uint64_t k[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const uint64_t i = b + (uint64_t)e * kKvWG + threadIdx.x;
            k[e] = a.keys[i < hi ? i : lo];
        }
#pragma unroll
        for (int e = 0; e < 2; ++e)
            if (b + (uint64_t)e * kKvWG + threadIdx.x < hi) ts_offer(t, k[e], estimate(cm, a, k[e]));
        __syncthreads();
        if (t.count > kSortCap - kRound) ts_compact(t, a.cand);
    }
    const uint32_t n = ts_sort(t);
    uint64_t* ok = a.unit_key + (uint64_t)u * a.cand;
    uint32_t* oe = a.unit_est + (uint64_t)u * a.cand;
    for (uint32_t x = threadIdx.x; x < a.cand; x += kKvWG) {
        ok[x] = x < n ? t.sk[x] : 0ull;
        oe[x] = x < n ? t.se[x] : 0u;
    }
}

// one workgroup per service: previous candidates + this batch's unit lists (+ extra lists)
__global__ __launch_bounds__(kKvWG) void k_kv_merge(KvArgs a, uint32_t use_units) {
    extern __shared__ uint32_t cm[];
    __shared__ TopSet t;
    const uint32_t s = blockIdx.x;
    load_cm(cm, a, s);
    ts_init(t);
    const uint32_t C = a.cand;
    const uint32_t u0 = use_units ? a.unit_base[s] : 0, u1 = use_units ? a.unit_base[s + 1] : 0;
    // flattened source list: [prev | units u0..u1 | extra lists], each C entries
    const uint64_t nsrc = (uint64_t)(1 + (u1 - u0) + a.extra_lists) * C;
    for (uint64_t b = 0; b < nsrc; b += kRound) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const uint64_t i = b + (uint64_t)e * kKvWG + threadIdx.x;
            if (i >= nsrc) continue;
            const uint64_t list = i / C, x = i % C;
            uint64_t key;
            uint32_t old;
            if (list == 0) {
                key = a.cand_key[(uint64_t)s * C + x];
                old = a.cand_est[(uint64_t)s * C + x];
            } else if (list <= (uint64_t)(u1 - u0)) {
                const uint64_t u = u0 + list - 1;
                key = a.unit_key[u * C + x];
                old = a.unit_est[u * C + x];
            } else {
                const uint64_t l = list - 1 - (u1 - u0);
                key = a.extra_key[(l * a.S + s) * C + x];
                old = a.extra_est[(l * a.S + s) * C + x];
            }
            if (old) ts_offer(t, key, estimate(cm, a, key));
        }
        __syncthreads();
        if (t.count > kSortCap - kRound) ts_compact(t, C);
    }
    const uint32_t n = ts_sort(t);
    for (uint32_t x = threadIdx.x; x < C; x += kKvWG) {
        a.cand_key[(uint64_t)s * C + x] = x < n ? t.sk[x] : 0ull;
        a.cand_est[(uint64_t)s * C + x] = x < n ? t.se[x] : 0u;
    }
}

__global__ void k_kv_estimate(KvArgs a, uint32_t s, const uint64_t* __restrict__ keys, uint64_t n,
                              uint32_t* __restrict__ est) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t* g = a.cm + (uint64_t)s * a.depth * a.width;
    est[i] = estimate(g, a, keys[i]);
}

}  // namespace

hipError_t launch_kv_sketch(const KvArgs& a, hipStream_t s) {
    if (!a.max_units) return hipSuccess;
    hipLaunchKernelGGL(k_kv_sketch, dim3(a.max_units), dim3(kKvWG), (size_t)a.depth * a.width * 4, s, a);
    return hipGetLastError();
}

hipError_t launch_kv_candidates(const KvArgs& a, hipStream_t s) {
    if (!a.max_units) return hipSuccess;
    hipLaunchKernelGGL(k_kv_candidates, dim3(a.max_units), dim3(kKvWG), (size_t)a.depth * a.width * 4, s, a);
    return hipGetLastError();
}

hipError_t launch_kv_merge(const KvArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_kv_merge, dim3(a.S), dim3(kKvWG), (size_t)a.depth * a.width * 4, s, a,
                       a.max_units ? 1u : 0u);
    return hipGetLastError();
}

hipError_t launch_kv_estimate(const KvArgs& a, uint32_t svc, const uint64_t* keys, uint64_t n, uint32_t* est,
                              hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_kv_estimate, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, svc, keys, n, est);
    return hipGetLastError();
}

}  // namespace zk
