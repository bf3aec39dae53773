// zk_reduce.hip — K3 link_reduce: per-tile link lists -> exact limb table (.group.sum,
// ZipkinAggregateJob.scala:39-40, DependencyLink.sg / MomentsGroup.plus made exact).
//
// A link is (cell << 40) | d. Its contribution to the cell is m0 += 1 and S_k += d^k (k = 1..4),
// laid out as 15 u64 limbs that each absorb 32-bit chunks (no carries before finalize). The 16 lanes
// of a lane group own one link and add the 15 limbs of one 128-byte cell, so a wave instruction
// issues four contiguous 128-B cell updates instead of 64 scattered 8-B ones (measured 5.7x faster,
// profiles/r01_atomics_microbench.txt).
#include "zk_internal.h"

namespace zk {
namespace {

// chunk q (0..14) of the link's contribution vector (m0, d, d^2, d^3, d^4 in 32-bit chunks)
__device__ __forceinline__ uint64_t limb_value(int q, uint64_t d) {
    constexpr uint64_t M = 0xFFFFFFFFull;
    if (q == kLimbM0) return 1;
    if (q < kLimbS2) return (d >> (32 * (q - kLimbS1))) & M;
    const unsigned __int128 d2 = (unsigned __int128)d * d;
    if (q < kLimbS3) return (uint64_t)(d2 >> (32 * (q - kLimbS2))) & M;
    const unsigned __int128 d3 = d2 * d;
    if (q < kLimbS4) return (uint64_t)(d3 >> (32 * (q - kLimbS3))) & M;
    const uint64_t lo = (uint64_t)d3, hi = (uint64_t)(d3 >> 64);
    const unsigned __int128 p0 = (unsigned __int128)lo * d;
    const unsigned __int128 p1 = (unsigned __int128)hi * d + (uint64_t)(p0 >> 64);
    const int c = q - kLimbS4;  // 0..4 over the 160-bit d^4 = p1:lo64(p0)
    if (c < 2) return ((uint64_t)p0 >> (32 * c)) & M;
    return (uint64_t)(p1 >> (32 * (c - 2))) & M;
}

__global__ __launch_bounds__(256) void k_link_reduce_atomic(const uint64_t* __restrict__ links,
                                                            const uint32_t* __restrict__ counts, uint64_t stride,
                                                            uint64_t tiles, uint64_t* __restrict__ table) {
    const int q = threadIdx.x & 15;
    const int g = threadIdx.x >> 4;  // 16 lane groups per workgroup
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const uint32_t c = counts[t];
        const uint64_t* L = links + t * stride;
        for (uint32_t i = g; i < c; i += 16) {
            const uint64_t v = L[i];
            const uint64_t cell = v >> 40, d = v & (kMaxDuration - 1);
            if (q < 15) {
                const uint64_t x = limb_value(q, d);
                if (x) atomicAdd((unsigned long long*)(table + cell * kLimbs + q), (unsigned long long)x);
            }
        }
    }
}

// ---- partitioned reduce ----------------------------------------------------------------------
// K1 already counted its links per cell bucket (hist[b][w], bucket-major). K2a scans every bucket
// column (exclusive offsets of each K1 list inside the bucket), K2b scans the bucket totals, K2c
// scatters every list into bucket order, K3 reduces each bucket in LDS (a bucket of <= 1024 cells
// x 15 limbs fits one CU) and adds it to the table with plain loads/stores: every cell has exactly
// one owner, so no global atomic is issued (when a bucket is split over several workgroups for
// parallelism, the few flush adds are atomic).

__device__ __forceinline__ uint32_t block_excl_scan_1024(uint32_t v, uint32_t* s_tmp, uint32_t* total) {
    // blockDim.x == 1024 (16 waves)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) s_tmp[wave] = incl;
    __syncthreads();
    if (wave == 0) {
        uint32_t w = lane < 16 ? s_tmp[lane] : 0u;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const uint32_t o = __shfl_up(w, off);
            if (lane >= off) w += o;
        }
        if (lane < 16) s_tmp[16 + lane] = w;  // inclusive wave totals
    }
    __syncthreads();
    *total = s_tmp[16 + 15];
    return (wave ? s_tmp[16 + wave - 1] : 0u) + incl - v;
}

__global__ __launch_bounds__(1024) void k_bucket_colscan(const uint32_t* __restrict__ hist, uint32_t lists,
                                                         uint32_t* __restrict__ col_off, uint64_t* __restrict__ totals) {
    __shared__ uint32_t s_tmp[32];
    const uint32_t b = blockIdx.x;
    uint64_t carry = 0;
    for (uint32_t base = 0; base < lists; base += 1024) {
        const uint32_t w = base + threadIdx.x;
        const uint32_t v = w < lists ? hist[(uint64_t)b * lists + w] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan_1024(v, s_tmp, &tot);
        if (w < lists) col_off[(uint64_t)b * lists + w] = (uint32_t)carry + ex;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) totals[b] = carry;
}

__global__ __launch_bounds__(1024) void k_bucket_base(uint64_t* __restrict__ base, uint32_t nb) {
    // in: base[b] = bucket total (nb <= 1024); out: exclusive prefix, base[nb] = grand total
    __shared__ uint32_t s_tmp[32];
    const uint32_t b = threadIdx.x;
    const uint32_t v = b < nb ? (uint32_t)base[b] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan_1024(v, s_tmp, &tot);
    __syncthreads();
    if (b < nb) base[b] = ex;
    if (b == 0) base[nb] = tot;
}

__global__ __launch_bounds__(256) void k_link_scatter(ReduceArgs r) {
    __shared__ uint32_t s_cur[kMaxBuckets];
    const uint32_t w = blockIdx.x;
    for (uint32_t b = threadIdx.x; b < r.nb; b += 256)
        s_cur[b] = (uint32_t)r.bucket_base[b] + r.col_off[(uint64_t)b * r.lists + w];
    __syncthreads();
    const uint32_t c = r.counts[w];
    const uint64_t* __restrict__ L = r.links + (uint64_t)w * r.stride;
    const int lane = threadIdx.x & 63;
    for (uint32_t base = 0; base < c; base += 256) {
        const uint32_t i = base + threadIdx.x;
        const bool in = i < c;
        const uint64_t v = in ? L[i] : 0;
        const uint32_t b = (uint32_t)((v >> 40) >> r.cb_shift);
        if (r.nb <= 32) {
            // few buckets: aggregate the wave's lanes per bucket before touching the LDS cursor
            uint64_t todo = __ballot(in);
            while (todo) {
                const int l0 = __ffsll((unsigned long long)todo) - 1;
                const uint32_t b0 = __shfl(b, l0);
                const uint64_t same = __ballot(in && b == b0) & todo;
                uint32_t basepos = 0;
                if (lane == l0) basepos = atomicAdd(&s_cur[b0], (uint32_t)__popcll(same));
                basepos = __shfl(basepos, l0);
                if ((same >> lane) & 1ull) {
                    const uint32_t rank = (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
                    r.sorted[basepos + rank] = v;
                }
                todo &= ~same;
            }
        } else if (in) {
            r.sorted[atomicAdd(&s_cur[b], 1u)] = v;
        }
    }
}

template <int CB_SHIFT>
__global__ __launch_bounds__(1024) void k_bucket_reduce(ReduceArgs r, uint32_t splits) {
    constexpr int CB = 1 << CB_SHIFT;
    extern __shared__ __attribute__((aligned(16))) uint64_t s_acc[];  // [CB][15]
    const uint32_t b = blockIdx.x / splits, part = blockIdx.x % splits;
    for (uint32_t x = threadIdx.x; x < (uint32_t)CB * 15; x += blockDim.x) s_acc[x] = 0;
    __syncthreads();
    const uint64_t lo = r.bucket_base[b], hi = r.bucket_base[b + 1];
    const uint64_t per = (hi - lo + splits - 1) / splits;
    const uint64_t s0 = lo + per * part;
    const uint64_t s1 = (s0 + per < hi) ? s0 + per : hi;
    const uint64_t cell0 = (uint64_t)b << CB_SHIFT;
    const int q = threadIdx.x & 15;
    const uint32_t groups = blockDim.x >> 4;
    for (uint64_t i = s0 + (threadIdx.x >> 4); i < s1; i += groups) {
        const uint64_t v = r.sorted[i];
        const uint32_t cl = (uint32_t)((v >> 40) - cell0);
        const uint64_t d = v & (kMaxDuration - 1);
        if (q < 15) {
            const uint64_t x = limb_value(q, d);
            if (x) atomicAdd((unsigned long long*)&s_acc[cl * 15 + q], (unsigned long long)x);
        }
    }
    __syncthreads();
    const uint64_t ncell = (cell0 + CB <= r.cells) ? CB : r.cells - cell0;
    for (uint32_t x = threadIdx.x; x < ncell * 16; x += blockDim.x) {
        const uint32_t cl = x >> 4, l = x & 15;
        if (l == 15) continue;
        const uint64_t v = s_acc[cl * 15 + l];
        if (!v) continue;
        uint64_t* dst = r.table + (cell0 + cl) * kLimbs + l;
        if (splits == 1)
            *dst += v;  // this workgroup owns the cell
        else
            atomicAdd((unsigned long long*)dst, (unsigned long long)v);
    }
}

}  // namespace

void bucket_geometry(uint32_t S, uint32_t* nb, uint32_t* cb_shift) {
    const uint64_t cells = (uint64_t)S * S;
    *nb = 0;
    *cb_shift = 0;
    for (uint32_t sh = 9; sh <= 10; ++sh) {
        const uint64_t n = (cells + (1ull << sh) - 1) >> sh;
        if (n <= kMaxBuckets) {
            *nb = (uint32_t)n;
            *cb_shift = sh;
            return;
        }
    }
}

hipError_t launch_partitioned_reduce(const ReduceArgs& r, hipStream_t s) {
    if (!r.nb || !r.lists) return hipSuccess;
    hipLaunchKernelGGL(k_bucket_colscan, dim3(r.nb), dim3(1024), 0, s, r.hist, r.lists, r.col_off, r.bucket_base);
    hipLaunchKernelGGL(k_bucket_base, dim3(1), dim3(1024), 0, s, r.bucket_base, r.nb);
    hipLaunchKernelGGL(k_link_scatter, dim3(r.lists), dim3(256), 0, s, r);
    const uint32_t splits = r.nb >= 256 ? 1u : (512u + r.nb - 1) / r.nb;
    const size_t lds = (size_t)(1u << r.cb_shift) * 15 * sizeof(uint64_t);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_bucket_reduce<9>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)((1u << 9) * 15 * sizeof(uint64_t)));
        (void)hipFuncSetAttribute((const void*)k_bucket_reduce<10>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)((1u << 10) * 15 * sizeof(uint64_t)));
        attr_set = true;
    }
    if (r.cb_shift == 9)
        hipLaunchKernelGGL(k_bucket_reduce<9>, dim3(r.nb * splits), dim3(1024), lds, s, r, splits);
    else
        hipLaunchKernelGGL(k_bucket_reduce<10>, dim3(r.nb * splits), dim3(1024), lds, s, r, splits);
    return hipGetLastError();
}

hipError_t launch_link_reduce(const uint64_t* links, const uint32_t* counts, uint64_t stride, uint64_t tiles,
                              uint64_t* table, hipStream_t s) {
    if (!tiles) return hipSuccess;
    const uint64_t grid = tiles < 4096 ? tiles : 4096;
    hipLaunchKernelGGL(k_link_reduce_atomic, dim3((unsigned)grid), dim3(256), 0, s, links, counts, stride, tiles, table);
    return hipGetLastError();
}

}  // namespace zk
