// zk_reduce.hip — K3 link_reduce: per-tile link lists -> exact limb table (.group.sum,
// ZipkinAggregateJob.scala:39-40, DependencyLink.sg / MomentsGroup.plus made exact).
//
// A link is (cell << 40) | d. Its contribution to the cell is m0 += 1 and S_k += d^k (k = 1..4),
// laid out as 15 u64 limbs that each absorb 32-bit chunks (no carries before finalize). The 16 lanes
// of a lane group own one link and add the 15 limbs of one 128-byte cell, so a wave instruction
// issues four contiguous 128-B cell updates instead of 64 scattered 8-B ones (measured 5.7x faster,
// profiles/r01_atomics_microbench.txt).
#include "zk_block.h"
#include "zk_internal.h"
#include "zk_launch.h"

constexpr int kK2U = 8;      // links per thread per K2 chunk
constexpr int kK2WG = 1024;  // K2 workgroup: 8192-link chunks (512 threads: 0.236 -> 0.199 ms on C2)
constexpr int kK3U = 4;      // links per thread per K3 iteration (the next iteration's links prefetched)

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

__global__ __launch_bounds__(1024) void k_bucket_colscan(const uint32_t* __restrict__ hist, uint32_t lists,
                                                         uint32_t* __restrict__ col_off, uint64_t* __restrict__ totals) {
    __shared__ uint32_t s_tmp[32];
    const uint32_t b = blockIdx.x;
    uint64_t carry = 0;
    for (uint32_t base = 0; base < lists; base += 1024) {
        const uint32_t w = base + threadIdx.x;
        const uint32_t v = w < lists ? hist[(uint64_t)b * lists + w] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan<16>(v, s_tmp, &tot);
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
    const uint32_t ex = block_excl_scan<16>(v, s_tmp, &tot);
    __syncthreads();
    if (b < nb) base[b] = ex;
    if (b == 0) base[nb] = tot;
}

// K2c: one workgroup per K1 list. Chunks of C links are counting-sorted by bucket in LDS and
// written out in sorted order, and each bucket's tail that does not yet fill a 64-byte line stays
// in an LDS carry until the next chunk completes it: every line of the output is written whole,
// from one workgroup, within one chunk (the per-link version wrote 64 scattered 8-byte words per
// store instruction, at ~2.3x write amplification in WRITE_SIZE).
constexpr int kScatterLine = 8;  // links per 64-byte line (128-byte lines: WRITE_SIZE 571 -> 396 MB, but
                                 // their LDS carry halves the resident workgroups: 1.4x slower)
// One workgroup walks LPW consecutive K1 lists as one stream: within every bucket, list w+1's range
// follows list w's (col_off is an exclusive scan over lists), so the per-bucket cursors and line
// carries run on across the list boundaries and K2's grid stays ~256 workgroups (one per CU)
// whatever K1's grid: K2 0.221 -> 0.201 ms on C2 against ~1024 workgroups of 4 lists
// (profiles/r04/ab_k2_grid.txt; 512: 0.211 ms).
constexpr int kScatterMaxLPW = 16;
constexpr uint32_t kScatterGrid = 256;  // (512 workgroups: 0.211 ms; 4096-link chunks at two workgroups
                                        // per CU: 0.229 ms, at one: 0.250 ms -- ab_k2_grid.txt)
template <int U, int WG>
__global__ __launch_bounds__(WG) void k_link_scatter(ReduceArgs r, uint32_t lpw) {
    constexpr int C = WG * U;
    __shared__ uint32_t s_pre[kScatterMaxLPW + 4];  // exclusive prefix of the group's list counts (+ ~0 pads)
    __shared__ uint32_t s_cur[kMaxBuckets];   // output position of each bucket's first pending link
    __shared__ uint32_t s_hist[kMaxBuckets];  // links of the chunk per bucket
    __shared__ uint32_t s_off[kMaxBuckets];   // exclusive offsets in the sorted chunk
    __shared__ uint32_t s_cc[kMaxBuckets];    // carried links per bucket (< kScatterLine)
    __shared__ uint64_t s_sorted[C];
    __shared__ uint32_t s_tmp[32];
    extern __shared__ __attribute__((aligned(16))) uint64_t s_carry[];  // [nb][kScatterLine]
    // XCD-aware order (dispatch puts block i on XCD i % 8): the blocks of one XCD take consecutive
    // list groups, so the per-bucket ranges of neighbouring lists (which share their boundary
    // lines) are written through one L2. Same box, clustered C2 (profiles/r03/ab_k2_xcd.txt): K2
    // 0.221 -> 0.217 ms, K3 0.149 -> 0.143 ms
    const uint32_t gx = gridDim.x / 8, gr = gridDim.x % 8, xi = blockIdx.x % 8;
    const uint32_t w = (xi * gx + (xi < gr ? xi : gr) + blockIdx.x / 8) * lpw;  // first list of the group
    const uint32_t nl = (r.lists - w) < lpw ? (r.lists - w) : lpw;
    const int tid = threadIdx.x;
    constexpr int BPT = (kMaxBuckets + WG - 1) / WG;  // buckets per thread in the scan
    for (uint32_t b = tid; b < r.nb; b += WG) {
        s_cur[b] = (uint32_t)r.bucket_base[b] + r.col_off[(uint64_t)b * r.lists + w];
        s_hist[b] = 0u;
        s_cc[b] = 0u;
    }
    if (tid == 0) {
        uint32_t acc = 0;
        for (uint32_t q = 0; q < nl; ++q) {
            s_pre[q] = acc;
            acc += r.counts[w + q];
        }
        s_pre[nl] = acc;
        for (uint32_t q = nl + 1; q < kScatterMaxLPW + 4; ++q) s_pre[q] = 0xFFFFFFFFu;
    }
    __syncthreads();
    const uint32_t c = s_pre[nl];  // links of the group
    uint32_t pre[kScatterMaxLPW + 1];
#pragma unroll
    for (int q = 0; q <= kScatterMaxLPW; ++q) pre[q] = q <= (int)nl ? s_pre[q] : 0xFFFFFFFFu;
    // element i of the group's stream (i < c): list q with pre[q] <= i < pre[q + 1]
    auto at = [&](uint32_t i) -> const uint64_t* {
        uint32_t q = 0;
#pragma unroll
        for (int k = 1; k < kScatterMaxLPW; ++k) q += (i >= pre[k]) ? 1u : 0u;
        q = q < nl - 1 ? q : nl - 1;  // an empty group (c == 0) reads element 0 of its last list
        return r.links + (uint64_t)(w + q) * r.stride + (i - pre[q]);
    };
    // the links of the chunk starting at element b0 into dst. Lists hold ~C links or more, so a
    // chunk nearly always meets at most two list boundaries: its elements are then placed with two
    // compares against the (uniform) bounds after its first list, found by a walk that only moves
    // forward (q0); other chunks compare against every bound.
    uint32_t q0 = 0;
    auto load_chunk = [&](uint64_t (&dst)[U], uint32_t b0) {
        if (b0 >= c) {  // uniform: past the group's end
#pragma unroll
            for (int k = 0; k < U; ++k) dst[k] = r.links[(uint64_t)w * r.stride];
            return;
        }
        while (q0 + 1 < nl && b0 >= s_pre[q0 + 1]) ++q0;  // uniform
        const uint32_t pa = s_pre[q0], p1 = s_pre[q0 + 1], p2 = s_pre[q0 + 2], p3 = s_pre[q0 + 3];
        if ((uint64_t)b0 + C <= p3) {  // uniform
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const uint32_t i = b0 + tid + WG * k;
                const uint32_t ii = i < c ? i : b0;
                const uint32_t q = q0 + (ii >= p1 ? 1u : 0u) + (ii >= p2 ? 1u : 0u);
                const uint32_t lo = ii >= p2 ? p2 : (ii >= p1 ? p1 : pa);
                dst[k] = r.links[(uint64_t)(w + q) * r.stride + (ii - lo)];
            }
        } else {
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const uint32_t i = b0 + tid + WG * k;
                dst[k] = *at(i < c ? i : 0);
            }
        }
    };
    uint64_t nxt[U];
    load_chunk(nxt, 0u);
    for (uint32_t base = 0; base < c; base += C) {
        const uint32_t cnt = (c - base) < (uint32_t)C ? (c - base) : (uint32_t)C;
        const bool last = base + C >= c;
        uint64_t v[U];
        uint32_t bk[U], rank[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = nxt[k];
        load_chunk(nxt, base + C);  // next chunk in flight
#pragma unroll
        for (int k = 0; k < U; ++k) {
            bk[k] = (uint32_t)((v[k] >> 40) >> r.cb_shift);
            rank[k] = (tid + WG * k < (int)cnt) ? atomicAdd(&s_hist[bk[k]], 1u) : 0u;
        }
        __syncthreads();
        {
            uint32_t h[BPT], sum = 0;
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                const uint32_t bin = tid * BPT + q;
                h[q] = bin < r.nb ? s_hist[bin] : 0u;
                sum += h[q];
            }
            uint32_t tot;
            uint32_t ex = block_excl_scan<WG / 64>(sum, s_tmp, &tot);
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                const uint32_t bin = tid * BPT + q;
                if (bin < r.nb) s_off[bin] = ex;
                ex += h[q];
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (tid + WG * k < (int)cnt) s_sorted[s_off[bk[k]] + rank[k]] = v[k];
        // carried links: write those whose line the chunk completes, shift the rest down
        for (uint32_t b = tid; b < r.nb; b += WG) {
            const uint32_t cc = s_cc[b], pos = s_cur[b];
            const uint32_t end = pos + cc + s_hist[b];
            const uint32_t lim = last ? end : max(pos, end & ~(uint32_t)(kScatterLine - 1));
            uint64_t* cb = s_carry + (uint64_t)b * kScatterLine;
            for (uint32_t k = 0; k < cc; ++k) {
                const uint32_t dest = pos + k;
                if (dest < lim)
                    r.sorted[dest] = cb[k];
                else
                    cb[dest - lim] = cb[k];  // dest - lim <= k: ascending order is safe
            }
        }
        __syncthreads();
        for (uint32_t i = tid; i < cnt; i += WG) {
            const uint64_t x = s_sorted[i];
            const uint32_t b = (uint32_t)((x >> 40) >> r.cb_shift);
            const uint32_t pos = s_cur[b], cc = s_cc[b];
            const uint32_t end = pos + cc + s_hist[b];
            const uint32_t lim = last ? end : max(pos, end & ~(uint32_t)(kScatterLine - 1));
            const uint32_t dest = pos + cc + (i - s_off[b]);
            if (dest < lim)
                r.sorted[dest] = x;
            else
                s_carry[(uint64_t)b * kScatterLine + (dest - lim)] = x;
        }
        __syncthreads();
        for (uint32_t b = tid; b < r.nb; b += WG) {
            const uint32_t pos = s_cur[b];
            const uint32_t end = pos + s_cc[b] + s_hist[b];
            // never below the bucket's own first pending position: the line's head may belong to
            // the previous workgroup's range of this bucket
            const uint32_t lim = last ? end : max(pos, end & ~(uint32_t)(kScatterLine - 1));
            s_cur[b] = lim;
            s_cc[b] = end - lim;
            s_hist[b] = 0u;
        }
        __syncthreads();
    }
}

// Exact sums of one run of durations (<= 4096 links of one cell), kept in registers.
struct RunSums {
    uint64_t n, s1;          // s1 < 2^52
    unsigned __int128 s2;    // < 2^92
    unsigned __int128 s3;    // low 128 bits of s3 (< 2^132)
    uint64_t s3h;
    uint64_t s4[3];          // < 2^172
    __device__ __forceinline__ void clear() {
        n = s1 = s3h = 0;
        s2 = s3 = 0;
        s4[0] = s4[1] = s4[2] = 0;
    }
    __device__ __forceinline__ void add(uint64_t d) {
        const unsigned __int128 d2 = (unsigned __int128)d * d;  // < 2^80
        const unsigned __int128 d3 = d2 * d;                    // < 2^120
        const unsigned __int128 p0 = (unsigned __int128)(uint64_t)d3 * d;
        const unsigned __int128 p1 = (unsigned __int128)(uint64_t)(d3 >> 64) * d + (uint64_t)(p0 >> 64);
        ++n;
        s1 += d;
        s2 += d2;
        const unsigned __int128 t3 = s3 + d3;
        s3h += (t3 < s3);
        s3 = t3;
        // s4 += d^4 = p1:lo64(p0)
        const uint64_t w0 = (uint64_t)p0, w1 = (uint64_t)p1, w2 = (uint64_t)(p1 >> 64);
        const unsigned __int128 a0 = (unsigned __int128)s4[0] + w0;
        const unsigned __int128 a1 = (unsigned __int128)s4[1] + w1 + (uint64_t)(a0 >> 64);
        s4[0] = (uint64_t)a0;
        s4[1] = (uint64_t)a1;
        s4[2] += w2 + (uint64_t)(a1 >> 64);
    }
    // d < 2^32 (durations under 71 minutes, i.e. nearly all): d^2 fits 64 bits, so d^3 and d^4
    // are 64x32 and 64x64 products (5 32-bit multiplies instead of ~18)
    __device__ __forceinline__ void add_small(uint32_t d) {
        const uint64_t d2 = (uint64_t)d * d;
        const unsigned __int128 d3 = (unsigned __int128)d2 * d;   // < 2^96
        const unsigned __int128 d4 = (unsigned __int128)d2 * d2;  // < 2^128
        ++n;
        s1 += d;
        s2 += d2;
        const unsigned __int128 t3 = s3 + d3;
        s3h += (t3 < s3);
        s3 = t3;
        const uint64_t w0 = (uint64_t)d4, w1 = (uint64_t)(d4 >> 64);
        const unsigned __int128 a0 = (unsigned __int128)s4[0] + w0;
        const unsigned __int128 a1 = (unsigned __int128)s4[1] + w1 + (uint64_t)(a0 >> 64);
        s4[0] = (uint64_t)a0;
        s4[1] = (uint64_t)a1;
        s4[2] += (uint64_t)(a1 >> 64);
    }
    // add the run as 32-bit chunks to 15 register limbs (same layout as flush)
    __device__ __forceinline__ void to_limbs(uint64_t* l) const {
        constexpr uint64_t M = 0xFFFFFFFFull;
        const uint64_t s2lo = (uint64_t)s2, s2hi = (uint64_t)(s2 >> 64);
        const uint64_t s3lo = (uint64_t)s3, s3mid = (uint64_t)(s3 >> 64);
        l[0] += n;
        l[1] += s1 & M;
        l[2] += s1 >> 32;
        l[3] += s2lo & M;
        l[4] += s2lo >> 32;
        l[5] += s2hi;
        l[6] += s3lo & M;
        l[7] += s3lo >> 32;
        l[8] += s3mid & M;
        l[9] += (s3mid >> 32) | (s3h << 32);
        l[10] += s4[0] & M;
        l[11] += s4[0] >> 32;
        l[12] += s4[1] & M;
        l[13] += s4[1] >> 32;
        l[14] += s4[2];
    }
    // add the run as 32-bit chunks into the 15 limbs of an LDS cell (the topmost limb of each sum
    // may receive more than 32 bits: the table only needs value = sum of limb_k * 2^(32k))
    __device__ __forceinline__ void flush(uint64_t* cell) const {
        constexpr uint64_t M = 0xFFFFFFFFull;
        uint64_t v[15];
        v[0] = n;
        v[1] = s1 & M;
        v[2] = s1 >> 32;
        const uint64_t s2lo = (uint64_t)s2, s2hi = (uint64_t)(s2 >> 64);
        v[3] = s2lo & M;
        v[4] = s2lo >> 32;
        v[5] = s2hi;
        const uint64_t s3lo = (uint64_t)s3, s3mid = (uint64_t)(s3 >> 64);
        v[6] = s3lo & M;
        v[7] = s3lo >> 32;
        v[8] = s3mid & M;
        v[9] = (s3mid >> 32) | (s3h << 32);
        v[10] = s4[0] & M;
        v[11] = s4[0] >> 32;
        v[12] = s4[1] & M;
        v[13] = s4[1] >> 32;
        v[14] = s4[2];
#pragma unroll
        for (int q = 0; q < 15; ++q)
            if (v[q]) atomicAdd((unsigned long long*)&cell[q], (unsigned long long)v[q]);
    }
};

// One cell bucket (CB = 512 or 1024 cells) per workgroup of CB threads; thread t owns cell t for
// the whole kernel and keeps its 15 exact limbs in registers. Links come in chunks of C = P*CB:
// counting-sorted by cell in LDS (histogram, scan, place), after which every owner sums its own
// cell's run in registers -- no atomics and no LDS accumulator -- and finally adds its limbs to
// the table with plain stores (the workgroup owns the bucket; atomics only when a small bucket
// count is split over several workgroups).
template <int CB_SHIFT, int P>
__global__ __launch_bounds__(1 << CB_SHIFT) void k_bucket_reduce(ReduceArgs r, uint32_t splits) {
    constexpr int CB = 1 << CB_SHIFT, WG = CB, C = P * WG;
    static_assert(WG <= 1024, "one thread per cell");
    __shared__ uint32_t s_tmp[32];
    __shared__ uint32_t s_hist[CB];
    __shared__ uint32_t s_off[CB];
    __shared__ uint64_t s_d[C];  // the chunk's durations grouped by cell
    const int tid = threadIdx.x;
    const uint32_t b = blockIdx.x / splits, part = blockIdx.x % splits;
    s_hist[tid] = 0u;
    const uint64_t lo = r.bucket_base[b], hi = r.bucket_base[b + 1];
    const uint64_t per = (hi - lo + splits - 1) / splits;
    const uint64_t s0 = lo + per * part;
    const uint64_t s1 = (s0 + per < hi) ? s0 + per : hi;
    const uint64_t cell0 = (uint64_t)b << CB_SHIFT;
    uint64_t lim[15];
#pragma unroll
    for (int q = 0; q < 15; ++q) lim[q] = 0;
    uint64_t nxt[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const uint64_t i = s0 + tid + (uint64_t)k * WG;
        nxt[k] = r.sorted[i < s1 ? i : 0];
    }
    __syncthreads();
    for (uint64_t base = s0; base < s1; base += C) {
        const int cnt = (int)((s1 - base) < (uint64_t)C ? (s1 - base) : (uint64_t)C);
        uint64_t v[P];
        uint32_t cl[P], rank[P];
#pragma unroll
        for (int k = 0; k < P; ++k) {
            v[k] = nxt[k];
            const uint64_t i = base + C + tid + (uint64_t)k * WG;
            nxt[k] = r.sorted[i < s1 ? i : 0];  // next chunk in flight during this one
        }
#pragma unroll
        for (int k = 0; k < P; ++k) {
            cl[k] = (uint32_t)((v[k] >> 40) - cell0);
            rank[k] = (tid + k * WG < cnt) ? atomicAdd(&s_hist[cl[k]], 1u) : 0u;
        }
        __syncthreads();
        const uint32_t h = s_hist[tid];
        uint32_t tot;
        const uint32_t ex = block_excl_scan<WG / 64>(h, s_tmp, &tot);
        s_off[tid] = ex;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < P; ++k)
            if (tid + k * WG < cnt) s_d[s_off[cl[k]] + rank[k]] = v[k] & (kMaxDuration - 1);
        __syncthreads();
        RunSums run;
        run.clear();
        for (uint32_t q = 0; q < h; ++q) {
            const uint64_t d = s_d[ex + q];
            if (d >> 32)
                run.add(d);
            else
                run.add_small((uint32_t)d);
        }
        run.to_limbs(lim);
        s_hist[tid] = 0u;
        __syncthreads();
    }
    const uint64_t cell = cell0 + tid;
    if (cell < r.cells) {
        uint64_t* dst = r.table + cell * kLimbs;
#pragma unroll
        for (int q = 0; q < 15; ++q) {
            if (!lim[q]) continue;
            if (splits == 1)
                dst[q] += lim[q];  // this workgroup owns the cell
            else
                atomicAdd((unsigned long long*)&dst[q], (unsigned long long)lim[q]);
        }
    }
}

// K3 (cell buckets of 512): one bucket per workgroup; every link adds its contributions to the
// bucket's table in LDS with non-returning 64-bit LDS atomics -- no counting sort, no per-chunk
// barriers and no run-length imbalance (every thread handles the same number of links); the next
// iteration's links are in flight while this one's atomics run (profiles/r02/ab_k3lds.txt: equal to
// the counting-sort K3 serially, pipelined steps 1.63 -> 1.57 ms). Wide rows (round 3): fewer atomics per link. Each power
// sum is kept as 42-bit pieces instead of 32-bit chunks -- S1 one piece, S2 two, S3 three, S4 four,
// each row summing < 2^42 per link over a sub-part of < 2^20 links (< 2^62) -- and a link with d <
// 2^21 adds m0 and S1 as one packed word (2^42 + d): 6 LDS atomics for such a link (d^2 < 2^42 is one
// piece; d^3 < 2^63 and d^4 < 2^84 two each) against 8 with 32-bit chunks. At the flush every
// thread rebuilds its cell's exact S1..S4 from the pieces and cuts them into the table's 32-bit
// limbs with carries: all but the top limb of a sum receive < 2^32 per flush, and a flush holds at
// least one link, so with < 2^32 links since reset those limbs stay < 2^64; the top limb receives
// floor(S / 2^(32 top)) <= sum over the flush's links of (floor(d^k / 2^(32 top)) + 1) <= 2^32 per
// link (tests/test_reduce_bounds.py checks these bounds against the limb layout at d = 2^40 - 1).
template <int CB_SHIFT, int WG>
__global__ __launch_bounds__(WG) void k_bucket_lds_reduce_wide(ReduceArgs r, uint32_t splits) {
    constexpr int CB = 1 << CB_SHIFT;
    static_assert(CB == WG, "one thread per cell at the flush");
    constexpr int ROWS = 12;  // 0 m0, 1 S1, 2-3 S2, 4-6 S3, 7-10 S4, 11 packed m0|S1
    constexpr int RS = CB + 1;
    constexpr int CS = 17;  // staging stride of a cell's 15 limbs (odd: conflict-free both ways)
    constexpr int WORDS = (ROWS * RS > CB * CS) ? ROWS * RS : CB * CS;
    constexpr uint64_t P42 = (1ull << 42) - 1;
    constexpr uint64_t M = 0xFFFFFFFFull;
    constexpr uint64_t kSub = 1ull << 20;  // links per sub-part (row sums < 2^62)
    __shared__ unsigned long long s_t[WORDS];
    const int tid = threadIdx.x;
    const uint32_t b = blockIdx.x / splits, part = blockIdx.x % splits;
    const uint64_t lo = r.bucket_base[b], hi = r.bucket_base[b + 1];
    const uint64_t per = (hi - lo + splits - 1) / splits;
    const uint64_t p0 = lo + per * part;
    const uint64_t p1 = (p0 + per < hi) ? p0 + per : hi;
    const uint64_t cell0 = (uint64_t)b << CB_SHIFT;
    for (uint64_t s0 = p0; s0 < p1 || s0 == p0; s0 += kSub) {
        const uint64_t s1 = (s0 + kSub < p1) ? s0 + kSub : p1;
        for (int x = tid; x < ROWS * RS; x += WG) s_t[x] = 0ull;
        uint64_t nxt[kK3U];
#pragma unroll
        for (int k = 0; k < kK3U; ++k) {
            const uint64_t i = s0 + tid + (uint64_t)k * WG;
            nxt[k] = i < s1 ? r.sorted[i] : ~0ull;
        }
        __syncthreads();
        for (uint64_t base = s0; base < s1; base += (uint64_t)WG * kK3U) {
            uint64_t v[kK3U];
#pragma unroll
            for (int k = 0; k < kK3U; ++k) {
                v[k] = nxt[k];
                const uint64_t i = base + (uint64_t)WG * kK3U + tid + (uint64_t)k * WG;
                nxt[k] = i < s1 ? r.sorted[i] : ~0ull;
            }
#pragma unroll
            for (int k = 0; k < kK3U; ++k) {
                if (v[k] == ~0ull) continue;
                const uint32_t c = (uint32_t)((v[k] >> 40) - cell0);
                const uint64_t d = v[k] & (kMaxDuration - 1);
                unsigned long long* t = s_t + c;
#define ZK_K3W_ADD(q, x)                                            \
    do {                                                            \
        const uint64_t x_ = (x);                                    \
        if (x_) atomicAdd(&t[(q) * RS], (unsigned long long)x_);    \
    } while (0)
                if (d < (1ull << 21)) {
                    const uint64_t d2 = d * d;                           // < 2^42
                    const uint64_t d3 = d2 * d;                          // < 2^63
                    const unsigned __int128 d4 = (unsigned __int128)d2 * d2;  // < 2^84
                    atomicAdd(&t[11 * RS], (1ull << 42) | d);
                    ZK_K3W_ADD(2, d2);
                    ZK_K3W_ADD(4, d3 & P42);
                    ZK_K3W_ADD(5, d3 >> 42);
                    ZK_K3W_ADD(7, (uint64_t)d4 & P42);
                    ZK_K3W_ADD(8, (uint64_t)(d4 >> 42));
                } else {
                    // d < 2^40: d^2 < 2^80, d^3 < 2^120, d^4 < 2^160 as 64-bit words
                    const unsigned __int128 d2 = (unsigned __int128)d * d;
                    const unsigned __int128 d3 = d2 * d;
                    const uint64_t d3lo = (uint64_t)d3, d3hi = (uint64_t)(d3 >> 64);
                    const unsigned __int128 q0 = (unsigned __int128)d3lo * d;
                    const unsigned __int128 q1 = (unsigned __int128)d3hi * d + (uint64_t)(q0 >> 64);
                    const uint64_t w0 = (uint64_t)q0, w1 = (uint64_t)q1, w2 = (uint64_t)(q1 >> 64);  // d^4
                    atomicAdd(&t[0 * RS], 1ull);
                    ZK_K3W_ADD(1, d);
                    ZK_K3W_ADD(2, (uint64_t)d2 & P42);
                    ZK_K3W_ADD(3, (uint64_t)(d2 >> 42));
                    ZK_K3W_ADD(4, d3lo & P42);
                    ZK_K3W_ADD(5, (uint64_t)(d3 >> 42) & P42);
                    ZK_K3W_ADD(6, (uint64_t)(d3 >> 84));
                    ZK_K3W_ADD(7, w0 & P42);
                    ZK_K3W_ADD(8, ((w0 >> 42) | (w1 << 22)) & P42);
                    ZK_K3W_ADD(9, ((w1 >> 20) | (w2 << 44)) & P42);
                    ZK_K3W_ADD(10, (w1 >> 62) | (w2 << 2));
                }
#undef ZK_K3W_ADD
            }
        }
        __syncthreads();
        // rebuild the cell's exact sums from the pieces and cut them into 32-bit limbs
        uint64_t limb[15];
        {
            const int c = tid;
            uint64_t rv[ROWS];
#pragma unroll
            for (int q = 0; q < ROWS; ++q) rv[q] = s_t[q * RS + c];
            const uint64_t m0 = rv[0] + (rv[11] >> 42);
            const uint64_t S1 = rv[1] + (rv[11] & P42);  // < 2^63
            // S2 = rv2 + rv3 * 2^42 (< 2^104)
            const unsigned __int128 S2 = (unsigned __int128)rv[2] + ((unsigned __int128)rv[3] << 42);
            // S3 = rv4 + rv5 * 2^42 + rv6 * 2^84 (< 2^147): as lo128 + hi
            unsigned __int128 a3 = (unsigned __int128)rv[4] + ((unsigned __int128)rv[5] << 42);
            const unsigned __int128 t6 = (unsigned __int128)rv[6] << 20;  // rv6 * 2^84 = (rv6 << 20) * 2^64
            unsigned __int128 s3lo = a3 + ((unsigned __int128)(uint64_t)t6 << 64);
            uint64_t s3hi = (uint64_t)(t6 >> 64) + (s3lo < a3 ? 1u : 0u);
            // S4 = rv7 + rv8 * 2^42 + rv9 * 2^84 + rv10 * 2^126 (< 2^189): as 3 words
            const unsigned __int128 a4 = (unsigned __int128)rv[7] + ((unsigned __int128)rv[8] << 42);  // < 2^105
            const unsigned __int128 b4 = (unsigned __int128)rv[9] << 20;   // rv9 * 2^84 in units of 2^64
            const unsigned __int128 c4 = (unsigned __int128)rv[10] << 62;  // rv10 * 2^126 in units of 2^64
            // word 0 and the carry into word 1
            const uint64_t s4w0 = (uint64_t)a4;
            const unsigned __int128 hi = (a4 >> 64) + b4 + c4;  // the sum in units of 2^64 (< 2^125)
            const uint64_t s4w1 = (uint64_t)hi, s4w2 = (uint64_t)(hi >> 64);
            limb[0] = m0;
            limb[1] = S1 & M;
            limb[2] = S1 >> 32;
            limb[3] = (uint64_t)S2 & M;
            limb[4] = ((uint64_t)S2) >> 32;
            limb[5] = (uint64_t)(S2 >> 64);
            limb[6] = (uint64_t)s3lo & M;
            limb[7] = ((uint64_t)s3lo) >> 32;
            limb[8] = (uint64_t)(s3lo >> 64) & M;
            limb[9] = ((uint64_t)(s3lo >> 96)) | (s3hi << 32);
            limb[10] = s4w0 & M;
            limb[11] = s4w0 >> 32;
            limb[12] = s4w1 & M;
            limb[13] = s4w1 >> 32;
            limb[14] = s4w2;
        }
        __syncthreads();  // every row read before the staging overwrites them
#pragma unroll
        for (int q = 0; q < 15; ++q) s_t[tid * CS + q] = limb[q];
        __syncthreads();
        // 16 lanes per 128-byte cell: whole lines read-modify-written
        for (int x = tid; x < CB * kLimbs; x += WG) {
            const int c = x >> 4, q = x & 15;
            const uint64_t cell = cell0 + c;
            if (cell >= r.cells || q == 15) continue;
            const uint64_t v = s_t[c * CS + q];
            if (!v) continue;
            uint64_t* dst = r.table + cell * kLimbs + q;
            if (splits == 1)
                *dst += v;  // this workgroup owns the cell
            else
                atomicAdd((unsigned long long*)dst, (unsigned long long)v);
        }
        __syncthreads();  // the staging is read before the next sub-part clears the rows
        if (s1 >= p1) break;
    }
}

}  // namespace

// smallest cell bucket: 2^9 cells (2^8: 977 buckets at S = 500, measured 0.46 -> 0.53 ms for
// K2 + K3: K2's per-bucket LDS carry doubles)
constexpr uint32_t kCbMinShift = 9;

void bucket_geometry(uint32_t S, uint32_t* nb, uint32_t* cb_shift) {
    const uint64_t cells = (uint64_t)S * S;
    *nb = 0;
    *cb_shift = 0;
    for (uint32_t sh = kCbMinShift; sh <= 10; ++sh) {
        const uint64_t n = (cells + (1ull << sh) - 1) >> sh;
        if (n <= kMaxBuckets) {
            *nb = (uint32_t)n;
            *cb_shift = sh;
            return;
        }
    }
}

uint64_t reduce_scatter_dyn_lds(uint32_t S) {
    uint32_t nb = 0, sh = 0;
    bucket_geometry(S, &nb, &sh);
    return (uint64_t)nb * kScatterLine * 8;  // K2's per-bucket line carry
}

hipError_t launch_partitioned_reduce(const ReduceArgs& r, hipStream_t s) {
    if (!r.nb || !r.lists) return hipSuccess;
    hipError_t e = launch_checked("k_bucket_colscan", k_bucket_colscan, dim3(r.nb), dim3(1024), 0, s, r.hist, r.lists,
                                  r.col_off, r.bucket_base);
    if (e != hipSuccess) return e;
    e = launch_checked("k_bucket_base", k_bucket_base, dim3(1), dim3(1024), 0, s, r.bucket_base, r.nb);
    if (e != hipSuccess) return e;
    // ~kScatterGrid K2 workgroups: a K1 grid larger than that is walked LPW lists per workgroup
    uint32_t lpw = (r.lists + kScatterGrid - 1) / kScatterGrid;
    if (lpw > (uint32_t)kScatterMaxLPW) lpw = kScatterMaxLPW;
    const uint32_t k2_grid = (r.lists + lpw - 1) / lpw;
    e = launch_checked("k_link_scatter", k_link_scatter<kK2U, kK2WG>, dim3(k2_grid), dim3(kK2WG),
                       (size_t)r.nb * kScatterLine * 8, s, r, lpw);
    if (e != hipSuccess) return e;
    const uint32_t splits = r.nb >= 256 ? 1u : (512u + r.nb - 1) / r.nb;
    // buckets of 512 cells (S <= 724): the LDS-atomic K3; of 1024 cells: the counting-sort K3
    if (r.cb_shift == 9)
        return launch_checked("k_bucket_lds_reduce_wide<9>", k_bucket_lds_reduce_wide<9, 512>, dim3(r.nb * splits),
                              dim3(512), 0, s, r, splits);
    return launch_checked("k_bucket_reduce<10>", k_bucket_reduce<10, 4>, dim3(r.nb * splits), dim3(1024), 0, s, r, splits);
}

hipError_t launch_link_reduce(const uint64_t* links, const uint32_t* counts, uint64_t stride, uint64_t tiles,
                              uint64_t* table, hipStream_t s) {
    if (!tiles) return hipSuccess;
    const uint64_t grid = tiles < 4096 ? tiles : 4096;
    return launch_checked("k_link_reduce_atomic", k_link_reduce_atomic, dim3((unsigned)grid), dim3(256), 0, s, links,
                          counts, stride, tiles, table);
}

}  // namespace zk
