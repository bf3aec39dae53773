// zk_partition.hip — partition (service, payload) items into service-contiguous runs.
//
// Three launches, all streaming: (1) per-workgroup service histogram of a contiguous input range
// in LDS, written service-major (hist[s * grid + w]); (2) one exclusive scan of that matrix
// (hipcub), which makes every (service, workgroup) pair a disjoint output range, ordered by
// service first; (3) the scatter pass re-reads the range and appends each payload at its LDS
// cursor. Order inside one (service, workgroup) range follows LDS atomic order, which none of the
// sketches depends on (count-min and HyperLogLog are order-free; candidate selection is by
// final estimate).
#include <hipcub/hipcub.hpp>

#include "zk_block.h"
#include "zk_sketch_internal.h"
#include "zk_launch.h"

namespace zk {
namespace {

constexpr int kPartWG = 256;
constexpr int kPartU = 4;  // items per thread per iteration (loads issued before the LDS atomics)

// range of workgroup w: a slice of one flat array (counts == nullptr) or list w of the lists form
__device__ __forceinline__ void part_range(uint64_t n, uint64_t per, const uint32_t* counts, uint64_t* lo,
                                           uint64_t* hi) {
    if (counts) {
        *lo = (uint64_t)blockIdx.x * per;
        *hi = *lo + counts[blockIdx.x];
    } else {
        *lo = (uint64_t)blockIdx.x * per;
        *hi = *lo + per < n ? *lo + per : n;
    }
}

__global__ __launch_bounds__(kPartWG) void k_part_hist(const uint32_t* __restrict__ svc, uint64_t n, uint64_t per,
                                                        const uint32_t* __restrict__ counts, uint32_t S, uint32_t grid,
                                                        uint32_t* __restrict__ hist, unsigned long long* dropped) {
    extern __shared__ uint32_t h[];
    for (uint32_t i = threadIdx.x; i < S; i += kPartWG) h[i] = 0u;
    __syncthreads();
    uint64_t lo, hi;
    part_range(n, per, counts, &lo, &hi);
    uint32_t bad = 0;
    constexpr uint64_t BS = (uint64_t)kPartWG * kPartU;
    auto load = [&](uint32_t (&v)[kPartU], uint64_t b) {
#pragma unroll
        for (int e = 0; e < kPartU; ++e) {
            const uint64_t i = b + (uint64_t)e * kPartWG + threadIdx.x;
            v[e] = i < hi ? svc[i] : 0xFFFFFFFFu;
        }
    };
    auto count = [&](const uint32_t (&v)[kPartU], uint64_t b) {
#pragma unroll
        for (int e = 0; e < kPartU; ++e) {
            const uint64_t i = b + (uint64_t)e * kPartWG + threadIdx.x;
            if (v[e] < S)
                atomicAdd(&h[v[e]], 1u);
            else if (i < hi)
                ++bad;
        }
    };
    // two alternating load buffers (C4 partition 6.95 -> 6.77 ms, profiles/r02/ab_part_hist_pipe.txt)
    // two alternating buffers: one block's loads are in flight while the other is counted
    uint32_t va[kPartU], vb[kPartU];
    load(va, lo);
    for (uint64_t b = lo; b < hi; b += 2 * BS) {
        load(vb, b + BS);
        count(va, b);
        load(va, b + 2 * BS);
        count(vb, b + BS);  // past hi: every entry is the 0xFFFFFFFF sentinel and i >= hi
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < S; i += kPartWG) hist[(uint64_t)i * grid + blockIdx.x] = h[i];
    if (bad) atomicAdd(dropped, (unsigned long long)bad);
}

__global__ __launch_bounds__(kPartWG) void k_part_scatter(const uint32_t* __restrict__ svc,
                                                           const uint64_t* __restrict__ payload, uint64_t n,
                                                           uint64_t per, const uint32_t* __restrict__ counts,
                                                           uint32_t S, uint32_t grid,
                                                           const uint32_t* __restrict__ offs,
                                                           uint64_t* __restrict__ out, bool hash, uint64_t hash_seed) {
    extern __shared__ uint32_t cur[];  // absolute output cursor per service
    for (uint32_t i = threadIdx.x; i < S; i += kPartWG) cur[i] = offs[(uint64_t)i * grid + blockIdx.x];
    __syncthreads();
    uint64_t lo, hi;
    part_range(n, per, counts, &lo, &hi);
    for (uint64_t b = lo; b < hi; b += (uint64_t)kPartWG * kPartU) {
        uint32_t v[kPartU];
        uint64_t p[kPartU];
#pragma unroll
        for (int e = 0; e < kPartU; ++e) {
            const uint64_t i = b + (uint64_t)e * kPartWG + threadIdx.x;
            const bool in = i < hi;
            v[e] = in ? svc[i] : 0xFFFFFFFFu;
            p[e] = in ? payload[i] : 0ull;
            if (hash) p[e] = sk_mix64(p[e] ^ hash_seed);
        }
#pragma unroll
        for (int e = 0; e < kPartU; ++e)
            if (v[e] < S) out[atomicAdd(&cur[v[e]], 1u)] = p[e];
    }
}

// The same scatter with whole output lines (S <= kLineMaxS): chunks of C items are counting-sorted
// by service in LDS and written in runs; each service's tail that does not yet fill a 64-byte line
// stays in an LDS carry until a later chunk completes it (the item-by-item version above writes
// 8-byte pieces of 500 interleaved streams, ~8x write amplification). Same pattern as K2
// (zk_reduce.hip k_link_scatter), with the service taken from its own column.
constexpr uint32_t kLineMaxS = 1024;
constexpr int kLineU = 8;      // items per thread per chunk (line scatter): 8192-item chunks (4: 1.80 -> 1.43 ms on C4)
constexpr int kLineWG = 1024;  // line-scatter workgroup (512 threads x 4 items: 2.38 -> 1.76 ms on C4)
// Items per output line: 8 = 64 bytes. 128-byte lines (7168-item chunks, so that the S x 128 B carry
// fits) measured 8.99-9.03 ms against 6.93-7.00 ms for the C4 partition (profiles/r02/ab_part_lines.txt).
constexpr int kLineItems = 8;
template <int U, int WG>
__global__ __launch_bounds__(WG) void k_part_scatter_lines(const uint32_t* __restrict__ svc,
                                                            const uint64_t* __restrict__ payload, uint64_t n,
                                                            uint64_t per, const uint32_t* __restrict__ counts,
                                                            uint32_t S, uint32_t grid,
                                                            const uint32_t* __restrict__ offs,
                                                            uint64_t* __restrict__ out, bool hash, uint64_t hash_seed) {
    constexpr int C = WG * U;
    constexpr int BPT = (kLineMaxS + WG - 1) / WG;  // services per thread in the scan
    __shared__ uint32_t s_cur[kLineMaxS];  // output position of each service's first pending item
    __shared__ uint32_t s_hist[kLineMaxS];  // items of the chunk per service
    __shared__ uint32_t s_off[kLineMaxS];   // exclusive offsets in the sorted chunk
    __shared__ uint32_t s_cc[kLineMaxS];    // carried items per service (< kLineItems)
    __shared__ uint64_t s_sorted[C];
    __shared__ uint16_t s_svc[C];
    __shared__ uint32_t s_tmp[32];
    extern __shared__ __attribute__((aligned(16))) uint64_t s_carry[];  // [S][kLineItems]
    const int tid = threadIdx.x;
    for (uint32_t b = tid; b < S; b += WG) {
        s_cur[b] = offs[(uint64_t)b * grid + blockIdx.x];
        s_hist[b] = 0u;
        s_cc[b] = 0u;
    }
    uint64_t lo, hi;
    part_range(n, per, counts, &lo, &hi);
    const uint64_t lo0 = hi > lo ? lo : 0;  // an in-range index for the unconditional loads
    uint64_t nv[U];
    uint32_t ns[U];
    // loads are unconditional (clamped index) and masked at use: a conditional load, or a select
    // right after it, makes the compiler wait for it at once and the prefetch is lost
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const uint64_t i = lo + tid + (uint64_t)WG * k;
        ns[k] = svc[i < hi ? i : lo0];
        nv[k] = payload[i < hi ? i : lo0];
    }
    __syncthreads();
    for (uint64_t base = lo; base < hi; base += C) {
        const bool last = base + C >= hi;
        uint64_t v[U];
        uint32_t bk[U], rank[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            v[k] = hash ? sk_mix64(nv[k] ^ hash_seed) : nv[k];
            bk[k] = (base + tid + (uint64_t)WG * k < hi) ? ns[k] : 0xFFFFFFFFu;
            const uint64_t i = base + C + tid + (uint64_t)WG * k;  // next chunk in flight
            ns[k] = svc[i < hi ? i : lo0];
            nv[k] = payload[i < hi ? i : lo0];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) rank[k] = bk[k] < S ? atomicAdd(&s_hist[bk[k]], 1u) : 0u;
        __syncthreads();
        {
            uint32_t h[BPT], sum = 0;
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                const uint32_t bin = tid * BPT + q;
                h[q] = bin < S ? s_hist[bin] : 0u;
                sum += h[q];
            }
            uint32_t tot;
            uint32_t ex = block_excl_scan<WG / 64>(sum, s_tmp, &tot);
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                const uint32_t bin = tid * BPT + q;
                if (bin < S) s_off[bin] = ex;
                ex += h[q];
            }
            if (tid == 0) s_tmp[31] = tot;  // valid items of the chunk
        }
        __syncthreads();
        const uint32_t cnt = s_tmp[31];
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (bk[k] < S) {
                const uint32_t p = s_off[bk[k]] + rank[k];
                s_sorted[p] = v[k];
                s_svc[p] = (uint16_t)bk[k];
            }
        // carried items: write those whose line the chunk completes, shift the rest down
        for (uint32_t b = tid; b < S; b += WG) {
            const uint32_t cc = s_cc[b], pos = s_cur[b];
            const uint32_t end = pos + cc + s_hist[b];
            const uint32_t lim = last ? end : max(pos, end & ~(uint32_t)(kLineItems - 1));
            uint64_t* cb = s_carry + (uint64_t)b * kLineItems;
            for (uint32_t k = 0; k < cc; ++k) {
                const uint32_t dest = pos + k;
                if (dest < lim)
                    out[dest] = cb[k];
                else
                    cb[dest - lim] = cb[k];  // dest - lim <= k: ascending order is safe
            }
        }
        __syncthreads();
        for (uint32_t i = tid; i < cnt; i += WG) {
            const uint64_t x = s_sorted[i];
            const uint32_t b = s_svc[i];
            const uint32_t pos = s_cur[b], cc = s_cc[b];
            const uint32_t end = pos + cc + s_hist[b];
            const uint32_t lim = last ? end : max(pos, end & ~(uint32_t)(kLineItems - 1));
            const uint32_t dest = pos + cc + (i - s_off[b]);
            if (dest < lim)
                out[dest] = x;
            else
                s_carry[(uint64_t)b * kLineItems + (dest - lim)] = x;
        }
        __syncthreads();
        for (uint32_t b = tid; b < S; b += WG) {
            const uint32_t pos = s_cur[b];
            const uint32_t end = pos + s_cc[b] + s_hist[b];
            // never below the service's own first pending position: the line's head may belong to
            // the previous workgroup's range of this service
            const uint32_t lim = last ? end : max(pos, end & ~(uint32_t)(kLineItems - 1));
            s_cur[b] = lim;
            s_cc[b] = end - lim;
            s_hist[b] = 0u;
        }
        __syncthreads();
    }
}

// The scatter with write streams shared per XCD (flat input, S <= kLineMaxS): the
// input is cut into P <= 8 portions (groups of the histogram's workgroup ranges) and every
// service's output range into P sub-ranges, one per portion. Workgroups start on their XCD's
// portion (HW_REG_XCC_ID), take chunks of 8192 items in order, counting-sort a chunk by service
// in LDS and claim its runs at the portion's shared per-service cursors (one global atomic per
// service of the chunk): the ~32 workgroups of an XCD append to the same S streams, so adjacent
// runs fill their lines through one L2 (the per-workgroup ranges of k_part_scatter_lines keep
// grid x S streams apart and need LDS carries for whole lines). A workgroup whose portion is
// drained takes chunks of the others: placement changes only speed. Same pattern as the
// clustering pass (zk_cluster.hip k_cl_xscatter, profiles/r03/ab_cluster_writes.txt).
constexpr uint32_t kPartParts = 8;
#ifndef ZK_PX_U
#define ZK_PX_U 8  // items per thread of a chunk (A/B knob)
#endif
#ifndef ZK_PX_PER_CU
#define ZK_PX_PER_CU 1  // scatter workgroups per CU (A/B knob; 2 needs ZK_PX_U <= 4 for the LDS)
#endif
constexpr int kPxWG = 1024;  // XCD scatter workgroup (chunks of 8 items per thread), one per CU
constexpr int kPxU = ZK_PX_U;
constexpr uint32_t kPxChunk = kPxWG * kPxU;

struct PartX {
    const uint32_t* svc;
    const uint64_t* payload;
    uint64_t* out;
    uint32_t S, parts;
    unsigned int* cursor;        // [P][S]
    const uint64_t* part_lo;     // P + 1 portion bounds (items)
    const uint32_t* part_tiles;  // P + 1: chunks of the portions before p
    unsigned int* next;          // P chunk counters
    bool hash;
    uint64_t hash_seed;
};

__global__ void k_part_xprep(const uint32_t* __restrict__ offs, uint32_t S, uint32_t grid, uint32_t parts,
                             uint64_t per, uint64_t n, unsigned int* __restrict__ cursor, uint64_t* __restrict__ part_lo,
                             uint32_t* __restrict__ part_tiles, unsigned int* __restrict__ next) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < parts * S) {
        const uint32_t p = q / S, b = q % S;
        cursor[q] = offs[(uint64_t)b * grid + (uint64_t)p * grid / parts];
    }
    if (q == 0) {
        uint32_t t = 0;
        for (uint32_t p = 0; p <= parts; ++p) {
            const uint64_t lo = (uint64_t)p * grid / parts * per;
            part_lo[p] = lo < n ? lo : n;
        }
        for (uint32_t p = 0; p < parts; ++p) {
            part_tiles[p] = t;
            t += (uint32_t)((part_lo[p + 1] - part_lo[p] + kPxChunk - 1) / kPxChunk);
            next[p] = 0u;
        }
        part_tiles[parts] = t;
    }
}

// Portion p's chunks are taken in a static stride by the blocks dispatched to XCD p (block i runs on
// XCD i % 8), so no chunk claim is needed, and the next chunk's services and payloads load while this
// chunk is placed and stored: per chunk, the claim and the load round trips left the critical path
// (only the cursor claims' round trip stays on it; 5.41 -> 5.11-5.14 ms against claimed chunks).
__global__ __launch_bounds__(kPxWG, kPxWG / 256 * ZK_PX_PER_CU) void k_part_xscatter_static(PartX a) {
    constexpr int BPT = (kLineMaxS + kPxWG - 1) / kPxWG;  // services per thread in the scan
    __shared__ uint32_t s_cnt[kLineMaxS];  // items of the chunk per service
    __shared__ uint32_t s_off[kLineMaxS];  // exclusive offsets in the sorted chunk
    __shared__ uint32_t s_cur[kLineMaxS];  // output position of the chunk's run of each service
    __shared__ uint64_t s_sorted[kPxChunk];
    __shared__ uint16_t s_svc[kPxChunk];
    __shared__ uint32_t s_tmp[32];
    const int t = threadIdx.x;
    const uint32_t S = a.S;
    const uint32_t p = blockIdx.x % a.parts, xb = blockIdx.x / a.parts;
    const uint32_t nx = gridDim.x / a.parts + (p < gridDim.x % a.parts ? 1u : 0u);
    const uint32_t nj = a.part_tiles[p + 1] - a.part_tiles[p];
    const uint64_t plo = a.part_lo[p], phi = a.part_lo[p + 1];
    unsigned int* const cur = a.cursor + (uint64_t)p * S;
    for (uint32_t b = t; b < S; b += kPxWG) s_cnt[b] = 0u;
    // the zeros are published before any wave's first count (a wave's zeroing that waits behind a
    // slow global load would otherwise erase another wave's first counts)
    __syncthreads();
    uint64_t nv[kPxU];
    uint32_t nbk[kPxU];
    auto load = [&](uint32_t j) {
        const uint64_t lo = plo + (uint64_t)j * kPxChunk;
        const uint64_t hi = lo + kPxChunk < phi ? lo + kPxChunk : phi;
#pragma unroll
        for (int k = 0; k < kPxU; ++k) {
            const uint64_t i = lo + t + (uint64_t)kPxWG * k;
            nbk[k] = a.svc[i < hi ? i : lo];
            nv[k] = a.payload[i < hi ? i : lo];
        }
    };
    if (xb < nj) load(xb);
    for (uint32_t j = xb; j < nj; j += nx) {
        const uint64_t lo = plo + (uint64_t)j * kPxChunk;
        const uint64_t hi = lo + kPxChunk < phi ? lo + kPxChunk : phi;
        uint64_t v[kPxU];
        uint32_t bk[kPxU], rank[kPxU];
#pragma unroll
        for (int k = 0; k < kPxU; ++k) {
            v[k] = nv[k];
            bk[k] = nbk[k];
            if (lo + t + (uint64_t)kPxWG * k >= hi) bk[k] = 0xFFFFFFFFu;
            if (a.hash) v[k] = sk_mix64(v[k] ^ a.hash_seed);
            rank[k] = bk[k] < S ? atomicAdd(&s_cnt[bk[k]], 1u) : 0u;
        }
        __syncthreads();
        uint32_t cnt;
        {
            uint32_t h[BPT], sum = 0;
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                const uint32_t bin = t * BPT + q;
                h[q] = bin < S ? s_cnt[bin] : 0u;
                sum += h[q];
            }
            uint32_t ex = block_excl_scan<kPxWG / 64>(sum, s_tmp, &cnt);
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                const uint32_t bin = t * BPT + q;
                if (bin < S) {
                    s_off[bin] = ex;
                    s_cur[bin] = h[q] ? atomicAdd(&cur[bin], h[q]) : 0u;
                    s_cnt[bin] = 0u;  // every rank is taken: ready for the next chunk
                }
                ex += h[q];
            }
        }
        __syncthreads();
        // the next chunk's loads in flight while this one is placed and stored (issued after the
        // cursor claims, whose returns would otherwise wait for them)
        if (j + nx < nj) load(j + nx);
#pragma unroll
        for (int k = 0; k < kPxU; ++k)
            if (bk[k] < S) {
                const uint32_t q = s_off[bk[k]] + rank[k];
                s_sorted[q] = v[k];
                s_svc[q] = (uint16_t)bk[k];
            }
        __syncthreads();
        for (uint32_t i = t; i < cnt; i += kPxWG) {
            const uint32_t b = s_svc[i];
            a.out[s_cur[b] + (i - s_off[b])] = s_sorted[i];
        }
        // No barrier here: the next chunk's first LDS writes are its rank atomics on s_cnt (zeroed
        // before this chunk's second barrier); s_cur / s_off and s_sorted / s_svc are rewritten only
        // after its first barrier, which every thread reaches after these reads.
    }
}

// seg[s] = offs[s * grid], seg[S] = number of partitioned items
__global__ void k_part_seg(const uint32_t* __restrict__ offs, const uint32_t* __restrict__ hist, uint32_t S,
                           uint32_t grid, uint64_t* __restrict__ seg) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < S) seg[s] = offs[(uint64_t)s * grid];
    if (s == S) {
        const uint64_t last = (uint64_t)S * grid - 1;
        seg[S] = (uint64_t)offs[last] + hist[last];
    }
}

// unit_base = exclusive scan of ceil(len_s / unit_items); one workgroup of 1024 threads
__global__ __launch_bounds__(1024) void k_unit_plan(const uint64_t* __restrict__ seg, uint32_t S,
                                                     uint64_t unit_items, uint32_t* __restrict__ unit_base) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t b = 0; b < S; b += 1024) {
        const uint32_t s = b + threadIdx.x;
        const uint64_t len = s < S ? seg[s + 1] - seg[s] : 0;
        const uint32_t u = (uint32_t)((len + unit_items - 1) / unit_items);
        uint32_t incl = u;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = __shfl_up(incl, off);
            if (lane >= off) incl += o;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t before = carry;
        for (int w = 0; w < wave; ++w) before += wsum[w];
        if (s < S) unit_base[s] = before + incl - u;
        __syncthreads();
        if (threadIdx.x == 1023) carry = before + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) unit_base[S] = carry;
}

uint64_t scan_temp_bytes(uint64_t m) {
    size_t bytes = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)m);
    return (bytes + 255) & ~(uint64_t)255;
}

}  // namespace

int partition_scatter_choice(uint32_t S, uint64_t static_lines, uint64_t static_items, uint64_t* dyn) {
    const uint64_t carry = (uint64_t)S * kLineItems * 8;  // the line kernel's [S][8] u64 carry
    if (S <= kLineMaxS && lds_fits(static_lines, carry)) {
        *dyn = carry;
        return kScatterLines;
    }
    *dyn = (uint64_t)S * 4;  // the item kernel's per-service cursor
    return lds_fits(static_items, *dyn) ? kScatterItems : kScatterNone;
}

PartitionPlan partition_plan(uint64_t n, uint32_t S, uint32_t cus) {
    PartitionPlan p;
    p.S = S;
    // ~4 resident workgroups per CU; at least 16k items per workgroup so the S-entry histogram
    // column stays small next to the data
    uint64_t g = (uint64_t)cus * 4;
    const uint64_t by_items = (n + 16383) / 16384;
    if (g > by_items) g = by_items ? by_items : 1;
    p.grid = (uint32_t)g;
    p.per_wg = (n + g - 1) / g;
    if (p.per_wg == 0) p.per_wg = 1;
    return p;
}

// the XCD-stream scatter's cursors [8][S] and portion tables, after the scan temp
uint64_t part_x_bytes(uint32_t S) {
    return (((uint64_t)kPartParts * S * 4 + 255) & ~255ull) + 3 * 256;
}

uint64_t partition_scratch_bytes(const PartitionPlan& p) {
    const uint64_t m = (uint64_t)p.S * p.grid;
    const uint64_t a = (m * 4 + 255) & ~255ull;
    return 2 * a + scan_temp_bytes(m) + part_x_bytes(p.S);
}

namespace {
hipError_t partition_impl(const PartitionPlan& p, const uint32_t* svc, const uint64_t* payload, uint64_t n,
                          const uint32_t* counts, uint64_t* out, uint64_t* seg, unsigned long long* dropped,
                          void* scratch, hipStream_t s, bool hash, uint64_t hash_seed) {
    const uint64_t m = (uint64_t)p.S * p.grid;
    const uint64_t a = (m * 4 + 255) & ~255ull;
    uint32_t* hist = (uint32_t*)scratch;
    uint32_t* offs = (uint32_t*)((uint8_t*)scratch + a);
    void* temp = (uint8_t*)scratch + 2 * a;
    size_t temp_bytes = scan_temp_bytes(m);
    hipError_t e = hipSuccess;
    const bool xcd = !counts && p.S <= kLineMaxS && n > 0;
    PartX x{};
    uint32_t gx = 0;
    if (xcd) {
        x.svc = svc;
        x.payload = payload;
        x.out = out;
        x.S = p.S;
        x.hash = hash;
        x.hash_seed = hash_seed;
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        gx = (uint32_t)(cus > 0 ? cus : 256) * ZK_PX_PER_CU;
    }
    const size_t lds = (size_t)p.S * 4;
    e = launch_checked("k_part_hist", k_part_hist, dim3(p.grid), dim3(kPartWG), lds, s, svc, n, p.per_wg, counts, p.S,
                       p.grid, hist, dropped);
    if (e != hipSuccess) return e;
    e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, hist, offs, (int)m, s);
    if (e != hipSuccess) return e;
    // whole lines while the line kernel's static LDS (read from its code object) plus the [S][8]
    // carry fit one CU (S <= 1022 at 8192-item chunks; S = 1024 faulted in round 2, before any
    // check), else item by item
    uint32_t st_lines = 0, st_items = 0, mt = 0;
    e = kernel_attrs((const void*)k_part_scatter_lines<kLineU, kLineWG>, &st_lines, &mt);
    if (e == hipSuccess) e = kernel_attrs((const void*)k_part_scatter, &st_items, &mt);
    if (e != hipSuccess) return e;
    uint64_t dyn = 0;
    const int choice = partition_scatter_choice(p.S, st_lines, st_items, &dyn);
    if (xcd) {
        // write streams shared per XCD: portion cursors claimed per chunk
        x.parts = p.grid < kPartParts ? p.grid : kPartParts;
        if (x.parts > gx) x.parts = gx;
        uint8_t* xp = (uint8_t*)temp + temp_bytes;
        x.cursor = (unsigned int*)xp;
        xp += ((uint64_t)kPartParts * p.S * 4 + 255) & ~255ull;
        uint64_t* part_lo = (uint64_t*)xp;
        uint32_t* part_tiles = (uint32_t*)(xp + 256);
        unsigned int* next = (unsigned int*)(xp + 512);
        x.part_lo = part_lo;
        x.part_tiles = part_tiles;
        x.next = next;
        e = launch_checked("k_part_xprep", k_part_xprep, dim3((x.parts * p.S + 255) / 256), dim3(256), 0, s,
                           (const uint32_t*)offs, p.S, p.grid, x.parts, p.per_wg, n, x.cursor, part_lo, part_tiles, next);
        if (e == hipSuccess)
            e = launch_checked("k_part_xscatter_static", k_part_xscatter_static, dim3(gx), dim3(kPxWG), 0, s, x);
    } else if (choice == kScatterLines)
        e = launch_checked("k_part_scatter_lines", k_part_scatter_lines<kLineU, kLineWG>, dim3(p.grid),
                           dim3(kLineWG), dyn, s, svc, payload, n, p.per_wg, counts, p.S, p.grid, offs, out, hash,
                           hash_seed);
    else
        e = launch_checked("k_part_scatter", k_part_scatter, dim3(p.grid), dim3(kPartWG), dyn, s, svc, payload, n,
                           p.per_wg, counts, p.S, p.grid, offs, out, hash, hash_seed);
    if (e != hipSuccess) return e;
    return launch_checked("k_part_seg", k_part_seg, dim3((p.S + 256) / 256), dim3(256), 0, s, offs, hist, p.S, p.grid,
                          seg);
}
}  // namespace

hipError_t launch_partition(const PartitionPlan& p, const uint32_t* svc, const uint64_t* payload, uint64_t n,
                            uint64_t* out, uint64_t* seg, unsigned long long* dropped, void* scratch,
                            hipStream_t s, bool hash, uint64_t hash_seed) {
    return partition_impl(p, svc, payload, n, nullptr, out, seg, dropped, scratch, s, hash, hash_seed);
}

PartitionPlan partition_plan_lists(uint32_t lists, uint32_t S) {
    PartitionPlan p;
    p.S = S;
    p.grid = lists;
    p.per_wg = 0;  // set by the caller through launch_partition_lists (the list stride)
    return p;
}

hipError_t launch_partition_lists(const PartitionPlan& p0, const uint32_t* svc, const uint64_t* payload,
                                  uint64_t stride, const uint32_t* counts, uint64_t* out, uint64_t* seg,
                                  unsigned long long* dropped, void* scratch, hipStream_t s) {
    PartitionPlan p = p0;
    p.per_wg = stride;
    return partition_impl(p, svc, payload, 0, counts, out, seg, dropped, scratch, s, false, 0);
}

hipError_t launch_unit_plan(const uint64_t* seg, uint32_t S, uint64_t unit_items, uint32_t* unit_base,
                            hipStream_t s) {
    return launch_checked("k_unit_plan", k_unit_plan, dim3(1), dim3(1024), 0, s, seg, S, unit_items, unit_base);
}

}  // namespace zk

// internal (not in include/): the partition's scatter choice for a CPU test of the LDS planner
extern "C" int zk_internal_partition_choice(uint32_t S, uint64_t static_lines, uint64_t static_items, uint64_t* dyn) {
    return zk::partition_scatter_choice(S, static_lines, static_items, dyn);
}
