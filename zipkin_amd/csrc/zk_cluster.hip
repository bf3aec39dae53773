// zk_cluster.hip — order-agnostic input: a hand-written traceId-hash partition, and the
// trace-clustering check.
//
// The reference job accepts span fragments in any order: Scalding shuffles them by key before
// every reduce (groupBy((id, traceId)) at ZipkinAggregateJob.scala:21-22, the (parentId, traceId)
// join key at :28-33). K1 merges and joins inside a trace segment, so it needs every fragment of a
// trace adjacent. The clustering pass makes a batch in any order trace-clustered, MSD-radix style
// on the digits of a hash of the traceId -- the traceId is in the shuffle key of both reference
// joins, so a trace never straddles two buckets:
//
//   P0 k_cl_hist     per-workgroup LDS histogram of the first digit (top hash bits) of a contiguous
//                    input range; one exclusive scan (hipcub) of the digit-major matrix gives every
//                    (digit, workgroup) pair a disjoint output range
//   P1 k_cl_xscatter each workgroup re-reads its range in chunks of 8192 records: digits ranked in
//      <global>      LDS (atomic counting sort), then column by column the chunk is loaded
//                    coalesced, staged in LDS in digit order and written as per-digit runs at the
//                    ranges' cursors
//   P2 k_cl_xscatter one workgroup per first-level bucket: an LDS histogram of the second digit over
//      <local>       the bucket, its scan (the sub-bucket bounds), then the same chunked scatter
//                    inside the bucket
//   P3 k_cl_traces   one workgroup per sub-bucket (~1k records): an LDS hash table of the
//                    sub-bucket's distinct traceIds counts each trace's records, a scan places the
//                    traces, and a second sweep writes every record to its trace's run -- the
//                    output is exactly trace-clustered (a sub-bucket larger than 2048 records is
//                    done in several rounds, each taking a hash range of its traceIds)
//
// Small batches run P3 alone over the whole batch. Traffic per record: 8 B (P0) + 104 B (P1:
// traceIds twice, every column once, written once) + 112 B (P2, plus its histogram sweep) + 104 B
// (P3). Round 2 used rocprim's radix_sort_pairs over the 64-bit traceIds and a gather of the
// columns by the sorted index (random 8-byte reads): 21 ms per 1e8 records on MI355X against
// 1.2 ms for K1 (profiles/r03/).
//
// The trace set (ZK_BATCH_VERIFY_TRACES): every trace segment start inserts its traceId into an
// open-addressing set of all traceIds accumulated since the last reset. A traceId found again
// means a trace split into two non-adjacent runs, or spread over two accumulate calls -- both
// would be mis-joined silently -- and is counted in ST_NOT_CLUSTERED (finalize then returns
// ZK_ERR_NOT_CLUSTERED). Exact: the set stores whole traceIds, so it has no false positives.
#include <stdlib.h>

#include <type_traits>

#include <hipcub/hipcub.hpp>

#include "zk_block.h"
#include "zk_cluster.h"
#include "zk_launch.h"
#include "zk_tracegen.h"

namespace zk {
namespace {

constexpr uint64_t kSetSalt = 0x6A09E667F3BCC909ull;
// the partition hash: independent of the shard function mix64(traceId) % world (zk_trace_shard)
// and of TraceGen's traceId construction (traceId = mix64^-1(k * world + rank))
constexpr uint64_t kPartSalt = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t kTraceSalt = 0x165667B19E3779F9ull;

__device__ __forceinline__ uint64_t part_hash(uint64_t tid) { return zk_mix64(tid ^ kPartSalt); }
__device__ __forceinline__ uint32_t digit_of(uint64_t h, uint32_t shift, uint32_t mask) {
    return (uint32_t)(h >> shift) & mask;
}

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

// ---- P0: per-workgroup digit histogram -----------------------------------------------------------
// One workgroup per CU (the P0 ranges are what P1's portions are cut from): 16 waves and two
// alternating load buffers, so one block's traceIds are in flight while the other is counted
// (256 threads with one buffer: 0.247 ms per 1e8 records, latency-bound at 4 waves per CU).
constexpr int kHistWG = 1024;
constexpr int kHistU = 4;

__global__ __launch_bounds__(kHistWG) void k_cl_hist(const uint64_t* __restrict__ tid, uint64_t n, uint64_t per,
                                                      uint32_t shift, uint32_t nd, uint32_t grid,
                                                      uint32_t* __restrict__ hist) {
    extern __shared__ uint32_t h[];
    for (uint32_t i = threadIdx.x; i < nd; i += kHistWG) h[i] = 0u;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * per;
    const uint64_t hi = lo + per < n ? lo + per : n;
    const uint32_t mask = nd - 1;
    constexpr uint64_t BS = (uint64_t)kHistWG * kHistU;
    auto load = [&](uint64_t (&v)[kHistU], uint64_t b) {
#pragma unroll
        for (int e = 0; e < kHistU; ++e) {
            const uint64_t i = b + (uint64_t)e * kHistWG + threadIdx.x;
            v[e] = tid[i < hi ? i : lo];
        }
    };
    auto count = [&](const uint64_t (&v)[kHistU], uint64_t b) {
#pragma unroll
        for (int e = 0; e < kHistU; ++e) {
            const uint64_t i = b + (uint64_t)e * kHistWG + threadIdx.x;
            if (i < hi) atomicAdd(&h[digit_of(part_hash(v[e]), shift, mask)], 1u);
        }
    };
    uint64_t va[kHistU], vb[kHistU];
    if (lo < hi) load(va, lo);  // a trailing workgroup may own no records
    for (uint64_t b = lo; b < hi; b += 2 * BS) {
        load(vb, b + BS);
        count(va, b);
        load(va, b + 2 * BS);
        count(vb, b + BS);  // past hi: nothing counted
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < nd; d += kHistWG) hist[(uint64_t)d * grid + blockIdx.x] = h[d];
}

// bucket bounds from the scanned matrix: base[d] = offs[d * grid] (the first workgroup's range of
// digit d), base[nd] = n
__global__ void k_cl_bounds(const uint32_t* __restrict__ offs, uint32_t nd, uint32_t grid, uint64_t n,
                            uint32_t* __restrict__ base) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < nd) base[d] = offs[(uint64_t)d * grid];
    if (d == nd) base[nd] = (uint32_t)n;
}

// ---- P1 / P2 helpers ---------------------------------------------------------------------------
constexpr uint32_t kMaxDigits = 2048;   // <= 11 bits per level
// levels of <= 256 digits (8 bits: every level up to 2^24 records) run a variant with byte digit
// tags and smaller digit arrays
constexpr uint32_t kSmallDigits = 256;
constexpr uint32_t kMidDigits = 512;  // (the group join's plans: 9-bit levels)

// column C (0..6) of a batch: the u64 columns first, then service_id and flags (u32)
template <int C>
__device__ __forceinline__ uint64_t col_load(const SpanColsDev& c, uint64_t i) {
    if constexpr (C == 0) return c.trace_id[i];
    if constexpr (C == 1) return c.span_id[i];
    if constexpr (C == 2) return c.parent_id[i];
    if constexpr (C == 3) return (uint64_t)c.first_ts[i];
    if constexpr (C == 4) return (uint64_t)c.last_ts[i];
    if constexpr (C == 5) return c.service_id[i];
    return c.flags[i];
}
template <int C>
__device__ __forceinline__ void col_store(const SpanColsMut& c, uint64_t i, uint64_t v) {
    if constexpr (C == 0) c.trace_id[i] = v;
    if constexpr (C == 1) c.span_id[i] = v;
    if constexpr (C == 2) c.parent_id[i] = v;
    if constexpr (C == 3) c.first_ts[i] = (int64_t)v;
    if constexpr (C == 4) c.last_ts[i] = (int64_t)v;
    if constexpr (C == 5) c.service_id[i] = (uint32_t)v;
    if constexpr (C == 6) c.flags[i] = (uint32_t)v;
}

// Move the seven columns of rows base + t + k*WG (k < U, those < cnt) through the LDS stage: row
// (t, k) goes to stage slot pos[k], and the thread writes stage slot t + k*WG to out row dest[k].
// v holds column 0 (the traceIds) of the thread's rows on entry.
// Coalesced loads and coalesced per-run stores; column C + 1's loads are issued before column C's
// stores, so a column's HBM latency hides behind the previous column's LDS round trip.
template <int U, int WG, int C = 0>
__device__ __forceinline__ void move_columns(const SpanColsDev& in, const SpanColsMut& out, uint64_t base,
                                             uint32_t cnt, const uint32_t (&pos)[U], const uint32_t (&dest)[U],
                                             uint64_t* stage, uint64_t (&v)[U]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < U; ++k)
        if (t + k * WG < cnt) stage[pos[k]] = v[k];
    __syncthreads();
    if constexpr (C < 6) {
#pragma unroll
        for (int k = 0; k < U; ++k) {  // the next column, in flight during this column's stores
            const uint32_t j = t + k * WG;
            v[k] = col_load<C + 1>(in, base + (j < cnt ? j : 0));
        }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const uint32_t i = t + k * WG;
        if (i < cnt) col_store<C>(out, dest[k], stage[i]);
    }
    __syncthreads();
    if constexpr (C < 6) move_columns<U, WG, C + 1>(in, out, base, cnt, pos, dest, stage, v);
}

// exclusive scan of s_cnt[0..nd) into out[d] = add + offset (one pass of the whole workgroup)
template <int WG, uint32_t MAXD>
__device__ __forceinline__ void scan_digits(const uint32_t* s_cnt, uint32_t nd, uint32_t add, uint32_t* out,
                                            uint32_t* s_tmp) {
    constexpr int DPT = (MAXD + WG - 1) / WG;
    const int t = threadIdx.x;
    uint32_t h[DPT], sum = 0;
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
        const uint32_t d = t * DPT + q;
        h[q] = d < nd ? s_cnt[d] : 0u;
        sum += h[q];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan<WG / 64>(sum, s_tmp, &tot);
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
        const uint32_t d = t * DPT + q;
        if (d < nd) out[d] = add + ex;
        ex += h[q];
    }
}

// ---- P1 / P2 with streams shared per XCD ----------------------------------------------------------
// With one output range per (workgroup, digit) -- the round-2/3 scatter and its write-combining
// successor, removed after round 3 -- 256 workgroups x 256 digits x 7 columns of write streams sit
// ~12 KB apart, and a run's partial tail line waits for the same workgroup's next chunk
// (profiles/r03/ab_cluster_writes.txt: 2.73 / 2.97 ms per pass vs 2.05 / 1.97 here). Here the input is cut into P <= 8 portions, and a digit's output
// range is cut into P sub-ranges, one per portion; a chunk of portion p claims its runs at the
// portion's shared cursors (one global atomic per digit of the chunk). Workgroups start on the
// portion of their XCD (HW_REG_XCC_ID) and take chunks in order, so at any moment the ~32
// workgroups of an XCD append to the same 256 x 7 streams: neighbouring runs are written through
// the same L2, and the open lines of an XCD are 256 x 7 instead of 32 x 256 x 7. Placement only
// changes speed: a workgroup whose portion is drained takes chunks of the others, and every
// portion's cursors belong to the portion, not to an XCD.
//   P1: portion p = the P0 ranges [p g / P, (p + 1) g / P); its cursors start at the scanned P0
//       offsets of its first range.
//   P2: portion p = the first-level buckets b = p, p + P, ...; a chunk lies inside one bucket and
//       claims its runs at the bucket's sub-bucket cursors (the scanned (bucket, digit) histogram
//       of P2h, which also gives the sub-bucket bounds).
constexpr uint32_t kParts = 8;
constexpr int kXsWG = 1024;  // one P1/P2 workgroup per CU (2 or 4 smaller ones: 3.77 / 4.60 ms per pass)
constexpr int kXsU = 8;      // records per thread per P1/P2 chunk
constexpr uint32_t kXsChunk = kXsWG * kXsU;

struct XArgs {
    SpanColsDev in;
    SpanColsMut out;
    uint32_t shift, nd;
    uint32_t parts;                    // P
    const uint32_t* part_tiles;        // P + 1: chunks of the portions before p
    unsigned int* next;                // P chunk counters
    unsigned int* cursor;              // global: [P][nd]; local: [nb1][nd] (absolute output positions)
    // global: portion p = records [part_lo[p], part_lo[p + 1])
    const uint32_t* part_lo;
    // local: portion p's buckets b = p + P m; bucket_tiles[p * (nbp + 1) + m] = chunks of its first m buckets
    const uint32_t* bucket;            // nb1 + 1 bucket bounds
    const uint32_t* bucket_tiles;
    uint32_t nb1, nbp;
    uint32_t* hist;                    // P2h: [nb1][nd] counts
};

// chunk j of portion p -> its records [lo, hi) and (local) its bucket
template <bool LOCAL>
__device__ __forceinline__ void xchunk(const XArgs& a, uint32_t p, uint32_t j, uint64_t* lo, uint64_t* hi,
                                       uint32_t* b) {
    if constexpr (!LOCAL) {
        *b = 0;
        *lo = (uint64_t)a.part_lo[p] + (uint64_t)j * kXsChunk;
        const uint64_t e = a.part_lo[p + 1];
        *hi = *lo + kXsChunk < e ? *lo + kXsChunk : e;
    } else {
        const uint32_t* bt = a.bucket_tiles + (uint64_t)p * (a.nbp + 1);
        // l = the last m with bt[m] <= j: every wave reads 64 entries at once and counts by ballot
        // (one load round trip per 64 buckets of the portion instead of a dependent binary search)
        const uint32_t lane = threadIdx.x & 63u;
        uint32_t l = 0;
        for (uint32_t m0 = 0; m0 < a.nbp; m0 += 64u) {  // uniform
            const uint32_t m = m0 + lane;
            const uint64_t le = __ballot(m < a.nbp && bt[m < a.nbp ? m : 0] <= j);
            l += (uint32_t)__popcll(le);
            if (le != ~0ull) break;  // bt rises: the first entry > j ends the count
        }
        l = l ? l - 1u : 0u;  // (bt[0] = 0 <= j always)
        const uint32_t bk = p + a.parts * l;
        *b = bk;
        *lo = (uint64_t)a.bucket[bk] + (uint64_t)(j - bt[l]) * kXsChunk;
        const uint64_t e = a.bucket[bk + 1];
        *hi = *lo + kXsChunk < e ? *lo + kXsChunk : e;
    }
}

// P1 cursors: cursor[p][d] = offs[d * grid + first P0 range of p]; portion bounds and chunk counts
__global__ void k_cl_xprep1(const uint32_t* __restrict__ offs, uint32_t nd, uint32_t grid, uint32_t parts,
                            uint64_t per, uint64_t n, unsigned int* __restrict__ cursor, uint32_t* __restrict__ part_lo,
                            uint32_t* __restrict__ part_tiles, unsigned int* __restrict__ next) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < parts * nd) {
        const uint32_t p = q / nd, d = q % nd;
        cursor[q] = offs[(uint64_t)d * grid + (uint64_t)p * grid / parts];
    }
    if (q == 0) {
        uint32_t t = 0;
        for (uint32_t p = 0; p <= parts; ++p) {
            const uint64_t lo = (uint64_t)p * grid / parts * per;
            part_lo[p] = (uint32_t)(lo < n ? lo : n);
        }
        for (uint32_t p = 0; p < parts; ++p) {
            part_tiles[p] = t;
            t += (part_lo[p + 1] - part_lo[p] + kXsChunk - 1) / kXsChunk;
            next[p] = 0u;
        }
        part_tiles[parts] = t;
    }
}

// P2 work lists: the chunks of each portion's buckets. One workgroup: the chunk counts of every
// bucket in parallel into LDS, then one thread per portion scans its buckets' counts (a single
// thread reading the bounds one bucket after another took 24 us).
constexpr int kPrep2WG = 1024;
__global__ __launch_bounds__(kPrep2WG) void k_cl_xprep2(const uint32_t* __restrict__ bucket, uint32_t nb1,
                                                        uint32_t parts, uint32_t nbp,
                                                        uint32_t* __restrict__ bucket_tiles,
                                                        uint32_t* __restrict__ part_tiles,
                                                        unsigned int* __restrict__ next) {
    __shared__ uint32_t s_c[kMaxDigits];
    __shared__ uint32_t s_tot[kParts];
    for (uint32_t bk = threadIdx.x; bk < nb1; bk += kPrep2WG)
        s_c[bk] = (bucket[bk + 1] - bucket[bk] + kXsChunk - 1) / kXsChunk;
    __syncthreads();
    const uint32_t p = threadIdx.x;
    if (p < parts) {
        uint32_t c = 0;
        uint32_t* bt = bucket_tiles + (uint64_t)p * (nbp + 1);
        for (uint32_t m = 0; m < nbp; ++m) {
            bt[m] = c;
            const uint32_t bk = p + parts * m;
            if (bk < nb1) c += s_c[bk];
        }
        bt[nbp] = c;
        s_tot[p] = c;
        next[p] = 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t q = 0; q < parts; ++q) {
            part_tiles[q] = t;
            t += s_tot[q];
        }
        part_tiles[parts] = t;
    }
}

// P2h: (bucket, second digit) counts; one workgroup per chunk of any portion
// (4 chunks per workgroup with the next chunk's loads in flight and one flush per bucket: 0.207 vs
// 0.197 ms, not kept: the global atomics and the load latency are not what bounds it)
__global__ __launch_bounds__(256) void k_cl_xhist2(XArgs a) {
    __shared__ uint32_t h[kMaxDigits];
    const uint32_t k = blockIdx.x;
    if (k >= a.part_tiles[a.parts]) return;
    uint32_t p = 0;
    while (p + 1 < a.parts && a.part_tiles[p + 1] <= k) ++p;
    uint64_t lo, hi;
    uint32_t b;
    xchunk<true>(a, p, k - a.part_tiles[p], &lo, &hi, &b);
    const uint32_t mask = a.nd - 1;
    for (uint32_t d = threadIdx.x; d < a.nd; d += 256) h[d] = 0u;
    __syncthreads();
    constexpr int U = kXsChunk / 256;
    uint64_t v[U];
#pragma unroll
    for (int e = 0; e < U; ++e) {
        const uint64_t i = lo + threadIdx.x + (uint64_t)e * 256;
        v[e] = a.in.trace_id[i < hi ? i : lo];
    }
#pragma unroll
    for (int e = 0; e < U; ++e)
        if (lo + threadIdx.x + (uint64_t)e * 256 < hi) atomicAdd(&h[digit_of(part_hash(v[e]), a.shift, mask)], 1u);
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < a.nd; d += 256)
        if (h[d]) atomicAdd(&a.hist[(uint64_t)b * a.nd + d], h[d]);
}

// sub-bucket bounds from the scanned (bucket, digit) counts (the scan itself is the P2 cursors)
__global__ void k_cl_xsub(const uint32_t* __restrict__ scanned, uint64_t m, uint64_t n, uint32_t* __restrict__ sub) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < m) sub[q] = scanned[q];
    if (q == m) sub[m] = (uint32_t)n;
}

template <bool LOCAL, uint32_t MAXD>
__global__ __launch_bounds__(kXsWG, kXsWG / 256) void k_cl_xscatter(XArgs a) {
    using DigT = typename std::conditional<(MAXD <= 256), uint8_t, uint16_t>::type;
    __shared__ uint32_t s_cur[MAXD];  // output position of the chunk's run of each digit
    __shared__ uint32_t s_cnt[MAXD];  // records of the chunk per digit
    __shared__ uint32_t s_off[MAXD];  // exclusive offsets of the digits inside the sorted chunk
    __shared__ DigT s_dig[kXsChunk];  // digit of the sorted chunk's record i
    __shared__ __align__(16) uint64_t s_stage[kXsChunk];
    __shared__ uint32_t s_tmp[32];
    __shared__ uint32_t s_job;
    const int t = threadIdx.x;
    const uint32_t nd = a.nd, mask = nd - 1;
    const uint32_t p0 = xcc_id() % a.parts;
    for (uint32_t d = t; d < nd; d += kXsWG) s_cnt[d] = 0u;
    for (uint32_t step = 0; step < a.parts;) {
        const uint32_t p = (p0 + step) % a.parts;
        __syncthreads();  // the previous chunk is done with s_job and the counts
        if (t == 0) s_job = atomicAdd(&a.next[p], 1u);
        __syncthreads();
        const uint32_t j = s_job;
        if (j >= a.part_tiles[p + 1] - a.part_tiles[p]) {  // this portion is drained: the next one
            ++step;
            continue;
        }
        uint64_t lo, hi;
        uint32_t bk;
        xchunk<LOCAL>(a, p, j, &lo, &hi, &bk);
        const uint32_t cnt = (uint32_t)(hi - lo);
        unsigned int* const cur = a.cursor + (uint64_t)(LOCAL ? bk : p) * nd;
        // 1. digits and ranks (LDS atomic counting sort: the order inside a digit is free)
        uint32_t dg[kXsU], rank[kXsU];
        uint64_t tids[kXsU];
#pragma unroll
        for (int k = 0; k < kXsU; ++k) {
            const uint32_t i = t + k * kXsWG;
            tids[k] = a.in.trace_id[lo + (i < cnt ? i : 0)];
        }
#pragma unroll
        for (int k = 0; k < kXsU; ++k) {
            dg[k] = digit_of(part_hash(tids[k]), a.shift, mask);
            rank[k] = (t + k * kXsWG < cnt) ? atomicAdd(&s_cnt[dg[k]], 1u) : 0u;
        }
        __syncthreads();
        // 2. digit offsets inside the chunk; the chunk's runs claimed at the shared cursors
        scan_digits<kXsWG, MAXD>(s_cnt, nd, 0u, s_off, s_tmp);
        for (uint32_t d = t; d < nd; d += kXsWG) {
            const uint32_t c = s_cnt[d];
            s_cur[d] = c ? atomicAdd(&cur[d], c) : 0u;
        }
        __syncthreads();
        // 3. sorted position of each loaded record; digit of each sorted slot
        uint32_t pos[kXsU], dest[kXsU];
#pragma unroll
        for (int k = 0; k < kXsU; ++k) {
            pos[k] = s_off[dg[k]] + rank[k];
            if (t + k * kXsWG < cnt) s_dig[pos[k]] = (DigT)dg[k];
        }
        __syncthreads();
        // 4. output position of each sorted slot this thread writes
#pragma unroll
        for (int k = 0; k < kXsU; ++k) {
            const uint32_t i = t + k * kXsWG;
            const uint32_t d = i < cnt ? s_dig[i] : 0u;
            dest[k] = i < cnt ? s_cur[d] + (i - s_off[d]) : 0u;
        }
        // 5. the columns through the LDS stage (the traceIds are in registers already)
        move_columns<kXsU, kXsWG, 0>(a.in, a.out, lo, cnt, pos, dest, s_stage, tids);
        for (uint32_t d = t; d < nd; d += kXsWG) s_cnt[d] = 0u;  // (move_columns ended on a barrier)
    }
}

// ---- P3: trace runs inside each sub-bucket --------------------------------------------------------
constexpr int kTrWG = 512;
constexpr uint32_t kTrGrid = 2;  // P3 workgroups per CU
constexpr uint32_t kTrSlots = 2048;  // LDS trace table: load <= 1/2 at <= kTrSlots / 2 records per round
constexpr uint64_t kEmptyKey = ~0ull;  // a traceId equal to it takes the extra slot kTrSlots
constexpr int kTrFast = 4096;          // sub-buckets up to this many records: the LDS-staged path
constexpr int kTrStage = 2 * kTrFast;  // s_cur words: the fast path's u64 column stage aliases it
static_assert(kTrStage >= kTrSlots + 1, "s_cur also counts placements per slot");

struct TraceArgs {
    SpanColsDev in;
    SpanColsMut out;
    const uint32_t* sub;  // nsub + 1 sub-bucket bounds
    uint32_t nsub;
    unsigned int* next;   // work counter: sub-buckets are handed out one at a time
    unsigned long long* fail;  // sub-buckets given up (ST_SPILL_OVERFLOW: finalize -> ZK_ERR_CAPACITY)
    // list mode (the group join's fallback): only the sub-buckets list[0 .. *list_n), each written
    // to a range claimed at out_cursor, so the listed traces end up clustered in [0, *out_cursor)
    const uint32_t* list;
    const unsigned int* list_n;
    unsigned long long* out_cursor;
};
// A round that overflows the LDS table restarts its sub-bucket with twice the rounds. Rounds split
// traces on bits 40.. of the trace hash, so traceIds crafted to share those bits (mix64 is invertible)
// would overflow at every doubling: after kTrMaxDoublings the sub-bucket is given up and counted
// (finalize fails with ZK_ERR_CAPACITY instead of the pass sweeping 2^24 rounds). Honest data needs
// no doubling: a round's expected records are <= kTrSlots / 2 and its distinct traces fewer still.
constexpr uint32_t kTrMaxDoublings = 6;

__device__ __forceinline__ uint64_t trace_hash(uint64_t tid) { return zk_mix64(tid ^ kTraceSalt); }

__global__ __launch_bounds__(kTrWG) void k_cl_traces(TraceArgs a) {
    __shared__ unsigned long long s_key[kTrSlots];
    __shared__ uint32_t s_cnt[kTrSlots + 1];  // records per trace, then the trace's run start (scan)
    // records placed per trace (large sub-buckets); the fast path's u64 column stage (2048 rows)
    __shared__ __align__(16) uint32_t s_cur[kTrStage];
    __shared__ uint32_t s_work;
    __shared__ uint32_t s_fail;
    __shared__ uint64_t s_obase;
    __shared__ uint32_t s_tmp[32];
    const int t = threadIdx.x;
    constexpr int SPT = (kTrSlots + 1 + kTrWG - 1) / kTrWG;
    for (;;) {
        __syncthreads();  // every thread is past the previous sub-bucket's reads of s_work and the table
        if (t == 0) {
            uint32_t w = atomicAdd(a.next, 1u);
            if (a.list) {
                w = w < *a.list_n ? a.list[w] : a.nsub;
                if (w < a.nsub) s_obase = atomicAdd(a.out_cursor, (unsigned long long)(a.sub[w + 1] - a.sub[w]));
            } else {
                s_obase = w < a.nsub ? a.sub[w] : 0ull;
            }
            s_work = w;
        }
        __syncthreads();
        const uint32_t w = s_work;
        if (w >= a.nsub) break;
        const uint64_t lo = a.sub[w], hi = a.sub[w + 1];
        const uint64_t len = hi - lo;
        const uint64_t obase = s_obase;  // output position of the sub-bucket's first record
        // fast path (nearly every sub-bucket): the traceIds stay in registers, each record's rank
        // inside its trace comes back from the count's atomic, and the columns move through an LDS
        // stage with coalesced loads and stores (move_columns). The table holds up to kTrSlots / 2
        // distinct traces; a sub-bucket with more (or more records than kTrFast) takes the rounds
        // path below.
        if (len <= (uint64_t)kTrFast) {
            constexpr int U = kTrFast / kTrWG;
            uint32_t slots = 64;
            while (slots < 2 * len && slots < kTrSlots) slots <<= 1;
            const uint32_t smask = slots - 1;
            uint64_t tids[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const uint32_t j = t + k * kTrWG;
                tids[k] = a.in.trace_id[lo + (j < len ? j : 0)];
            }
            for (uint32_t s = t; s < slots; s += kTrWG) {
                s_key[s] = kEmptyKey;
                s_cnt[s] = 0u;
            }
            if (t == 0) {
                s_cnt[kTrSlots] = 0u;
                s_fail = 0u;
            }
            __syncthreads();
            uint32_t slot[U], rank[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                slot[k] = kTrSlots;
                rank[k] = 0u;
                if (t + k * kTrWG >= len) continue;
                const uint64_t tid = tids[k];
                if (tid != kEmptyKey) {
                    uint32_t sl = (uint32_t)trace_hash(tid) & smask, probes = 0;
                    for (;;) {
                        const unsigned long long kk = s_key[sl];
                        if (kk == tid) break;
                        if (kk == kEmptyKey) {
                            const unsigned long long old = atomicCAS(&s_key[sl], kEmptyKey, (unsigned long long)tid);
                            if (old == kEmptyKey || old == tid) break;
                        }
                        sl = (sl + 1) & smask;
                        if (++probes >= slots) {  // more distinct traces than the table holds
                            s_fail = 1u;
                            sl = kTrSlots + 1;
                            break;
                        }
                    }
                    slot[k] = sl;
                }
                if (slot[k] <= kTrSlots) rank[k] = atomicAdd(&s_cnt[slot[k]], 1u);
            }
            __syncthreads();
            if (s_fail == 0u) {
                uint32_t h[SPT], sum = 0;
#pragma unroll
                for (int q = 0; q < SPT; ++q) {
                    const uint32_t sx = t * SPT + q;
                    h[q] = (sx < slots || sx == kTrSlots) ? s_cnt[sx] : 0u;
                    sum += h[q];
                }
                uint32_t tot;
                uint32_t ex = block_excl_scan<kTrWG / 64>(sum, s_tmp, &tot);
#pragma unroll
                for (int q = 0; q < SPT; ++q) {
                    const uint32_t sx = t * SPT + q;
                    if (sx < slots || sx == kTrSlots) s_cnt[sx] = ex;
                    ex += h[q];
                }
                __syncthreads();
                uint32_t pos[U];
                uint32_t dest[U];
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    pos[k] = s_cnt[slot[k]] + rank[k];
                    dest[k] = (uint32_t)obase + t + k * kTrWG;
                }
                move_columns<U, kTrWG, 0>(a.in, a.out, lo, (uint32_t)len, pos, dest,
                                          reinterpret_cast<uint64_t*>(s_cur), tids);
                continue;
            }
            __syncthreads();  // every thread read s_fail before the rounds path clears it
        }
        // rounds of <= 2048 records expected (a hash range of the traceIds each), and a table of a
        // power of two >= 2 x the round's records: the load stays <= 1/2 whatever the trace sizes
        // (a round's distinct traceIds are at most its records)
        uint32_t rounds = 1;
        while (len / rounds > kTrSlots / 2) rounds <<= 1;
        uint32_t doublings = 0;
        uint32_t slots = 64;
        while (slots < 2 * (len / rounds + 1) && slots < kTrSlots) slots <<= 1;
        uint32_t smask = slots - 1;
        uint64_t placed = obase;  // output position of this round's first record
        for (uint32_t r = 0; r < rounds; ++r) {
            for (uint32_t s = t; s < slots; s += kTrWG) {
                s_key[s] = kEmptyKey;
                s_cnt[s] = 0u;
                s_cur[s] = 0u;
            }
            if (t == 0) {
                s_cnt[kTrSlots] = 0u;
                s_cur[kTrSlots] = 0u;
                s_fail = 0u;
            }
            __syncthreads();
            // sweep 1: count each trace's records of this round
            for (uint64_t i = lo + t; i < hi; i += kTrWG) {
                const uint64_t tid = a.in.trace_id[i];
                const uint64_t th = trace_hash(tid);
                if (rounds > 1 && (uint32_t)(th >> 40) % rounds != r) continue;
                uint32_t slot = kTrSlots;
                if (tid != kEmptyKey) {
                    slot = (uint32_t)th & smask;
                    uint32_t probes = 0;
                    for (;;) {
                        const unsigned long long k = s_key[slot];
                        if (k == tid) break;
                        if (k == kEmptyKey) {
                            const unsigned long long old = atomicCAS(&s_key[slot], kEmptyKey, (unsigned long long)tid);
                            if (old == kEmptyKey || old == tid) break;
                        }
                        slot = (slot + 1) & smask;
                        if (++probes >= slots) {  // full: a hash range far above its share of traces
                            s_fail = 1u;
                            slot = kTrSlots + 1;
                            break;
                        }
                    }
                }
                if (slot <= kTrSlots) atomicAdd(&s_cnt[slot], 1u);
            }
            __syncthreads();
            if (s_fail) {
                if (++doublings > kTrMaxDoublings || rounds >= (1u << 24)) {
                    // colliding traceIds: give the sub-bucket up (its output rows stay unwritten)
                    if (t == 0) atomicAdd(a.fail, 1ull);
                    break;
                }
                // start the sub-bucket over with twice the rounds (every output position of the
                // sub-bucket is rewritten by the new layout)
                rounds <<= 1;
                slots = 64;
                while (slots < 2 * (len / rounds + 1) && slots < kTrSlots) slots <<= 1;
                smask = slots - 1;
                placed = obase;
                r = ~0u;  // the loop's ++r makes it round 0
                __syncthreads();  // every thread read s_fail before the next round clears it
                continue;
            }
            // scan: the run start of each trace of the round (slot order, the extra slot last)
            {
                uint32_t h[SPT], sum = 0;
#pragma unroll
                for (int q = 0; q < SPT; ++q) {
                    const uint32_t s = t * SPT + q;
                    h[q] = (s < slots || s == kTrSlots) ? s_cnt[s] : 0u;
                    sum += h[q];
                }
                uint32_t tot;
                uint32_t ex = block_excl_scan<kTrWG / 64>(sum, s_tmp, &tot);
                __syncthreads();  // every thread read its counts before any is overwritten
#pragma unroll
                for (int q = 0; q < SPT; ++q) {
                    const uint32_t s = t * SPT + q;
                    if (s < slots || s == kTrSlots) s_cnt[s] = ex;
                    ex += h[q];
                }
                if (t == 0) s_tmp[31] = tot;
            }
            __syncthreads();
            const uint32_t round_records = s_tmp[31];
            // sweep 2: every record of the round to its trace's run
            for (uint64_t i = lo + t; i < hi; i += kTrWG) {
                const uint64_t tid = a.in.trace_id[i];
                const uint64_t th = trace_hash(tid);
                if (rounds > 1 && (uint32_t)(th >> 40) % rounds != r) continue;
                uint32_t slot = kTrSlots;
                if (tid != kEmptyKey) {
                    slot = (uint32_t)th & smask;
                    while (s_key[slot] != tid) slot = (slot + 1) & smask;
                }
                const uint64_t j = placed + s_cnt[slot] + atomicAdd(&s_cur[slot], 1u);
                a.out.trace_id[j] = tid;
                a.out.span_id[j] = a.in.span_id[i];
                a.out.parent_id[j] = a.in.parent_id[i];
                a.out.first_ts[j] = a.in.first_ts[i];
                a.out.last_ts[j] = a.in.last_ts[i];
                a.out.service_id[j] = a.in.service_id[i];
                a.out.flags[j] = a.in.flags[i];
            }
            placed += round_records;
            __syncthreads();  // the round's placement reads are done before the next round clears
        }
    }
}

__global__ __launch_bounds__(256) void k_trace_set_insert(const uint64_t* __restrict__ tid, uint64_t n,
                                                          unsigned long long* __restrict__ set, uint64_t slots,
                                                          unsigned long long* __restrict__ dup,
                                                          const unsigned long long* __restrict__ n_dev,
                                                          const uint32_t* __restrict__ skip_dev) {
    uint32_t found = 0;
    const uint64_t mask = slots - 1;
    if (n_dev && *n_dev < n) n = *n_dev;
    const uint64_t i0 = (skip_dev && *skip_dev) ? 1 : 0;  // record 0's run: the held trace's
    for (uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
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

// ZK_BATCH_CONTINUES on the device (zk_cluster.h CarryState), one workgroup: the batch's edge runs
// (the first trace boundary in [1, min(n, L + 1)), the last in [max(1, n - L - 1), n), searched 256
// records at a time from each end, so a batch of short traces costs a few hundred bytes), then one
// thread applies the rules that zk_deps_accumulate documents for held traces to this batch (n > 0)
// or flushes the carry (n == 0), then the workgroup appends the batch's leading run to the carry.
__global__ __launch_bounds__(256) void k_carry_plan(CarryState* __restrict__ cs, SpanColsDev b, SpanColsMut m,
                                                    uint64_t L, uint32_t continues, uint32_t verify,
                                                    uint32_t k1_joins, unsigned long long* __restrict__ too_large,
                                                    unsigned int* __restrict__ spill_count,
                                                    unsigned long long* __restrict__ set, uint64_t slots,
                                                    unsigned long long* __restrict__ dup) {
    __shared__ unsigned long long s_e0, s_e1, s_at, s_len;
    const uint32_t t = threadIdx.x;
    const uint64_t n = b.n;
    const uint64_t* __restrict__ tid = b.trace_id;
    if (t == 0) {
        s_e0 = ~0ull;
        s_e1 = 0;
        if (spill_count) *spill_count = 0;  // the batch's K1 spill list starts empty
    }
    __syncthreads();
    if (n >= 2) {
        const uint64_t head = n < L + 1 ? n : L + 1;
        for (uint64_t base = 1; base < head; base += 256) {
            const uint64_t i = base + t;
            if (i < head && tid[i] != tid[i - 1]) atomicMin(&s_e0, (unsigned long long)i);
            __syncthreads();
            const bool found = s_e0 != ~0ull;
            __syncthreads();  // (read by all before another round's atomics)
            if (found) break;
        }
        const uint64_t tail0 = n > L + 1 ? n - L - 1 : 1;
        for (uint64_t top = n; top > tail0; top = top > tail0 + 256 ? top - 256 : tail0) {
            const uint64_t lo = top > tail0 + 256 ? top - 256 : tail0;
            const uint64_t i = lo + t;
            if (i < top && tid[i] != tid[i - 1]) atomicMax(&s_e1, (unsigned long long)i);
            __syncthreads();
            const bool found = s_e1 != 0;
            __syncthreads();
            if (found) break;
        }
    }
    if (t == 0) {
        constexpr uint64_t kUnknown = ~0ull;  // an edge run longer than the L + 1 records searched
        cs->append_n = 0;
        cs->append_at = 0;
        cs->flush_n = 0;
        cs->flush_vn = 0;
        cs->zero = 0;
        cs->skip = 0;
        cs->hi = 0;
        cs->tail_lo = kUnknown;
        const uint64_t held_tid = cs->tid;
        auto flush = [&]() {  // the held trace is complete: join it now
            cs->flush_n = cs->n;
            cs->flush_vn = cs->verify ? cs->n : 0;
            cs->n = 0;
            cs->verify = 0;
        };
        bool done = false;
        if (n == 0) {
            cs->dropped = 0;
            flush();
            done = true;
        }
        uint64_t lead = 0;
        if (!done) {
            const uint64_t e0 = s_e0, e1 = s_e1;
            const uint64_t t0 = tid[0], tn = tid[n - 1];
            // the whole batch is one trace: no boundary in the searched head (all of it when
            // n <= L + 1), or none in head and tail and the same traceId at both ends (trace-clustered)
            const bool no_head = e0 == ~0ull, no_tail = e1 == 0;
            const bool one_run = no_head && (n <= L + 1 || (no_tail && t0 == tn));
            // end of the leading run, start of the last one (a run longer than L + 1 is only known to
            // be long; a held run has at most L + 1 records, the carry holds L + 2)
            const uint64_t first_end = one_run ? n : (no_head ? kUnknown : e0);
            const uint64_t last_start = one_run ? (n <= L + 1 ? 0 : kUnknown) : (no_tail ? kUnknown : e1);
            if (cs->n || cs->dropped) {
                if (t0 == cs->tid) {
                    lead = first_end;
                    if (cs->dropped) {
                        // the rest of a trace already found too long: skipped like its beginning
                    } else if (lead == kUnknown || cs->n + lead > L) {
                        cs->n = 0;  // longer than max_trace_records: not aggregated, counted once
                        cs->dropped = 1;
                        atomicAdd(too_large, 1ull);
                    } else {
                        cs->append_at = cs->n;
                        cs->append_n = lead;
                        cs->n += lead;
                    }
                }
                cs->verify |= verify;
                if (lead == n && continues) {
                    done = true;  // the whole batch continues the held trace
                } else {
                    cs->dropped = 0;
                    flush();
                }
            }
            if (!done) {
                uint64_t hi = n;
                if (continues && last_start != kUnknown) {
                    // (a last run longer than L + 1 is not held: K1 reports it too large; the leading
                    // run ends at or before the last run's start unless the batch is one run)
                    const uint64_t ls = (lead != kUnknown && lead > last_start) ? lead : last_start;
                    if (ls < n) {
                        cs->tail_lo = ls;
                        cs->n = n - ls;
                        cs->tid = tn;
                        cs->verify = verify;
                        hi = ls;
                    }
                }
                cs->hi = hi;
                cs->skip = lead ? 1u : 0u;  // K1 starts at the first trace boundary after record 0
            }
        }
        // who joins a flushed carry: K1 over it (one workgroup, its own spill list, which K1 fills when
        // the trace outgrows a window) or, for a flush alone, the spill kernel (one list entry)
        cs->flush_cnt = (!k1_joins && cs->flush_n) ? 1u : 0u;
        // the held trace's run in the trace set (ZK_BATCH_VERIFY_TRACES): inserted when it is joined
        if (set && cs->flush_vn) {
            bool seen;
            if (held_tid == 0ull)
                seen = atomicAdd(&set[slots], 1ull) > 0ull;
            else
                seen = set_insert(set, slots - 1, held_tid);
            if (seen) atomicAdd(dup, 1ull);
        }
        s_at = cs->append_at;
        s_len = cs->append_n;
    }
    __syncthreads();
    const uint64_t at = s_at, len = s_len;
    for (uint64_t k = t; k < len; k += 256) {  // the leading run into the held trace
        m.trace_id[at + k] = b.trace_id[k];
        m.span_id[at + k] = b.span_id[k];
        m.parent_id[at + k] = b.parent_id[k];
        m.first_ts[at + k] = b.first_ts[k];
        m.last_ts[at + k] = b.last_ts[k];
        m.service_id[at + k] = b.service_id[k];
        m.flags[at + k] = b.flags[k];
    }
}

// the batch's tail [tail_lo, n) -> the carry (after the carry's join has read the old one)
__global__ __launch_bounds__(256) void k_carry_tail(const CarryState* __restrict__ cs, SpanColsDev b, SpanColsMut m) {
    const uint64_t lo = cs->tail_lo;
    const uint64_t len = lo < b.n ? b.n - lo : 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < len; k += stride) {
        const uint64_t i = lo + k;
        m.trace_id[k] = b.trace_id[i];
        m.span_id[k] = b.span_id[i];
        m.parent_id[k] = b.parent_id[i];
        m.first_ts[k] = b.first_ts[i];
        m.last_ts[k] = b.last_ts[i];
        m.service_id[k] = b.service_id[i];
        m.flags[k] = b.flags[i];
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

// one counter += v on the stream (a held trace dropped by the host-side continuation logic)
__global__ __launch_bounds__(64) void k_stat_add(unsigned long long* __restrict__ slot, unsigned long long v) {
    if (threadIdx.x == 0) atomicAdd(slot, v);
}

unsigned grid_for(uint64_t n) {
    const uint64_t g = (n + 255) / 256;
    return (unsigned)(g < 8192 ? (g ? g : 1) : 8192);
}

uint64_t align256(uint64_t b) { return (b + 255) & ~255ull; }

size_t scan_bytes(uint64_t m) {
    size_t b = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)m);
    return b;
}

}  // namespace

ClusterPlan cluster_plan(uint64_t n, uint32_t cus, bool groups) {
    ClusterPlan p{};
    p.n = n;
    // digit bits in all: sub-buckets of 1-2k records on average (P3's fast path takes up to 4096);
    // for the group join 3/8 of its LDS capacity, so that batches of whole sub-buckets fill it and
    // hardly any sub-bucket exceeds it
    uint32_t bits = 0;
    uint64_t target = groups ? group_join_capacity() * 3 / 8 : 2048;
#ifdef ZK_DIAG_ENV  // diagnostic builds only (tools/build_variant.py): A/B override of the sub-bucket target
    if (const char* e = groups ? getenv("ZK_CL_GROUP_TARGET") : nullptr) target = (uint64_t)atoi(e);
#endif
    while (bits < 22 && (n >> bits) > target) ++bits;
    if (n <= kClusterSmall) bits = 0;  // P3 alone: one workgroup over the whole batch
    if (bits <= 8) {
        p.b1 = bits;
        p.b2 = 0;
    } else {
        p.b1 = 8;
        p.b2 = bits - 8;
        if (p.b2 > 11) {  // > 2^29 records: widen the first level
            p.b1 = bits - 11;
            p.b2 = 11;
        }
    }
#ifdef ZK_DIAG_ENV  // diagnostic builds only: A/B override of the digit split
    if (const char* e1 = getenv("ZK_CL_B1")) {
        const uint32_t b1 = (uint32_t)atoi(e1);
        if (b1 <= bits && b1 <= 11 && bits - b1 <= 11 && (b1 > 0 || bits == 0)) {
            p.b1 = b1;
            p.b2 = bits - b1;
        }
    }
#endif
    p.nb1 = 1u << p.b1;
    p.nb2 = 1u << p.b2;
    // P0 geometry (the ranges P1's portions are cut from): one range per CU, whole chunks each
    uint64_t g = (uint64_t)(cus ? cus : 256);
    const uint64_t chunks = (n + kXsChunk - 1) / kXsChunk;
    if (g > chunks) g = chunks ? chunks : 1;
    p.grid = (uint32_t)g;
    p.per = ((n + g - 1) / g + kXsChunk - 1) / kXsChunk * kXsChunk;
    if (!p.per) p.per = kXsChunk;
    return p;
}

// the XCD-shared-stream path's extra scratch: P1 cursors, portion tables, P2 chunk lists, the
// (bucket, digit) counts and the P2 cursors
struct XLayout {
    uint64_t cur1, part, btiles, m2, total;
};
XLayout x_layout(const ClusterPlan& p) {
    XLayout l{};
    const uint64_t nbp = (p.nb1 + kParts - 1) / kParts;
    l.m2 = (uint64_t)p.nb1 * p.nb2 + 1;
    l.cur1 = align256((uint64_t)kParts * p.nb1 * 4);
    l.part = align256((kParts + 1) * 4);
    l.btiles = align256(kParts * (nbp + 1) * 4);
    l.total = l.cur1 + 3 * l.part + l.btiles + 2 * align256(l.m2 * 4);
    return l;
}

// the group join's list of long sub-buckets and its two counters, at the end of the scratch
uint64_t group_bytes(const ClusterPlan& p) { return align256((uint64_t)p.nb1 * p.nb2 * 4) + 256; }

uint64_t cluster_scratch_bytes(const ClusterPlan& p) {
    const uint64_t m = (uint64_t)p.nb1 * p.grid;
    const XLayout xl = x_layout(p);
    const uint64_t sm = m > xl.m2 ? m : xl.m2;
    return 2 * align256(m * 4) + align256(((uint64_t)p.nb1 + 1) * 4) + align256(((uint64_t)p.nb1 * p.nb2 + 1) * 4) +
           256 + xl.total + align256(scan_bytes(sm)) + group_bytes(p);
}

hipError_t launch_cluster(const ClusterPlan& p, const SpanColsDev& in, const SpanColsMut& A, const SpanColsMut& B,
                          void* scratch, uint32_t cus, hipStream_t s, int* result,
                          unsigned long long* capacity_fail, ClusterGroups* groups) {
    const uint64_t n = in.n;
    *result = 0;
    if (n == 0) return hipSuccess;
    const uint64_t m = (uint64_t)p.nb1 * p.grid;
    uint8_t* sp = (uint8_t*)scratch;
    uint32_t* hist = (uint32_t*)sp;
    uint32_t* offs = (uint32_t*)(sp + align256(m * 4));
    uint32_t* bucket = (uint32_t*)(sp + 2 * align256(m * 4));
    uint32_t* sub = (uint32_t*)((uint8_t*)bucket + align256(((uint64_t)p.nb1 + 1) * 4));
    unsigned int* next = (unsigned int*)((uint8_t*)sub + align256(((uint64_t)p.nb1 * p.nb2 + 1) * 4));
    const XLayout xl = x_layout(p);
    uint8_t* xp = (uint8_t*)next + 256;
    unsigned int* cursor1 = (unsigned int*)xp;
    uint32_t* part_lo = (uint32_t*)(xp + xl.cur1);
    uint32_t* part_tiles = (uint32_t*)(xp + xl.cur1 + xl.part);
    unsigned int* xnext = (unsigned int*)(xp + xl.cur1 + 2 * xl.part);
    uint32_t* bucket_tiles = (uint32_t*)(xp + xl.cur1 + 3 * xl.part);
    uint32_t* hist2 = (uint32_t*)(xp + xl.cur1 + 3 * xl.part + xl.btiles);
    unsigned int* cursor2 = (unsigned int*)((uint8_t*)hist2 + align256(xl.m2 * 4));
    void* temp = xp + xl.total;
    hipError_t e = hipMemsetAsync(next, 0, 4, s);
    if (e != hipSuccess) return e;
    auto dev = [n](const SpanColsMut& c) {
        return SpanColsDev{c.trace_id, c.span_id, c.parent_id, c.first_ts, c.last_ts, c.service_id, c.flags, n};
    };
    TraceArgs ta{};
    ta.next = next;
    ta.fail = capacity_fail;
    if (!p.b1) {  // P3 alone: in -> A
        const uint32_t h_sub[2] = {0u, (uint32_t)n};
        e = hipMemcpyAsync(sub, h_sub, 8, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
        ta.in = in;
        ta.out = A;
        ta.sub = sub;
        ta.nsub = 1;
        *result = 0;
        return launch_checked("k_cl_traces", k_cl_traces, dim3(1), dim3(kTrWG), 0, s, ta);
    }
    // P0 + scan + first-level bucket bounds
    const uint32_t sh1 = 64 - p.b1;
    e = launch_checked("k_cl_hist", k_cl_hist, dim3(p.grid), dim3(kHistWG), (size_t)p.nb1 * 4, s, in.trace_id, n, p.per,
                       sh1, p.nb1, p.grid, hist);
    if (e != hipSuccess) return e;
    size_t temp_bytes = scan_bytes(m);
    e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, hist, offs, (int)m, s);
    if (e != hipSuccess) return e;
    e = launch_checked("k_cl_bounds", k_cl_bounds, dim3((p.nb1 + 256) / 256), dim3(256), 0, s, offs, p.nb1, p.grid, n,
                       bucket);
    if (e != hipSuccess) return e;
    // P1: in -> A (first-level buckets)
    const uint32_t parts1 = p.grid < kParts ? p.grid : kParts;
    XArgs x1{};
    {
        x1.in = in;
        x1.out = A;
        x1.shift = sh1;
        x1.nd = p.nb1;
        x1.parts = parts1;
        x1.part_tiles = part_tiles;
        x1.next = xnext;
        x1.cursor = cursor1;
        x1.part_lo = part_lo;
        e = launch_checked("k_cl_xprep1", k_cl_xprep1, dim3((parts1 * p.nb1 + 255) / 256), dim3(256), 0, s,
                           (const uint32_t*)offs, p.nb1, p.grid, parts1, p.per, n, cursor1, part_lo, part_tiles, xnext);
        if (e != hipSuccess) return e;
    }
    const uint32_t gx = cus ? cus : 256;
    e = p.nb1 <= kSmallDigits
            ? launch_checked("k_cl_xscatter<global,256>", k_cl_xscatter<false, kSmallDigits>, dim3(gx), dim3(kXsWG), 0, s,
                             x1)
        : p.nb1 <= kMidDigits
            ? launch_checked("k_cl_xscatter<global,512>", k_cl_xscatter<false, kMidDigits>, dim3(gx), dim3(kXsWG), 0, s, x1)
            : launch_checked("k_cl_xscatter<global>", k_cl_xscatter<false, kMaxDigits>, dim3(gx), dim3(kXsWG), 0, s, x1);
    if (e != hipSuccess) return e;
    if (!p.b2) {  // P3: A -> B
        ta.in = dev(A);
        ta.out = B;
        ta.sub = bucket;
        ta.nsub = p.nb1;
        *result = 1;
    } else {  // P2: A -> B (sub-buckets), P3: B -> A
        const uint32_t parts2 = p.nb1 < kParts ? p.nb1 : kParts;
        const uint32_t nbp = (p.nb1 + parts2 - 1) / parts2;
        XArgs x2{};
        {
            x2.in = dev(A);
            x2.out = B;
            x2.shift = sh1 - p.b2;
            x2.nd = p.nb2;
            x2.parts = parts2;
            x2.part_tiles = part_tiles;
            x2.next = xnext;
            x2.cursor = cursor2;
            x2.bucket = bucket;
            x2.bucket_tiles = bucket_tiles;
            x2.nb1 = p.nb1;
            x2.nbp = nbp;
            x2.hist = hist2;
            const uint32_t maxchunks = (uint32_t)((n + kXsChunk - 1) / kXsChunk + p.nb1);
            size_t tb2 = scan_bytes(xl.m2);
            e = launch_checked("k_cl_xprep2", k_cl_xprep2, dim3(1), dim3(kPrep2WG), 0, s, (const uint32_t*)bucket, p.nb1,
                               parts2, nbp, bucket_tiles, part_tiles, xnext);
            if (e == hipSuccess) e = hipMemsetAsync(hist2, 0, xl.m2 * 4, s);
            if (e == hipSuccess) e = launch_checked("k_cl_xhist2", k_cl_xhist2, dim3(maxchunks), dim3(256), 0, s, x2);
            if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(temp, tb2, hist2, cursor2, (int)xl.m2, s);
            if (e == hipSuccess)
                e = launch_checked("k_cl_xsub", k_cl_xsub, dim3((unsigned)((xl.m2 + 255) / 256)), dim3(256), 0, s,
                                   (const uint32_t*)cursor2, xl.m2 - 1, n, sub);
            if (e != hipSuccess) return e;
        }
        e = p.nb2 <= kSmallDigits
                ? launch_checked("k_cl_xscatter<local,256>", k_cl_xscatter<true, kSmallDigits>, dim3(gx), dim3(kXsWG), 0,
                                 s, x2)
            : p.nb2 <= kMidDigits
                ? launch_checked("k_cl_xscatter<local,512>", k_cl_xscatter<true, kMidDigits>, dim3(gx), dim3(kXsWG), 0, s,
                                 x2)
                : launch_checked("k_cl_xscatter<local>", k_cl_xscatter<true, kMaxDigits>, dim3(gx), dim3(kXsWG), 0, s, x2);
        if (e != hipSuccess) return e;
        if (groups) {  // the group join takes the sub-buckets from here
            uint8_t* gp = (uint8_t*)scratch + cluster_scratch_bytes(p) - group_bytes(p);
            groups->sub = sub;
            groups->nsub = p.nb1 * p.nb2;
            groups->big_list = (uint32_t*)gp;
            groups->big_count = (unsigned int*)(gp + align256((uint64_t)p.nb1 * p.nb2 * 4));
            groups->out_cursor = (unsigned long long*)(gp + align256((uint64_t)p.nb1 * p.nb2 * 4) + 64);
            *result = 1;
            return hipMemsetAsync(groups->big_count, 0, 128, s);
        }
        ta.in = dev(B);
        ta.out = A;
        ta.sub = sub;
        ta.nsub = p.nb1 * p.nb2;
        *result = 0;
    }
    const uint32_t g3 = ta.nsub < kTrGrid * cus ? ta.nsub : kTrGrid * cus;
    return launch_checked("k_cl_traces", k_cl_traces, dim3(g3), dim3(kTrWG), 0, s, ta);
}

hipError_t launch_cluster_fallback(const ClusterPlan& p, const ClusterGroups& g, const SpanColsDev& B,
                                   const SpanColsMut& A, void* scratch, uint32_t cus, hipStream_t s,
                                   unsigned long long* capacity_fail) {
    // the work counter of launch_cluster's layout
    const uint64_t m = (uint64_t)p.nb1 * p.grid;
    uint8_t* bucket = (uint8_t*)scratch + 2 * align256(m * 4);
    uint8_t* sub = bucket + align256(((uint64_t)p.nb1 + 1) * 4);
    unsigned int* next = (unsigned int*)(sub + align256(((uint64_t)p.nb1 * p.nb2 + 1) * 4));
    hipError_t e = hipMemsetAsync(next, 0, 4, s);
    if (e != hipSuccess) return e;
    TraceArgs ta{};
    ta.in = B;
    ta.out = A;
    ta.sub = g.sub;
    ta.nsub = g.nsub;
    ta.next = next;
    ta.fail = capacity_fail;
    ta.list = g.big_list;
    ta.list_n = g.big_count;
    ta.out_cursor = g.out_cursor;
    // one workgroup per CU: normally the list is empty and every workgroup leaves at once
    return launch_checked("k_cl_traces<list>", k_cl_traces, dim3(cus ? cus : 256), dim3(kTrWG), 0, s, ta);
}

hipError_t launch_trace_set_insert(const uint64_t* trace_id, uint64_t n, uint64_t* set, uint64_t slots,
                                   unsigned long long* dup, hipStream_t s, const unsigned long long* n_dev,
                                   const uint32_t* skip_dev) {
    if (n == 0) return hipSuccess;
    return launch_checked("k_trace_set_insert", k_trace_set_insert, dim3(grid_for(n)), dim3(256), 0, s, trace_id, n,
                          (unsigned long long*)set, slots, dup, n_dev, skip_dev);
}

hipError_t launch_carry_plan(CarryState* cs, const SpanColsDev& batch, const SpanColsMut& carry, uint64_t max_trace,
                             uint32_t continues, uint32_t verify, uint32_t k1_joins, unsigned long long* too_large,
                             unsigned int* spill_count, uint64_t* set, uint64_t slots, unsigned long long* dup,
                             hipStream_t s) {
    return launch_checked("k_carry_plan", k_carry_plan, dim3(1), dim3(256), 0, s, cs, batch, carry, max_trace,
                          continues, verify, k1_joins, too_large, spill_count, (unsigned long long*)set, slots, dup);
}

hipError_t launch_carry_tail(const CarryState* cs, const SpanColsDev& batch, const SpanColsMut& carry, hipStream_t s) {
    return launch_checked("k_carry_tail", k_carry_tail, dim3(64), dim3(256), 0, s, cs, batch, carry);
}

hipError_t launch_trace_set_rehash(const uint64_t* old, uint64_t old_slots, uint64_t* set, uint64_t slots,
                                   hipStream_t s) {
    return launch_checked("k_trace_set_rehash", k_trace_set_rehash, dim3(grid_for(old_slots + 1)), dim3(256), 0, s,
                          (const unsigned long long*)old, old_slots, (unsigned long long*)set, slots);
}

hipError_t launch_stat_add(unsigned long long* slot, uint64_t v, hipStream_t s) {
    return launch_checked("k_stat_add", k_stat_add, dim3(1), dim3(64), 0, s, slot, (unsigned long long)v);
}

hipError_t launch_stats_fold(const unsigned long long* shards, unsigned long long* out, hipStream_t s) {
    return launch_checked("k_stats_fold", k_stats_fold, dim3(1), dim3(256), 0, s, shards, (int)kStatShards, out);
}

}  // namespace zk
