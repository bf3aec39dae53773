// zk_join.hip — K1 span_join: merge fragments, validate, parent join, emit links.
//
// Restates zipkin-aggregate/.../aggregate/ZipkinAggregateJob.scala:20-38 over trace-clustered
// columnar records (one record = one stored span fragment, 48 B):
//   :21-22  groupBy((id, traceId)).reduce(mergeSpan)    -> LDS hash on (spanId, trace segment);
//           Span.mergeSpan (Span.scala:148-169): annotations concatenated, so first = min,
//           last = max, core-annotation counts add; parentId is the left operand's (order
//           dependent: ambiguous when fragments disagree, see zk_stats.ambiguous)
//   :23     filter(isValid)           -> every core annotation at most once (Span.scala:236-240)
//   :25-33  parentSpans.join(childSpans) on (parentId, traceId) -> probe of the same LDS hash
//   :34-37  Moments(child.duration), DependencyLink(parent.serviceName.get, child.serviceName.get)
//           duration = last - first over all annotations (Span.scala:228-230)
//
// Mapping to CDNA4: one workgroup owns the traces STARTING in a fixed tile of TILE records and
// stages them (up to CAP records, the tail trace may overhang the tile) in LDS. Every record is
// read from HBM exactly once with coalesced 8/4-byte column loads; the merge and the join never
// leave LDS. Traces longer than the tile capacity are deferred to k_span_join_spill (global
// scratch, one trace per workgroup at a time).
#include "zk_internal.h"

namespace zk {
namespace {

constexpr int kSpillWG = 256;

__device__ __forceinline__ uint32_t slot_hash(uint64_t sid, uint32_t seg) {
    uint64_t x = sid ^ ((uint64_t)(seg + 1) * 0x9E3779B97F4A7C15ull);
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    return (uint32_t)x;
}

__device__ __forceinline__ uint32_t svc_key(uint32_t flags, uint32_t svc, uint32_t S, bool* range_err) {
    uint32_t kind = (flags & ZK_F_SVC_SERVER) ? 0u : (flags & ZK_F_SVC_CLIENT) ? 1u : 2u;
    if (kind == 2u) return kSvcNone;
    if (svc >= S) {
        *range_err = true;
        return kSvcNone;
    }
    return (kind << kSvcKindShift) | svc;
}

// Tile counts word: 13-bit occurrence counts of cs|cr|sr|ss (each fragment adds 0..2) and the
// number of fragments carrying a parentId in bits 52..63. CAP <= 2048 keeps every field in range.
__device__ __forceinline__ uint64_t pack_counts(uint32_t f) {
    const uint64_t cs = (f >> ZK_F_CS_SHIFT) & 3u, cr = (f >> ZK_F_CR_SHIFT) & 3u;
    const uint64_t sr = (f >> ZK_F_SR_SHIFT) & 3u, ss = (f >> ZK_F_SS_SHIFT) & 3u;
    return cs | (cr << 13) | (sr << 26) | (ss << 39) | ((uint64_t)(f & ZK_F_HAS_PARENT) << 52);
}
__device__ __forceinline__ bool counts_valid(uint64_t c) {
    return (c & 0x1FFFull) <= 1 && ((c >> 13) & 0x1FFFull) <= 1 && ((c >> 26) & 0x1FFFull) <= 1 &&
           ((c >> 39) & 0x1FFFull) <= 1;
}
__device__ __forceinline__ uint32_t counts_npar(uint64_t c) { return (uint32_t)(c >> 52); }

// ---- link emission: exact power sums as 32-bit chunks into u64 limbs (no carries) ----------
__device__ __forceinline__ void add_chunk(uint64_t* p, uint64_t v) {
    if (v) atomicAdd((unsigned long long*)p, (unsigned long long)v);
}

__device__ __forceinline__ void emit_link(uint64_t* __restrict__ table, uint32_t cell, uint64_t d) {
    uint64_t* c = table + (uint64_t)cell * kLimbs;
    constexpr uint64_t M = 0xFFFFFFFFull;
    atomicAdd((unsigned long long*)(c + kLimbM0), 1ull);
    add_chunk(c + kLimbS1 + 0, d & M);
    add_chunk(c + kLimbS1 + 1, d >> 32);
    const unsigned __int128 d2 = (unsigned __int128)d * d;  // < 2^80
    const uint64_t d2lo = (uint64_t)d2, d2hi = (uint64_t)(d2 >> 64);
    add_chunk(c + kLimbS2 + 0, d2lo & M);
    add_chunk(c + kLimbS2 + 1, d2lo >> 32);
    add_chunk(c + kLimbS2 + 2, d2hi);
    const unsigned __int128 d3 = d2 * d;  // < 2^120
    const uint64_t d3lo = (uint64_t)d3, d3hi = (uint64_t)(d3 >> 64);
    add_chunk(c + kLimbS3 + 0, d3lo & M);
    add_chunk(c + kLimbS3 + 1, d3lo >> 32);
    add_chunk(c + kLimbS3 + 2, d3hi & M);
    add_chunk(c + kLimbS3 + 3, d3hi >> 32);
    const unsigned __int128 p0 = (unsigned __int128)d3lo * d;
    const unsigned __int128 p1 = (unsigned __int128)d3hi * d + (uint64_t)(p0 >> 64);
    const uint64_t w0 = (uint64_t)p0, w1 = (uint64_t)p1, w2 = (uint64_t)(p1 >> 64);  // d^4 < 2^160
    add_chunk(c + kLimbS4 + 0, w0 & M);
    add_chunk(c + kLimbS4 + 1, w0 >> 32);
    add_chunk(c + kLimbS4 + 2, w1 & M);
    add_chunk(c + kLimbS4 + 3, w1 >> 32);
    add_chunk(c + kLimbS4 + 4, w2);
}

// packed per-thread stat counters: 4 x 16-bit fields per u64 (a tile never exceeds 2^16)
struct StatPack {
    uint64_t w[4] = {0, 0, 0, 0};
    __device__ __forceinline__ void inc(int s, uint32_t v = 1) { w[s >> 2] += (uint64_t)v << (16 * (s & 3)); }
};

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Per-thread packed counts -> per-wave sums (16-bit fields cannot overflow: a wave covers at most
// 64 x 512 records) -> u32 LDS totals -> one add per stat into a sharded global slot (the stats
// array holds kStatShards copies, summed by the host, so 1e5 tiles never hammer one address).
__device__ __forceinline__ void flush_stats(StatPack& sp, uint32_t* s_stat, unsigned long long* g_stats) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t v = wave_sum_u64(sp.w[i]);
        if (lane == 0 && v) {
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const uint32_t x = (uint32_t)((v >> (16 * f)) & 0xFFFFull);
                if (x) atomicAdd(&s_stat[i * 4 + f], x);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < ST_N) {
        const uint32_t v = s_stat[threadIdx.x];
        unsigned long long* slot = g_stats + (uint64_t)(blockIdx.x % kStatShards) * ST_N;
        if (v) atomicAdd(&slot[threadIdx.x], (unsigned long long)v);
    }
}

// =============================================================================================
// K1: tile kernel
//
// Workgroup = 256 threads owning the traces that START in records [lo, lo + TILE); a trace may
// overhang the tile by up to TILE records (CAP = 2 TILE), longer ones are spilled. Thread t holds
// records 2t, 2t+1 (+TILE for the overhang), so every u64 column is read with one 16-byte load
// per lane. LDS is 46 KB, i.e. three workgroups per CU: one loads while the others merge/join.
//
// Hash slot word (u32): bits 0..10 leader index + 1; bits 12..15 "seen >= 1" and 16..19
// "seen >= 2" for cs, cr, sr, ss (Span.isValid = no ">= 2" bit); bit 20 some fragment has a
// parentId, bit 21 some fragment has none. Fragments OR their bits into the slot, so validity and
// parent presence need no per-span counters.
// =============================================================================================
constexpr uint32_t kSlotIdx = 0x7FFu;
constexpr int kSlotA = 12;
constexpr int kSlotB = 16;
constexpr uint32_t kSlotP1 = 1u << 20;
constexpr uint32_t kSlotP0 = 1u << 21;

// own bits of a fragment and the "seen exactly once" core annotations it may promote to ">= 2"
__device__ __forceinline__ uint32_t frag_bits(uint32_t f, uint32_t* once) {
    uint32_t A = 0, B = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t k = (f >> (ZK_F_CS_SHIFT + 2 * c)) & 3u;
        A |= (k >= 1 ? 1u : 0u) << c;
        B |= (k >= 2 ? 1u : 0u) << c;
    }
    *once = A & ~B;
    return (A << kSlotA) | (B << kSlotB) | ((f & ZK_F_HAS_PARENT) ? kSlotP1 : kSlotP0);
}
__device__ __forceinline__ bool slot_valid(uint32_t w) { return ((w >> kSlotB) & 0xFu) == 0u; }

__device__ __forceinline__ uint64_t spread32(uint32_t x) {
    uint64_t v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
}

// two consecutive elements starting at i (i even, columns 16-byte aligned); zeros past `lim`
// Two consecutive elements starting at i (i even), RAW: elements at or past `lim` are garbage and
// every consumer masks by record index. Branch-free and unmasked on purpose: a conditional tail
// load, or a select right after the load, makes the compiler wait (vmcnt) for the load at once,
// which serialises the column loads and defeats the prefetch. Index i < lim reads the aligned pair
// at i (columns are 16-B / 8-B aligned, so the pair never crosses a page even when i + 1 == lim);
// i >= lim reads pair 0.
__device__ __forceinline__ void ld2_u64(const uint64_t* __restrict__ p, uint64_t i, uint64_t lim, uint64_t v[2]) {
    const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(p + (i < lim ? i : 0));
    v[0] = x.x;
    v[1] = x.y;
}
__device__ __forceinline__ void ld2_u32(const uint32_t* __restrict__ p, uint64_t i, uint64_t lim, uint32_t v[2]) {
    const uint2 x = *reinterpret_cast<const uint2*>(p + (i < lim ? i : 0));
    v[0] = x.x;
    v[1] = x.y;
}

// per-thread stat counters: 16-bit fields, two per u32 (a lane adds at most 2 per window, and a
// workgroup streams < 2^32 / 1024 records, so a field stays below 2^15)
struct StatPack16 {
    uint32_t w[7] = {0, 0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ void add(int s, bool c) { w[s >> 1] += (c ? 1u : 0u) << (16 * (s & 1)); }
};

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ __forceinline__ void flush_stats16(const StatPack16& sp, uint32_t* s_stat, unsigned long long* g_stats) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t v = wave_sum_u32((sp.w[i] >> (16 * h)) & 0xFFFFu);
            if (lane == 0 && v) atomicAdd(&s_stat[2 * i + h], v);
        }
    }
    __syncthreads();
    if (threadIdx.x < ST_N) {
        const uint32_t v = s_stat[threadIdx.x];
        unsigned long long* slot = g_stats + (uint64_t)(blockIdx.x % kStatShards) * ST_N;
        if (v) atomicAdd(&slot[threadIdx.x], (unsigned long long)v);
    }
}

struct Window {  // two consecutive records per thread
    uint64_t tid[2], sid[2], pid[2], first[2], last[2];
    uint32_t svc[2], flags[2];
    uint64_t prev;  // traceId of the record before this wave's first record
};

__device__ __forceinline__ void load_window(const JoinArgs& a, uint64_t ws, Window& w) {
    const uint64_t n = a.c.n;
    const uint64_t i = ws + 2 * threadIdx.x;
    ld2_u64(a.c.trace_id, i, n, w.tid);
    ld2_u64(a.c.span_id, i, n, w.sid);
    ld2_u64(a.c.parent_id, i, n, w.pid);
    ld2_u64((const uint64_t*)a.c.first_ts, i, n, w.first);
    ld2_u64((const uint64_t*)a.c.last_ts, i, n, w.last);
    ld2_u32(a.c.service_id, i, n, w.svc);
    ld2_u32(a.c.flags, i, n, w.flags);
    // traceId before the pair (only lane 0's is used); unconditional for the same reason as ld2
    w.prev = a.c.trace_id[(i > 0 && i - 1 < n) ? i - 1 : 0];
}

// =============================================================================================
// K1: persistent streaming span_join
//
// Workgroup w owns the traces that START in records [R0, R1) = [w, w+1) * per_wg. It streams
// through them in windows of TILE records (two per thread, 16-byte column loads): the trace
// boundaries of the window come from a ballot bitmask; the complete traces of the window are
// merged, validated and joined in LDS; the incomplete last trace starts the next window (its
// records are re-read, mostly from L2). The next window's columns are prefetched into registers
// right after its start is known, so HBM streams while the LDS phases run. A trace longer than a
// window goes to the spill kernel. Four workgroups per CU (24 KB LDS, <= 128 VGPRs).
//
// The per-record code is written branch-free wherever possible (pair stores into LDS, merges as
// unconditional atomics with neutral values, one insert loop and one probe loop covering both of
// a thread's records): divergent ifs cost exec-mask bookkeeping that dominated the instruction
// stream (profiles/pmc_r01_v5).
//
// Hash slot word (u32): bits 0..10 leader index + 1; bits 12..15 "seen >= 1" and 16..19
// "seen >= 2" for cs, cr, sr, ss (Span.isValid = no ">= 2" bit); bit 20 some fragment has a
// parentId, bit 21 some fragment has none.
// =============================================================================================
template <int TILE, int WG>
__global__ __launch_bounds__(WG, 4) void k_span_join_stream(JoinArgs a) {
    constexpr int H = 2 * TILE;
    constexpr int NWORD = TILE / 64;
    constexpr uint32_t DUMMY = H;  // hash slot written by lanes with nothing to merge
    static_assert(TILE == 2 * WG && TILE <= 2047 && H == 4 * WG, "two records per thread");
    __shared__ __attribute__((aligned(16))) uint64_t s_sid[TILE];
    __shared__ __attribute__((aligned(16))) long long s_first[TILE];
    __shared__ __attribute__((aligned(16))) long long s_last[TILE];
    __shared__ __attribute__((aligned(16))) uint64_t s_pid[TILE];
    __shared__ __attribute__((aligned(16))) uint32_t s_ht[H + 4];
    __shared__ __attribute__((aligned(16))) uint32_t s_svck[TILE];
    __shared__ __attribute__((aligned(16))) uint32_t s_seg2[WG];  // seg of records 2t | 2t+1 << 16
    __shared__ uint64_t s_mask[NWORD];
    __shared__ uint32_t s_stat[ST_N];
    __shared__ uint32_t s_wsum[WG / 64];
    __shared__ uint32_t s_hist[kMaxBuckets + 1];  // + a dummy bin for lanes without a link
    const uint16_t* s_seg = reinterpret_cast<const uint16_t*>(s_seg2);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int jj = 2 * tid;  // local index of this thread's first record
    const uint64_t n = a.c.n;
    const uint64_t R0 = (uint64_t)blockIdx.x * a.per_wg;
    if (R0 >= n) {
        if (tid == 0) a.link_count[blockIdx.x] = 0u;
        for (uint32_t x = tid; x < a.nb; x += WG) a.hist[(uint64_t)x * a.grid + blockIdx.x] = 0u;
        return;
    }
    const uint64_t R1 = (R0 + a.per_wg < n) ? R0 + a.per_wg : n;
    uint64_t* __restrict__ out = a.links + (uint64_t)blockIdx.x * a.link_stride;
    uint32_t nout = 0;  // links written by this workgroup (uniform)
    uint64_t nrec = 0;  // records aggregated (uniform)
    StatPack16 st;
    if (tid < ST_N) s_stat[tid] = 0u;
    if (tid < 4) s_ht[H + tid] = 0u;  // dummy slots (never cleared per window, only OR-ed with 0)
    for (uint32_t x = tid; x <= kMaxBuckets; x += WG) s_hist[x] = 0u;

    uint64_t ws = R0;    // window start (even)
    uint64_t seek = R0;  // first record that may start one of our traces
    Window cur, nxt;
    load_window(a, ws, cur);
    for (;;) {
        const int wn = (int)((n - ws) < (uint64_t)TILE ? (n - ws) : (uint64_t)TILE);
        // ---- 1. trace boundaries of the window -------------------------------------------------
        uint64_t wlo, whi;  // this wave's two mask words (uniform)
        {
            uint64_t prev = __shfl_up(cur.tid[1], 1);
            if (lane == 0) prev = (ws + jj > 0) ? cur.prev : ~cur.tid[0];
            const bool b0 = (jj < wn) && cur.tid[0] != prev;
            const bool b1 = (jj + 1 < wn) && cur.tid[1] != cur.tid[0];
            const uint64_t m0 = __ballot(b0), m1 = __ballot(b1);
            wlo = spread32((uint32_t)m0) | (spread32((uint32_t)m1) << 1);
            whi = spread32((uint32_t)(m0 >> 32)) | (spread32((uint32_t)(m1 >> 32)) << 1);
            if (lane == 0) {
                s_mask[2 * wave] = wlo;
                s_mask[2 * wave + 1] = whi;
            }
        }
        __syncthreads();
        // ---- 2. which records are ours, where the next window starts (uniform) ----------------
        const int lo_j = (int)(seek - ws);
        const int r1_j = (R1 - ws < (uint64_t)wn) ? (int)(R1 - ws) : wn;
        int start = -1, stop = -1, last_b = -1, cin = -1;  // cin: last boundary before this wave
#pragma unroll
        for (int w = 0; w < NWORD; ++w) {
            const uint64_t x = s_mask[w];
            if (!x) continue;
            const int base = 64 * w;
            last_b = base + 63 - (int)__clzll((long long)x);
            if (w < 2 * wave) cin = last_b;
            if (start < 0 && base + 63 >= lo_j) {
                const uint64_t y = lo_j > base ? (x & (~0ull << (lo_j - base))) : x;
                if (y) start = base + (int)__ffsll((unsigned long long)y) - 1;
            }
            if (stop < 0 && base + 63 >= r1_j) {
                const uint64_t y = r1_j > base ? (x & (~0ull << (r1_j - base))) : x;
                if (y) stop = base + (int)__ffsll((unsigned long long)y) - 1;
            }
        }
        const bool at_end = ws + (uint64_t)wn >= n;
        int m;  // records [start, m) are processed in this window
        bool done = false;
        uint64_t next_seek = 0;
        if (start < 0 || (stop >= 0 && stop <= start)) {
            done = (start >= 0) || at_end || ws + (uint64_t)TILE >= R1;  // nothing of ours here
            next_seek = ws + (uint64_t)TILE;
            start = m = 0;
        } else if (stop >= 0) {
            m = stop;  // traces starting at/after R1 belong to the next workgroup
            done = true;
        } else if (at_end) {
            m = wn;
            done = true;
        } else if (last_b > start) {
            m = last_b;  // the last trace may continue past the window: it starts the next one
            next_seek = ws + (uint64_t)last_b;
        } else if (start > 1) {
            m = start;  // a single long trace starts mid-window: give it a window of its own
            next_seek = ws + (uint64_t)start;
        } else {
            // the trace at `start` is longer than a window: spill it, then seek past it
            if (tid == 0) {
                const unsigned int idx = atomicAdd(a.spill_count, 1u);
                if (idx < a.spill_cap) a.spill_list[idx] = ws + (uint64_t)start;
                atomicAdd(&a.stats[ST_SPILLED], 1ull);
            }
            m = start;
            next_seek = ws + (uint64_t)TILE;
        }
        if (!done && next_seek >= R1) done = true;
        const uint64_t next_ws = next_seek & ~1ull;
        load_window(a, done ? ws : next_ws, nxt);  // in flight during the LDS phases (unconditional: see ld2)
        nrec += (uint64_t)(m - start);

        // ---- 3. segment ids (from this wave's mask words) and LDS staging ---------------------
        bool in[2], rerr[2];
        int seg[2];
        uint32_t svck[2], bits[2], once[2];
        {
            const uint64_t myword = lane < 32 ? wlo : whi;
            int pre = cin;
            if (lane >= 32 && wlo) pre = 64 * (2 * wave) + 63 - (int)__clzll((long long)wlo);
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int j = jj + e;
                const uint64_t b = myword & ((2ull << (j & 63)) - 1ull);
                seg[e] = b ? (j & ~63) + 63 - (int)__clzll((long long)b) : pre;
                in[e] = j >= start && j < m;
                rerr[e] = false;
                svck[e] = svc_key(cur.flags[e], cur.svc[e], a.S, &rerr[e]);
                bits[e] = frag_bits(cur.flags[e], &once[e]);
            }
            // pair stores (records outside [start, m) are written too: nothing ever reads them)
            const bool ha0 = (cur.flags[0] & ZK_F_HAS_ANNOTATIONS) != 0;
            const bool ha1 = (cur.flags[1] & ZK_F_HAS_ANNOTATIONS) != 0;
            *reinterpret_cast<ulonglong2*>(&s_sid[jj]) = make_ulonglong2(cur.sid[0], cur.sid[1]);
            *reinterpret_cast<longlong2*>(&s_first[jj]) =
                make_longlong2(ha0 ? (long long)cur.first[0] : LLONG_MAX, ha1 ? (long long)cur.first[1] : LLONG_MAX);
            *reinterpret_cast<longlong2*>(&s_last[jj]) =
                make_longlong2(ha0 ? (long long)cur.last[0] : LLONG_MIN, ha1 ? (long long)cur.last[1] : LLONG_MIN);
            *reinterpret_cast<ulonglong2*>(&s_pid[jj]) =
                make_ulonglong2((cur.flags[0] & ZK_F_HAS_PARENT) ? cur.pid[0] : ~0ull,
                                (cur.flags[1] & ZK_F_HAS_PARENT) ? cur.pid[1] : ~0ull);
            *reinterpret_cast<uint2*>(&s_svck[jj]) = make_uint2(svck[0], svck[1]);
            s_seg2[tid] = (uint32_t)(seg[0] & 0xFFFF) | ((uint32_t)(seg[1] & 0xFFFF) << 16);
            *reinterpret_cast<uint4*>(&s_ht[4 * tid]) = make_uint4(0u, 0u, 0u, 0u);
        }
        __syncthreads();

        // ---- 4. groupBy((id, traceId)): one insert loop for both records ------------------------
        int lead[2] = {-1, -1};
        uint32_t slot_of[2] = {DUMMY, DUMMY};
        {
            int e = in[0] ? 0 : (in[1] ? 1 : 2);
            uint64_t key = e == 0 ? cur.sid[0] : cur.sid[1];
            uint32_t sg = (uint32_t)(e == 0 ? seg[0] : seg[1]);
            uint32_t mine = (uint32_t)(jj + (e == 0 ? 0 : 1) + 1) | (e == 0 ? bits[0] : bits[1]);
            uint32_t slot = slot_hash(key, sg) & (H - 1);
            while (e < 2) {
                const uint32_t old = atomicCAS(&s_ht[slot], 0u, mine);
                int found = -1;
                if (old == 0u) {
                    found = jj + e;
                } else {
                    const int o = (int)(old & kSlotIdx) - 1;
                    if (s_sid[o] == key && s_seg[o] == sg) found = o;
                }
                if (found >= 0) {
                    if (e == 0) {
                        lead[0] = found;
                        slot_of[0] = slot;
                    } else {
                        lead[1] = found;
                        slot_of[1] = slot;
                    }
                    e = (e == 0 && in[1]) ? 1 : 2;
                    key = cur.sid[1];
                    sg = (uint32_t)seg[1];
                    mine = (uint32_t)(jj + 2) | bits[1];
                    slot = slot_hash(key, sg) & (H - 1);
                } else {
                    slot = (slot + 1) & (H - 1);
                }
            }
        }
        __syncthreads();

        // ---- 5. reduce(mergeSpan): unconditional atomics, neutral for leaders / other records --
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const bool nl = lead[e] >= 0 && lead[e] != jj + e;  // fragment to fold into its leader
            const int tgt = nl ? lead[e] : jj + e;
            const uint32_t f = cur.flags[e];
            const bool ha = nl && (f & ZK_F_HAS_ANNOTATIONS);
            atomicMin(&s_first[tgt], ha ? (long long)cur.first[e] : LLONG_MAX);
            atomicMax(&s_last[tgt], ha ? (long long)cur.last[e] : LLONG_MIN);
            atomicMin(&s_svck[tgt], nl ? svck[e] : kSvcNone);
            atomicMin((unsigned long long*)&s_pid[tgt],
                      (unsigned long long)((nl && (f & ZK_F_HAS_PARENT)) ? cur.pid[e] : ~0ull));
            // lanes with nothing to fold OR zero into a slot of their own (no same-address pile-up)
            const uint32_t hs = nl ? slot_of[e] : (in[e] ? slot_of[e] : (uint32_t)((jj + e) & (H - 1)));
            const uint32_t old = atomicOr(&s_ht[hs], nl ? bits[e] : 0u);
            const uint32_t promote = nl ? (once[e] & (old >> kSlotA) & 0xFu) : 0u;  // second occurrence
            atomicOr(&s_ht[hs], promote << kSlotB);
        }
        __syncthreads();

        // ---- 6. filter(isValid), join on (parentId, traceId), (cell, duration) links ----------
        uint32_t w[2], sL[2];
        uint64_t pL[2];
        bool leader[2], child[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int L = in[e] ? lead[e] : jj + e;
            w[e] = s_ht[slot_of[e]];
            sL[e] = s_svck[L];
            pL[e] = s_pid[L];
            const uint32_t f = cur.flags[e];
            bool amb = (f & ZK_F_HAS_PARENT) ? (cur.pid[e] != pL[e]) : ((w[e] & kSlotP1) != 0u);
            const uint32_t sk = svck[e];
            amb = amb || (sk != kSvcNone && (sk >> kSvcKindShift) == (sL[e] >> kSvcKindShift) && sk != sL[e]);
            leader[e] = in[e] && lead[e] == jj + e;
            const bool valid = slot_valid(w[e]);
            child[e] = leader[e] && valid && (w[e] & kSlotP1);
            st.add(ST_AMBIGUOUS, in[e] && amb);
            st.add(ST_SVC_RANGE, in[e] && rerr[e]);
            st.add(ST_MERGED, leader[e]);
            st.add(ST_VALID, leader[e] && valid);
            st.add(ST_INVALID, leader[e] && !valid);
            st.add(ST_CHILD, child[e]);
        }
        // parent probes: one loop for both records
        uint32_t pw[2] = {0u, 0u};
        {
            int e = child[0] ? 0 : (child[1] ? 1 : 2);
            uint64_t key = e == 0 ? pL[0] : pL[1];
            uint32_t sg = (uint32_t)(e == 0 ? seg[0] : seg[1]);
            uint32_t slot = slot_hash(key, sg) & (H - 1);
            while (e < 2) {
                const uint32_t o = s_ht[slot];
                bool stop_e = o == 0u;
                if (!stop_e) {
                    const int oi = (int)(o & kSlotIdx) - 1;
                    if (s_sid[oi] == key && s_seg[oi] == sg) {
                        stop_e = true;
                        if (e == 0)
                            pw[0] = o;
                        else
                            pw[1] = o;
                    }
                }
                if (stop_e) {
                    e = (e == 0 && child[1]) ? 1 : 2;
                    key = pL[1];
                    sg = (uint32_t)seg[1];
                    slot = slot_hash(key, sg) & (H - 1);
                } else {
                    slot = (slot + 1) & (H - 1);
                }
            }
        }
        uint64_t link[2];
        uint32_t nl = 0;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int j = jj + e;
            const bool pok = child[e] && pw[e] != 0u && slot_valid(pw[e]);
            const uint32_t sp = s_svck[pok ? (int)(pw[e] & kSlotIdx) - 1 : j];
            const bool nosvc = pok && (sp == kSvcNone || sL[e] == kSvcNone);
            const uint64_t d = (uint64_t)s_last[j] - (uint64_t)s_first[j];
            const bool dbad = pok && !nosvc && d >= kMaxDuration;
            const bool has = pok && !nosvc && !dbad;
            const uint64_t cell = (uint64_t)(sp & kSvcIdMask) * a.S + (sL[e] & kSvcIdMask);
            link[e] = has ? ((cell << 40) | d) : ~0ull;
            nl += has ? 1u : 0u;
            st.add(ST_MISSING_PARENT, child[e] && !pok);
            st.add(ST_JOINED, pok);
            st.add(ST_NO_SERVICE, nosvc);
            st.add(ST_DUR_RANGE, dbad);
            // lanes without a link add 0 to a bin of their own (no same-address pile-up)
            atomicAdd(&s_hist[(has && a.nb) ? (uint32_t)(cell >> a.cb_shift) : (uint32_t)(j & (kMaxBuckets - 1))],
                      has ? 1u : 0u);
        }
        // ---- 7. append the window's links to this workgroup's list -----------------------------
        uint32_t incl = nl;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = __shfl_up(incl, off);
            if (lane >= off) incl += o;
        }
        if (lane == 63) s_wsum[wave] = incl;
        __syncthreads();
        uint32_t base = 0, total = 0;
#pragma unroll
        for (int w2 = 0; w2 < WG / 64; ++w2) {
            const uint32_t v = s_wsum[w2];
            if (w2 < wave) base += v;
            total += v;
        }
        if (!a.ablate) {
            uint32_t pos = nout + base + incl - nl;
            if (link[0] != ~0ull) out[pos++] = link[0];
            if (link[1] != ~0ull) out[pos] = link[1];
            nout += total;
        }
        if (done) break;
        ws = next_ws;
        seek = next_seek;
        cur = nxt;
        __syncthreads();  // s_wsum / s_mask reuse
    }
    if (tid == 0) {
        a.link_count[blockIdx.x] = nout;
        atomicAdd(&a.stats[(uint64_t)(blockIdx.x % kStatShards) * ST_N + ST_RECORDS], (unsigned long long)nrec);
    }
    flush_stats16(st, s_stat, a.stats);  // its barrier also publishes s_hist
    for (uint32_t x = tid; x < a.nb; x += WG)
        a.hist[(uint64_t)x * a.grid + blockIdx.x] = a.ablate ? 0u : s_hist[x];
}

// =============================================================================================
// Spill kernel: one trace longer than a tile, in per-workgroup global scratch.
// Every scratch access is an agent-scope atomic or an sc1 (L1-bypassing) load/store, so the
// merge never reads a stale L1 line left by this workgroup's previous trace.
// =============================================================================================
struct SpillScratch {
    uint64_t* sid;
    long long* first;
    long long* last;
    uint64_t* cntA;  // cs | cr << 21 | sr << 42
    uint64_t* cntB;  // ss | npar << 21
    uint64_t* pid;
    uint32_t* svck;
    uint32_t* ht;
};

__host__ __device__ inline uint64_t pow2ceil(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

__host__ __device__ inline uint64_t spill_ht_slots(uint32_t max_trace) { return pow2ceil(2ull * max_trace); }

__host__ __device__ inline SpillScratch spill_carve(uint8_t* base, uint32_t L) {
    SpillScratch s;
    uint8_t* p = base;
    s.sid = (uint64_t*)p;
    p += 8ull * L;
    s.first = (long long*)p;
    p += 8ull * L;
    s.last = (long long*)p;
    p += 8ull * L;
    s.cntA = (uint64_t*)p;
    p += 8ull * L;
    s.cntB = (uint64_t*)p;
    p += 8ull * L;
    s.pid = (uint64_t*)p;
    p += 8ull * L;
    s.svck = (uint32_t*)p;
    p += 4ull * L + 4ull * (L & 1);
    s.ht = (uint32_t*)p;
    return s;
}

template <class T>
__device__ __forceinline__ T ld_sc(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_sc(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void spill_counts(uint32_t f, uint64_t* A, uint64_t* B) {
    *A = (uint64_t)((f >> ZK_F_CS_SHIFT) & 3u) | ((uint64_t)((f >> ZK_F_CR_SHIFT) & 3u) << 21) |
         ((uint64_t)((f >> ZK_F_SR_SHIFT) & 3u) << 42);
    *B = (uint64_t)((f >> ZK_F_SS_SHIFT) & 3u) | ((uint64_t)(f & ZK_F_HAS_PARENT) << 21);
}
__device__ __forceinline__ bool spill_valid(uint64_t A, uint64_t B) {
    constexpr uint64_t F = (1ull << 21) - 1;
    return (A & F) <= 1 && ((A >> 21) & F) <= 1 && ((A >> 42) & F) <= 1 && (B & F) <= 1;
}

__global__ __launch_bounds__(kSpillWG) void k_span_join_spill(JoinArgs a) {
    __shared__ unsigned long long s_end;
    __shared__ uint32_t s_stat[ST_N];
    const uint32_t total = min(*a.spill_count, (unsigned int)a.spill_cap);
    const uint64_t n = a.c.n;
    const uint64_t* __restrict__ tr = a.c.trace_id;
    uint8_t* base = a.spill_scratch + (uint64_t)blockIdx.x * a.spill_scratch_stride;
    StatPack st;
    if (threadIdx.x < ST_N) s_stat[threadIdx.x] = 0u;
    for (uint32_t e = blockIdx.x; e < total; e += gridDim.x) {
        const uint64_t s = a.spill_list[e];
        const uint64_t t0 = tr[s];
        if (threadIdx.x == 0) s_end = ~0ull;
        __syncthreads();
        // trace extent: first index after s whose traceId differs (clustered input)
        for (uint64_t b0 = s + 1;; b0 += kSpillWG) {
            const uint64_t i = b0 + threadIdx.x;
            if (i >= n || tr[i] != t0) atomicMin(&s_end, (unsigned long long)i);
            __syncthreads();
            const uint64_t e_now = s_end;
            __syncthreads();
            if (e_now != ~0ull || b0 - s > (uint64_t)a.max_trace) break;
        }
        const uint64_t end = s_end;
        __syncthreads();
        if (end == ~0ull || end - s > (uint64_t)a.max_trace) {
            if (threadIdx.x == 0) atomicAdd(&a.stats[ST_TOO_LARGE], 1ull);
            continue;
        }
        const uint32_t L = (uint32_t)(end - s);
        const uint32_t H = (uint32_t)pow2ceil(2ull * L);
        const SpillScratch sc = spill_carve(base, a.max_trace);
        for (uint32_t j = threadIdx.x; j < L; j += kSpillWG) {
            const uint64_t gi = s + j;
            const uint32_t f = a.c.flags[gi];
            const bool ha = (f & ZK_F_HAS_ANNOTATIONS) != 0;
            bool rerr = false;
            uint64_t A, B;
            spill_counts(f, &A, &B);
            st_sc(&sc.sid[j], a.c.span_id[gi]);
            st_sc(&sc.first[j], ha ? (long long)a.c.first_ts[gi] : LLONG_MAX);
            st_sc(&sc.last[j], ha ? (long long)a.c.last_ts[gi] : LLONG_MIN);
            st_sc(&sc.cntA[j], A);
            st_sc(&sc.cntB[j], B);
            st_sc(&sc.pid[j], (uint64_t)((f & ZK_F_HAS_PARENT) ? a.c.parent_id[gi] : ~0ull));
            st_sc(&sc.svck[j], svc_key(f, a.c.service_id[gi], a.S, &rerr));
            if (rerr) st.inc(ST_SVC_RANGE);
        }
        for (uint32_t x = threadIdx.x; x < H; x += kSpillWG) st_sc(&sc.ht[x], 0u);
        __syncthreads();
        // insert
        for (uint32_t j = threadIdx.x; j < L; j += kSpillWG) {
            const uint64_t sid = a.c.span_id[s + j];
            uint32_t slot = slot_hash(sid, 0) & (H - 1);
            for (;;) {
                const uint32_t old = atomicCAS(&sc.ht[slot], 0u, j + 1);
                if (old == 0u) break;
                if (ld_sc(&sc.sid[old - 1]) == sid) break;
                slot = (slot + 1) & (H - 1);
            }
        }
        __syncthreads();
        // merge non-leaders into leaders
        for (uint32_t j = threadIdx.x; j < L; j += kSpillWG) {
            const uint64_t gi = s + j;
            const uint64_t sid = a.c.span_id[gi];
            uint32_t slot = slot_hash(sid, 0) & (H - 1);
            uint32_t Ld;
            for (;;) {
                const uint32_t o = ld_sc(&sc.ht[slot]);
                if (ld_sc(&sc.sid[o - 1]) == sid) {
                    Ld = o - 1;
                    break;
                }
                slot = (slot + 1) & (H - 1);
            }
            if (Ld != j) {
                const uint32_t f = a.c.flags[gi];
                if (f & ZK_F_HAS_ANNOTATIONS) {
                    atomicMin(&sc.first[Ld], (long long)a.c.first_ts[gi]);
                    atomicMax(&sc.last[Ld], (long long)a.c.last_ts[gi]);
                }
                uint64_t A, B;
                spill_counts(f, &A, &B);
                atomicAdd((unsigned long long*)&sc.cntA[Ld], (unsigned long long)A);
                atomicAdd((unsigned long long*)&sc.cntB[Ld], (unsigned long long)B);
                bool rerr = false;
                const uint32_t sk = svc_key(f, a.c.service_id[gi], a.S, &rerr);
                if (sk != kSvcNone) atomicMin(&sc.svck[Ld], sk);
                if (f & ZK_F_HAS_PARENT) atomicMin((unsigned long long*)&sc.pid[Ld], (unsigned long long)a.c.parent_id[gi]);
            }
        }
        __syncthreads();
        // validate, join, emit
        for (uint32_t j = threadIdx.x; j < L; j += kSpillWG) {
            const uint64_t gi = s + j;
            const uint64_t sid = a.c.span_id[gi];
            const uint32_t f = a.c.flags[gi];
            uint32_t slot = slot_hash(sid, 0) & (H - 1);
            uint32_t Ld;
            for (;;) {
                const uint32_t o = ld_sc(&sc.ht[slot]);
                if (ld_sc(&sc.sid[o - 1]) == sid) {
                    Ld = o - 1;
                    break;
                }
                slot = (slot + 1) & (H - 1);
            }
            const uint64_t A = ld_sc(&sc.cntA[Ld]), B = ld_sc(&sc.cntB[Ld]);
            const uint32_t npar = (uint32_t)(B >> 21);
            const uint32_t sL = ld_sc(&sc.svck[Ld]);
            const uint64_t pL = ld_sc(&sc.pid[Ld]);
            bool rerr = false;
            const uint32_t sk = svc_key(f, a.c.service_id[gi], a.S, &rerr);
            bool amb = (f & ZK_F_HAS_PARENT) ? (a.c.parent_id[gi] != pL) : (npar > 0);
            if (sk != kSvcNone && (sk >> kSvcKindShift) == (sL >> kSvcKindShift) && sk != sL) amb = true;
            if (amb) st.inc(ST_AMBIGUOUS);
            if (Ld != j) continue;
            st.inc(ST_MERGED);
            const bool valid = spill_valid(A, B);
            st.inc(valid ? ST_VALID : ST_INVALID);
            if (!(valid && npar > 0)) continue;
            st.inc(ST_CHILD);
            uint32_t ps = slot_hash(pL, 0) & (H - 1);
            int64_t P = -1;
            for (;;) {
                const uint32_t o = ld_sc(&sc.ht[ps]);
                if (o == 0u) break;
                if (ld_sc(&sc.sid[o - 1]) == pL) {
                    P = o - 1;
                    break;
                }
                ps = (ps + 1) & (H - 1);
            }
            if (P >= 0 && spill_valid(ld_sc(&sc.cntA[P]), ld_sc(&sc.cntB[P]))) {
                st.inc(ST_JOINED);
                const uint32_t spv = ld_sc(&sc.svck[P]);
                if (spv == kSvcNone || sL == kSvcNone) {
                    st.inc(ST_NO_SERVICE);
                } else {
                    const uint64_t d = (uint64_t)(ld_sc(&sc.last[Ld]) - ld_sc(&sc.first[Ld]));
                    if (d >= kMaxDuration)
                        st.inc(ST_DUR_RANGE);
                    else
                        emit_link(a.table, (spv & kSvcIdMask) * a.S + (sL & kSvcIdMask), d);
                }
            } else {
                st.inc(ST_MISSING_PARENT);
            }
        }
        if (threadIdx.x == 0) atomicAdd(&a.stats[ST_RECORDS], (unsigned long long)L);
        // flush per trace so the per-thread 16-bit fields never overflow
        flush_stats(st, s_stat, a.stats);
        st = StatPack();
        __syncthreads();
        if (threadIdx.x < ST_N) s_stat[threadIdx.x] = 0u;
        __syncthreads();
    }
}

// tile geometry of the shipped K1
constexpr int kTileWG = 256;
constexpr int kTile = 2 * kTileWG;

}  // namespace

uint64_t spill_scratch_bytes_per_wg(uint32_t max_trace) {
    const uint64_t L = max_trace;
    uint64_t b = 8ull * L * 6 + 4ull * L + 4ull * (L & 1) + 4ull * spill_ht_slots(max_trace);
    return (b + 255) & ~255ull;
}

hipError_t launch_join(const JoinArgs& a, hipStream_t s) {
    if (a.c.n == 0) return hipSuccess;
    hipLaunchKernelGGL((k_span_join_stream<kTile, kTileWG>), dim3((unsigned)a.grid), dim3(kTileWG), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_spill(const JoinArgs& a, uint32_t spill_wgs, hipStream_t s) {
    if (a.c.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_span_join_spill, dim3(spill_wgs), dim3(kSpillWG), 0, s, a);
    return hipGetLastError();
}

uint64_t join_tile_records() { return kTile; }

void join_geometry(uint64_t n, uint32_t cus, uint32_t* grid, uint64_t* per_wg, uint64_t* link_stride) {
    const uint64_t windows = (n + kTile - 1) / kTile;
    uint64_t g = (uint64_t)cus * 4;  // four resident workgroups per CU (<= 128 VGPRs, 23 KB LDS)
    if (g > windows) g = windows ? windows : 1;
    const uint64_t per = ((n + g - 1) / g + kTile - 1) / kTile * kTile;
    *grid = (uint32_t)g;
    *per_wg = per ? per : kTile;
    *link_stride = *per_wg + kTile;  // a workgroup's last trace may overhang its range by < TILE
}

}  // namespace zk
