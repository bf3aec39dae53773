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
#include "zk_launch.h"
#include "zk_sketch_internal.h"

#ifndef ZK_HASH_FACTOR
#define ZK_HASH_FACTOR 8
#endif
#ifndef ZK_K1_WGS_PER_CU
#define ZK_K1_WGS_PER_CU 4  // resident K1 workgroups per CU (one wave per SIMD each)
#endif
namespace zk {
namespace {

constexpr int kSpillWG = 256;

// ---- diagnostic phase stamps (separate build with -DZK_STAMPS; never in the product .so) -------
#ifdef ZK_STAMPS
__device__ unsigned long long g_zk_stamps[16];
__device__ __forceinline__ unsigned long long zk_memtime() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define ZK_STAMP_DECL                                 \
    unsigned long long zk_t_prev = zk_memtime();      \
    unsigned long long zk_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#define ZK_STAMP(k)                                   \
    do {                                              \
        const unsigned long long zk_t = zk_memtime(); \
        zk_acc[k] += zk_t - zk_t_prev;                \
        zk_t_prev = zk_t;                             \
    } while (0)
#define ZK_STAMP_FLUSH()                                                              \
    do {                                                                              \
        if ((threadIdx.x & 63) == 0)                                                  \
            for (int q = 0; q < 9; ++q) atomicAdd(&g_zk_stamps[q], zk_acc[q]);        \
    } while (0)
#else
#define ZK_STAMP_DECL
#define ZK_STAMP(k)
#define ZK_STAMP_FLUSH()
#endif
// a workgroup barrier that ends phase k: the stamps build books the wait itself to slot 8
#define ZK_PHASE_SYNC(k) \
    do {                 \
        ZK_STAMP(k);     \
        __syncthreads(); \
        ZK_STAMP(8);     \
    } while (0)

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

// packed per-thread stat counters of K1: 4 x 16-bit fields per u64 (a thread adds <= 2 per stat per
// window; folded every kFoldWindows windows, so a wave sum of 64 lanes stays below 2^16)
struct StatPack {
    uint64_t w[4] = {0, 0, 0, 0};
    __device__ __forceinline__ void inc(int s, uint32_t v = 1) { w[s >> 2] += (uint64_t)v << (16 * (s & 3)); }
};
// the spill kernel's counters: one u64 per stat (a spilled trace can hold up to 2^20 records, more
// than 16-bit wave sums can count)
struct StatWide {
    uint64_t w[ST_N] = {};
    __device__ __forceinline__ void inc(int s, uint32_t v = 1) { w[s] += v; }
};

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// spill kernel: per-thread counts -> per-wave sums -> u64 LDS totals -> one add per stat into a
// sharded global slot (the stats array holds kStatShards copies, summed by the host, so 1e5 tiles
// never hammer one address)
__device__ __forceinline__ void flush_stats(StatWide& sp, unsigned long long* s_stat, unsigned long long* g_stats) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < ST_N; ++i) {
        const uint64_t v = wave_sum_u64(sp.w[i]);
        if (lane == 0 && v) atomicAdd(&s_stat[i], (unsigned long long)v);
    }
    __syncthreads();
    if (threadIdx.x < ST_N) {
        const unsigned long long v = s_stat[threadIdx.x];
        unsigned long long* slot = g_stats + (uint64_t)(blockIdx.x % kStatShards) * ST_N;
        if (v) atomicAdd(&slot[threadIdx.x], v);
    }
}

// =============================================================================================
// K1 LDS hash
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
// bits 22..30 of the slot word: the leader's trace segment (< 512)
constexpr int kSlotSegShift = 22;

// own bits of a fragment and the "seen exactly once" core annotations it may promote to ">= 2":
// the four 2-bit counts of cs|cr|sr|ss (bits 8..15) give ">= 1" (either bit) and ">= 2" (the high
// bit) per field, compressed from every other bit to four contiguous bits -- ten bit operations
// instead of a compare and select per field and threshold
__device__ __forceinline__ uint32_t frag_bits(uint32_t f, uint32_t* once) {
    static_assert(ZK_F_SR_SHIFT == ZK_F_CS_SHIFT + 4 && ZK_F_CR_SHIFT == ZK_F_CS_SHIFT + 2 &&
                      ZK_F_SS_SHIFT == ZK_F_CS_SHIFT + 6, "cs, cr, sr, ss counts in consecutive 2-bit fields");
    const uint32_t f8 = (f >> ZK_F_CS_SHIFT) & 0xFFu;
    const uint32_t hi = (f8 >> 1) & 0x55u;
    uint32_t y = (f8 & 0x55u) | hi | (hi << 8);  // ">= 1" spread in the low byte, ">= 2" in the high byte
    y = (y | (y >> 1)) & 0x3333u;
    y = (y | (y >> 2)) & 0x0F0Fu;
    const uint32_t A = y & 0xFu, B = y >> 8;
    *once = A & ~B;
    return (A << kSlotA) | (B << kSlotB) | ((f & ZK_F_HAS_PARENT) ? kSlotP1 : kSlotP0);
}
__device__ __forceinline__ bool slot_valid(uint32_t w) { return ((w >> kSlotB) & 0xFu) == 0u; }

// Two consecutive elements starting at i (i even), RAW: elements at or past `lim` are garbage and
// every consumer masks by record index. Branch-free and unmasked on purpose: a conditional tail
// load, or a select right after the load, makes the compiler wait (vmcnt) for the load at once,
// which serialises the column loads and defeats the prefetch. Index i < lim reads the aligned pair
// at i (columns are 16-B / 8-B aligned, so the pair never crosses a page even when i + 1 == lim);
// i >= lim reads pair 0.
// Diagnostic builds only (results wrong; profiles/r06/k1_sensitivity_ab.txt): ZK_K1_DIAG_HOT
// redirects every column load into the first 2^16 records (L2-resident: K1 with HBM reads taken
// out), ZK_K1_DIAG_NOFIRST drops the first_ts column (8 B / record fewer read), ZK_K1_DIAG_NOSTORE
// drops the link stores, ZK_K1_DIAG_TRASHONLY sends both stores of every lane to the trash slot.
// Each reports no links (K2/K3 then index nothing).
#ifdef ZK_K1_DIAG_HOT
#define ZK_HOTIDX(i) ((i) & 0xFFFFull)
#else
#define ZK_HOTIDX(i) (i)
#endif
#if defined(ZK_K1_DIAG_HOT) || defined(ZK_K1_DIAG_NOFIRST) || defined(ZK_K1_DIAG_NOSTORE) || defined(ZK_K1_DIAG_TRASHONLY)
#define ZK_K1_DIAG 1
#endif
__device__ __forceinline__ void ld2_u64(const uint64_t* __restrict__ p, uint64_t i, uint64_t lim, uint64_t v[2]) {
    const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(p + ZK_HOTIDX(i < lim ? i : 0));
    v[0] = x.x;
    v[1] = x.y;
}
__device__ __forceinline__ void ld2_u32(const uint32_t* __restrict__ p, uint64_t i, uint64_t lim, uint32_t v[2]) {
    const uint2 x = *reinterpret_cast<const uint2*>(p + ZK_HOTIDX(i < lim ? i : 0));
    v[0] = x.x;
    v[1] = x.y;
}

// K1 stat counters: the per-thread 16-bit pack (StatPack) is folded into the workgroup's u32 LDS
// totals every kFoldWindows windows (a lane adds <= 2 per stat per window, so a wave sum of 64
// lanes stays below 2^16), and the totals go to a sharded global slot once at the end.
constexpr int kFoldWindows = 256;

__device__ __forceinline__ void fold_stats(StatPack& sp, uint32_t* s_stat) {
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
        sp.w[i] = 0;
    }
}

__device__ __forceinline__ void publish_stats(const uint32_t* s_stat, unsigned long long* g_stats) {
    __syncthreads();
    if (threadIdx.x < ST_N) {
        const uint32_t v = s_stat[threadIdx.x];
        unsigned long long* slot = g_stats + (uint64_t)(blockIdx.x % kStatShards) * ST_N;
        if (v) atomicAdd(&slot[threadIdx.x], (unsigned long long)v);
    }
}

// ---- window boundary masks ---------------------------------------------------------------------
// A wave's 128 records (thread t holds records 2t, 2t+1) are described by two ballots: ev (bit t:
// record 2t starts a trace) and od (bit t: record 2t+1 does). Positions below are local (0..127).
__device__ __forceinline__ int first_ge(uint64_t ev, uint64_t od, int q) {  // first boundary >= q
    if (q < 0) q = 0;
    if (q >= 128) return -1;
    const int se = (q + 1) >> 1, so = q >> 1;  // 2t >= q <=> t >= se;  2t+1 >= q <=> t >= so
    const uint64_t me = se >= 64 ? 0ull : (ev & (~0ull << se));
    const uint64_t mo = od & (~0ull << so);
    const int pe = me ? 2 * (__ffsll((unsigned long long)me) - 1) : 256;
    const int po = mo ? 2 * (__ffsll((unsigned long long)mo) - 1) + 1 : 256;
    const int p = pe < po ? pe : po;
    return p < 256 ? p : -1;
}
__device__ __forceinline__ int last_of(uint64_t ev, uint64_t od) {  // last boundary, or -1
    const int pe = ev ? 2 * (63 - (int)__clzll((long long)ev)) : -1;
    const int po = od ? 2 * (63 - (int)__clzll((long long)od)) + 1 : -1;
    return pe > po ? pe : po;
}
// lane l-1's value (wave_shr:1 DPP, no LDS round trip); lane 0 gets garbage
__device__ __forceinline__ uint64_t lane_shr1(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x138, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x138, 0xF, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {  // set bits of m in lanes < this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

struct Window {  // two consecutive records per thread
    uint64_t tid[2], sid[2], pid[2], first[2], last[2];
    uint32_t svc[2], flags[2];
    uint64_t prev;  // traceId of the record before this wave's first record
};

// boundary ballots of a window starting at ws with wn records: ev bit t = record 2t starts a trace,
// od bit t = record 2t+1 does (this wave's lanes)
__device__ __forceinline__ void window_ballots(const Window& w, uint64_t ws, int wn, uint64_t* ev, uint64_t* od) {
    const int t = threadIdx.x, lane = t & 63;
    uint64_t prev = lane_shr1(w.tid[1]);
    if (lane == 0) prev = (ws + 2 * t > 0) ? w.prev : ~w.tid[0];
    const bool b0 = (2 * t < wn) && w.tid[0] != prev;
    const bool b1 = (2 * t + 1 < wn) && w.tid[1] != w.tid[0];
    *ev = __ballot(b0);
    *od = __ballot(b1);
}

// Column loads of a window, in three groups issued at different points of the loop (round 2,
// profiles/r02/ab_late.txt, ab_early_cols.txt): the traceIds (what the boundary phase needs) a
// whole window ahead; spanId, first/last and service right after the window before passed its
// merge barrier (phase 6 no longer reads them); parentId and flags at the top of the window's own
// iteration. 26 -> 6 registers of prefetch against loading everything a window ahead (120 -> 101
// VGPRs, K1 1.251 -> 1.227 -> 1.160 ms).
__device__ __forceinline__ void load_tid(const JoinArgs& a, uint64_t n, uint64_t ws, Window& w) {
    const uint64_t i = ws + 2 * threadIdx.x;
    ld2_u64(a.c.trace_id, i, n, w.tid);
    w.prev = a.c.trace_id[ZK_HOTIDX((i > 0 && i - 1 < n) ? i - 1 : 0)];
}
__device__ __forceinline__ void load_early(const JoinArgs& a, uint64_t n, uint64_t ws, Window& w) {
    const uint64_t i = ws + 2 * threadIdx.x;
    ld2_u64(a.c.span_id, i, n, w.sid);
#ifndef ZK_K1_DIAG_NOFIRST
    ld2_u64((const uint64_t*)a.c.first_ts, i, n, w.first);
#endif
    ld2_u64((const uint64_t*)a.c.last_ts, i, n, w.last);
#ifdef ZK_K1_DIAG_NOFIRST
    w.first[0] = w.last[0] - 5;
    w.first[1] = w.last[1] - 5;
#endif
    ld2_u32(a.c.service_id, i, n, w.svc);
}
template <bool JOIN>
__device__ __forceinline__ void load_late(const JoinArgs& a, uint64_t n, uint64_t ws, Window& w) {
    const uint64_t i = ws + 2 * threadIdx.x;
    if constexpr (JOIN) {
        ld2_u64(a.c.parent_id, i, n, w.pid);
    } else {  // sketch-only pass: parentId is not read (40 B per record)
        w.pid[0] = w.pid[1] = 0ull;
    }
    ld2_u32(a.c.flags, i, n, w.flags);
}

// =============================================================================================
// K1: persistent streaming span_join
//
// Workgroup w owns the traces that START in records [R0, R1) = [w, w+1) * per_wg. It streams
// through them in windows of TILE records (two per thread, 16-byte column loads): the trace
// boundaries of the window come from a ballot bitmask; the complete traces of the window are
// merged, validated and joined in LDS; the incomplete last trace starts the next window (its
// records are re-read, mostly from L2). The next window's columns are prefetched into registers,
// so HBM streams while the LDS phases run. A trace longer than a window goes to the spill kernel.
// Four workgroups per CU (<= 40 KB LDS, <= 128 VGPRs). Three barriers per window: boundaries,
// staging, merge; waves claim their slice of the link list with one LDS atomic (no append barrier),
// and hash slots are emptied one window later by their leaders.
//
// Hash slot word (u32): bits 0..10 leader index + 1; bits 12..15 "seen >= 1" and 16..19
// "seen >= 2" for cs, cr, sr, ss (Span.isValid = no ">= 2" bit); bit 20 some fragment has a
// parentId, bit 21 some fragment has none; bits 22..30 the leader's trace segment, so a probe
// compares the segment from the word it read and loads the occupant's spanId only on a match.
// =============================================================================================
// MODE bits: kModeJoin = the dependency path (parent join, links); kModeEmit = one sketch item
// per merged valid span with a service (zk_rt.hip). The product dependency pass is kModeJoin.
constexpr int kModeJoin = 1;
constexpr int kModeEmit = 2;
constexpr int kModeLinks = 4;  // with kModeJoin: a realtime link item beside every link (zk_rl)
template <int TILE, int WG, int MODE>
// launch bounds: minimum waves per SIMD = resident workgroups per CU x waves per workgroup / 4 SIMDs
__global__ __launch_bounds__(WG, ZK_K1_WGS_PER_CU * WG / 256) void k_span_join_stream(JoinArgs a) {
    constexpr int H = ZK_HASH_FACTOR * TILE;  // load <= 1/16 (distinct spans / slots): short probe chains, since a wave waits for its longest
    constexpr int NWORD = TILE / 64;
    static_assert(TILE == 2 * WG && TILE <= 512, "two records per thread; the segment field of the slot word is 9 bits");
    __shared__ __align__(16) uint64_t s_sid[TILE];
    __shared__ __align__(16) long long s_first[TILE];
    __shared__ __align__(16) long long s_last[TILE];
    __shared__ __align__(16) uint64_t s_pid[TILE];
    __shared__ __align__(16) uint32_t s_svck[TILE];
    __shared__ __align__(16) uint32_t s_ht[H];
    __shared__ __align__(16) uint64_t s_mask[NWORD];
    __shared__ uint32_t s_stat[ST_N];
    __shared__ uint64_t s_cursor;  // links (low 32) and sketch items (high 32) appended so far
    __shared__ uint32_t s_hist[kMaxBuckets];  // links per cell bucket (K2's scatter offsets)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // the group join's fallback: n on the device, ranges cut from it (per_wg bounds them)
    const uint64_t n = a.n_dev ? (uint64_t)*a.n_dev : a.c.n;
    uint64_t per = a.per_wg;
    if (a.n_dev) {
        const uint64_t q = ((n + a.grid - 1) / a.grid + TILE - 1) / TILE * TILE;
        if (q < per) per = q ? q : TILE;
    }
    const uint64_t R0 = (uint64_t)blockIdx.x * per;
    if (R0 >= n) {
        if (a.append) return;  // the lists and histogram keep what the group join wrote
        if (tid == 0) {
            a.link_count[blockIdx.x] = 0u;
            if (a.rt_count) a.rt_count[blockIdx.x] = 0u;
        }
        for (uint32_t x = tid; x < a.nb; x += WG) a.hist[(uint64_t)x * a.grid + blockIdx.x] = 0u;
        return;
    }
    const uint64_t R1 = (R0 + per < n) ? R0 + per : n;
    uint64_t* __restrict__ out = a.links + (uint64_t)blockIdx.x * a.link_stride;
    const uint64_t trash = a.link_stride - 1;  // never a real link slot (join_geometry)
    uint64_t* __restrict__ it_pay = a.rt_pay + (uint64_t)blockIdx.x * a.link_stride;
    uint32_t* __restrict__ it_svc = a.rt_svc + (uint64_t)blockIdx.x * a.link_stride;
    uint64_t nrec = 0;  // records aggregated (uniform)
    StatPack st;
    int fold_in = kFoldWindows;  // windows until the next stat fold (uniform)
    if (tid < ST_N) s_stat[tid] = 0u;
    if (tid == 0) s_cursor = a.append ? (uint64_t)a.link_count[blockIdx.x] : 0ull;
    for (uint32_t x = tid; x < a.nb; x += WG) s_hist[x] = a.append ? a.hist[(uint64_t)x * a.grid + blockIdx.x] : 0u;
    constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
    uint32_t r_clear[2] = {kNoSlot, kNoSlot};  // hash slots this thread's leaders of the last window hold

    Window cur, nxt;
    constexpr bool JOIN = (MODE & kModeJoin) != 0, EMIT = (MODE & kModeEmit) != 0, LINKS = (MODE & kModeLinks) != 0;
    static_assert(!LINKS || (JOIN && !EMIT), "link items ride on the join's links");
#pragma unroll
    for (int x = tid; x < H / 4; x += WG) reinterpret_cast<uint4*>(s_ht)[x] = make_uint4(0u, 0u, 0u, 0u);
    uint64_t m_ev, m_od;  // this wave's boundary ballots of the current window (uniform; phase 3 reuses them)
    ZK_STAMP_DECL
    uint64_t ws = R0;         // window start (even)
    // first record that may start one of our traces (skip: record 0's run is the held trace's,
    // decided on the device when the batch continues one, zk_cluster.hip k_carry_plan)
    const uint32_t skip0 = a.skip_dev ? *a.skip_dev : a.skip;
    uint64_t seek = R0 + (blockIdx.x == 0 ? skip0 : 0u);
    bool seek_start = false;  // seek is known to be a trace start (uniform)
    load_tid(a, n, ws, cur);
    load_early(a, n, ws, cur);
    // the first window's ballots; later windows' are taken at the end of the window before (below)
    window_ballots(cur, ws, (int)((n - ws) < (uint64_t)TILE ? (n - ws) : (uint64_t)TILE), &m_ev, &m_od);
    if (lane == 0) *reinterpret_cast<ulonglong2*>(&s_mask[2 * wave]) = make_ulonglong2(m_ev, m_od);
    for (;;) {
        load_late<JOIN>(a, n, ws, cur);
        const int wn = (int)((n - ws) < (uint64_t)TILE ? (n - ws) : (uint64_t)TILE);
        // ---- 1. trace boundaries of the window (ballots taken at the end of the window before) --
        ZK_PHASE_SYNC(0);
        // ---- 2. which records are ours, where the next window starts (uniform) ----------------
        const int lo_j = (int)(seek - ws);
        const int r1_j = (R1 - ws < (uint64_t)wn) ? (int)(R1 - ws) : wn;
        // lane w < NW holds wave w's masks: the first boundary >= lo_j (start), the first >= r1_j
        // (stop), the last of the window (last_b) and the last before this wave's records (prev_b)
        int start = -1, stop = -1, last_b = -1, prev_b = -1;  // wave-uniform (SGPRs)
        {
            constexpr int NW = WG / 64;
            uint64_t ev = 0ull, od = 0ull;
            if (lane < NW) {
                const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(&s_mask[2 * lane]);
                ev = x.x;
                od = x.y;
            }
            const int base = 128 * lane;
            // steady state: the window starts at the trace start `seek` that the window before
            // found, and the range end R1 is beyond it -- start = lo_j, stop = none, with no search
            // (the search would return exactly these: bit lo_j is set in the masks)
            const bool fast = seek_start && lo_j < wn && R1 - ws >= (uint64_t)wn;
            if (fast) {
                start = lo_j;
            } else {
                const int fs = lane < NW ? first_ge(ev, od, lo_j - base) : -1;
                const int ft = lane < NW ? first_ge(ev, od, r1_j - base) : -1;
                const uint64_t bs = __ballot(fs >= 0), bt = __ballot(ft >= 0);
                if (bs) {
                    const int w = __ffsll((unsigned long long)bs) - 1;
                    start = 128 * w + __builtin_amdgcn_readlane(fs, w);
                }
                if (bt) {
                    const int w = __ffsll((unsigned long long)bt) - 1;
                    stop = 128 * w + __builtin_amdgcn_readlane(ft, w);
                }
            }
            const int lb = last_of(ev, od);
            const uint64_t bl = __ballot(lb >= 0);
            if (bl) {
                const int w = 63 - (int)__clzll((long long)bl);
                last_b = 128 * w + __builtin_amdgcn_readlane(lb, w);
            }
            const uint64_t bp = bl & ((1ull << wave) - 1ull);
            if (bp) {
                const int w = 63 - (int)__clzll((long long)bp);
                prev_b = 128 * w + __builtin_amdgcn_readlane(lb, w);
            }
        }
        const bool at_end = ws + (uint64_t)wn >= n;
        int m;                  // records [start, m) are processed in this window
        bool done = false;
        uint64_t next_seek = 0;
        bool next_seek_start = false;  // next_seek is a trace start (uniform)
        if (start < 0 || (stop >= 0 && stop <= start)) {
            // no trace of ours starts in the rest of this window
            done = (start >= 0) || at_end || ws + (uint64_t)TILE >= R1;
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
            next_seek_start = true;
        } else if (start > 1) {
            m = start;  // a single long trace starts mid-window: give it a window of its own
            next_seek = ws + (uint64_t)start;
            next_seek_start = true;
        } else {
            // the trace at `start` is longer than a window: spill it, then seek past it
            if (tid == 0) {
                const unsigned int idx = atomicAdd(a.spill_count, 1u);
                if (idx < a.spill_cap)
                    a.spill_list[idx] = ws + (uint64_t)start;
                else
                    atomicAdd(&a.stats[ST_SPILL_OVERFLOW], 1ull);
                atomicAdd(&a.stats[ST_SPILLED], 1ull);
            }
            m = start;
            next_seek = ws + (uint64_t)TILE;
        }
        if (!done && next_seek >= R1) done = true;
        const uint64_t next_ws = next_seek & ~1ull;
        load_tid(a, n, done ? ws : next_ws, nxt);  // in flight during the LDS phases below (unconditional: see ld2)
        ZK_STAMP(1);
        nrec += (uint64_t)(m - start);
        uint64_t n_ev = 0, n_od = 0;  // the next window's ballots

        // the last window's leaders empty their hash slots (see phase 7)
#pragma unroll
        for (int e = 0; e < 2; ++e)
            if (r_clear[e] != kNoSlot) s_ht[r_clear[e]] = 0u;
        // ---- 3. segment ids and LDS staging ----------------------------------------------------
        // seg = index of the trace's first record in the window (the last boundary <= j), from the
        // wave's own ballots: record 2t+1 is its own segment start or shares 2t's. Staging stores
        // are unconditional 16-B pairs (entries outside [start, m) are never read).
        int r_seg[2];
        uint32_t r_svck[2];
        bool r_rerr[2];
        {
            const int j0 = 2 * tid;
            // last boundary <= j0 among this wave's records, else the one before the wave (it exists
            // when j0 >= start, since start is a boundary)
            const int p = last_of(m_ev & ((2ull << lane) - 1ull), m_od & ((1ull << lane) - 1ull));
            const bool b1 = (m_od >> lane) & 1ull;
            int seg0 = -1;
            if (j0 >= start && j0 < m) seg0 = p >= 0 ? 128 * wave + p : prev_b;
            r_seg[0] = seg0;
            r_seg[1] = (j0 + 1 >= start && j0 + 1 < m) ? (b1 ? j0 + 1 : seg0) : -1;
            uint64_t v_first[2], v_last[2], v_pid[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                r_rerr[e] = false;
                r_svck[e] = svc_key(cur.flags[e], cur.svc[e], a.S, &r_rerr[e]);
                const uint32_t f = cur.flags[e];
                const bool ha = (f & ZK_F_HAS_ANNOTATIONS) != 0;
                v_first[e] = ha ? cur.first[e] : (uint64_t)LLONG_MAX;
                v_last[e] = ha ? cur.last[e] : (uint64_t)LLONG_MIN;
                v_pid[e] = (f & ZK_F_HAS_PARENT) ? cur.pid[e] : ~0ull;
            }
            *reinterpret_cast<ulonglong2*>(&s_sid[j0]) = make_ulonglong2(cur.sid[0], cur.sid[1]);
            *reinterpret_cast<ulonglong2*>(&s_first[j0]) = make_ulonglong2(v_first[0], v_first[1]);
            *reinterpret_cast<ulonglong2*>(&s_last[j0]) = make_ulonglong2(v_last[0], v_last[1]);
            *reinterpret_cast<ulonglong2*>(&s_pid[j0]) = make_ulonglong2(v_pid[0], v_pid[1]);
            *reinterpret_cast<uint2*>(&s_svck[j0]) = make_uint2(r_svck[0], r_svck[1]);
        }
        ZK_PHASE_SYNC(2);  // (the hash table is empty here: cleared once, then by its leaders)

        // ---- 4. groupBy((id, traceId)): the first fragment to claim a slot leads --------------
        // Both records of the thread probe together (one LDS round trip per step for the pair).
        int r_leader[2];
        uint32_t r_slot[2];
        {
            bool act[2];
            uint32_t word[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                r_leader[e] = -1;
                r_slot[e] = slot_hash(cur.sid[e], (uint32_t)(r_seg[e] & 0xFFFF)) & (H - 1);
                act[e] = r_seg[e] >= 0;
                uint32_t once;
                word[e] = (uint32_t)(2 * tid + e + 1) | frag_bits(cur.flags[e], &once) |
                          (((uint32_t)r_seg[e] & 0x1FFu) << kSlotSegShift);
            }
            while (act[0] || act[1]) {
                uint32_t old[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) old[e] = act[e] ? atomicCAS(&s_ht[r_slot[e]], 0u, word[e]) : 0u;
                int o[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    o[e] = (int)(old[e] & kSlotIdx) - 1;
                    if (act[e] && old[e] == 0u) {
                        r_leader[e] = 2 * tid + e;
                        act[e] = false;
                    }
                }
                uint64_t osid[2];
                uint16_t oseg[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    oseg[e] = (uint16_t)((old[e] >> kSlotSegShift) & 0x1FFu);
                    osid[e] = (act[e] && oseg[e] == (uint16_t)r_seg[e]) ? s_sid[o[e]] : ~cur.sid[e];
                }
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    if (!act[e]) continue;
                    if (osid[e] == cur.sid[e] && oseg[e] == (uint16_t)r_seg[e]) {
                        r_leader[e] = o[e];
                        act[e] = false;
                    } else {
                        r_slot[e] = (r_slot[e] + 1) & (H - 1);
                    }
                }
            }
        }
        ZK_STAMP(3);

        // ---- 5. reduce(mergeSpan) ------------------------------------------------------------------
        // No barrier before this: a fragment merges into its leader as soon as it has found it (the
        // leader's staged values are in place since phase 3; OR-ing bits into a claimed slot leaves
        // its index field, which is all a concurrent probe reads, unchanged).
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int j = 2 * tid + e;
            const int L = r_leader[e];
            if (L >= 0 && L != j) {
                const uint32_t f = cur.flags[e];
                if (f & ZK_F_HAS_ANNOTATIONS) {
                    atomicMin(&s_first[L], (long long)cur.first[e]);
                    atomicMax(&s_last[L], (long long)cur.last[e]);
                }
                if (r_svck[e] != kSvcNone) atomicMin(&s_svck[L], r_svck[e]);
                if (f & ZK_F_HAS_PARENT) atomicMin((unsigned long long*)&s_pid[L], (unsigned long long)cur.pid[e]);
                uint32_t once;
                const uint32_t bits = frag_bits(f, &once);
                uint32_t* const wp = &s_ht[r_slot[e]];
                const uint32_t old = atomicOr(wp, bits);
                const uint32_t promote = once & (old >> kSlotA) & 0xFu;  // second occurrence
                if (promote) atomicOr(wp, promote << kSlotB);
            }
        }
        ZK_PHASE_SYNC(4);
        load_early(a, n, done ? ws : next_ws, cur);  // phase 6 no longer reads these registers

        // ---- 6. filter(isValid), join on (parentId, traceId), (cell, duration) links ----------
        uint64_t r_link[2], r_item[2];
        uint32_t r_isvc[2];
        uint64_t r_lkey[2] = {0, 0};  // kModeLinks: the link's realtime item key (child-major cell | d)
        uint32_t nl = 0, ni = 0;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            r_link[e] = ~0ull;
            r_item[e] = ~0ull;
            r_isvc[e] = 0u;
            const int L = r_leader[e];
            if (L < 0) continue;
            const int j = 2 * tid + e;
            const uint32_t f = cur.flags[e];
            const uint32_t w = s_ht[r_slot[e]];
            const uint32_t sL = s_svck[L];
            const uint64_t pL = s_pid[L];
            bool amb = (f & ZK_F_HAS_PARENT) ? (cur.pid[e] != pL) : ((w & kSlotP1) != 0u);
            const uint32_t sk = r_svck[e];
            if (sk != kSvcNone && (sk >> kSvcKindShift) == (sL >> kSvcKindShift) && sk != sL) amb = true;
            if (amb) st.inc(ST_AMBIGUOUS);
            if (r_rerr[e]) st.inc(ST_SVC_RANGE);
            if (L != j) continue;
            st.inc(ST_MERGED);
            const bool valid = slot_valid(w);
            st.inc(valid ? ST_VALID : ST_INVALID);
            if constexpr (EMIT) {
                // realtime sketch item: (service, traceId, duration) of the merged span
                if (valid && sL != kSvcNone && s_first[j] != LLONG_MAX) {
                    const uint64_t d = (uint64_t)(s_last[j] - s_first[j]);
                    if (d < kMaxDuration) {
                        r_item[e] = rt_payload(cur.tid[e], d, a.rt_p, a.rt_seed);
                        r_isvc[e] = sL & kSvcIdMask;
                        ++ni;
                    } else {
                        st.inc(ST_RT_DUR_RANGE);
                    }
                }
            }
            if constexpr (!JOIN) continue;
            if (!(valid && (w & kSlotP1))) continue;
            st.inc(ST_CHILD);
            const uint16_t seg = (uint16_t)r_seg[e];
            uint32_t slot = slot_hash(pL, seg) & (H - 1);
            uint32_t pw = 0, sp = kSvcNone;
            for (;;) {
                const uint32_t o = s_ht[slot];
                if (o == 0u) break;
                const int oi = (int)(o & kSlotIdx) - 1;
                if (((o >> kSlotSegShift) & 0x1FFu) == seg) {
                    const uint64_t osid = s_sid[oi];
                    const uint32_t osvc = s_svck[oi];  // read with the spanId: one round trip
                    if (osid == pL) {
                        pw = o;
                        sp = osvc;
                        break;
                    }
                }
                slot = (slot + 1) & (H - 1);
            }
            if (pw == 0u || !slot_valid(pw)) {
                st.inc(ST_MISSING_PARENT);
                continue;
            }
            st.inc(ST_JOINED);
            if (sp == kSvcNone || sL == kSvcNone) {
                st.inc(ST_NO_SERVICE);
                continue;
            }
            const uint64_t d = (uint64_t)(s_last[j] - s_first[j]);
            if (d >= kMaxDuration) {
                st.inc(ST_DUR_RANGE);
                continue;
            }
            const uint64_t cell = (uint64_t)(sp & kSvcIdMask) * a.S + (sL & kSvcIdMask);
            r_link[e] = (cell << 40) | d;
            if constexpr (LINKS) r_lkey[e] = (((uint64_t)(sL & kSvcIdMask) * a.S + (sp & kSvcIdMask)) << 40) | d;
            if (a.nb) atomicAdd(&s_hist[cell >> a.cb_shift], 1u);
            ++nl;
        }
        ZK_STAMP(5);
        // ---- 7. append the window's links (and sketch items) to this workgroup's lists ----------
        // no barrier: each wave claims its slice of the workgroup's lists with ONE LDS atomic on a
        // cursor (links in the low 32 bits, sketch items in the high 32); lane offsets from ballots
        // (nl, ni are 0..2). The waves' order inside a list is whatever the atomics give -- the
        // reduce adds exact integers, so it is free.
        const uint64_t l1 = __ballot(nl >= 1u), l2 = __ballot(nl >= 2u);
        const uint64_t i1 = EMIT ? __ballot(ni >= 1u) : 0ull, i2 = EMIT ? __ballot(ni >= 2u) : 0ull;
        uint32_t lbase = 0, ibase = 0;
        {
            const uint64_t wtot = (uint64_t)(__popcll(l1) + __popcll(l2)) | ((uint64_t)(__popcll(i1) + __popcll(i2)) << 32);
            uint64_t old = 0;
            if (lane == 0 && wtot) old = atomicAdd((unsigned long long*)&s_cursor, (unsigned long long)wtot);
            old = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(old >> 32), 0) << 32) | (uint32_t)__shfl((int)(uint32_t)old, 0);
            lbase = (uint32_t)old + lanes_below(l1) + lanes_below(l2);
            ibase = (uint32_t)(old >> 32) + lanes_below(i1) + lanes_below(i2);
        }
        // the next window's ballots, BEFORE this window's link stores: the prefetched traceIds are
        // then waited for while only they are in flight, not behind the stores (vmcnt is one queue
        // for loads and stores, and the first use of a prefetched value waits for everything older
        // in the compiler's model). s_mask is free: every wave read it in phase 2, before the
        // phase-3 barrier; the next window's phase-1 barrier publishes the new masks.
        if (!done) {
            const uint64_t nws = next_ws;
            window_ballots(nxt, nws, (int)((n - nws) < (uint64_t)TILE ? (n - nws) : (uint64_t)TILE), &n_ev, &n_od);
            if (lane == 0) *reinterpret_cast<ulonglong2*>(&s_mask[2 * wave]) = make_ulonglong2(n_ev, n_od);
        }
        if constexpr (JOIN) {
            // exactly two stores per thread on every path (absent links go to the list's trash
            // slot), so the loop-end wait for the prefetched window can count them: vmcnt(2)
            uint32_t pos = lbase;
#if defined(ZK_K1_DIAG_TRASHONLY)
            out[trash] = r_link[0];
            out[trash] = r_link[1];
#elif !defined(ZK_K1_DIAG_NOSTORE)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const bool v = r_link[e] != ~0ull;
                const uint64_t at = v ? (uint64_t)pos : trash;
                out[at] = r_link[e];
                if constexpr (LINKS) {  // the realtime link item at the link's own position
                    a.lk_key[(uint64_t)blockIdx.x * a.link_stride + at] = r_lkey[e];
                    a.lk_tid[(uint64_t)blockIdx.x * a.link_stride + at] = cur.tid[e];
                }
                pos += v ? 1u : 0u;
            }
#else
            if (pos == 0xFFFFFFFFu) out[0] = r_link[0];
#endif
        }
        if constexpr (EMIT) {
            uint32_t pos = ibase;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const bool v = r_item[e] != ~0ull;
                const uint64_t at = v ? (uint64_t)pos : trash;
                it_pay[at] = r_item[e];
                it_svc[at] = r_isvc[e];
                pos += v ? 1u : 0u;
            }
        }
        // every leader empties its own slot in the NEXT window, after its phase-1 barrier (which
        // every wave reaches only when done probing this window) and before its phase-3 barrier
        // (after which that window inserts)
#pragma unroll
        for (int e = 0; e < 2; ++e) r_clear[e] = (r_leader[e] == 2 * tid + e) ? r_slot[e] : kNoSlot;
        ZK_STAMP(6);
        if (--fold_in == 0) {
            fold_stats(st, s_stat);
            fold_in = kFoldWindows;
        }
        if (done) break;
        ws = next_ws;
        seek = next_seek;
        seek_start = next_seek_start;
        m_ev = n_ev;
        m_od = n_od;
        cur.tid[0] = nxt.tid[0];
        cur.tid[1] = nxt.tid[1];
        cur.prev = nxt.prev;
        // no loop-end barrier: the next window's phase-1 barrier already separates this window's
        // last LDS reads (phase 6-7) from its writes (phase 3 on), and phase 1's s_mask writes
        // from this window's reads (phases 2-3, before the barrier that ends phase 3)
        ZK_STAMP(7);
    }
    ZK_STAMP_FLUSH();
    __syncthreads();  // every wave's last append is in the cursor
#ifdef ZK_K1_DIAG
    if (tid == 0) s_cursor = 0ull;  // the lists hold no links K2/K3 may read
    for (uint32_t x = tid; x < a.nb; x += WG) s_hist[x] = 0u;
    __syncthreads();
#endif
    const uint32_t nout = (uint32_t)s_cursor;
    const uint32_t nitem = (uint32_t)(s_cursor >> 32);
    if (tid == 0) {
        a.link_count[blockIdx.x] = nout;
        if constexpr (EMIT) a.rt_count[blockIdx.x] = nitem;
        atomicAdd(&a.stats[(uint64_t)(blockIdx.x % kStatShards) * ST_N + ST_RECORDS], (unsigned long long)nrec);
    }
    fold_stats(st, s_stat);
    publish_stats(s_stat, a.stats);  // its barrier also publishes s_hist
    if constexpr (EMIT) {
        if (tid == 0 && s_stat[ST_RT_DUR_RANGE]) atomicAdd(&a.rt_dropped[1], (unsigned long long)s_stat[ST_RT_DUR_RANGE]);
    }
    if constexpr (JOIN) {
        for (uint32_t x = tid; x < a.nb; x += WG) a.hist[(uint64_t)x * a.grid + blockIdx.x] = s_hist[x];
    } else {
        for (uint32_t x = tid; x < a.nb; x += WG) a.hist[(uint64_t)x * a.grid + blockIdx.x] = 0u;
    }
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
    __shared__ unsigned long long s_stat[ST_N];
    const uint32_t total = min(*a.spill_count, (unsigned int)a.spill_cap);
    const uint64_t n = a.n_dev ? (uint64_t)*a.n_dev : a.c.n;
    const uint64_t* __restrict__ tr = a.c.trace_id;
    uint8_t* base = a.spill_scratch + (uint64_t)blockIdx.x * a.spill_scratch_stride;
    StatWide st;
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
            st_sc(&sc.pid[j], (uint64_t)((f & ZK_F_HAS_PARENT) ? (a.join ? a.c.parent_id[gi] : 0ull) : ~0ull));
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
                if (f & ZK_F_HAS_PARENT)
                    atomicMin((unsigned long long*)&sc.pid[Ld], (unsigned long long)(a.join ? a.c.parent_id[gi] : 0ull));
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
            bool amb = (f & ZK_F_HAS_PARENT) ? ((a.join ? a.c.parent_id[gi] : 0ull) != pL) : (npar > 0);
            if (sk != kSvcNone && (sk >> kSvcKindShift) == (sL >> kSvcKindShift) && sk != sL) amb = true;
            if (amb) st.inc(ST_AMBIGUOUS);
            if (Ld != j) continue;
            st.inc(ST_MERGED);
            const bool valid = spill_valid(A, B);
            st.inc(valid ? ST_VALID : ST_INVALID);
            if (a.rt_pay && valid && sL != kSvcNone) {
                // sketch item of the merged span, appended to list `grid` (capacity >= records)
                const long long f0 = ld_sc(&sc.first[Ld]);
                if (f0 != LLONG_MAX) {
                    const uint64_t d = (uint64_t)(ld_sc(&sc.last[Ld]) - f0);
                    if (d < kMaxDuration) {
                        const uint64_t at = (uint64_t)a.grid * a.link_stride + atomicAdd(&a.rt_count[a.grid], 1u);
                        a.rt_pay[at] = rt_payload(a.c.trace_id[gi], d, a.rt_p, a.rt_seed);
                        a.rt_svc[at] = sL & kSvcIdMask;
                    } else {
                        atomicAdd(&a.rt_dropped[1], 1ull);
                    }
                }
            }
            if (!a.join) continue;
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
                    if (d >= kMaxDuration) {
                        st.inc(ST_DUR_RANGE);
                    } else {
                        emit_link(a.table, (spv & kSvcIdMask) * a.S + (sL & kSvcIdMask), d);
                        if (a.lk_key) {  // the realtime link item, appended to the spill list
                            const uint32_t q = atomicAdd(a.lk_spill_count, 1u);
                            if (q < a.lk_spill_cap) {
                                const uint64_t at = (uint64_t)a.grid * a.link_stride + q;
                                a.lk_key[at] = (((uint64_t)(sL & kSvcIdMask) * a.S + (spv & kSvcIdMask)) << 40) | d;
                                a.lk_tid[at] = a.c.trace_id[gi];
                            }
                        }
                    }
                }
            } else {
                st.inc(ST_MISSING_PARENT);
            }
        }
        if (threadIdx.x == 0) atomicAdd(&a.stats[ST_RECORDS], (unsigned long long)L);
        // flush per trace so the per-thread 16-bit fields never overflow
        flush_stats(st, s_stat, a.stats);
        st = StatWide();
        __syncthreads();
        if (threadIdx.x < ST_N) s_stat[threadIdx.x] = 0ull;
        __syncthreads();
    }
}

// =============================================================================================
// K1G: the join over hash groups (unclustered batches)
//
// The clustering pass's partition (zk_cluster.hip P0-P2) leaves every trace inside one sub-bucket,
// its records in any order. Instead of clustering each sub-bucket (P3) and streaming K1 over the
// result, one workgroup per CU takes runs of whole consecutive sub-buckets (batches of <= kGCap
// records) into LDS and keys the same merge and join by (traceId, spanId) and (traceId, parentId):
// the groupBy((id, traceId)) and the (parentId, traceId) join of ZipkinAggregateJob.scala:21-33 with
// the traceId in the key, as the reference has it, instead of a trace segment. Every record is read
// from HBM once (48 B); P3's 104 B per record and K1's second read of the columns are gone. Two
// register windows alternate: the batch after next loads into the current batch's registers in
// three groups, each as soon as the registers it overwrites are dead. Sub-buckets longer than kGCap
// (a trace of > 2k records, or an unlucky hash range) are listed and left to the fallback: P3 over
// the listed sub-buckets only, then K1 (append mode) over its output, into the same link lists.
//
// Slot word (u32): bits 0..11 leader position + 1; 12..21 the fragment bits of K1's slot word;
// 22..31 a 10-bit fingerprint of the key hash, so a probe loads the occupant's traceId and spanId
// only when the fingerprint matches.
// =============================================================================================
#ifndef ZK_GJ_WG
#define ZK_GJ_WG 1024  // group-join workgroup: 2 x WG positions of LDS per batch
#endif
#ifndef ZK_GJ_HF
#define ZK_GJ_HF 8  // hash slots per LDS position (4: +0.13 ms per 1e8 records, longer probe chains)
#endif
constexpr int kGWG = ZK_GJ_WG;
constexpr int kGCap = 2 * kGWG;      // positions of a batch in LDS (two per thread, pair-aligned)
constexpr int kGH = ZK_GJ_HF * kGCap;  // hash slots: load <= 1/8 (~1/16 at the plan's batches)
constexpr int kGPerCU = kGWG >= 1024 ? 1 : kGWG >= 512 ? 2 : 4;  // resident workgroups per CU (LDS)
constexpr uint32_t kGIdx = 0xFFFu;
constexpr int kGFpShift = 22;
static_assert(kGCap < (int)kGIdx && kSlotP0 < (1u << kGFpShift), "slot word fields");

// the 32-bit hash of key (traceId, x): tmix = traceId * golden, computed once per record
__device__ __forceinline__ uint32_t group_hash(uint64_t tmix, uint64_t x) {
    uint64_t h = x ^ tmix;
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 33;
    return (uint32_t)h;
}

__device__ __forceinline__ void load_group(const JoinArgs& a, uint64_t base, Window& w) {
    ld2_u64(a.c.trace_id, base + 2 * threadIdx.x, a.c.n, w.tid);
    load_early(a, a.c.n, base, w);
    load_late<true>(a, a.c.n, base, w);
}

__global__ __launch_bounds__(kGWG, kGPerCU * kGWG / 256) void k_group_join(JoinArgs a) {
    __shared__ __align__(16) uint64_t s_tid[kGCap];
    __shared__ __align__(16) uint64_t s_sid[kGCap];
    __shared__ __align__(16) long long s_first[kGCap];
    __shared__ __align__(16) long long s_last[kGCap];
    __shared__ __align__(16) uint64_t s_pid[kGCap];
    __shared__ __align__(16) uint32_t s_svck[kGCap];
    __shared__ __align__(16) uint32_t s_ht[kGH];
    __shared__ uint32_t s_stat[ST_N];
    __shared__ uint32_t s_hist[kMaxBuckets];
    __shared__ uint32_t s_cursor;
    __shared__ uint32_t s_find[2];

    const int tid = threadIdx.x, lane = tid & 63;
    const uint64_t n = a.c.n;
    const uint32_t nsub = a.nsub;
    ZK_STAMP_DECL
    const uint64_t R0 = (uint64_t)blockIdx.x * a.per_wg;
    const uint64_t R1 = (R0 + a.per_wg < n) ? R0 + a.per_wg : n;
    if (tid < ST_N) s_stat[tid] = 0u;
    if (tid == 0) {
        s_cursor = 0u;
        s_find[0] = kGWG;
        s_find[1] = nsub;
    }
    for (uint32_t x = tid; x < a.nb; x += kGWG) s_hist[x] = 0u;
    for (int x = tid; x < kGH / 4; x += kGWG) reinterpret_cast<uint4*>(s_ht)[x] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    // first owned sub-bucket: the first g with sub[g] >= R0, in two parallel rounds (sub[nsub] = n > R0)
    uint32_t g0 = nsub;
    if (R0 < n) {
        // samples min(t * step, nsub), t < kGWG: the last one is nsub, so some sample is >= R0
        const uint32_t step = nsub / (kGWG - 1) + 1;
        {
            const uint32_t x = (uint32_t)tid * step < nsub ? (uint32_t)tid * step : nsub;
            if (a.sub[x] >= R0) atomicMin(&s_find[0], (uint32_t)tid);
        }
        __syncthreads();
        const uint32_t c = s_find[0];  // the first sample >= R0: g0 lies in (sample c-1, sample c]
        const uint32_t lo_g = c == 0 ? 0u : (c - 1) * step + 1;
        const uint32_t hi_g = c * step < nsub ? c * step : nsub;
        for (uint32_t x = lo_g + tid; x <= hi_g; x += kGWG)
            if (a.sub[x] >= R0) atomicMin(&s_find[1], x);
        __syncthreads();
        g0 = s_find[1];
    }
    // Batches: runs of whole consecutive sub-buckets of <= kGCap records in all (the keys carry the
    // traceId, so sub-buckets share the LDS table freely). Every wave holds the bounds of the next 64
    // sub-buckets in a lane each (one vector load, issued a batch ahead) and cuts the batch with two
    // ballots: the longest prefix that fits and whose sub-buckets start in this workgroup's range.
    // A sub-bucket longer than kGCap alone is listed for the fallback. (uniform)
    auto fetch = [&](uint32_t gs) -> uint32_t {
        const uint32_t g = gs + (uint32_t)lane;
        return a.sub[g < nsub ? g : nsub];
    };
    // -> next first sub-bucket; [*lo, *hi) the batch's records (empty: none, or a window of only
    // empty / listed sub-buckets, *more = 1: fetch at the returned index and cut again)
    auto cut = [&](uint32_t gs, uint32_t bv, uint32_t* lo, uint32_t* hi, bool* more) -> uint32_t {
        *lo = *hi = 0u;
        *more = false;
        const uint64_t own = __ballot(gs + (uint32_t)lane < nsub && bv < R1);  // sub-buckets starting in range
        int o = 0;
        for (;;) {
            if (o >= 63) {
                *more = true;
                return gs + (uint32_t)o;
            }
            if (!((own >> o) & 1ull)) return nsub;  // the rest belongs to the next workgroups
            const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bv, o);
            const uint32_t off = b0 & 1u;
            // lane l > o ends a batch of sub-buckets o..l-1 that fits (a prefix: the bounds rise)
            const uint64_t fit = __ballot(lane > o && gs + (uint32_t)lane <= nsub && bv - b0 + off <= (uint32_t)kGCap);
            // ends up to the first sub-bucket not in range
            const uint64_t notown = ~own & (~0ull << o);
            const int q = notown ? __ffsll((unsigned long long)notown) - 1 : 64;
            int l = o + __popcll(fit);
            if (l > q) l = q;
            if (l > o) {
                *lo = b0;
                *hi = (uint32_t)__builtin_amdgcn_readlane((int)bv, l);
                if (*hi == b0) *more = true;  // empty sub-buckets only
                return gs + (uint32_t)l;
            }
            // sub-bucket o alone is longer than the LDS capacity
            if (tid == 0) a.big_list[atomicAdd(a.big_count, 1u)] = gs + (uint32_t)o;  // (every wave cuts alike)
            ++o;
        }
    };
    // the next batch with records at or after gs (bv = fetch(gs)); *lo == *hi: none left
    auto next_batch = [&](uint32_t gs, uint32_t bv, uint32_t* lo, uint32_t* hi) -> uint32_t {
        for (;;) {
            bool more;
            gs = cut(gs, bv, lo, hi, &more);
            if (!more) return gs;
            bv = fetch(gs);
        }
    };

    StatPack st;
    int fold_in = kFoldWindows;
    uint64_t nrec = 0;
    constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
    uint32_t r_clear[2] = {kNoSlot, kNoSlot};
    uint64_t* __restrict__ out = a.links + (uint64_t)blockIdx.x * a.link_stride;
    const uint64_t trash = a.link_stride - 1;

    uint32_t gs = g0;
    uint32_t bv = fetch(gs);
    // Join batch [lo, hi) from `cur`; then cut the batch after the one in flight and load it into
    // `cur` (no longer read) BEFORE the closing barrier: the waves issue their loads as they finish,
    // not all at once after it (the stamps build showed 18 % of wave cycles in the load issue).
    auto run_group = [&](Window& cur, uint32_t lo, uint32_t hi, uint32_t* nlo, uint32_t* nhi) {
        const uint32_t len = hi - lo;
        // The batch after the one in flight, and its column loads into `cur` spread over this batch's
        // phases as `cur`'s registers fall free (service after staging; spanId and first/last after the
        // merge; traceId, parentId and flags after the join), so the waves' load issue interleaves with
        // compute instead of coming as one 98-KB burst (one burst before the closing barrier: 1.84 vs
        // 1.57 ms per 1e8 records, profiles/r04/ab_group_join_spread.txt). Unconditional (base 0 when
        // there is none).
        gs = next_batch(gs, bv, nlo, nhi);
        const uint64_t nbase = *nhi > *nlo ? (uint64_t)(*nlo & ~1u) : 0ull;
        bv = fetch(gs);
        const int off = (int)(lo & 1u);
        nrec += len;
        // ---- stage: transformed values at positions 2t, 2t+1 (position p = record lo - off + p) ---
#pragma unroll
        for (int e = 0; e < 2; ++e)
            if (r_clear[e] != kNoSlot) s_ht[r_clear[e]] = 0u;  // the previous group's leaders
        const int j0 = 2 * tid;
        bool act[2];
        uint32_t r_svck[2];
        bool r_rerr[2];
        uint64_t tmix[2];
        {
            uint64_t v_first[2], v_last[2], v_pid[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                act[e] = j0 + e >= off && j0 + e < off + (int)len;
                tmix[e] = cur.tid[e] * 0x9E3779B97F4A7C15ull;
                r_rerr[e] = false;
                r_svck[e] = svc_key(cur.flags[e], cur.svc[e], a.S, &r_rerr[e]);
                const uint32_t f = cur.flags[e];
                const bool ha = (f & ZK_F_HAS_ANNOTATIONS) != 0;
                v_first[e] = ha ? cur.first[e] : (uint64_t)LLONG_MAX;
                v_last[e] = ha ? cur.last[e] : (uint64_t)LLONG_MIN;
                v_pid[e] = (f & ZK_F_HAS_PARENT) ? cur.pid[e] : ~0ull;
            }
            *reinterpret_cast<ulonglong2*>(&s_tid[j0]) = make_ulonglong2(cur.tid[0], cur.tid[1]);
            *reinterpret_cast<ulonglong2*>(&s_sid[j0]) = make_ulonglong2(cur.sid[0], cur.sid[1]);
            *reinterpret_cast<ulonglong2*>(&s_first[j0]) = make_ulonglong2(v_first[0], v_first[1]);
            *reinterpret_cast<ulonglong2*>(&s_last[j0]) = make_ulonglong2(v_last[0], v_last[1]);
            *reinterpret_cast<ulonglong2*>(&s_pid[j0]) = make_ulonglong2(v_pid[0], v_pid[1]);
            *reinterpret_cast<uint2*>(&s_svck[j0]) = make_uint2(r_svck[0], r_svck[1]);
        }
        ZK_PHASE_SYNC(1);  // staged; every slot of the previous group is empty
        ld2_u32(a.c.service_id, nbase + 2 * threadIdx.x, a.c.n, cur.svc);
        // ---- groupBy((id, traceId)): the first fragment to claim a slot leads ------------------
        int r_leader[2];
        uint32_t r_slot[2];
        {
            uint32_t word[2], fp[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                r_leader[e] = -1;
                const uint32_t h = group_hash(tmix[e], cur.sid[e]);
                r_slot[e] = h & (kGH - 1);
                fp[e] = h >> kGFpShift;
                uint32_t once;
                word[e] = (uint32_t)(j0 + e + 1) | frag_bits(cur.flags[e], &once) | (fp[e] << kGFpShift);
            }
            bool pend[2] = {act[0], act[1]};
            while (pend[0] || pend[1]) {
                uint32_t old[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) old[e] = pend[e] ? atomicCAS(&s_ht[r_slot[e]], 0u, word[e]) : 0u;
                int o[2];
                bool cand[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    o[e] = (int)(old[e] & kGIdx) - 1;
                    if (pend[e] && old[e] == 0u) {
                        r_leader[e] = j0 + e;
                        pend[e] = false;
                    }
                    cand[e] = pend[e] && (old[e] >> kGFpShift) == fp[e];
                }
                uint64_t osid[2], otid[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    osid[e] = cand[e] ? s_sid[o[e]] : ~cur.sid[e];
                    otid[e] = cand[e] ? s_tid[o[e]] : ~cur.tid[e];
                }
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    if (!pend[e]) continue;
                    if (osid[e] == cur.sid[e] && otid[e] == cur.tid[e]) {
                        r_leader[e] = o[e];
                        pend[e] = false;
                    } else {
                        r_slot[e] = (r_slot[e] + 1) & (kGH - 1);
                    }
                }
            }
        }
        ZK_STAMP(2);
        // ---- reduce(mergeSpan) into the leader (no barrier: see K1 phase 5) ----------------------
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int j = j0 + e;
            const int L = r_leader[e];
            if (L >= 0 && L != j) {
                const uint32_t f = cur.flags[e];
                if (f & ZK_F_HAS_ANNOTATIONS) {
                    atomicMin(&s_first[L], (long long)cur.first[e]);
                    atomicMax(&s_last[L], (long long)cur.last[e]);
                }
                if (r_svck[e] != kSvcNone) atomicMin(&s_svck[L], r_svck[e]);
                if (f & ZK_F_HAS_PARENT) atomicMin((unsigned long long*)&s_pid[L], (unsigned long long)cur.pid[e]);
                uint32_t once;
                const uint32_t bits = frag_bits(f, &once);
                uint32_t* const wp = &s_ht[r_slot[e]];
                const uint32_t old = atomicOr(wp, bits);
                const uint32_t promote = once & (old >> kSlotA) & 0xFu;
                if (promote) atomicOr(wp, promote << kSlotB);
            }
        }
        ZK_PHASE_SYNC(3);  // merged
        ld2_u64(a.c.span_id, nbase + 2 * threadIdx.x, a.c.n, cur.sid);
        ld2_u64((const uint64_t*)a.c.first_ts, nbase + 2 * threadIdx.x, a.c.n, cur.first);
        ld2_u64((const uint64_t*)a.c.last_ts, nbase + 2 * threadIdx.x, a.c.n, cur.last);
        // ---- filter(isValid), join on (parentId, traceId), links ---------------------------------
        uint64_t r_link[2];
        uint32_t nl = 0;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            r_link[e] = ~0ull;
            const int L = r_leader[e];
            if (L < 0) continue;
            const int j = j0 + e;
            const uint32_t f = cur.flags[e];
            const uint32_t w = s_ht[r_slot[e]];
            const uint32_t sL = s_svck[L];
            const uint64_t pL = s_pid[L];
            bool amb = (f & ZK_F_HAS_PARENT) ? (cur.pid[e] != pL) : ((w & kSlotP1) != 0u);
            const uint32_t sk = r_svck[e];
            if (sk != kSvcNone && (sk >> kSvcKindShift) == (sL >> kSvcKindShift) && sk != sL) amb = true;
            if (amb) st.inc(ST_AMBIGUOUS);
            if (r_rerr[e]) st.inc(ST_SVC_RANGE);
            if (L != j) continue;
            st.inc(ST_MERGED);
            const bool valid = slot_valid(w);
            st.inc(valid ? ST_VALID : ST_INVALID);
            if (!(valid && (w & kSlotP1))) continue;
            st.inc(ST_CHILD);
            const uint32_t hp = group_hash(tmix[e], pL);
            const uint32_t pfp = hp >> kGFpShift;
            uint32_t slot = hp & (kGH - 1);
            uint32_t pw = 0, sp = kSvcNone;
            for (;;) {
                const uint32_t o = s_ht[slot];
                if (o == 0u) break;
                if ((o >> kGFpShift) == pfp) {
                    const int oi = (int)(o & kGIdx) - 1;
                    const uint64_t osid = s_sid[oi];
                    const uint64_t otid = s_tid[oi];
                    const uint32_t osvc = s_svck[oi];
                    if (osid == pL && otid == cur.tid[e]) {
                        pw = o;
                        sp = osvc;
                        break;
                    }
                }
                slot = (slot + 1) & (kGH - 1);
            }
            if (pw == 0u || !slot_valid(pw)) {
                st.inc(ST_MISSING_PARENT);
                continue;
            }
            st.inc(ST_JOINED);
            if (sp == kSvcNone || sL == kSvcNone) {
                st.inc(ST_NO_SERVICE);
                continue;
            }
            const uint64_t d = (uint64_t)(s_last[j] - s_first[j]);
            if (d >= kMaxDuration) {
                st.inc(ST_DUR_RANGE);
                continue;
            }
            const uint64_t cell = (uint64_t)(sp & kSvcIdMask) * a.S + (sL & kSvcIdMask);
            r_link[e] = (cell << 40) | d;
            if (a.nb) atomicAdd(&s_hist[cell >> a.cb_shift], 1u);
            ++nl;
        }
        ZK_STAMP(4);
        ld2_u64(a.c.trace_id, nbase + 2 * threadIdx.x, a.c.n, cur.tid);
        ld2_u64(a.c.parent_id, nbase + 2 * threadIdx.x, a.c.n, cur.pid);
        ld2_u32(a.c.flags, nbase + 2 * threadIdx.x, a.c.n, cur.flags);
        // ---- append: one LDS atomic per wave claims its slice of the workgroup's list ------------
        const uint64_t l1 = __ballot(nl >= 1u), l2 = __ballot(nl >= 2u);
        uint32_t lbase = 0;
        {
            const uint32_t wtot = (uint32_t)(__popcll(l1) + __popcll(l2));
            uint32_t old = 0;
            if (lane == 0 && wtot) old = atomicAdd(&s_cursor, wtot);
            lbase = (uint32_t)__shfl((int)old, 0) + lanes_below(l1) + lanes_below(l2);
        }
        uint32_t pos = lbase;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const bool v = r_link[e] != ~0ull;
            out[v ? (uint64_t)pos : trash] = r_link[e];
            pos += v ? 1u : 0u;
        }
#pragma unroll
        for (int e = 0; e < 2; ++e) r_clear[e] = (r_leader[e] == j0 + e) ? r_slot[e] : kNoSlot;
        if (--fold_in == 0) {
            fold_stats(st, s_stat);
            fold_in = kFoldWindows;
        }
        ZK_PHASE_SYNC(5);  // every probe of this group is done before the next one is staged
    };

    // two register windows: one batch's columns load while the other batch is joined; the bounds
    // of the batch after both load while the first is joined
    Window wa, wb;
    uint32_t la = 0, ha = 0, lb = 0, hb = 0;
    gs = next_batch(gs, bv, &la, &ha);
    if (ha > la) load_group(a, la & ~1u, wa);
    bv = fetch(gs);
    gs = next_batch(gs, bv, &lb, &hb);
    if (hb > lb) load_group(a, lb & ~1u, wb);
    bv = fetch(gs);
    ZK_STAMP(6);
    for (;;) {
        if (ha <= la) break;
        run_group(wa, la, ha, &la, &ha);
        ZK_STAMP(6);
        if (hb <= lb) break;
        run_group(wb, lb, hb, &lb, &hb);
        ZK_STAMP(6);
    }
    ZK_STAMP_FLUSH();
    __syncthreads();
    if (tid == 0) {
        a.link_count[blockIdx.x] = s_cursor;
        atomicAdd(&a.stats[(uint64_t)(blockIdx.x % kStatShards) * ST_N + ST_RECORDS], (unsigned long long)nrec);
    }
    fold_stats(st, s_stat);
    publish_stats(s_stat, a.stats);  // its barrier also publishes s_hist
    for (uint32_t x = tid; x < a.nb; x += kGWG) a.hist[(uint64_t)x * a.grid + blockIdx.x] = s_hist[x];
}

// tile geometry of the shipped K1
#ifndef ZK_K1_WG
#define ZK_K1_WG 256  // K1 workgroup; a window is two records per thread
#endif
constexpr int kTileWG = ZK_K1_WG;
constexpr int kTile = 2 * kTileWG;

}  // namespace

uint64_t spill_scratch_bytes_per_wg(uint32_t max_trace) {
    const uint64_t L = max_trace;
    uint64_t b = 8ull * L * 6 + 4ull * L + 4ull * (L & 1) + 4ull * spill_ht_slots(max_trace);
    return (b + 255) & ~255ull;
}

hipError_t launch_join(const JoinArgs& a, hipStream_t s, uint32_t blocks) {
    if (a.c.n == 0) return hipSuccess;
    const dim3 g((unsigned)(blocks ? blocks : a.grid)), b(kTileWG);
    const bool emit = a.rt_pay != nullptr, join = a.join != 0;
    if (a.lk_key && join && !emit)
        return launch_checked("k_span_join_stream<join|links>", k_span_join_stream<kTile, kTileWG, kModeJoin | kModeLinks>,
                              g, b, 0, s, a);
    if (emit && join)
        return launch_checked("k_span_join_stream<join|emit>", k_span_join_stream<kTile, kTileWG, kModeJoin | kModeEmit>,
                              g, b, 0, s, a);
    if (emit)
        return launch_checked("k_span_join_stream<emit>", k_span_join_stream<kTile, kTileWG, kModeEmit>, g, b, 0, s, a);
    return launch_checked("k_span_join_stream<join>", k_span_join_stream<kTile, kTileWG, kModeJoin>, g, b, 0, s, a);
}

hipError_t launch_spill(const JoinArgs& a, uint32_t spill_wgs, hipStream_t s) {
    if (a.c.n == 0) return hipSuccess;
    return launch_checked("k_span_join_spill", k_span_join_spill, dim3(spill_wgs), dim3(kSpillWG), 0, s, a);
}

uint64_t join_tile_records() { return kTile; }

hipError_t launch_group_join(const JoinArgs& a, hipStream_t s) {
    if (a.c.n == 0) return hipSuccess;
    return launch_checked("k_group_join", k_group_join, dim3(a.grid), dim3(kGWG), 0, s, a);
}

uint32_t group_join_capacity() { return kGCap; }

void group_join_geometry(uint64_t n, uint32_t cus, uint32_t* grid, uint64_t* per_wg, uint64_t* link_stride) {
    uint64_t g = (uint64_t)(cus ? cus : 256) * kGPerCU;
    const uint64_t by_n = (n + kGCap - 1) / kGCap;
    if (g > by_n) g = by_n ? by_n : 1;
    const uint64_t per = (n + g - 1) / g;
    *grid = (uint32_t)g;
    *per_wg = per ? per : 1;
    // the group join's links (its sub-buckets start in its range: <= per + kGCap records), then the
    // fallback K1's (a range of <= per_wg rounded to tiles, + an overhanging trace), + the trash slot
    const uint64_t fb = (*per_wg + kTile - 1) / kTile * kTile + kTile;
    *link_stride = *per_wg + kGCap + fb + 1;
}

#ifdef ZK_STAMPS
extern "C" int zk_debug_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_zk_stamps), 16 * 8) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_zk_stamps), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif

void join_geometry(uint64_t n, uint32_t cus, uint32_t* grid, uint64_t* per_wg, uint64_t* link_stride) {
    const uint64_t windows = (n + kTile - 1) / kTile;
#ifndef ZK_K1_GRID_MULT
// workgroups per resident slot (1: persistent, every workgroup resident at once). 4: a quarter of
// the range per workgroup, so the last workgroups' imbalance is smaller and a K1 launch shares the
// chip gracefully with the other table set's K2/K3 (same box, interleaved, profiles/r02/
// ab_grid_mult_overlap.txt: serial K1 1.226 -> 1.187 ms, two-set step with full overlap 1.63-1.68 ->
// 1.56-1.57 ms; 8: slower). A persistent grid claiming ranges from a guided schedule instead:
// K1 alone -0.6 %, pipelined step +3.7 % (profiles/r04/ab_k1_guided.txt). K2 walks 4 lists per
// workgroup, so its grid stays 1024.
#define ZK_K1_GRID_MULT 4
#endif
    uint64_t g = (uint64_t)cus * ZK_K1_WGS_PER_CU * ZK_K1_GRID_MULT;  // <= 128 VGPRs, <= 40 KB LDS per WG
    if (g > windows) g = windows ? windows : 1;
    const uint64_t per = ((n + g - 1) / g + kTile - 1) / kTile * kTile;
    *grid = (uint32_t)g;
    *per_wg = per ? per : kTile;
    // a workgroup's last trace may overhang its range by < TILE; then the trash slot of K1's stores
    *link_stride = *per_wg + kTile + 1;
}}  // namespace zk
