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
// =============================================================================================
template <int TILE, int CAP, int WG>
__global__ __launch_bounds__(WG) void k_span_join_tile(JoinArgs a) {
    static_assert(CAP % WG == 0 && CAP >= TILE && (CAP & (CAP - 1)) == 0 && CAP <= 4096, "tile");
    constexpr int PT = CAP / WG;
    constexpr int H = 2 * CAP;
    constexpr int NC = CAP / 64;
    __shared__ uint64_t s_sid[CAP];
    __shared__ long long s_first[CAP];
    __shared__ long long s_last[CAP];
    __shared__ uint64_t s_cnt[CAP];
    __shared__ uint64_t s_pid[CAP];
    __shared__ uint32_t s_svck[CAP];
    __shared__ uint16_t s_seg[CAP];
    __shared__ uint32_t s_ht[H];
    __shared__ int s_chunk_last[NC];
    __shared__ int s_chunk_pref[NC];
    __shared__ uint32_t s_stat[ST_N];
    __shared__ uint64_t s_start, s_end;
    __shared__ int s_tail, s_cut;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t n = a.c.n;
    const uint64_t lo = (uint64_t)blockIdx.x * TILE;
    const uint64_t hi = (lo + TILE < n) ? lo + TILE : n;
    const uint64_t* __restrict__ tr = a.c.trace_id;

    // ---- 1. which traces does this tile own: those starting in [lo, hi) -------------------
    if (tid < ST_N) s_stat[tid] = 0u;
    if (wave == 0) {
        uint64_t start = hi;
        for (uint64_t base = lo; base < hi; base += 64) {
            const uint64_t i = base + lane;
            bool b = false;
            if (i < hi) b = (i == 0) || (tr[i] != tr[i - 1]);
            const uint64_t m = __ballot(b);
            if (m) {
                start = base + (uint64_t)(__ffsll((unsigned long long)m) - 1);
                break;
            }
        }
        int tail = 0;
        uint64_t end = start;
        if (start < hi) {
            const uint64_t limit = start + CAP;  // records [start, limit) fit the tile
            end = ~0ull;
            for (uint64_t base = hi; base <= limit; base += 64) {
                const uint64_t i = base + lane;
                bool b = false;
                if (i <= limit) b = (i >= n) || (tr[i] != tr[i - 1]);
                const uint64_t m = __ballot(b);
                if (m) {
                    end = base + (uint64_t)(__ffsll((unsigned long long)m) - 1);
                    break;
                }
            }
            if (end == ~0ull) {  // the last owned trace does not fit: spill it
                tail = 1;
                end = hi;
            }
        }
        if (lane == 0) {
            s_start = start;
            s_end = end;
            s_tail = tail;
        }
    }
    __syncthreads();
    const uint64_t start = s_start;
    if (start >= hi) return;
    const int tail = s_tail;
    const int m_load = (int)(s_end - start);

    // ---- 2. coalesced column loads + trace segmentation (ballot of traceId changes) -------
    uint64_t r_sid[PT], r_pid[PT];
    long long r_first[PT], r_last[PT];
    uint32_t r_flags[PT], r_svck[PT];
    int r_seg[PT], r_leader[PT];
    bool r_rerr[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k) {
        const int j = tid + k * WG;
        const bool in = j < m_load;
        const uint64_t gi = start + (uint64_t)j;
        uint64_t t = 0;
        r_sid[k] = 0;
        r_pid[k] = 0;
        r_first[k] = 0;
        r_last[k] = 0;
        r_flags[k] = 0;
        r_rerr[k] = false;
        uint32_t svc = 0;
        if (in) {
            t = tr[gi];
            r_sid[k] = a.c.span_id[gi];
            r_pid[k] = a.c.parent_id[gi];
            r_first[k] = a.c.first_ts[gi];
            r_last[k] = a.c.last_ts[gi];
            svc = a.c.service_id[gi];
            r_flags[k] = a.c.flags[gi];
        }
        r_svck[k] = svc_key(r_flags[k], svc, a.S, &r_rerr[k]);
        uint64_t tprev = __shfl_up(t, 1);
        if (lane == 0 && in && j > 0) tprev = tr[gi - 1];
        const bool b = in && (j == 0 || t != tprev);
        const uint64_t mask = __ballot(b);
        const int c = (k * WG + wave * 64) >> 6;
        if (lane == 0) s_chunk_last[c] = mask ? (c * 64 + 63 - __clzll((long long)mask)) : -1;
        const uint64_t pm = mask & ((2ull << lane) - 1ull);
        r_seg[k] = pm ? (c * 64 + 63 - __clzll((long long)pm)) : -1;
    }
    __syncthreads();
    if (wave == 0) {
        int v = lane < NC ? s_chunk_last[lane] : -1;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(v, off);
            if (lane >= off) v = v > o ? v : o;
        }
        int ex = __shfl_up(v, 1);
        if (lane == 0) ex = -1;
        if (lane < NC) s_chunk_pref[lane] = ex;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; ++k) {
        const int j = tid + k * WG;
        if (r_seg[k] < 0) r_seg[k] = s_chunk_pref[j >> 6];
        if (j < m_load) {
            const uint32_t f = r_flags[k];
            const bool ha = (f & ZK_F_HAS_ANNOTATIONS) != 0;
            s_sid[j] = r_sid[k];
            s_seg[j] = (uint16_t)r_seg[k];
            s_first[j] = ha ? r_first[k] : LLONG_MAX;
            s_last[j] = ha ? r_last[k] : LLONG_MIN;
            s_cnt[j] = pack_counts(f);
            s_pid[j] = (f & ZK_F_HAS_PARENT) ? r_pid[k] : ~0ull;
            s_svck[j] = r_svck[k];
            if (tail && j == m_load - 1) s_cut = r_seg[k];
        }
    }
    for (int x = tid; x < H; x += WG) s_ht[x] = 0u;
    __syncthreads();
    const int m = tail ? s_cut : m_load;
    if (tail && tid == 0) {
        const unsigned int idx = atomicAdd(a.spill_count, 1u);
        if (idx < a.spill_cap) a.spill_list[idx] = start + (uint64_t)m;
        atomicAdd(&a.stats[ST_SPILLED], 1ull);
    }

    // ---- 3. groupBy((id, traceId)): insert into the LDS hash, first fragment leads --------
#pragma unroll
    for (int k = 0; k < PT; ++k) {
        const int j = tid + k * WG;
        r_leader[k] = -1;
        if (j < m) {
            const uint64_t sid = r_sid[k];
            const uint16_t seg = (uint16_t)r_seg[k];
            uint32_t slot = slot_hash(sid, seg) & (H - 1);
            for (;;) {
                const uint32_t old = atomicCAS(&s_ht[slot], 0u, (uint32_t)(j + 1));
                if (old == 0u) {
                    r_leader[k] = j;
                    break;
                }
                const int o = (int)old - 1;
                if (s_sid[o] == sid && s_seg[o] == seg) {
                    r_leader[k] = o;
                    break;
                }
                slot = (slot + 1) & (H - 1);
            }
        }
    }
    __syncthreads();

    // ---- 4. reduce(mergeSpan): fold every other fragment into its leader -------------------
#pragma unroll
    for (int k = 0; k < PT; ++k) {
        const int j = tid + k * WG;
        const int L = r_leader[k];
        if (j < m && L != j) {
            const uint32_t f = r_flags[k];
            if (f & ZK_F_HAS_ANNOTATIONS) {
                atomicMin(&s_first[L], r_first[k]);
                atomicMax(&s_last[L], r_last[k]);
            }
            atomicAdd((unsigned long long*)&s_cnt[L], (unsigned long long)pack_counts(f));
            if (r_svck[k] != kSvcNone) atomicMin(&s_svck[L], r_svck[k]);
            if (f & ZK_F_HAS_PARENT) atomicMin((unsigned long long*)&s_pid[L], (unsigned long long)r_pid[k]);
        }
    }
    __syncthreads();

    // ---- 5. filter(isValid), join on (parentId, traceId), emit DependencyLink moments ------
    StatPack st;
#pragma unroll
    for (int k = 0; k < PT; ++k) {
        const int j = tid + k * WG;
        if (j < m) {
            const int L = r_leader[k];
            const uint32_t f = r_flags[k];
            const uint64_t cL = s_cnt[L];
            const uint32_t npar = counts_npar(cL);
            const uint32_t sL = s_svck[L];
            bool amb = (f & ZK_F_HAS_PARENT) ? (r_pid[k] != s_pid[L]) : (npar > 0);
            const uint32_t sk = r_svck[k];
            if (sk != kSvcNone && (sk >> kSvcKindShift) == (sL >> kSvcKindShift) && sk != sL) amb = true;
            if (amb) st.inc(ST_AMBIGUOUS);
            if (r_rerr[k]) st.inc(ST_SVC_RANGE);
            if (L == j) {
                st.inc(ST_MERGED);
                const bool valid = counts_valid(cL);
                st.inc(valid ? ST_VALID : ST_INVALID);
                if (valid && npar > 0) {
                    st.inc(ST_CHILD);
                    const uint64_t p = s_pid[j];
                    const uint16_t seg = (uint16_t)r_seg[k];
                    uint32_t slot = slot_hash(p, seg) & (H - 1);
                    int P = -1;
                    for (;;) {
                        const uint32_t o = s_ht[slot];
                        if (o == 0u) break;
                        if (s_sid[o - 1] == p && s_seg[o - 1] == seg) {
                            P = (int)o - 1;
                            break;
                        }
                        slot = (slot + 1) & (H - 1);
                    }
                    if (P >= 0 && counts_valid(s_cnt[P])) {
                        st.inc(ST_JOINED);
                        const uint32_t sp = s_svck[P];
                        if (sp == kSvcNone || sL == kSvcNone) {
                            st.inc(ST_NO_SERVICE);
                        } else {
                            const uint64_t d = (uint64_t)(s_last[j] - s_first[j]);
                            if (d >= kMaxDuration) {
                                st.inc(ST_DUR_RANGE);
                            } else {
                                if (!a.ablate) emit_link(a.table, (sp & kSvcIdMask) * a.S + (sL & kSvcIdMask), d);
                            }
                        }
                    } else {
                        st.inc(ST_MISSING_PARENT);
                    }
                }
            }
        }
    }
    if (tid == 0) st.inc(ST_RECORDS, (uint32_t)m);
    flush_stats(st, s_stat, a.stats);
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
constexpr int kTile = 1024;
constexpr int kCap = 2048;
constexpr int kTileWG = 256;

}  // namespace

uint64_t spill_scratch_bytes_per_wg(uint32_t max_trace) {
    const uint64_t L = max_trace;
    uint64_t b = 8ull * L * 6 + 4ull * L + 4ull * (L & 1) + 4ull * spill_ht_slots(max_trace);
    return (b + 255) & ~255ull;
}

hipError_t launch_join(const JoinArgs& a, hipStream_t s) {
    if (a.c.n == 0) return hipSuccess;
    const uint64_t tiles = (a.c.n + kTile - 1) / kTile;
    hipLaunchKernelGGL((k_span_join_tile<kTile, kCap, kTileWG>), dim3((unsigned)tiles), dim3(kTileWG), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_spill(const JoinArgs& a, uint32_t spill_wgs, hipStream_t s) {
    if (a.c.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_span_join_spill, dim3(spill_wgs), dim3(kSpillWG), 0, s, a);
    return hipGetLastError();
}

uint64_t join_tile_records() { return kTile; }

}  // namespace zk
