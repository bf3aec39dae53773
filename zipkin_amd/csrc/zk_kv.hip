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
#include "zk_launch.h"

namespace zk {
namespace {

constexpr int kKvWG = 512;  // (256: candidates 1.55 -> 1.41 ms with 512 on C4)
#ifndef ZK_KV_SET_BITS
#define ZK_KV_SET_BITS 10  // LDS hash-set slots = 2^bits (11: 2.34 -> 10: 2.03 ms candidates with three workgroups per CU)
#endif
constexpr uint32_t kSetBits = ZK_KV_SET_BITS;
constexpr uint32_t kSetCap = 1u << kSetBits;  // LDS hash-set slots (load <= 0.5); RowHash.set: the top kSetBits bits
constexpr uint32_t kSortCap = kSetCap / 2;    // compaction sort buffer
constexpr uint32_t kRound = kSortCap / 2;     // merge: entries offered between compaction checks (<= kSortCap / 2)
// candidates, a block with more survivors than the sort buffer takes: inserted kInsStep threads at a
// time, each step after a compaction down to <= kKvMaxCand entries, so the set never holds more than
// kSortCap keys
constexpr uint32_t kInsStep = kSortCap - kKvMaxCand < 512u ? kSortCap - kKvMaxCand : 512u;
static_assert(kSortCap >= 2 * kKvMaxCand && kInsStep >= 64, "sort buffer too small for the candidate lists");
// candidate rounds of keys in flight per thread (two alternating buffers of 2 x 4 keys: the next
// block's keys load while this block is estimated and inserted, C4: 3.46 -> 3.22-3.26 ms,
// profiles/r02/ab_kv_cand_pipe.txt)
#ifndef ZK_KV_PREFETCH
#define ZK_KV_PREFETCH 2  // (4 with 128 VGPRs and two workgroups per CU before round 6)
#endif
#ifndef ZK_KV_CAND_WAVES
#define ZK_KV_CAND_WAVES 6  // candidate pass: min waves per SIMD, 6 = three 512-thread workgroups per CU (<= 80 VGPRs)
#endif
constexpr int kPrefetch = ZK_KV_PREFETCH;
constexpr uint64_t kEmptyKey = ~0ull;

__device__ __forceinline__ bool beats(uint32_t e1, uint64_t k1, uint32_t e2, uint64_t k2) {
    return e1 > e2 || (e1 == e2 && k1 < k2);
}

// Row indices of a key: ONE splitmix64 of (key ^ seed_0), split into h1 (low half) and h2 (high
// half, odd); row r uses the top log2(width) bits of h1 + r * h2 (mod 2^32) -- double hashing
// (Kirsch & Mitzenmacher 2006), so a key costs one 64-bit mix instead of one per row, and the next
// row's index is one 32-bit add away.
struct RowHash {
    uint32_t x, h2, sh, set;  // set: the key's first slot in a workgroup's candidate hash set
    RowHash() = default;
    __device__ __forceinline__ RowHash(uint64_t key, uint64_t seed, uint32_t wbits) { init(sk_mix64(key ^ seed), wbits); }
    // from the key's hash h = sk_mix64(key ^ seed): the partition writes h, so the sketch and
    // candidate passes skip the 64-bit mix
    __device__ static __forceinline__ RowHash from_hash(uint64_t h, uint32_t wbits) {
        RowHash r;
        r.init(h, wbits);
        return r;
    }
    __device__ __forceinline__ void init(uint64_t h, uint32_t wbits) {
        set = (uint32_t)(h >> (64 - kSetBits));  // top kSetBits bits
        x = (uint32_t)h;
        h2 = (uint32_t)(h >> 32) | 1u;
        sh = 32u - wbits;
    }
    __device__ __forceinline__ uint32_t next() {  // index in the current row, then advance a row
        const uint32_t i = x >> sh;
        x += h2;
        return i;
    }
};

__device__ __forceinline__ uint32_t estimate_rh(const uint32_t* cm, const KvArgs& a, RowHash rh) {
    uint32_t e = 0xFFFFFFFFu;
    for (uint32_t r = 0; r < a.depth; ++r) e = min(e, cm[r * a.width + rh.next()]);
    return e;
}
__device__ __forceinline__ uint32_t estimate(const uint32_t* cm, const KvArgs& a, uint64_t key) {
    return estimate_rh(cm, a, RowHash(key, a.seeds[0], a.wbits));
}

// a key's count-min hash and back (sk_mix64 is a bijection)
__device__ __forceinline__ uint64_t kv_hash(uint64_t key, uint64_t seed) { return sk_mix64(key ^ seed); }
__device__ __forceinline__ uint64_t kv_key(uint64_t h, uint64_t seed) { return sk_unmix64(h) ^ seed; }

// Distinct (key, estimate) set keeping the best `keep` entries (estimate desc, key asc). The hash set
// hk holds the keys' HASHES (kv_hash: distinct keys, distinct hashes); the sort buffer sk and the
// threshold hold the keys themselves, so ties order by key as the oracle does.
struct TopSet {
    uint64_t hk[kSetCap];
    uint32_t he[kSetCap];
    uint64_t sk[kSortCap];
    uint32_t se[kSortCap];
    uint32_t count, gcount;
    uint32_t pending[3];  // survivors of the current block (candidates kernel), block k's in pending[k % 3]
    uint32_t has_thr, thr_est;
    uint64_t thr_key;
    uint32_t special, special_est;  // the key whose hash equals the empty sentinel
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

__device__ __forceinline__ void ts_insert(TopSet& t, uint64_t key, uint32_t est, uint32_t slot) {  // key: a hash
    if (key == kEmptyKey) {
        if (atomicCAS(&t.special, 0u, 1u) == 0u) {
            t.special_est = est;
            atomicAdd(&t.count, 1u);
        }
        return;
    }
    // Read before CAS: the heavy keys (the ones that keep beating the threshold, i.e. most offers
    // under a skewed key distribution) are already in the set, and a CAS on their slot from many
    // lanes at once serialises. Slots only go empty -> key between compactions, so a plain read
    // that shows the key (or another key) is final; one that shows empty is settled by the CAS.
    for (;;) {
        const uint64_t cur = __hip_atomic_load(&t.hk[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == key) return;
        if (cur == kEmptyKey) {
            const unsigned long long old =
                atomicCAS((unsigned long long*)&t.hk[slot], (unsigned long long)kEmptyKey, (unsigned long long)key);
            if (old == kEmptyKey) {
                t.he[slot] = est;
                atomicAdd(&t.count, 1u);
                return;
            }
            if (old == key) return;
        }
        slot = (slot + 1) & (kSetCap - 1);
    }
}

// read-only membership probe (the set only grows between compactions)
__device__ __forceinline__ bool ts_contains(TopSet& t, uint64_t key, uint32_t slot) {
    if (key == kEmptyKey) return __hip_atomic_load(&t.special, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u;
    for (;;) {
        const uint64_t cur = __hip_atomic_load(&t.hk[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == key) return true;
        if (cur == kEmptyKey) return false;
        slot = (slot + 1) & (kSetCap - 1);
    }
}

// offer a key (threshold test on the key itself) whose hash is h
__device__ __forceinline__ void ts_offer(TopSet& t, uint64_t key, uint64_t h, uint32_t est) {
    if (est == 0u) return;
    if (t.has_thr && !beats(est, key, t.thr_est, t.thr_key)) return;
    ts_insert(t, h, est, (uint32_t)(h >> (64 - kSetBits)));
}

// gather + sort (best first) into sk/se, hashes turned back into keys; returns the number of
// entries. Clears the set.
__device__ uint32_t ts_sort(TopSet& t, uint64_t seed) {
    if (threadIdx.x == 0) t.gcount = 0;
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < kSetCap; x += kKvWG) {
        const uint64_t k = t.hk[x];
        if (k != kEmptyKey) {
            const uint32_t p = atomicAdd(&t.gcount, 1u);
            t.sk[p] = kv_key(k, seed);
            t.se[p] = t.he[x];
        }
        t.hk[x] = kEmptyKey;
    }
    __syncthreads();
    if (threadIdx.x == 0 && t.special) {
        const uint32_t p = t.gcount++;
        t.sk[p] = kv_key(kEmptyKey, seed);
        t.se[p] = t.special_est;
    }
    __syncthreads();
    const uint32_t n = t.gcount;
    // the bitonic network over the next power of two >= n only (a small unit or a merge of few lists
    // sorts 64-256 entries: 21-36 barrier stages instead of 55)
    uint32_t P = 2;
    while (P < n) P <<= 1;
    for (uint32_t x = n + threadIdx.x; x < P; x += kKvWG) {
        t.sk[x] = kEmptyKey;
        t.se[x] = 0u;  // padding never beats a real entry (real estimates are >= 1)
    }
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t x = threadIdx.x; x < P; x += kKvWG) {
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
__device__ void ts_compact(TopSet& t, uint32_t keep, uint64_t seed) {
    const uint32_t n = ts_sort(t, seed);
    const uint32_t m = n < keep ? n : keep;
    if (threadIdx.x == 0 && m == keep && keep > 0) {
        t.has_thr = 1;
        t.thr_est = t.se[m - 1];
        t.thr_key = t.sk[m - 1];
    }
    for (uint32_t x = threadIdx.x; x < m; x += kKvWG) {
        const uint64_t h = kv_hash(t.sk[x], seed);
        ts_insert(t, h, t.se[x], (uint32_t)(h >> (64 - kSetBits)));
    }
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

// Unit u of service s: the service's run is cut into unit_base[s+1] - unit_base[s] equal parts
// (at most unit_items keys each), so no unit is a small remainder.
__device__ __forceinline__ void unit_range(const KvArgs& a, uint32_t s, uint32_t u, uint64_t* lo, uint64_t* hi) {
    const uint64_t b = a.seg[s], e = a.seg[s + 1];
    const uint64_t parts = a.unit_base[s + 1] - a.unit_base[s];
    const uint64_t len = (e - b + parts - 1) / parts;
    *lo = b + (uint64_t)(u - a.unit_base[s]) * len;
    *hi = *lo + len < e ? *lo + len : e;
}

// kSmall (batches of a few thousand keys per service, StoredSpanJob's per-batch sketches): the
// counters stay in global memory -- the sketch adds to them with global atomics, the candidate and
// merge passes estimate from them -- instead of a 4 x width row block per unit moved through LDS (the
// per-unit fixed cost that dominated small batches: 64 KB in, 64 KB flushed, per service and batch).
// The sums and the estimates are the same integers either way.
template <bool kSmall>
__global__ __launch_bounds__(kKvWG) void k_kv_sketch(KvArgs a) {
    extern __shared__ uint32_t cm_lds[];
    const uint32_t u = blockIdx.x;
    if (u >= a.unit_base[a.S]) return;
    const uint32_t s = find_service(a.unit_base, a.S, u);
    uint64_t lo, hi;
    unit_range(a, s, u, &lo, &hi);
    const uint32_t cells = a.depth * a.width;
    uint32_t* const g = a.cm + (uint64_t)s * cells;
    uint32_t* const cm = kSmall ? g : cm_lds;
    if constexpr (!kSmall) {
        for (uint32_t x = threadIdx.x; x < cells; x += kKvWG) cm[x] = 0u;
        __syncthreads();
    }
    // two alternating 4-key buffers (C4 sketch 2.00 -> 1.96-1.97 ms; the pass is LDS-atomic-bound,
    // profiles/r02/ab_kv_sketch_pipe.txt)
    constexpr int U = 4;
    constexpr uint64_t BS = (uint64_t)kKvWG * U;
    auto load = [&](uint64_t (&k)[U], uint64_t b) {
#pragma unroll
        for (int e = 0; e < U; ++e) {
            const uint64_t i = b + (uint64_t)e * kKvWG + threadIdx.x;
            k[e] = a.keys[i < hi ? i : lo];
        }
    };
    // Under a skewed key distribution several lanes of one atomic instruction hold the same hot key and
    // their adds to the same counters serialise in LDS. Each wave tracks one hot key (wave-uniform):
    // the lanes holding it are counted by a ballot and their first lane adds the count. The hot key
    // is learned on the fly: every instruction also tests the key of a rotating lane and adopts it
    // when more lanes hold it. (Only which lane adds what changes: every counter gets the same total.)
    const int lane = threadIdx.x & 63;
    uint64_t hot = ~0ull;
    int probe = 0;
    auto add = [&](const uint64_t (&k)[U], uint64_t b) {
        // row hashes unconditionally, so the loads are not sunk into the conditional (see candidates)
        RowHash rh[U];
#pragma unroll
        for (int e = 0; e < U; ++e) rh[e] = RowHash::from_hash(k[e], a.wbits);  // keys arrive hashed
#pragma unroll
        for (int e = 0; e < U; ++e) {
            const bool valid = b + (uint64_t)e * kKvWG + threadIdx.x < hi;
            const uint64_t cand = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(k[e] >> 32), probe) << 32) |
                                  (uint32_t)__builtin_amdgcn_readlane((uint32_t)k[e], probe);
            probe = (probe + 1) & 63;
            uint64_t mh = __ballot(valid && k[e] == hot);
            const uint64_t mc = __ballot(valid && k[e] == cand);
            if (__popcll(mc) > __popcll(mh)) {
                hot = cand;
                mh = mc;
            }
            const bool in = (mh >> lane) & 1ull;
            const uint32_t inc = in ? (lane == __ffsll((unsigned long long)mh) - 1 ? (uint32_t)__popcll(mh) : 0u)
                                    : (valid ? 1u : 0u);
            if (inc)
                for (uint32_t r = 0; r < a.depth; ++r) atomicAdd(&cm[r * a.width + rh[e].next()], inc);
        }
    };
    uint64_t ka[U], kb[U];
    load(ka, lo);
    for (uint64_t b = lo; b < hi; b += 2 * BS) {
        load(kb, b + BS);
        add(ka, b);
        load(ka, b + 2 * BS);
        add(kb, b + BS);  // past hi: every key is masked
    }
    if constexpr (!kSmall) {
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < cells; x += kKvWG) {
            const uint32_t v = cm[x];
            if (v) atomicAdd(&g[x], v);
        }
    }
    if (threadIdx.x == 0) atomicAdd((unsigned long long*)&a.totals[s], (unsigned long long)(hi - lo));
}

__device__ void load_cm(uint32_t* cm, const KvArgs& a, uint32_t s) {
    const uint32_t cells = a.depth * a.width;
    const uint32_t* g = a.cm + (uint64_t)s * cells;
    for (uint32_t x = threadIdx.x; x < cells; x += kKvWG) cm[x] = g[x];
}

template <bool kSmall>
#if ZK_KV_CAND_WAVES
__global__ __launch_bounds__(kKvWG, ZK_KV_CAND_WAVES) void k_kv_candidates(KvArgs a) {
#else
__global__ __launch_bounds__(kKvWG) void k_kv_candidates(KvArgs a) {
#endif
    extern __shared__ uint32_t cm_lds[];
    __shared__ TopSet t;
    const uint32_t u = blockIdx.x;
    if (u >= a.unit_base[a.S]) return;
    const uint32_t s = find_service(a.unit_base, a.S, u);
    uint64_t lo, hi;
    unit_range(a, s, u, &lo, &hi);
    const uint32_t* const cm = kSmall ? a.cm + (uint64_t)s * a.depth * a.width : cm_lds;
    if constexpr (!kSmall) load_cm(cm_lds, a, s);
    ts_init(t);  // contains the barrier that publishes cm
    // Blocks of J = 8 keys per thread (4096 per workgroup), in two alternating key buffers: one
    // block's loads are in flight while the other is processed (a register ring carried across the
    // back edge instead makes the compiler copy it at the loop head, waiting for every load in
    // flight). Per block: every key is estimated and filtered against the current threshold and the
    // set (read-only probes: under a skewed key distribution most survivors are already in the set);
    // the survivors are counted (B1) and, when they fit the sort buffer, inserted at once (B2) --
    // two barriers per block instead of one per workgroup of keys. A block with too many survivors
    // (the start of a unit) is inserted one workgroup of keys at a time with a compaction check in
    // between.
    constexpr int J = 2 * kPrefetch;
    constexpr uint64_t BS = (uint64_t)kKvWG * J;  // keys per block
    uint32_t rot = 0;  // this block's survivor counter
    if (threadIdx.x == 0) t.pending[0] = t.pending[1] = t.pending[2] = 0u;
    __syncthreads();
    auto load_block = [&](uint64_t (&kq)[J], uint64_t b) {
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint64_t i = b + (uint64_t)j * kKvWG + threadIdx.x;
            kq[j] = a.keys[i < hi ? i : lo];
        }
    };
    auto run_block = [&](const uint64_t (&kq)[J], uint64_t b) {
        // estimates unconditionally (clamped keys past the end are harmless): a load whose only
        // uses sit in a conditional block is sunk into it, and then every key waits for HBM
        uint32_t est[J], slot[J];
        {  // rows outer, keys inner: one loop step per row for all J keys (2.86-2.93 -> 2.49-2.52 ms)
            RowHash rh[J];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                rh[j] = RowHash::from_hash(kq[j], a.wbits);  // kq: the keys' hashes
                est[j] = 0xFFFFFFFFu;
                slot[j] = rh[j].set;
            }
            for (uint32_t r = 0; r < a.depth; ++r) {
                const uint32_t* row = cm + r * a.width;
#pragma unroll
                for (int j = 0; j < J; ++j) est[j] = min(est[j], row[rh[j].next()]);
            }
        }
        const uint32_t has_thr = t.has_thr, thr_est = t.thr_est;
        const uint64_t thr_key = t.thr_key;
        uint32_t need = 0;
        // the first slot of every key read at once (J independent LDS reads instead of J dependent
        // probe chains): under a skewed distribution most live keys sit in their first slot; only
        // a collision walks on. No insert runs between here and B1, so plain reads are final.
        uint64_t h0[J];
#pragma unroll
        for (int j = 0; j < J; ++j) h0[j] = t.hk[slot[j]];
        // Decisions as bit masks (no short-circuit branches: every divergent branch costs the scalar
        // unit exec-mask bookkeeping, and the pass was bound by scalar issue, profiles/r03/
        // ab_kv_candidates.txt). The first two probe slots of every key are read at once; only a
        // threshold tie (decided on the unhashed key), the sentinel key and a key whose two slots hold
        // other keys take a branch.
        uint64_t h1[J];
#pragma unroll
        for (int j = 0; j < J; ++j) h1[j] = t.hk[(slot[j] + 1) & (kSetCap - 1)];
        uint32_t live_m = 0, tie_m = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const bool valid = (b + (uint64_t)j * kKvWG + threadIdx.x < hi) & (est[j] != 0u);
            live_m |= (uint32_t)(valid & ((has_thr == 0u) | (est[j] > thr_est))) << j;
            tie_m |= (uint32_t)(valid & (has_thr != 0u) & (est[j] == thr_est)) << j;
        }
        if (tie_m) {
#pragma unroll
            for (int j = 0; j < J; ++j)
                if ((tie_m >> j) & 1u) live_m |= (uint32_t)(kv_key(kq[j], a.seeds[0]) < thr_key) << j;
        }
        uint32_t slow_m = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const bool special = kq[j] == kEmptyKey;
            const bool hit = (h0[j] == kq[j]) | ((h0[j] != kEmptyKey) & (h1[j] == kq[j]));
            const bool absent = (h0[j] == kEmptyKey) | ((h0[j] != kq[j]) & (h1[j] == kEmptyKey));
            const uint32_t lv = (live_m >> j) & 1u;
            need |= (lv & (uint32_t)(!special & absent & !hit)) << j;
            slow_m |= (lv & (uint32_t)(special | (!hit & !absent))) << j;
        }
        if (slow_m) {
#pragma unroll
            for (int j = 0; j < J; ++j)
                if (((slow_m >> j) & 1u) && !ts_contains(t, kq[j], kq[j] == kEmptyKey ? slot[j] : (slot[j] + 2) & (kSetCap - 1)))
                    need |= 1u << j;
        }
        // the next block's counter, last read right after the previous block's B1 (three counters: a
        // block without survivors skips B2, so a fast thread may add to the next block's counter
        // before a slow one has passed this block's B1)
        const uint32_t nxt = rot == 2u ? 0u : rot + 1u;
        if (threadIdx.x == 0) t.pending[nxt] = 0u;
        if (need) atomicAdd(&t.pending[rot], (uint32_t)__popc(need));
        __syncthreads();  // B1: survivors counted
        const uint32_t pend = t.pending[rot];
        rot = nxt;
        // no survivors (most blocks once the threshold has risen): the set, its count and the threshold
        // stay as they are, so the next block may filter at once (no B2)
        if (pend == 0u) return;
        if (t.count + pend > kSortCap && t.count > a.cand) ts_compact(t, a.cand, a.seeds[0]);
        if (t.count + pend <= kSortCap) {
            if (need) {  // (most threads insert nothing: one branch instead of J)
#pragma unroll
                for (int j = 0; j < J; ++j)
                    if (need & (1u << j)) ts_insert(t, kq[j], est[j], slot[j]);
            }
            __syncthreads();  // B2: the set and count are complete for the next block's filter
        } else {
#pragma unroll
            for (int j = 0; j < J; ++j) {
                for (uint32_t t0 = 0; t0 < (uint32_t)kKvWG; t0 += kInsStep) {
                    if (threadIdx.x - t0 < kInsStep && (need & (1u << j))) ts_insert(t, kq[j], est[j], slot[j]);
                    __syncthreads();
                    if (t.count > kSortCap - kInsStep) ts_compact(t, a.cand, a.seeds[0]);
                }
            }
        }
    };
    // two key buffers, alternating: the next block's loads are in flight while this one is
    // estimated and inserted (each buffer is loaded and consumed in fixed places, so nothing is
    // copied across the back edge)
    uint64_t ka[J], kb[J];
    load_block(ka, lo);
    for (uint64_t b = lo; b < hi; b += 2 * BS) {
        load_block(kb, b + BS);
        run_block(ka, b);
        load_block(ka, b + 2 * BS);
        if (b + BS < hi) run_block(kb, b + BS);
    }
    const uint32_t n = ts_sort(t, a.seeds[0]);
    uint64_t* ok = a.unit_key + (uint64_t)u * a.cand;
    uint32_t* oe = a.unit_est + (uint64_t)u * a.cand;
    for (uint32_t x = threadIdx.x; x < a.cand; x += kKvWG) {
        ok[x] = x < n ? t.sk[x] : 0ull;
        oe[x] = x < n ? t.se[x] : 0u;
    }
}

// one workgroup per service: previous candidates + this batch's unit lists (+ extra lists)
template <bool kSmall>
__global__ __launch_bounds__(kKvWG) void k_kv_merge(KvArgs a, uint32_t use_units) {
    extern __shared__ uint32_t cm_lds[];
    __shared__ TopSet t;
    const uint32_t s = blockIdx.x;
    const uint32_t* const cm = kSmall ? a.cm + (uint64_t)s * a.depth * a.width : cm_lds;
    if constexpr (!kSmall) load_cm(cm_lds, a, s);
    ts_init(t);
    const uint32_t C = a.cand;
    const uint32_t u0 = use_units ? a.unit_base[s] : 0, u1 = use_units ? a.unit_base[s + 1] : 0;
    // flattened source list: [prev | units u0..u1 | extra lists], each C entries
    const uint64_t nsrc = (uint64_t)(1 + (u1 - u0) + a.extra_lists) * C;
    for (uint64_t b = 0; b < nsrc; b += kRound) {
#pragma unroll
        for (int e = 0; e < (int)((kRound + kKvWG - 1) / kKvWG); ++e) {
            const uint64_t i = b + (uint64_t)e * kKvWG + threadIdx.x;
            if (i >= nsrc || (uint64_t)e * kKvWG + threadIdx.x >= kRound) continue;
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
            if (old) {
                const uint64_t h = kv_hash(key, a.seeds[0]);
                ts_offer(t, key, h, estimate_rh(cm, a, RowHash::from_hash(h, a.wbits)));
            }
        }
        __syncthreads();
        if (t.count > kSortCap - kRound) ts_compact(t, C, a.seeds[0]);
    }
    const uint32_t n = ts_sort(t, a.seeds[0]);
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

hipError_t launch_kv_sketch(const KvArgs& a, hipStream_t s, bool small) {
    if (!a.max_units) return hipSuccess;
    if (small) return launch_checked("k_kv_sketch", k_kv_sketch<true>, dim3(a.max_units), dim3(kKvWG), 0, s, a);
    return launch_checked("k_kv_sketch", k_kv_sketch<false>, dim3(a.max_units), dim3(kKvWG),
                          (size_t)a.depth * a.width * 4, s, a);
}

hipError_t launch_kv_candidates(const KvArgs& a, hipStream_t s, bool small) {
    if (!a.max_units) return hipSuccess;
    if (small)
        return launch_checked("k_kv_candidates", k_kv_candidates<true>, dim3(a.max_units), dim3(kKvWG), 0, s, a);
    return launch_checked("k_kv_candidates", k_kv_candidates<false>, dim3(a.max_units), dim3(kKvWG),
                          (size_t)a.depth * a.width * 4, s, a);
}

hipError_t launch_kv_merge(const KvArgs& a, hipStream_t s, bool small) {
    if (small) return launch_checked("k_kv_merge", k_kv_merge<true>, dim3(a.S), dim3(kKvWG), 0, s, a, a.max_units ? 1u : 0u);
    return launch_checked("k_kv_merge", k_kv_merge<false>, dim3(a.S), dim3(kKvWG), (size_t)a.depth * a.width * 4, s, a,
                          a.max_units ? 1u : 0u);
}

hipError_t launch_kv_estimate(const KvArgs& a, uint32_t svc, const uint64_t* keys, uint64_t n, uint32_t* est,
                              hipStream_t s) {
    if (!n) return hipSuccess;
    return launch_checked("k_kv_estimate", k_kv_estimate, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, svc,
                          keys, n, est);
}

}  // namespace zk
