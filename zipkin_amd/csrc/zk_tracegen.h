// zk_tracegen.h — counter-based restatement of zipkin-tracegen's workload shape.
//
// Follows zipkin-tracegen/src/main/scala/com/twitter/zipkin/tracegen/TraceGen.scala:
//   :53-59   per trace: start = now - U{1..8} h, root depth U{0..maxDepth-1}, root service
//   :69-88   withEndpoint: a service not already on the call path (loop avoidance)
//   :90-142  doRpc: sr at t+1ms, 1-3 binary annotations, U{0..9} ms of work, 2-6 custom
//            annotations each followed by U{0..4} ms, U{2..depth+1} parallel downstream calls
//            (client fragment cs at cur+delay, delay = U{0..9} us with p = 0.3, cr at the
//            callee's return + 1 ms, both carrying the CALLEE's endpoint), ss at the max return.
// Records are emitted in TraceGen's own order (each client fragment right after its callee's
// subtree, the server fragment after all its calls: post-order), so a trace is contiguous.
//
// Differences from TraceGen, all deliberate and documented in DESIGN.md:
//  - java.util.Random is replaced by a per-trace splitmix64 stream keyed by (seed, traceId) so
//    that the host and the device produce bit-identical records in parallel;
//  - when loop avoidance fails after S attempts TraceGen invents a new suffixed name (:80-81);
//    here the first service id not on the path is taken (ids must stay < S);
//  - traceIds are a bijection of (seed, trace index, shard) so that they are unique and
//    zk_trace_shard(traceId, world) == rank.
//
// Shared by the device generator kernel (zkagg.hip) and the host generator; ZK_HD marks the
// functions for both sides when compiled by hipcc.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ZK_HD __host__ __device__ __forceinline__
#else
#define ZK_HD static inline
#endif

#define ZK_TG_MAX_DEPTH 16

ZK_HD uint64_t zk_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

ZK_HD uint64_t zk_unmix64(uint64_t z) {
    z = z ^ (z >> 31) ^ (z >> 62);
    z *= 0x319642B2D24D8EC3ull;
    z = z ^ (z >> 27) ^ (z >> 54);
    z *= 0x96DE1B173F119089ull;
    z = z ^ (z >> 30) ^ (z >> 60);
    return z;
}

ZK_HD uint32_t zk_shard_of(uint64_t trace_id, uint32_t world) {
    return world <= 1 ? 0u : (uint32_t)(zk_mix64(trace_id) % world);
}

// traceId for trace k of shard (rank, world): v = world * u + rank with u unique per (seed, k),
// traceId = mix64^-1(v)  =>  mix64(traceId) % world == rank and traceIds are pairwise distinct.
ZK_HD uint64_t zk_tg_trace_id(uint64_t seed, uint64_t k, uint32_t rank, uint32_t world) {
    const uint64_t w = world ? world : 1;
    const uint64_t u = (k & ((1ull << 40) - 1)) | ((zk_mix64(seed) & 0xFFFFull) << 40);
    return zk_unmix64(u * w + rank);
}

// Global trace set (zk_tracegen_params.global_ids): trace k of ONE set shared by every world size,
// traceId = mix64^-1(v) with v = k | (seed bits << 40) unique per (seed, k). Its shard is
// mix64(traceId) % world = v % world, so shard (rank, world) owns the traces k = k0, k0 + world, ...
// with k0 = the first k >= 0 whose v % world == rank: the same records for every world, split.
ZK_HD uint64_t zk_tg_global_v(uint64_t seed, uint64_t k) {
    return (k & ((1ull << 40) - 1)) | ((zk_mix64(seed) & 0xFFFFull) << 40);
}
ZK_HD uint64_t zk_tg_global_trace_id(uint64_t seed, uint64_t k) { return zk_unmix64(zk_tg_global_v(seed, k)); }
// first global trace of shard (rank, world)
ZK_HD uint64_t zk_tg_global_k0(uint64_t seed, uint32_t rank, uint32_t world) {
    const uint64_t w = world ? world : 1;
    const uint64_t base = zk_tg_global_v(seed, 0) % w;  // v(k) % w = (base + k) % w for k < 2^40
    return ((uint64_t)rank + w - base) % w;
}

struct zk_rng {
    uint64_t s;
};

ZK_HD uint64_t zk_rng_next(zk_rng* r) {
    r->s += 0x9E3779B97F4A7C15ull;
    return zk_mix64(r->s);
}

// uniform in [0, bound) (bound >= 1), multiply-shift on the high 32 bits
ZK_HD uint32_t zk_rng_below(zk_rng* r, uint32_t bound) {
    return (uint32_t)(((zk_rng_next(r) >> 32) * (uint64_t)bound) >> 32);
}

struct zk_tg_rec {
    uint64_t trace_id, span_id, parent_id;
    int64_t first_ts, last_ts;
    uint32_t service_id, flags;
};

struct zk_tg_frame {
    uint64_t span_id, parent_id;
    int64_t sr_ts, cur, maxt;
    // pending downstream call (client fragment of the child being generated)
    uint64_t pend_child;
    int64_t pend_cs;
    uint32_t pend_svc;
    uint32_t svc, depth, nchild, child_idx, has_parent;
};

// TraceGen.withEndpoint service choice (TraceGen.scala:70-88) against the services on the path.
ZK_HD uint32_t zk_tg_pick_service(zk_rng* r, uint32_t S, const zk_tg_frame* stk, int sp) {
    uint32_t svc = zk_rng_below(r, S);
    uint32_t attempts = S;
    for (;;) {
        bool on_path = false;
        for (int i = 0; i < sp; ++i) on_path |= (stk[i].svc == svc);
        if (!on_path) return svc;
        if (attempts == 0) break;
        svc = zk_rng_below(r, S);
        --attempts;
    }
    // deterministic replacement for TraceGen's "new suffixed name"
    for (uint32_t c = 0; c < S; ++c) {
        bool on_path = false;
        for (int i = 0; i < sp; ++i) on_path |= (stk[i].svc == c);
        if (!on_path) return c;
    }
    return svc;  // S <= path length: a repeat is unavoidable
}

// doRpc prologue (TraceGen.scala:98-115): sr, binary annotations, work, custom annotations.
ZK_HD void zk_tg_enter(zk_rng* r, zk_tg_frame* f, int64_t time, uint32_t depth, uint32_t svc,
                       uint64_t span_id, uint64_t parent_id, uint32_t has_parent) {
    f->span_id = span_id;
    f->parent_id = parent_id;
    f->has_parent = has_parent;
    f->svc = svc;
    f->depth = depth;
    int64_t cur = time + 1000;                         // time + 1.millisecond
    f->sr_ts = cur;                                    // SERVER_RECV
    const uint32_t nbin = zk_rng_below(r, 3) + 1;      // (0 to nextInt(3)) binary annotations
    for (uint32_t b = 0; b < nbin; ++b) {
        (void)zk_rng_next(r);                          // key word, value word
    }
    cur += (int64_t)zk_rng_below(r, 10) * 1000;        // work: nextInt(10) ms
    const uint32_t ncustom = zk_rng_below(r, 5) + 2;   // (0 to nextInt(5)+1) custom annotations
    for (uint32_t a = 0; a < ncustom; ++a) {
        cur += (int64_t)zk_rng_below(r, 5) * 1000;     // annotation at cur, then += nextInt(5) ms
    }
    f->cur = cur;
    f->maxt = cur;
    f->nchild = depth > 0 ? zk_rng_below(r, depth) + 2 : 0;  // (0 to nextInt(depth)+1)
    f->child_idx = 0;
}

// Generate one trace with the given traceId; Emit is called once per span fragment, in TraceGen
// order. Returns the number of fragments. The trace's content depends on (seed, traceId) only.
template <class Emit>
ZK_HD uint32_t zk_tg_trace_body(uint64_t seed, uint64_t trace_id, uint32_t max_depth, uint32_t S, int64_t base_ts,
                                Emit& emit) {
    zk_rng r;
    r.s = zk_mix64(seed ^ zk_mix64(trace_id ^ 0x5DEECE66Dull));
    zk_tg_frame stk[ZK_TG_MAX_DEPTH + 1];
    int sp = 0;
    uint32_t nrec = 0;
    const int64_t start = base_ts - (int64_t)(zk_rng_below(&r, 8) + 1) * 3600000000ll;
    const uint32_t depth0 = zk_rng_below(&r, max_depth);
    const uint32_t svc0 = zk_tg_pick_service(&r, S, stk, 0);
    zk_tg_enter(&r, &stk[0], start, depth0, svc0, zk_rng_next(&r), 0, 0);
    sp = 1;
    while (sp > 0) {
        zk_tg_frame* f = &stk[sp - 1];
        if (f->child_idx < f->nchild) {
            // withEndpoint { nextEp => ... } (TraceGen.scala:119-134)
            const uint32_t nsvc = zk_tg_pick_service(&r, S, stk, sp);
            const uint64_t child = zk_rng_next(&r);
            const int64_t delay = (zk_rng_below(&r, 10) > 6) ? (int64_t)zk_rng_below(&r, 10) : 0;
            f->pend_child = child;
            f->pend_cs = f->cur + delay;               // CLIENT_SEND at curTime + delay
            f->pend_svc = nsvc;
            const uint32_t cdepth = zk_rng_below(&r, f->depth);
            zk_tg_enter(&r, &stk[sp], f->cur, cdepth, nsvc, child, f->span_id, 1);
            ++sp;
            continue;
        }
        if (f->nchild > 0) f->cur = f->maxt;           // curTime = times.max
        zk_tg_rec rec;
        rec.trace_id = trace_id;
        rec.span_id = f->span_id;
        rec.parent_id = f->parent_id;
        rec.first_ts = f->sr_ts;
        rec.last_ts = f->cur;                          // SERVER_SEND
        rec.service_id = f->svc;
        rec.flags = (f->has_parent ? 1u : 0u) | (1u << 1) | (1u << 3) | (1u << 12) | (1u << 14);
        emit(rec);
        ++nrec;
        const int64_t ret = f->cur;
        --sp;
        if (sp == 0) break;
        zk_tg_frame* p = &stk[sp - 1];
        const int64_t t = ret + 1000;                  // doRpc(...) + 1.millisecond
        rec.span_id = p->pend_child;
        rec.parent_id = p->span_id;
        rec.first_ts = p->pend_cs;                     // CLIENT_SEND
        rec.last_ts = t;                               // CLIENT_RECV
        rec.service_id = p->pend_svc;                  // callee endpoint (TraceGen.scala:127,129)
        rec.flags = 1u | (1u << 1) | (1u << 2) | (1u << 8) | (1u << 10);
        emit(rec);
        ++nrec;
        if (t > p->maxt) p->maxt = t;                  // times.max (every t > the call's start)
        p->child_idx++;
    }
    return nrec;
}

// trace k of shard (rank, world): a per-shard traceId (zk_tg_trace_id), or trace k of the global set
// (zk_tg_global_trace_id) when `global` -- then k is the global trace index
template <class Emit>
ZK_HD uint32_t zk_tg_trace(uint64_t seed, uint64_t k, uint32_t rank, uint32_t world, uint32_t max_depth, uint32_t S,
                           int64_t base_ts, Emit& emit, bool global = false) {
    const uint64_t trace_id = global ? zk_tg_global_trace_id(seed, k) : zk_tg_trace_id(seed, k, rank, world);
    return zk_tg_trace_body(seed, trace_id, max_depth, S, base_ts, emit);
}
