// zk_rt.hip — realtime span sketches per service (include/zksketch.h, zk_rt_*):
// HyperLogLog registers of distinct traceIds and a log-linear histogram of span durations.
//
// The reference declares these aggregates without an implementation (RealtimeAggregates.scala:
// 26-38; QueryService.scala:416-430 answers "Not Implemented"). Items are produced per merged,
// valid span with a service name by K1 (zk_join.hip, MODE_EMIT) or from already-merged spans by
// k_rt_items below; they are partitioned by service (zk_partition.hip), then one workgroup per
// unit (<= 64k items of one service) keeps that service's registers and bins in LDS and merges
// them into the global sketch once: byte-wise MAX for registers, SUM for bins. Both merges are
// order-independent, so the sketch state is bit-identical for any batching or GPU count.
#include "zk_sketch_internal.h"
#include "zk_launch.h"

namespace zk {
namespace {

constexpr int kRtWG = 256;

__device__ __forceinline__ uint32_t find_unit_service(const uint32_t* __restrict__ unit_base, uint32_t S, uint32_t u) {
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

// byte-wise max of v into the byte lane `sh` of *w (LDS or global), CAS loop, skipped when no gain
template <class P>
__device__ __forceinline__ void max_byte(P* w, uint32_t sh, uint32_t v) {
    uint32_t old = *w;
    while (((old >> sh) & 0xFFu) < v) {
        const uint32_t nw = (old & ~(0xFFu << sh)) | (v << sh);
        const uint32_t prev = atomicCAS(w, old, nw);
        if (prev == old) break;
        old = prev;
    }
}

__device__ __forceinline__ uint32_t bytewise_max(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t x = (a >> (8 * k)) & 0xFFu, y = (b >> (8 * k)) & 0xFFu;
        r |= (x > y ? x : y) << (8 * k);
    }
    return r;
}

// (two alternating load buffers, as in the KV passes, measured within noise: pipelined C5 1.43-1.46
// vs 1.44-1.47 ms, serial equal, profiles/r02/ab_rt_sketch_pipe.txt -- one buffer kept)
__global__ __launch_bounds__(kRtWG) void k_rt_sketch(RtArgs a) {
    extern __shared__ uint32_t lds[];
    const uint32_t R = 1u << a.p;        // registers per service
    uint32_t* s_reg = lds;               // R / 4 words (4 registers per word)
    uint32_t* s_bin = lds + (R >> 2);    // nbins
    const uint32_t u = blockIdx.x;
    if (u >= a.unit_base[a.S]) return;
    const uint32_t s = find_unit_service(a.unit_base, a.S, u);
    const uint64_t lo = a.seg[s] + (uint64_t)(u - a.unit_base[s]) * a.unit_items;
    const uint64_t end = a.seg[s + 1];
    const uint64_t hi = lo + a.unit_items < end ? lo + a.unit_items : end;
    for (uint32_t x = threadIdx.x; x < (R >> 2); x += kRtWG) s_reg[x] = 0u;
    for (uint32_t x = threadIdx.x; x < a.nbins; x += kRtWG) s_bin[x] = 0u;
    __syncthreads();
    constexpr int U = 4;
    constexpr uint64_t BS = (uint64_t)kRtWG * U;
    auto load = [&](uint64_t (&v)[U], uint64_t b) {
#pragma unroll
        for (int e = 0; e < U; ++e) {
            const uint64_t i = b + (uint64_t)e * kRtWG + threadIdx.x;
            v[e] = a.items[i < hi ? i : lo];
        }
    };
    auto add = [&](const uint64_t (&v)[U], uint64_t b) {
#pragma unroll
        for (int e = 0; e < U; ++e) {
            if (b + (uint64_t)e * kRtWG + threadIdx.x >= hi) continue;
            const uint32_t idx = (uint32_t)(v[e] >> kRtPayShiftIdx);
            const uint32_t rho = (uint32_t)(v[e] >> kRtPayShiftRho) & 63u;
            const uint64_t d = v[e] & ((1ull << kRtPayShiftRho) - 1ull);
            max_byte(&s_reg[idx >> 2], 8u * (idx & 3u), rho);
            atomicAdd(&s_bin[rt_bin(d, a.m)], 1u);
        }
    };
    for (uint64_t b = lo; b < hi; b += BS) {
        uint64_t v[U];
        load(v, b);
        add(v, b);
    }
    __syncthreads();
    uint32_t* g_reg = (uint32_t*)(a.regs + (uint64_t)s * R);
    for (uint32_t x = threadIdx.x; x < (R >> 2); x += kRtWG) {
        const uint32_t v = s_reg[x];
        if (!v) continue;
        uint32_t old = g_reg[x];
        for (;;) {
            const uint32_t nw = bytewise_max(old, v);
            if (nw == old) break;
            const uint32_t prev = atomicCAS(&g_reg[x], old, nw);
            if (prev == old) break;
            old = prev;
        }
    }
    uint32_t* g_bin = a.hist + (uint64_t)s * a.nbins;
    for (uint32_t x = threadIdx.x; x < a.nbins; x += kRtWG) {
        const uint32_t c = s_bin[x];
        if (c) atomicAdd(&g_bin[x], c);
    }
}

__global__ void k_rt_items(const uint32_t* __restrict__ svc, const uint64_t* __restrict__ tid,
                           const int64_t* __restrict__ dur, uint64_t n, uint32_t S, uint32_t p, uint64_t seed,
                           uint32_t* __restrict__ out_svc, uint64_t* __restrict__ out_pay,
                           unsigned long long* dropped) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool bad_s = false, bad_d = false;
    if (i < n) {
        const uint32_t s = svc[i];
        const int64_t d = dur[i];
        bad_s = s >= S;
        bad_d = !bad_s && (d < 0 || (uint64_t)d >= (1ull << kRtPayShiftRho));
        out_svc[i] = (bad_s || bad_d) ? 0xFFFFFFFFu : s;
        out_pay[i] = (bad_s || bad_d) ? 0ull : rt_payload(tid[i], (uint64_t)d, p, seed);
    }
    const uint64_t ms = __ballot(bad_s), md = __ballot(bad_d);
    if ((threadIdx.x & 63) == 0) {
        if (ms) atomicAdd(&dropped[0], (unsigned long long)__popcll(ms));
        if (md) atomicAdd(&dropped[1], (unsigned long long)__popcll(md));
    }
}

// Queries of every service at once (zk_rt_distinct_traces, zk_rt_quantiles_all), one workgroup per
// service: the exact HyperLogLog sum z = sum_j 2^(64 - M[j]) as a 128-bit integer (from a count of
// each register value, so the result does not depend on the summation order) and the zero count;
// the histogram's total N; for each quantile q[i] the bin holding the nearest rank
// max(1, ceil(q N)). out row s: [z_lo, z_hi, zeros, N, bin_0 .. bin_{nq-1}]. The host finishes the
// estimate with the same double arithmetic as hll_estimate, so both give identical results.
__global__ __launch_bounds__(kRtWG) void k_rt_query(const uint8_t* __restrict__ regs, const uint32_t* __restrict__ hist,
                                                   uint32_t p, uint32_t nbins, const double* __restrict__ q, uint32_t nq,
                                                   unsigned long long* __restrict__ out) {
    __shared__ uint32_t cnt[65];
    __shared__ unsigned long long part[kRtWG];
    __shared__ unsigned long long s_n;
    const uint32_t s = blockIdx.x, t = threadIdx.x;
    if (t < 65) cnt[t] = 0u;
    __syncthreads();
    const uint32_t R = 1u << p;
    const uint32_t* rw = (const uint32_t*)(regs + (uint64_t)s * R);
    for (uint32_t x = t; x < (R >> 2); x += kRtWG) {
        const uint32_t w = rw[x];
#pragma unroll
        for (int k = 0; k < 4; ++k) atomicAdd(&cnt[(w >> (8 * k)) & 0xFFu], 1u);
    }
    // the histogram: each thread one contiguous chunk of bins
    const uint32_t chunk = (nbins + kRtWG - 1) / kRtWG;
    const uint32_t b0 = t * chunk < nbins ? t * chunk : nbins, b1 = b0 + chunk < nbins ? b0 + chunk : nbins;
    const uint32_t* h = hist + (uint64_t)s * nbins;
    unsigned long long local = 0;
    for (uint32_t b = b0; b < b1; ++b) local += h[b];
    part[t] = local;
    __syncthreads();
    unsigned long long* o = out + (uint64_t)s * (4u + nq);
    if (t == 0) {
        unsigned __int128 z = 0;
        for (int v = 0; v <= 64; ++v) z += (unsigned __int128)cnt[v] << (64 - v);
        unsigned long long N = 0;
        for (uint32_t k = 0; k < kRtWG; ++k) {  // exclusive prefix of the chunks, in place
            const unsigned long long c = part[k];
            part[k] = N;
            N += c;
        }
        o[0] = (unsigned long long)z;
        o[1] = (unsigned long long)(z >> 64);
        o[2] = cnt[0];
        o[3] = N;
        for (uint32_t i = 0; i < nq; ++i) o[4 + i] = 0ull;
        s_n = N;
    }
    __syncthreads();
    const unsigned long long N = s_n;
    if (N == 0) return;
    const unsigned long long excl = part[t];
    for (uint32_t i = 0; i < nq; ++i) {
        unsigned long long rank = (unsigned long long)ceil(q[i] * (double)N);
        if (rank < 1) rank = 1;
        if (rank > N) rank = N;
        if (excl < rank && excl + local >= rank) {
            unsigned long long cum = excl;
            for (uint32_t b = b0; b < b1; ++b) {
                cum += h[b];
                if (cum >= rank) {
                    o[4 + i] = b;
                    break;
                }
            }
        }
    }
}

}  // namespace

hipError_t launch_rt_query(const uint8_t* regs, const uint32_t* hist, uint32_t S, uint32_t p, uint32_t nbins,
                           const double* q, uint32_t nq, unsigned long long* out, hipStream_t s) {
    return launch_checked("k_rt_query", k_rt_query, dim3(S), dim3(kRtWG), 0, s, regs, hist, p, nbins, q, nq, out);
}

hipError_t launch_rt_sketch(const RtArgs& a, hipStream_t s) {
    if (!a.max_units) return hipSuccess;
    const size_t lds = (size_t)((1u << a.p) / 4 + a.nbins) * 4;
    return launch_checked("k_rt_sketch", k_rt_sketch, dim3(a.max_units), dim3(kRtWG), lds, s, a);
}

hipError_t launch_rt_items(const uint32_t* svc, const uint64_t* trace_id, const int64_t* dur, uint64_t n, uint32_t S,
                           uint32_t p, uint64_t seed, uint32_t* out_svc, uint64_t* out_pay,
                           unsigned long long* dropped, hipStream_t s) {
    if (!n) return hipSuccess;
    return launch_checked("k_rt_items", k_rt_items, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, svc, trace_id,
                          dur, n, S, p, seed, out_svc, out_pay, dropped);
}

}  // namespace zk
