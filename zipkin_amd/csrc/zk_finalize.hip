// zk_finalize.hip — K5: exact power sums -> Algebird Moments (m0, m1..m4), rounded once.
//
// Algebird (algebird-core 0.8.1, not vendored; called from ZipkinAggregateJob.scala:35,40 and
// Dependencies.scala:41) represents a distribution as Moments(m0 = count, m1 = mean,
// m2 = sum (x-mean)^2, m3 = sum (x-mean)^3, m4 = sum (x-mean)^4) — the meaning is pinned by
// zipkinDependencies.thrift:24-30 and the accessors in zipkin-web momentAnnotations.js:6-11.
// The reference folds these pairwise in fp64 (MomentsGroup.plus), so its last bits depend on the
// reduce order. Here every cell holds the exact integer sums S1..S4 of d^k, and
//   m1 = S1/n
//   m2 = (n S2 - S1^2)/n
//   m3 = (n^2 S3 - 3 n S1 S2 + 2 S1^3)/n^2
//   m4 = (n^3 S4 - 4 n^2 S1 S3 + 6 n S1^2 S2 - 3 S1^4)/n^3
// are evaluated in 384-bit integers and divided with one round-to-nearest-even: the result is the
// correctly rounded value of the exact moments, independent of order, GPU count and batching.
#include "zk_internal.h"
#include "zk_launch.h"

namespace zk {
namespace {

constexpr int W = 6;  // 384-bit: every numerator is < 2^300 (n < 2^32, d < 2^40)
struct U512 {
    uint64_t w[W];
};

__device__ __forceinline__ U512 u_zero() {
    U512 r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = 0;
    return r;
}

__device__ __forceinline__ U512 u_add(const U512& a, const U512& b) {
    U512 r;
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        const uint64_t s = a.w[i] + b.w[i];
        const uint64_t c1 = s < a.w[i];
        r.w[i] = s + c;
        const uint64_t c2 = r.w[i] < s;
        c = c1 | c2;
    }
    return r;
}

__device__ __forceinline__ U512 u_sub(const U512& a, const U512& b) {  // a >= b
    U512 r;
    uint64_t br = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        const uint64_t d = a.w[i] - b.w[i];
        const uint64_t b1 = a.w[i] < b.w[i];
        r.w[i] = d - br;
        const uint64_t b2 = d < br;
        br = b1 | b2;
    }
    return r;
}

__device__ __forceinline__ int u_cmp(const U512& a, const U512& b) {
#pragma unroll
    for (int i = W - 1; i >= 0; --i) {
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
    }
    return 0;
}

__device__ __forceinline__ bool u_is_zero(const U512& a) {
    uint64_t o = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) o |= a.w[i];
    return o == 0;
}

// truncated product (inputs are small enough that nothing is lost)
__device__ __forceinline__ U512 u_mul(const U512& a, const U512& b) {
    U512 r = u_zero();
#pragma unroll
    for (int i = 0; i < W; ++i) {
        uint64_t carry = 0;
#pragma unroll
        for (int j = 0; i + j < W; ++j) {
            const unsigned __int128 p =
                (unsigned __int128)a.w[i] * b.w[j] + r.w[i + j] + carry;
            r.w[i + j] = (uint64_t)p;
            carry = (uint64_t)(p >> 64);
        }
    }
    return r;
}

__device__ __forceinline__ U512 u_mul_small(const U512& a, uint64_t m) {
    U512 r;
    uint64_t carry = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        const unsigned __int128 p = (unsigned __int128)a.w[i] * m + carry;
        r.w[i] = (uint64_t)p;
        carry = (uint64_t)(p >> 64);
    }
    return r;
}

__device__ __forceinline__ int u_bitlen(const U512& a) {
    int L = 0;
#pragma unroll
    for (int i = 0; i < W; ++i)
        if (a.w[i]) L = 64 * i + 64 - __clzll((long long)a.w[i]);
    return L;
}

// word shifts select among compile-time variants so the words stay in registers (a runtime
// word index would put the number in scratch)
__device__ __forceinline__ U512 u_shl(const U512& a, int s) {
    const int ws = s >> 6, bs = s & 63;
    U512 t = u_zero();
#pragma unroll
    for (int k = 0; k < W; ++k) {
        if (k == ws) {
#pragma unroll
            for (int i = 0; i < W; ++i) t.w[i] = i >= k ? a.w[i - k] : 0;
        }
    }
    if (!bs) return t;
    U512 r;
#pragma unroll
    for (int i = W - 1; i >= 0; --i) r.w[i] = (t.w[i] << bs) | (i ? t.w[i - 1] >> (64 - bs) : 0);
    return r;
}

__device__ __forceinline__ void u_shr1(U512& a) {
#pragma unroll
    for (int i = 0; i < W - 1; ++i) a.w[i] = (a.w[i] >> 1) | (a.w[i + 1] << 63);
    a.w[W - 1] >>= 1;
}

// sum_k limb[k] * 2^(32k)
template <int NCHUNKS>
__device__ __forceinline__ U512 from_chunks(const uint64_t* limb) {
    U512 r = u_zero();
#pragma unroll
    for (int k = 0; k < NCHUNKS; ++k) {
        // limb[k] * 2^(32k): word k/2, shifted by 32 if k is odd
        U512 t = u_zero();
        if (k & 1) {
            t.w[k / 2] = limb[k] << 32;
            if (k / 2 + 1 < W) t.w[k / 2 + 1] = limb[k] >> 32;
        } else {
            t.w[k / 2] = limb[k];
        }
        r = u_add(r, t);
    }
    return r;
}

__device__ __forceinline__ U512 u_shr(const U512& a, int s) {
    const int ws = s >> 6, bs = s & 63;
    U512 t = u_zero();
#pragma unroll
    for (int k = 0; k < W; ++k) {
        if (k == ws) {
#pragma unroll
            for (int i = 0; i < W; ++i) t.w[i] = i + k < W ? a.w[i + k] : 0;
        }
    }
    if (!bs) return t;
    U512 r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = (t.w[i] >> bs) | (i + 1 < W ? t.w[i + 1] << (64 - bs) : 0);
    return r;
}

// low `s` bits of a are all zero?
__device__ __forceinline__ bool u_low_zero(const U512& a, int s) {
    uint64_t o = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        const int rem = s - 64 * i;
        const uint64_t m = rem >= 64 ? ~0ull : (rem <= 0 ? 0ull : ((1ull << rem) - 1ull));
        o |= a.w[i] & m;
    }
    return o == 0;
}

__device__ __forceinline__ double u_to_double(const U512& a) {
    double x = 0.0;
    for (int i = W - 1; i >= 0; --i) x = x * 18446744073709551616.0 + (double)a.w[i];
    return x;
}

// correctly rounded (RNE) value of A / D for A, D > 0.
// Scale so that Q = floor(A 2^s / D) has 58..59 bits; when s < 0 the low -s bits of A are
// shifted out and kept as a sticky flag (floor(floor(A/2^k)/D) = floor(A/(2^k D))), so every
// operand stays below ~2^160. Q is found by double-precision estimates that never overshoot,
// each followed by an exact remainder update, then the 59-bit Q is rounded to 53 bits.
__device__ __forceinline__ double div_round(U512 A, const U512& D) {
    if (u_is_zero(A)) return 0.0;
    const int a = u_bitlen(A), b = u_bitlen(D);
    const int s = 58 - a + b;  // floor(A 2^s / D) in [2^57, 2^59)
    bool sticky = false;
    if (s >= 0) {
        A = u_shl(A, s);
    } else {
        sticky = !u_low_zero(A, -s);
        A = u_shr(A, -s);
    }
    const double dd = u_to_double(D);
    uint64_t q = 0;
    for (int it = 0; it < 4; ++it) {
        if (u_cmp(A, D) < 0) break;
        double t = u_to_double(A) / dd * (1.0 - 0x1p-48);
        uint64_t ti = t < 1.0 ? 1ull : (uint64_t)t;  // underestimate (>= 1: A >= D)
        A = u_sub(A, u_mul_small(D, ti));
        q += ti;
    }
    while (u_cmp(A, D) >= 0) {  // at most a couple of steps after the estimates
        A = u_sub(A, D);
        ++q;
    }
    sticky = sticky || !u_is_zero(A);
    const int L = 64 - __clzll((long long)q);  // 58 or 59
    int r = L - 53;
    uint64_t mant = q >> r;
    const uint64_t rem = q & ((1ull << r) - 1);
    const uint64_t half = 1ull << (r - 1);
    if (rem > half || (rem == half && (sticky || (mant & 1)))) ++mant;
    if (mant == (1ull << 53)) {
        mant >>= 1;
        ++r;
    }
    return ldexp((double)mant, r - s);
}

__device__ __forceinline__ double signed_ratio(const U512& P, const U512& Q, const U512& D) {
    const int c = u_cmp(P, Q);
    if (c == 0) return 0.0;
    if (c > 0) return div_round(u_sub(P, Q), D);
    return -div_round(u_sub(Q, P), D);
}

__global__ __launch_bounds__(256) void k_finalize(const uint64_t* __restrict__ table, uint64_t cells,
                                                  uint64_t* m0o, double* m1o, double* m2o, double* m3o,
                                                  double* m4o, uint8_t* pres) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cells) return;
    uint64_t L[kLimbs];
    const uint4* src = reinterpret_cast<const uint4*>(table + c * kLimbs);
#pragma unroll
    for (int i = 0; i < kLimbs / 2; ++i) {
        const uint4 v = src[i];
        L[2 * i] = (uint64_t)v.x | ((uint64_t)v.y << 32);
        L[2 * i + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
    const uint64_t n = L[kLimbM0];
    double m1 = 0, m2 = 0, m3 = 0, m4 = 0;
    if (n) {
        const U512 S1 = from_chunks<2>(L + kLimbS1);
        const U512 S2 = from_chunks<3>(L + kLimbS2);
        const U512 S3 = from_chunks<4>(L + kLimbS3);
        const U512 S4 = from_chunks<5>(L + kLimbS4);
        U512 N1 = u_zero();
        N1.w[0] = n;
        const U512 N2 = u_mul_small(N1, n);
        const U512 N3 = u_mul_small(N2, n);
        const U512 S1sq = u_mul(S1, S1);
        const U512 S1cu = u_mul(S1sq, S1);
        m1 = div_round(S1, N1);
        // m2 = (n S2 - S1^2) / n
        m2 = signed_ratio(u_mul_small(S2, n), S1sq, N1);
        // m3 = (n^2 S3 + 2 S1^3 - 3 n S1 S2) / n^2
        {
            const U512 P = u_add(u_mul(N2, S3), u_mul_small(S1cu, 2));
            const U512 Q = u_mul_small(u_mul(S1, S2), 3 * n);
            m3 = signed_ratio(P, Q, N2);
        }
        // m4 = (n^3 S4 + 6 n S1^2 S2 - 4 n^2 S1 S3 - 3 S1^4) / n^3
        {
            const U512 P = u_add(u_mul(N3, S4), u_mul_small(u_mul(S1sq, S2), 6 * n));
            const U512 Q = u_add(u_mul_small(u_mul(N2, u_mul(S1, S3)), 4), u_mul_small(u_mul(S1sq, S1sq), 3));
            m4 = signed_ratio(P, Q, N3);
        }
    }
    m0o[c] = n;
    m1o[c] = m1;
    m2o[c] = m2;
    m3o[c] = m3;
    m4o[c] = m4;
    pres[c] = n ? 1 : 0;
}

}  // namespace

hipError_t launch_finalize(const uint64_t* table, uint32_t S, const zk_link_table* out, hipStream_t s) {
    const uint64_t cells = (uint64_t)S * S;
    if (!cells) return hipSuccess;
    return launch_checked("k_finalize", k_finalize, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, table, cells,
                          out->m0, out->m1, out->m2, out->m3, out->m4, out->present);
}

}  // namespace zk
