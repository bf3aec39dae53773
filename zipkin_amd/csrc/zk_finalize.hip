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
// are evaluated in 512-bit integers and divided with one round-to-nearest-even: the result is the
// correctly rounded value of the exact moments, independent of order, GPU count and batching.
#include "zk_internal.h"

namespace zk {
namespace {

constexpr int W = 8;  // 512-bit
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
__device__ U512 u_mul(const U512& a, const U512& b) {
    U512 r = u_zero();
    for (int i = 0; i < W; ++i) {
        if (a.w[i] == 0) continue;
        uint64_t carry = 0;
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
    for (int i = W - 1; i >= 0; --i) {
        if (a.w[i]) return 64 * i + 64 - __clzll((long long)a.w[i]);
    }
    return 0;
}

__device__ U512 u_shl(const U512& a, int s) {
    U512 r = u_zero();
    const int ws = s >> 6, bs = s & 63;
    for (int i = W - 1; i >= ws; --i) {
        uint64_t v = a.w[i - ws] << bs;
        if (bs && i - ws - 1 >= 0) v |= a.w[i - ws - 1] >> (64 - bs);
        r.w[i] = v;
    }
    return r;
}

__device__ __forceinline__ void u_shr1(U512& a) {
#pragma unroll
    for (int i = 0; i < W - 1; ++i) a.w[i] = (a.w[i] >> 1) | (a.w[i + 1] << 63);
    a.w[W - 1] >>= 1;
}

// sum_k limb[k] * 2^(32k)
__device__ __forceinline__ U512 from_chunks(const uint64_t* limb, int nchunks) {
    U512 r = u_zero();
    for (int k = 0; k < nchunks; ++k) {
        U512 t = u_zero();
        t.w[0] = limb[k];
        r = u_add(r, u_shl(t, 32 * k));
    }
    return r;
}

// correctly rounded (RNE) value of A / D for A, D > 0
__device__ double div_round(U512 A, U512 D) {
    if (u_is_zero(A)) return 0.0;
    const int a = u_bitlen(A), b = u_bitlen(D);
    const int s = 58 - a + b;  // scale so that floor(A 2^s / D) is in [2^57, 2^59)
    if (s >= 0)
        A = u_shl(A, s);
    else
        D = u_shl(D, -s);
    U512 Dsh = u_shl(D, 58);
    uint64_t q = 0;
    for (int i = 58; i >= 0; --i) {
        if (u_cmp(A, Dsh) >= 0) {
            A = u_sub(A, Dsh);
            q |= 1ull << i;
        }
        u_shr1(Dsh);
    }
    const bool sticky = !u_is_zero(A);
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

__device__ double signed_ratio(const U512& P, const U512& Q, const U512& D) {
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
        const U512 S1 = from_chunks(L + kLimbS1, 2);
        const U512 S2 = from_chunks(L + kLimbS2, 3);
        const U512 S3 = from_chunks(L + kLimbS3, 4);
        const U512 S4 = from_chunks(L + kLimbS4, 5);
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
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, table, cells,
                       out->m0, out->m1, out->m2, out->m3, out->m4, out->present);
    return hipGetLastError();
}

}  // namespace zk
