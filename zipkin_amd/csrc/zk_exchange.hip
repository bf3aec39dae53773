// zk_exchange.hip — the packed exchange form of the exact link table for the N > 1 all-reduce.
//
// The accumulator (zk_internal.h) keeps S1..S4 as sums of 32-bit chunks in 15 u64 limbs per cell
// (128 B with padding): carry-free, so K1/K3 add without carries. For the cross-rank SUM of
// ZipkinAggregateJob.scala:39-43 (`.group.sum` / `.sum` across reducers) that is 32 MB at S = 500.
// zk_deps_partial instead carry-normalises every cell into 56-bit limbs -- m0 one, S1 two, S2 two,
// S3 three, S4 four: 12 u64 = 96 B per cell, 24 MB at S = 500 -- each < 2^56 except a sum's top limb,
// which holds that sum's bits above the others. With fewer than 2^32 records since reset and
// d < 2^40 us: S1 < 2^72 (top limb < 2^16), S2 < 2^112 (top limb = bits 56..111: up to 2^56 - 1, the
// tightest), S3 < 2^152 (top limb = bits 112..151 < 2^40), S4 < 2^192 (top limb = bits 168..191 <
// 2^24). Every limb is therefore <= 2^56 - 1 and a SUM all-reduce over up to 256 ranks never carries
// out of a u64 (256 x (2^56 - 1) < 2^64) -- 256 ranks is the hard limit, set by S2's top limb and by
// every low limb alike (tests/test_multirank.py sums 256 copies of the largest cell). zk_deps_note_merged
// rebuilds the exact sums from the summed limbs and writes them back into the accumulator in its own
// chunk layout.
#include "zk_internal.h"
#include "zk_launch.h"

namespace zk {
namespace {

constexpr int kXLimbs = 12;
// (offset, limbs) of m0, S1..S4 in the packed cell, and of S1..S4 in the accumulator's chunk layout
constexpr int kXOff[5] = {0, 1, 3, 5, 8};
constexpr int kXCnt[5] = {1, 2, 2, 3, 4};
constexpr int kCOff[5] = {kLimbM0, kLimbS1, kLimbS2, kLimbS3, kLimbS4};
constexpr int kCCnt[5] = {1, 2, 3, 4, 5};
constexpr uint64_t kM56 = (1ull << 56) - 1;

// 256-bit accumulator: w += x << shift (shift < 192)
__device__ __forceinline__ void add_shifted(uint64_t (&w)[4], uint64_t x, int shift) {
    const int q = shift >> 6, r = shift & 63;
    const uint64_t lo = r ? (x << r) : x;
    const uint64_t hi = r ? (x >> (64 - r)) : 0ull;
    unsigned __int128 s = (unsigned __int128)w[q] + lo;
    w[q] = (uint64_t)s;
    uint64_t c = (uint64_t)(s >> 64);
    if (q + 1 < 4) {
        s = (unsigned __int128)w[q + 1] + hi + c;
        w[q + 1] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
        for (int k = q + 2; k < 4; ++k) {
            s = (unsigned __int128)w[k] + c;
            w[k] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
    }
}

// bits [off, off + 64) of w (zero above 256)
__device__ __forceinline__ uint64_t bits_at(const uint64_t (&w)[4], int off) {
    const int q = off >> 6, r = off & 63;
    if (q >= 4) return 0ull;
    uint64_t v = w[q] >> r;
    if (r && q + 1 < 4) v |= w[q + 1] << (64 - r);
    return v;
}

__global__ __launch_bounds__(256) void k_table_pack(const uint64_t* __restrict__ table, uint64_t cells,
                                                     uint64_t* __restrict__ xchg) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c < cells) {
        const uint64_t* v = table + c * kLimbs;
        uint64_t* o = xchg + c * kXLimbs;
#pragma unroll
        for (int s = 0; s < 5; ++s) {
            uint64_t w[4] = {0, 0, 0, 0};
            for (int j = 0; j < kCCnt[s]; ++j) add_shifted(w, v[kCOff[s] + j], 32 * j);
            for (int i = 0; i < kXCnt[s]; ++i) {
                const uint64_t x = bits_at(w, 56 * i);
                o[kXOff[s] + i] = (i + 1 < kXCnt[s]) ? (x & kM56) : x;  // the top limb takes the rest
            }
        }
    }
    if (c < kStatTailWords) xchg[cells * kXLimbs + c] = table[cells * kLimbs + c];  // the counter tail
}

__global__ __launch_bounds__(256) void k_table_unpack(const uint64_t* __restrict__ xchg, uint64_t cells,
                                                       uint64_t* __restrict__ table) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c < cells) {
        const uint64_t* x = xchg + c * kXLimbs;
        uint64_t out[kLimbs];
#pragma unroll
        for (int s = 0; s < 5; ++s) {
            uint64_t w[4] = {0, 0, 0, 0};
            for (int i = 0; i < kXCnt[s]; ++i) add_shifted(w, x[kXOff[s] + i], 56 * i);
            for (int j = 0; j < kCCnt[s]; ++j) {
                const uint64_t b = bits_at(w, 32 * j);
                out[kCOff[s] + j] = (j + 1 < kCCnt[s]) ? (b & 0xFFFFFFFFull) : b;
            }
        }
        out[15] = 0ull;
        uint64_t* t = table + c * kLimbs;
#pragma unroll
        for (int j = 0; j < kLimbs; ++j) t[j] = out[j];
    }
    if (c < kStatTailWords) table[cells * kLimbs + c] = xchg[cells * kXLimbs + c];
}

}  // namespace

uint64_t exchange_bytes(uint32_t S) { return (uint64_t)S * S * kXLimbs * 8 + kStatTailWords * 8; }

hipError_t launch_table_pack(const uint64_t* table, uint32_t S, uint64_t* xchg, hipStream_t s) {
    const uint64_t cells = (uint64_t)S * S;
    const uint64_t n = cells > kStatTailWords ? cells : kStatTailWords;
    return launch_checked("k_table_pack", k_table_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, table,
                          cells, xchg);
}

hipError_t launch_table_unpack(const uint64_t* xchg, uint32_t S, uint64_t* table, hipStream_t s) {
    const uint64_t cells = (uint64_t)S * S;
    const uint64_t n = cells > kStatTailWords ? cells : kStatTailWords;
    return launch_checked("k_table_unpack", k_table_unpack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                          xchg, cells, table);
}

}  // namespace zk
