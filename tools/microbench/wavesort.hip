// Microbenchmark (not product code): the cost floor of the north_star's K1 design -- a register
// bitonic sort of each wave's records by (trace segment, spanId) plus a binary-search parent join
// over the sorted lanes -- on the real C2 column stream, to set against K1's LDS hash (SURVEY §8,
// row N1; VERDICT r04 "Next round" 4).
//
// Each wave streams its own range in windows of 128 records (two per lane, 16-B pair loads of the
// traceId, spanId and parentId columns: 24 of K1's 48 B per record). Variants (template MODE):
//   0 stream:  loads + trace boundaries (ballots) + segment ids; values folded so nothing is dead
//   1 sort:    + a 128-element bitonic sort of the 64-bit keys (segment << 57 | spanId >> 7) with the
//              record index as payload; element i lives in lane i / 2, slot i % 2; partners across
//              lanes move by __shfl_xor (ds_bpermute / DPP), 28 compare-exchange stages
//   2 join:    + each record's parent found by a 7-step binary search of (segment, parentId) over
//              the sorted keys (a __shfl per probe), the found index folded
// Nothing merges fragments, validates spans or emits links: it is a lower bound on the sorted
// design's time, to compare with K1's full kernel time on the same batch.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const int lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int l) {
    const int lo = __shfl((int)(uint32_t)v, l), hi = __shfl((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_wavesort(const uint64_t* __restrict__ tid, const uint64_t* __restrict__ sid,
                                                   const uint64_t* __restrict__ pid, uint64_t n,
                                                   unsigned long long* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t per = (n + nwaves - 1) / nwaves;
    const uint64_t r0 = wave * per, r1 = r0 + per < n ? r0 + per : n;
    uint64_t acc = 0;
    for (uint64_t ws = r0 & ~1ull; ws < r1; ws += 128) {
        const uint64_t i = ws + 2 * lane;
        const uint64_t j = i < n ? i : 0;
        const ulonglong2 t = *reinterpret_cast<const ulonglong2*>(tid + j);
        const ulonglong2 s = *reinterpret_cast<const ulonglong2*>(sid + j);
        const ulonglong2 p = *reinterpret_cast<const ulonglong2*>(pid + j);
        // trace boundaries and segment ids (the position of the record's trace start in the window)
        uint64_t prev;
        {
            const int lo = __shfl_up((int)(uint32_t)t.y, 1), hi = __shfl_up((int)(uint32_t)(t.y >> 32), 1);
            prev = ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
            if (lane == 0) prev = ~t.x;
        }
        const uint64_t ev = __ballot(t.x != prev), od = __ballot(t.y != t.x);
        const uint64_t mask_le = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
        const uint64_t me = ev & mask_le, mo = od & ((1ull << lane) - 1ull);
        const int pe = me ? 2 * (63 - __clzll(me)) : -1, po = mo ? 2 * (63 - __clzll(mo)) + 1 : -1;
        const int seg0 = pe > po ? pe : po;
        const int seg1 = ((od >> lane) & 1ull) ? 2 * lane + 1 : seg0;
        if constexpr (MODE == 0) {
            acc += s.x ^ s.y ^ p.x ^ p.y ^ (uint64_t)(seg0 + 3 * seg1);
            continue;
        }
        uint64_t key[2] = {((uint64_t)(seg0 & 127) << 57) | (s.x >> 7), ((uint64_t)(seg1 & 127) << 57) | (s.y >> 7)};
        uint32_t val[2] = {(uint32_t)(2 * lane), (uint32_t)(2 * lane + 1)};
        // bitonic sort: element e = 2 * lane + slot
#pragma unroll
        for (int k = 2; k <= 128; k <<= 1) {
#pragma unroll
            for (int jj = k >> 1; jj >= 1; jj >>= 1) {
                if (jj == 1) {  // partner in the same lane
                    {
                        const int e0 = 2 * lane;
                        const bool up = (e0 & k) == 0;
                        const bool sw = up ? (key[0] > key[1]) : (key[0] < key[1]);
                        const uint64_t a = key[0], b = key[1];
                        const uint32_t va = val[0], vb = val[1];
                        key[0] = sw ? b : a;
                        key[1] = sw ? a : b;
                        val[0] = sw ? vb : va;
                        val[1] = sw ? va : vb;
                    }
                } else {
                    const int lm = jj >> 1;  // partner lane = lane ^ lm, same slot
#pragma unroll
                    for (int sl = 0; sl < 2; ++sl) {
                        const int e = 2 * lane + sl;
                        const uint64_t ok = shfl_xor64(key[sl], lm);
                        const uint32_t ov = (uint32_t)__shfl_xor((int)val[sl], lm);
                        const bool up = (e & k) == 0;
                        const bool lower = (e & jj) == 0;
                        // the lower element of an ascending pair keeps the min
                        const bool take_min = (up == lower);
                        const bool other_smaller = ok < key[sl] || (ok == key[sl] && ov < val[sl]);
                        const bool take = take_min ? other_smaller : !other_smaller;
                        key[sl] = take ? ok : key[sl];
                        val[sl] = take ? ov : val[sl];
                    }
                }
            }
        }
        if constexpr (MODE == 1) {
            acc += key[0] ^ key[1] ^ val[0] ^ ((uint64_t)val[1] << 32) ^ p.x ^ p.y;
            continue;
        }
        // binary search of each record's (segment, parentId) among the 128 sorted keys
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
            const int sg = sl ? seg1 : seg0;
            const uint64_t want = ((uint64_t)(sg & 127) << 57) | ((sl ? p.y : p.x) >> 7);
            int lo = 0;
#pragma unroll
            for (int step = 64; step >= 1; step >>= 1) {
                const int probe = lo + step - 1;  // element index
                const uint64_t k0 = shfl64(key[0], probe >> 1), k1 = shfl64(key[1], probe >> 1);
                const uint64_t kp = (probe & 1) ? k1 : k0;
                if (kp < want) lo += step;
            }
            const uint64_t k0 = shfl64(key[0], (lo & 127) >> 1), k1 = shfl64(key[1], (lo & 127) >> 1);
            const uint32_t v0 = (uint32_t)__shfl((int)val[0], (lo & 127) >> 1), v1 = (uint32_t)__shfl((int)val[1], (lo & 127) >> 1);
            const uint64_t kf = (lo & 1) ? k1 : k0;
            acc += (kf == want) ? (uint64_t)((lo & 1) ? v1 : v0) : 7ull;
        }
    }
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

}  // namespace

extern "C" int ws_run(const uint64_t* tid, const uint64_t* sid, const uint64_t* pid, uint64_t n, int mode,
                      unsigned long long* out, int grid, int reps, float* ms) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(k_wavesort<0>, dim3(grid), dim3(256), 0, 0, tid, sid, pid, n, out);
        else if (mode == 1) hipLaunchKernelGGL(k_wavesort<1>, dim3(grid), dim3(256), 0, 0, tid, sid, pid, n, out);
        else hipLaunchKernelGGL(k_wavesort<2>, dim3(grid), dim3(256), 0, 0, tid, sid, pid, n, out);
    };
    launch();
    hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    hipEventElapsedTime(ms, a, b);
    *ms /= reps;
    hipEventDestroy(a);
    hipEventDestroy(b);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
