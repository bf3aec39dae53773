// Microbenchmark: how fast can scattered u64 adds into a 32 MB link table go on MI355X?
// Decides the link-reduce design. Not product code.
//   A  device-scope atomicAdd, one lane per (cell, limb), 11 limbs per link, random cells
//   B  device-scope atomicAdd, 16 lanes cooperate on one 128-B cell (4 links per wave-instr)
//   C  workgroup-scope atomics into a per-XCD copy of the table (XCC_ID from the hardware)
//   D  same as C, cooperative 16-lane cells
//   E  plain scattered 8-B stores (no atomics) for reference
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return (uint32_t)x;
}

__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 7;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_links(uint64_t* table, uint64_t cells, uint64_t links, uint64_t copy_stride) {
    const uint64_t gtid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    uint64_t* base = table;
    if (MODE == 2 || MODE == 3) base = table + (uint64_t)xcc_id() * copy_stride;
    if (MODE == 0 || MODE == 2 || MODE == 4) {
        for (uint64_t l = gtid; l < links; l += nthreads) {
            const uint32_t cell = hash32(l * 0x9E3779B97F4A7C15ull) % cells;
            const uint64_t d = 1000 + (l & 1023);
            uint64_t* c = base + (uint64_t)cell * 16;
#pragma unroll
            for (int k = 0; k < 11; ++k) {
                if (MODE == 0) atomicAdd((unsigned long long*)&c[k], (unsigned long long)(d + k));
                else if (MODE == 2) __hip_atomic_fetch_add((unsigned long long*)&c[k], (unsigned long long)(d + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else c[k] = d + k;
            }
        }
    } else {
        // 16 lanes per link: lane q of the group handles limb q (q < 11)
        const int q = threadIdx.x & 15;
        const uint64_t g = gtid >> 4, ng = nthreads >> 4;
        for (uint64_t l = g; l < links; l += ng) {
            const uint32_t cell = hash32(l * 0x9E3779B97F4A7C15ull) % cells;
            const uint64_t d = 1000 + (l & 1023);
            uint64_t* c = base + (uint64_t)cell * 16;
            if (q < 11) {
                if (MODE == 1) atomicAdd((unsigned long long*)&c[q], (unsigned long long)(d + q));
                else __hip_atomic_fetch_add((unsigned long long*)&c[q], (unsigned long long)(d + q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
}

int main() {
    const uint64_t cells = 250000, links = 50000000;
    const uint64_t stride = cells * 16;
    uint64_t* t;
    CHECK(hipMalloc(&t, stride * 8 * 8));
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const char* names[] = {"A dev-scope lane/limb", "B dev-scope 16-lane cell", "C wg-scope per-XCD lane/limb",
                           "D wg-scope per-XCD 16-lane", "E plain scattered stores"};
    for (int mode = 0; mode < 5; ++mode) {
        std::vector<float> ts;
        for (int rep = 0; rep < 4; ++rep) {
            CHECK(hipMemset(t, 0, stride * 8 * 8));
            CHECK(hipEventRecord(a));
            dim3 grid(256 * 8), blk(256);
            switch (mode) {
                case 0: hipLaunchKernelGGL(k_links<0>, grid, blk, 0, 0, t, cells, links, stride); break;
                case 1: hipLaunchKernelGGL(k_links<1>, grid, blk, 0, 0, t, cells, links, stride); break;
                case 2: hipLaunchKernelGGL(k_links<2>, grid, blk, 0, 0, t, cells, links, stride); break;
                case 3: hipLaunchKernelGGL(k_links<3>, grid, blk, 0, 0, t, cells, links, stride); break;
                case 4: hipLaunchKernelGGL(k_links<4>, grid, blk, 0, 0, t, cells, links, stride); break;
            }
            CHECK(hipGetLastError());
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms; hipEventElapsedTime(&ms, a, b); ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        // correctness of the per-XCD copies: sum of limb 0 across copies must be sum over links of d
        std::vector<uint64_t> h(stride * 8);
        CHECK(hipMemcpy(h.data(), t, stride * 8 * 8, hipMemcpyDeviceToHost));
        unsigned __int128 s = 0;
        for (int x = 0; x < 8; ++x) for (uint64_t c = 0; c < cells; ++c) s += h[x * stride + c * 16];
        unsigned __int128 want = 0;
        for (uint64_t l = 0; l < links; ++l) want += 1000 + (l & 1023);
        printf("%-32s median %.3f ms  min %.3f ms  -> %.2e links/s  limb0 sum %s\n", names[mode], ts[ts.size() / 2], ts[0],
               links / (ts[0] * 1e-3), mode == 4 ? "n/a" : (s == want * 4 ? "ok(x4 reps)" : (s == want ? "ok" : "MISMATCH")));
    }
    return 0;
}
