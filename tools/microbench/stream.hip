// Microbenchmark: achievable HBM read bandwidth for a 4.8 GB columnar read (the K1 input size),
// 16 B per lane, grid-stride, result folded so nothing is dead-code eliminated. Not product code.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ p, uint64_t n16, unsigned* out) {
    unsigned acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t bytes = 4800000000ull;
    uint4* p;
    unsigned* o;
    if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
    (void)hipMemset(p, 1, bytes);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int grid : {1024, 2048, 4096, 8192}) {
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, p, bytes / 16, o);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        printf("grid %5d: %.3f ms  %.0f GB/s\n", grid, best, bytes / (best * 1e-3) / 1e9);
    }
    return 0;
}
