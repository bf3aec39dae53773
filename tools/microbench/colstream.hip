// Microbenchmark: what K1's HBM access pattern alone reaches. 7 span columns (5 x u64, 2 x u32)
// of 1e8 records, 256-thread workgroups, 512-record windows, two records per thread (16-B / 8-B
// pair loads), values folded so nothing is dead. Variants:
//   contig   workgroup w streams its own contiguous range (K1 today: 4096 ranges, 7 streams each)
//   chunkK   ranges of K windows dealt round-robin to workgroups (fewer concurrent DRAM pages)
//   pre      + the next window's 7 columns loaded before this window's values are folded
// An LDS allocation of 40 KB holds occupancy at K1's 4 workgroups per CU. Not product code.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

struct Cols {
    const uint64_t *a, *b, *c, *d, *e;
    const uint32_t *f, *g;
    uint64_t n;
};

struct W {
    ulonglong2 a, b, c, d, e;
    uint2 f, g;
};

__device__ __forceinline__ void ld(const Cols& C, uint64_t i, W& w) {
    i = i < C.n ? i : 0;
    w.a = *reinterpret_cast<const ulonglong2*>(C.a + i);
    w.b = *reinterpret_cast<const ulonglong2*>(C.b + i);
    w.c = *reinterpret_cast<const ulonglong2*>(C.c + i);
    w.d = *reinterpret_cast<const ulonglong2*>(C.d + i);
    w.e = *reinterpret_cast<const ulonglong2*>(C.e + i);
    w.f = *reinterpret_cast<const uint2*>(C.f + i);
    w.g = *reinterpret_cast<const uint2*>(C.g + i);
}
__device__ __forceinline__ uint64_t fold(const W& w) {
    return w.a.x ^ w.a.y ^ w.b.x ^ w.b.y ^ w.c.x ^ w.c.y ^ w.d.x ^ w.d.y ^ w.e.x ^ w.e.y ^ w.f.x ^ w.f.y ^
           ((uint64_t)w.g.x << 32) ^ w.g.y;
}

// windows of 512 records; chunk = windows per dealt range (0: one contiguous range per workgroup)
template <bool PRE>
__global__ __launch_bounds__(256, 4) void k_cols(Cols C, uint64_t chunk, unsigned long long* out) {
    __shared__ uint64_t s_pad[40 * 1024 / 8];
    const uint64_t nwin = (C.n + 511) / 512;
    uint64_t acc = 0;
    uint64_t w0, w1, step;
    if (chunk == 0) {
        const uint64_t per = (nwin + gridDim.x - 1) / gridDim.x;
        w0 = blockIdx.x * per;
        w1 = w0 + per < nwin ? w0 + per : nwin;
        step = 0;
    } else {
        w0 = blockIdx.x * chunk;
        w1 = w0 + chunk;
        step = (uint64_t)gridDim.x * chunk;
    }
    for (; w0 < nwin; w0 += step, w1 += step) {
        const uint64_t e = w1 < nwin ? w1 : nwin;
        W cur, nxt;
        ld(C, w0 * 512 + 2 * threadIdx.x, cur);
        for (uint64_t w = w0; w < e; ++w) {
            if (PRE) {
                ld(C, (w + 1) * 512 + 2 * threadIdx.x, nxt);
                acc ^= fold(cur);
                cur = nxt;
            } else {
                if (w > w0) ld(C, w * 512 + 2 * threadIdx.x, cur);
                acc ^= fold(cur);
            }
        }
        if (step == 0) break;
    }
    s_pad[threadIdx.x] = acc;
    __syncthreads();
    if (s_pad[(threadIdx.x + 1) & 255] == 0x1234567890ull) out[0] = acc;
}

int main() {
    const uint64_t n = 100000000ull;
    void* base;
    const uint64_t bytes = n * 48 + 4096;
    unsigned long long* o;
    if (hipMalloc(&base, bytes) != hipSuccess || hipMalloc(&o, 8) != hipSuccess) return 1;
    (void)hipMemset(base, 1, bytes);
    char* p = (char*)base;
    Cols C;
    C.a = (const uint64_t*)p; p += n * 8;
    C.b = (const uint64_t*)p; p += n * 8;
    C.c = (const uint64_t*)p; p += n * 8;
    C.d = (const uint64_t*)p; p += n * 8;
    C.e = (const uint64_t*)p; p += n * 8;
    C.f = (const uint32_t*)p; p += n * 4;
    C.g = (const uint32_t*)p;
    C.n = n;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    struct V { const char* name; int grid; uint64_t chunk; bool pre; };
    const V vs[] = {
        {"contig g4096", 4096, 0, false}, {"contig g4096 pre", 4096, 0, true},
        {"contig g1024", 1024, 0, false}, {"contig g1024 pre", 1024, 0, true},
        {"chunk1 g1024", 1024, 1, false}, {"chunk8 g1024", 1024, 8, false}, {"chunk8 g1024 pre", 1024, 8, true},
        {"chunk32 g1024 pre", 1024, 32, true}, {"chunk8 g4096 pre", 4096, 8, true},
    };
    for (const V& v : vs) {
        float best = 1e9;
        for (int r = 0; r < 7; ++r) {
            (void)hipEventRecord(a);
            if (v.pre)
                hipLaunchKernelGGL(k_cols<true>, dim3(v.grid), dim3(256), 0, 0, C, v.chunk, o);
            else
                hipLaunchKernelGGL(k_cols<false>, dim3(v.grid), dim3(256), 0, 0, C, v.chunk, o);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            if (r > 0 && ms < best) best = ms;
        }
        printf("%-20s %.3f ms  %.0f GB/s\n", v.name, best, n * 48.0 / (best * 1e-3) / 1e9);
    }
    return 0;
}
