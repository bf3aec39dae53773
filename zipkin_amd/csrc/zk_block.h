// zk_block.h — workgroup-level device helpers shared by the reduce and partition kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zk {

// the XCD this wave runs on (0..7): a placement hint for speed only (MI355X_MICROARCH.md,
// "Workgroup dispatch, XCD placement")
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x;
}

// Exclusive prefix sum over the workgroup (one value per thread) and the workgroup total.
// NW = waves per block (blockDim.x == 64 * NW, NW <= 16); s_tmp: 32 u32 of LDS. Two barriers.
template <int NW>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_tmp, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) s_tmp[wave] = incl;
    __syncthreads();
    if (wave == 0) {
        uint32_t w = lane < NW ? s_tmp[lane] : 0u;
#pragma unroll
        for (int off = 1; off < NW; off <<= 1) {
            const uint32_t o = __shfl_up(w, off);
            if (lane >= off) w += o;
        }
        if (lane < NW) s_tmp[16 + lane] = w;  // inclusive wave totals
    }
    __syncthreads();
    *total = s_tmp[16 + NW - 1];
    return (wave ? s_tmp[16 + wave - 1] : 0u) + incl - v;
}

}  // namespace zk
