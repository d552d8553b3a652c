// kd_join.h — device helpers shared by the join kernels (classify2 / classify3).
#pragma once
#include "kd_internal.h"

namespace kd {

__device__ __forceinline__ bool oid_ne(const u32* __restrict__ x, const u32* __restrict__ y) {
    return ((x[0] ^ y[0]) | (x[1] ^ y[1]) | (x[2] ^ y[2]) | (x[3] ^ y[3]) | (x[4] ^ y[4])) != 0;
}

__device__ bool names_eq(const u8* __restrict__ na, const u64* __restrict__ oa, u64 i, const u8* __restrict__ nb,
                         const u64* __restrict__ ob, u64 j) {
    u64 a0 = oa[i], a1 = oa[i + 1], b0 = ob[j], b1 = ob[j + 1];
    if (a1 - a0 != b1 - b0) return false;
    for (u64 k = 0; k < a1 - a0; k++)
        if (na[a0 + k] != nb[b0 + k]) return false;
    return true;
}

// block-wide exclusive scan of one u32 per thread; returns the block total via *total
template <int NT>
__device__ __forceinline__ u32 block_excl_scan(u32 v, u32* s_wave, u32* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    u32 x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        u32 y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_wave[wid] = x;
    __syncthreads();
    u32 wpre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        u32 s = s_wave[w];
        if (w < wid) wpre += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return wpre + x - v;
}

template <int NT>
__device__ __forceinline__ u32 block_sum(u32 v, u32* s_wave) {
    u32 tot;
    block_excl_scan<NT>(v, s_wave, &tot);
    return tot;
}

}  // namespace kd
