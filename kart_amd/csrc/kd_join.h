// kd_join.h — device helpers shared by the join kernels (classify2 / classify3).
#pragma once
#include "kd_internal.h"

namespace kd {

__device__ __forceinline__ bool oid_ne(const u32* __restrict__ x, const u32* __restrict__ y) {
    return ((x[0] ^ y[0]) | (x[1] ^ y[1]) | (x[2] ^ y[2]) | (x[3] ^ y[3]) | (x[4] ^ y[4])) != 0;
}

// Filename equality, four bytes per step: each name is read as the aligned dwords that hold it and
// realigned with v_alignbyte, so a 24-byte name costs ~7 dword loads per side instead of 24
// dependent byte loads.  Only dwords holding at least one byte of the name are loaded (dword k+1
// of a name at byte offset s is needed iff 4k + 4 < s + len), so nothing past the arena is read.
__device__ __forceinline__ u32 name_word(const u32* __restrict__ w, u32 s, u32 len, u32 k, u32 prev, u32* next) {
    const u32 nx = (4 * k + 4 < s + len) ? w[k + 1] : 0u;
    *next = nx;
    return __builtin_amdgcn_alignbyte(nx, prev, s);
}

__device__ bool names_eq(const u8* __restrict__ na, const u64* __restrict__ oa, u64 i, const u8* __restrict__ nb,
                         const u64* __restrict__ ob, u64 j) {
    const u64 a0 = oa[i], a1 = oa[i + 1], b0 = ob[j], b1 = ob[j + 1];
    if (a1 - a0 != b1 - b0) return false;
    const u32 len = (u32)(a1 - a0);
    if (len == 0) return true;
    const u32 sa = (u32)(a0 & 3), sb = (u32)(b0 & 3);
    const u32* wa = (const u32*)(na + (a0 - sa));
    const u32* wb = (const u32*)(nb + (b0 - sb));
    u32 pa = wa[0], pb = wb[0], diff = 0;
    const u32 nw = (len + 3) >> 2;
    for (u32 k = 0; k < nw; k++) {
        u32 xa_next, xb_next;
        const u32 x = name_word(wa, sa, len, k, pa, &xa_next);
        const u32 y = name_word(wb, sb, len, k, pb, &xb_next);
        const u32 rem = len - 4 * k;
        const u32 m = rem >= 4 ? 0xFFFFFFFFu : ((1u << (8 * rem)) - 1u);
        diff |= (x ^ y) & m;
        pa = xa_next;
        pb = xb_next;
    }
    return diff == 0;
}

// bytes [a, a + n) and [b, b + n) of LDS (byte addresses) equal: the aligned words of each side
// read four at a time and realigned with v_alignbyte, the whole words unmasked and only the tail
// masked (reads may run 4 bytes past a range: still LDS, masked).  (The k_join3b matched-pair compare
// is ~8 % of C4's join; the 16-byte-block form with a mask per word spent twice the VALU.)
__device__ __forceinline__ bool lds_eq_bytes(u32 a, u32 b, u32 n) {
    typedef const __attribute__((address_space(3))) u32* l32;
    auto rd = [](u32 addr) { return *(l32)(size_t)addr; };
    const u32 sa = a & 3, sb = b & 3;
    u32 wa = a - sa, wb = b - sb;
    u32 pa = rd(wa), pb = rd(wb), diff = 0;
    const u32 nw = n >> 2;
    u32 w = 0;
    for (; w + 4 <= nw; w += 4) {
        u32 xa[4], xb[4];
#pragma unroll
        for (int j = 0; j < 4; j++) { xa[j] = rd(wa + 4 * j + 4); xb[j] = rd(wb + 4 * j + 4); }
        diff |= __builtin_amdgcn_alignbyte(xa[0], pa, sa) ^ __builtin_amdgcn_alignbyte(xb[0], pb, sb);
#pragma unroll
        for (int j = 1; j < 4; j++)
            diff |= __builtin_amdgcn_alignbyte(xa[j], xa[j - 1], sa) ^ __builtin_amdgcn_alignbyte(xb[j], xb[j - 1], sb);
        pa = xa[3]; pb = xb[3];
        wa += 16; wb += 16;
    }
    for (; w < nw; w++) {
        const u32 xa = rd(wa + 4), xb = rd(wb + 4);
        diff |= __builtin_amdgcn_alignbyte(xa, pa, sa) ^ __builtin_amdgcn_alignbyte(xb, pb, sb);
        pa = xa; pb = xb;
        wa += 4; wb += 4;
    }
    const u32 rem = n & 3;
    if (rem) {
        const u32 xa = rd(wa + 4), xb = rd(wb + 4);
        diff |= (__builtin_amdgcn_alignbyte(xa, pa, sa) ^ __builtin_amdgcn_alignbyte(xb, pb, sb)) & ((1u << (8 * rem)) - 1u);
    }
    return diff == 0;
}

// K filename comparisons at once, all loads issued before any compare: each name's offsets, then a
// W-dword window of each name (the dwords holding its bytes; past its last dword the window
// re-reads dword 0, so every load stays inside the name).  Bit k of the result = pair k is active
// and its names differ.  A name whose window would exceed W dwords (byte offset mod 4 + length >
// 4W) takes names_eq.
template <int K, int W>
__device__ __forceinline__ u32 names_ne_batch(const u8* __restrict__ na, const u64* __restrict__ oa, const u32* ia,
                                              const u8* __restrict__ nb, const u64* __restrict__ ob, const u32* jb,
                                              u32 act) {
    u64 a0[K], a1[K], b0[K], b1[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const u64 i = (act >> k) & 1 ? ia[k] : 0, j = (act >> k) & 1 ? jb[k] : 0;
        a0[k] = oa[i]; a1[k] = oa[i + 1];
        b0[k] = ob[j]; b1[k] = ob[j + 1];
    }
    u32 wa[K][W], wb[K][W];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const u32 la = (u32)(a1[k] - a0[k]), lb = (u32)(b1[k] - b0[k]);
        const u32 sa = (u32)(a0[k] & 3), sb = (u32)(b0[k] & 3);
        const u32 nwa = (sa + la + 3) >> 2, nwb = (sb + lb + 3) >> 2;
        // an empty name has no dword of its own: read the offsets array instead (valid memory)
        const u32* pa = la ? (const u32*)(na + (a0[k] - sa)) : (const u32*)oa;
        const u32* pb = lb ? (const u32*)(nb + (b0[k] - sb)) : (const u32*)ob;
#pragma unroll
        for (int w = 0; w < W; w++) {
            wa[k][w] = pa[(u32)w < nwa ? w : 0];
            wb[k][w] = pb[(u32)w < nwb ? w : 0];
        }
    }
    u32 ne = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
        if (!((act >> k) & 1)) continue;
        const u32 la = (u32)(a1[k] - a0[k]), lb = (u32)(b1[k] - b0[k]);
        if (la != lb) { ne |= 1u << k; continue; }
        const u32 sa = (u32)(a0[k] & 3), sb = (u32)(b0[k] & 3);
        if (sa + la > 4 * W || sb + la > 4 * W) {
            if (!names_eq(na, oa, ia[k], nb, ob, jb[k])) ne |= 1u << k;
            continue;
        }
        u32 diff = 0;
#pragma unroll
        for (int w = 0; w < W; w++) {
            const u32 x = __builtin_amdgcn_alignbyte(w + 1 < W ? wa[k][w + 1] : 0u, wa[k][w], sa);
            const u32 y = __builtin_amdgcn_alignbyte(w + 1 < W ? wb[k][w + 1] : 0u, wb[k][w], sb);
            const u32 rem = la > 4u * w ? la - 4u * w : 0u;
            const u32 m = rem >= 4 ? 0xFFFFFFFFu : ((1u << (8 * rem)) - 1u);
            diff |= (x ^ y) & m;
        }
        if (diff) ne |= 1u << k;
    }
    return ne;
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

// ---------------------------------------------------------------------------------------------
// decoupled look-back (k_join2p, k_resolve3)
// ---------------------------------------------------------------------------------------------
// Look-back descriptors, two words per tile (own flag each, looked back independently):
//   word 0 = flag << 62 | deltas << 31 | updates,   word 1 = flag << 62 | deletes
// flag 0 = not yet, 1 = the tile's own counts (aggregate), 2 = inclusive prefix through the tile.
// Fields are 31 bits (side sizes are checked on the host), so payloads add without carries.
constexpr u64 LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_PAY = (1ull << 62) - 1;

__device__ __forceinline__ void lb_store(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ u64 lb_load(u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Wave 0 of the tile's workgroup: publish the aggregates, walk back over earlier tiles' descriptors
// (32 at a time per word, lanes 0-31 word 0 and lanes 32-63 word 1) until an inclusive prefix is
// found, publish the tile's own inclusive prefix; returns the exclusive payload of this lane's word.
// Every workgroup is resident (the grid is sized by occupancy) and tiles are taken in increasing
// order, so every predecessor's descriptor is eventually published.
__device__ __forceinline__ u64 lookback(u64* __restrict__ desc, u64 ntiles, u64 t, u64 agg0, u64 agg1) {
    const int lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31;
    u64* D = desc + (u64)h * ntiles;
    const u64 agg = h ? agg1 : agg0;
    if (l == 0) lb_store(D + t, (t == 0 ? LB_INC : LB_AGG) | agg);
    u64 excl = 0;
    bool done = t == 0;
    i64 pos = (i64)t - 1;
    while (true) {
        const bool act = !done;
        if (__ballot(act) == 0) break;
        u64 v = LB_INC;  // before tile 0: an inclusive prefix of zero
        const i64 idx = pos - l;
        if (act && idx >= 0) v = lb_load(D + idx);
        const u32 f = (u32)(v >> 62);
        const u32 mx = (u32)(__ballot(act && f == 0) >> (32 * h));
        const u32 mp = (u32)(__ballot(act && f == 2) >> (32 * h));
        const int fp = mp ? __ffs(mp) - 1 : 32, fx = mx ? __ffs(mx) - 1 : 32;
        const bool take_all = mp == 0 && mx == 0;  // 32 aggregates: add them and look further back
        const bool finish = mp != 0 && fp < fx;    // aggregates up to an inclusive prefix
        u64 s = (act && (take_all || (finish && l <= fp))) ? (v & LB_PAY) : 0;
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);  // sum within the 32-lane half
        if (act && (take_all || finish)) excl += s;
        if (act && finish) done = true;
        if (act && take_all) pos -= 32;
        if (act && !take_all && !finish) __builtin_amdgcn_s_sleep(1);  // a predecessor not published yet
    }
    if (l == 0) lb_store(D + t, LB_INC | (excl + agg));
    return excl;
}

}  // namespace kd
