// kd_sort.hip — packing a side on the GPU: join keys sorted with an LDS-ranked LSD radix sort,
// OIDs permuted by the sort order, duplicate keys detected.
//
// Replaces the sort the host packer did after decoding the leaf paths (Dataset3's leaves arrive in
// git path order — kart/dataset3.py:225-231 walks the trees — which is not join-key order: base64
// tree names sort by ASCII, not by bucket value, and b64(msgpack(pk)) filenames do not sort by pk).
//
// Only the bits that differ between keys are sorted: int keys of pks below 2^30 vary in 30 of 64
// bits (bucket24 | pk % 64), so four 8-bit passes instead of eight.  Per pass:
//   k_rs_hist    one wave per 4096-key tile: digit counts of the tile (ballot ranking, LDS counters)
//   k_rs_scan    one block per digit: exclusive scan of that digit's tile counts (digit-major)
//   k_rs_scatter one wave per tile: the same ranking again (stable: rounds in item order, lanes in
//                lane order), digit base + earlier tiles' count + rank -> destination of (key, index)
// A digit's rank inside a 64-item round comes from 8 ballots (lanes whose digit bits all agree),
// its running count from one LDS counter per digit updated by the lowest lane of each digit group.
#include "kd_internal.h"

namespace kd {

constexpr int RS_TILE = 4096;          // keys per tile (one wave, 64 rounds of 64)
constexpr int RS_ROUNDS = RS_TILE / 64;

// lanes of the wave holding the same 8-bit digit as this lane
__device__ __forceinline__ u64 digit_peers(u32 d, bool valid) {
    u64 m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const u64 v = __ballot(valid && ((d >> b) & 1));
        m &= ((d >> b) & 1) ? v : ~v;
    }
    return m;
}

__device__ __forceinline__ u32 lanes_below(u64 m) {
    return __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0));
}

// varying bits of the keys: OR of (key ^ key[0]) over all keys
__global__ __launch_bounds__(256) void k_rs_bits(const u64* __restrict__ key, u64 n, u64* __restrict__ out) {
    const u64 k0 = key[0];
    u64 x = 0;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) x |= key[i] ^ k0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, 64);
    if ((threadIdx.x & 63) == 0 && x) atomicOr((unsigned long long*)out, (unsigned long long)x);
}

__global__ __launch_bounds__(64) void k_rs_hist(const u64* __restrict__ key, u64 n, int shift, u32 ntiles,
                                               u32* __restrict__ hist) {
    __shared__ u32 s_cnt[256];
    const int lane = threadIdx.x;
    for (int i = lane; i < 256; i += 64) s_cnt[i] = 0;
    __builtin_amdgcn_wave_barrier();
    const u64 t0 = (u64)blockIdx.x * RS_TILE;
    for (int r = 0; r < RS_ROUNDS; r++) {
        const u64 i = t0 + (u64)r * 64 + lane;
        const bool v = i < n;
        const u32 d = v ? (u32)(key[i] >> shift) & 0xFF : 0;
        const u64 m = digit_peers(d, v);
        if (v && lanes_below(m) == 0) s_cnt[d] += (u32)__popcll(m);  // one lane per digit group
        __builtin_amdgcn_wave_barrier();
    }
    for (int i = lane; i < 256; i += 64) hist[(u64)i * ntiles + blockIdx.x] = s_cnt[i];  // digit-major
}

// one block per digit: exclusive scan of hist[d][0..ntiles) in place, the digit's total to tot[d]
__global__ __launch_bounds__(256) void k_rs_scan(u32* __restrict__ hist, u32 ntiles, u32* __restrict__ tot) {
    __shared__ u32 s_w[4];
    u32* h = hist + (u64)blockIdx.x * ntiles;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    u32 carry = 0;
    for (u32 base = 0; base < ntiles; base += 256) {
        const u32 i = base + tid;
        const u32 x = i < ntiles ? h[i] : 0;
        u32 s = x;  // inclusive wave scan
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
        if (lane == 63) s_w[wid] = s;
        __syncthreads();
        u32 wp = 0, all = 0;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            if (w < wid) wp += s_w[w];
            all += s_w[w];
        }
        if (i < ntiles) h[i] = carry + wp + s - x;
        carry += all;
        __syncthreads();
    }
    if (tid == 0) tot[blockIdx.x] = carry;
}

// stable scatter of one pass; pass 0 takes the item index as its value
__global__ __launch_bounds__(64) void k_rs_scatter(const u64* __restrict__ key, const u32* __restrict__ val, u64 n,
                                                  int shift, u32 ntiles, const u32* __restrict__ hist,
                                                  const u32* __restrict__ tot, u64* __restrict__ okey,
                                                  u32* __restrict__ oval) {
    __shared__ u32 s_off[256];
    const int lane = threadIdx.x;
    // digit bases: exclusive scan of the 256 totals (4 per lane) + this tile's earlier-tile counts
    {
        u32 t[4], s = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) { t[j] = tot[4 * lane + j]; s += t[j]; }
        u32 inc = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        u32 ex = inc - s;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const u32 d = 4 * lane + j;
            s_off[d] = ex + hist[(u64)d * ntiles + blockIdx.x];
            ex += t[j];
        }
    }
    __builtin_amdgcn_wave_barrier();
    const u64 t0 = (u64)blockIdx.x * RS_TILE;
    for (int r = 0; r < RS_ROUNDS; r++) {
        const u64 i = t0 + (u64)r * 64 + lane;
        const bool v = i < n;
        const u64 k = v ? key[i] : 0;
        const u32 x = v ? (val ? val[i] : (u32)i) : 0;
        const u32 d = (u32)(k >> shift) & 0xFF;
        const u64 m = digit_peers(d, v);
        const u32 below = lanes_below(m);
        const u32 base = s_off[d];  // read by every lane before the leader moves it
        __builtin_amdgcn_wave_barrier();
        if (v && below == 0) s_off[d] = base + (u32)__popcll(m);
        __builtin_amdgcn_wave_barrier();
        if (v) {
            okey[base + below] = k;
            oval[base + below] = x;
        }
    }
}

// rows of 20 bytes gathered by the sort order: out[k] = in[order[k]]
__global__ __launch_bounds__(256) void k_gather_oid(const u8* __restrict__ in, const u32* __restrict__ order, u64 n,
                                                    u8* __restrict__ out) {
    typedef const __attribute__((address_space(1))) u32* gp32;
    for (u64 k = (u64)blockIdx.x * 256 + threadIdx.x; k < n; k += (u64)gridDim.x * 256) {
        const gp32 s = (gp32)(in + 20ull * order[k]);  // 20-B rows: 4-B aligned
        u32* d = (u32*)(out + 20ull * k);
        const u32 a = s[0], b = s[1], c = s[2], e = s[3], f = s[4];
        d[0] = a; d[1] = b; d[2] = c; d[3] = e; d[4] = f;
    }
}

__global__ __launch_bounds__(256) void k_iota_u32(u32* __restrict__ out, u64 n) {
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) out[i] = (u32)i;
}

// sorted keys strictly ascending?  *dup |= 1 on an equal (or descending) neighbour
__global__ __launch_bounds__(256) void k_check_sorted(const u64* __restrict__ key, u64 n, u32* __restrict__ dup) {
    bool bad = false;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x + 1; i < n; i += (u64)gridDim.x * 256) bad |= key[i - 1] >= key[i];
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(dup, 1u);
}

}  // namespace kd

using namespace kd;

extern "C" int kd_sort_side(kd_ctx* ctx, uint64_t* d_key, uint8_t* d_oid, uint32_t* d_order, uint64_t n,
                            uint32_t* h_dup) {
    KD_CHECK(ctx && (n == 0 || (d_key && d_order)), "kd_sort_side: NULL");
    KD_CHECK(n < 0xFFFFFFFFull, "kd_sort_side: side too large for uint32 indices");
    KD_HIP(hipSetDevice(ctx->device));
    if (h_dup) *h_dup = 0;
    if (n == 0) return KD_OK;
    int rc;
    const u32 ntiles = (u32)((n + RS_TILE - 1) / RS_TILE);
    void *bits, *hist, *tot, *k2, *v2, *dup;
    if ((rc = ensure(ctx, "rs.bits", 16, &bits))) return rc;
    if ((rc = ensure(ctx, "rs.hist", (u64)ntiles * 256 * 4, &hist))) return rc;
    if ((rc = ensure(ctx, "rs.tot", 256 * 4, &tot))) return rc;
    if ((rc = ensure(ctx, "rs.k2", n * 8, &k2))) return rc;
    if ((rc = ensure(ctx, "rs.v2", n * 4, &v2))) return rc;
    if ((rc = ensure(ctx, "rs.dup", 16, &dup))) return rc;
    const unsigned gs = (unsigned)std::max<u64>(1, std::min<u64>((n + 255) / 256, (u64)ctx->n_cu * 8));
    // ---- which bits vary (one 8-byte read-back decides the pass count) ----
    KD_HIP(hipMemsetAsync(bits, 0, 16, ctx->stream));
    rc = launch(ctx, "k_rs_bits", [&] {
        hipLaunchKernelGGL(k_rs_bits, dim3(gs), dim3(256), 0, ctx->stream, (const u64*)d_key, n, (u64*)bits);
    });
    if (rc) return rc;
    u64 vary = 0;
    KD_HIP(hipMemcpyAsync(&vary, bits, 8, hipMemcpyDeviceToHost, ctx->stream));
    KD_HIP(hipStreamSynchronize(ctx->stream));
    int lo = 0, hi = -1;
    if (vary) { lo = __builtin_ctzll(vary); hi = 63 - __builtin_clzll(vary); }
    const int passes = vary ? (hi - lo + 8) / 8 : 0;
    // ---- LSD passes, ping-ponging between the caller's arrays and scratch ----
    u64* ka = d_key;
    u32* va = nullptr;  // pass 0: values are the item indices
    u64* kb = (u64*)k2;
    u32* vb = (u32*)v2;
    for (int p = 0; p < passes; p++) {
        const int shift = lo + 8 * p;
        if ((rc = launch(ctx, "k_rs_hist", [&] {
                 hipLaunchKernelGGL(k_rs_hist, dim3(ntiles), dim3(64), 0, ctx->stream, (const u64*)ka, n, shift, ntiles,
                                    (u32*)hist);
             })))
            return rc;
        if ((rc = launch(ctx, "k_rs_scan", [&] {
                 hipLaunchKernelGGL(k_rs_scan, dim3(256), dim3(256), 0, ctx->stream, (u32*)hist, ntiles, (u32*)tot);
             })))
            return rc;
        if ((rc = launch(ctx, "k_rs_scatter", [&] {
                 hipLaunchKernelGGL(k_rs_scatter, dim3(ntiles), dim3(64), 0, ctx->stream, (const u64*)ka, (const u32*)va,
                                    n, shift, ntiles, (const u32*)hist, (const u32*)tot, kb, vb);
             })))
            return rc;
        // next pass reads what this one wrote; the value array alternates between d_order and scratch
        std::swap(ka, kb);
        if (p == 0) { va = vb; vb = d_order; }
        else std::swap(va, vb);
    }
    // ---- results into the caller's arrays ----
    if (passes == 0) {  // all keys equal (n == 1, or duplicates): identity order
        rc = launch(ctx, "k_iota", [&] {
            hipLaunchKernelGGL(k_iota_u32, dim3(gs), dim3(256), 0, ctx->stream, d_order, n);
        });
        if (rc) return rc;
    } else {
        if (ka != d_key) KD_HIP(hipMemcpyAsync(d_key, ka, n * 8, hipMemcpyDeviceToDevice, ctx->stream));
        if (va != d_order) KD_HIP(hipMemcpyAsync(d_order, va, n * 4, hipMemcpyDeviceToDevice, ctx->stream));
    }
    if (d_oid) {  // OIDs permuted by the order (through scratch, then back in place)
        void* o2;
        if ((rc = ensure(ctx, "rs.oid", n * 20, &o2))) return rc;
        if ((rc = launch(ctx, "k_gather_oid", [&] {
                 hipLaunchKernelGGL(k_gather_oid, dim3(gs), dim3(256), 0, ctx->stream, (const u8*)d_oid, (const u32*)d_order, n,
                                    (u8*)o2);
             })))
            return rc;
        KD_HIP(hipMemcpyAsync(d_oid, o2, n * 20, hipMemcpyDeviceToDevice, ctx->stream));
    }
    KD_HIP(hipMemsetAsync(dup, 0, 4, ctx->stream));
    if ((rc = launch(ctx, "k_check_sorted", [&] {
             hipLaunchKernelGGL(k_check_sorted, dim3(gs), dim3(256), 0, ctx->stream, (const u64*)d_key, n, (u32*)dup);
         })))
        return rc;
    if (h_dup) {
        KD_HIP(hipMemcpyAsync(h_dup, dup, 4, hipMemcpyDeviceToHost, ctx->stream));
        KD_HIP(hipStreamSynchronize(ctx->stream));
    }
    return KD_OK;
}
