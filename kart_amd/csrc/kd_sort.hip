// kd_sort.hip — packing a side on the GPU: join keys sorted by an LDS-staged onesweep LSD radix
// sort, OIDs permuted by the sort order, duplicate keys detected.
//
// Replaces the sort the host packer did after decoding the leaf paths (Dataset3's leaves arrive in
// git path order — kart/dataset3.py:225-231 walks the trees — which is not join-key order: base64
// tree names sort by ASCII, not by bucket value, and b64(msgpack(pk)) filenames do not sort by pk).
//
// 1. k_rs_bits     OR of key ^ key[0]: the bits that vary.  One 8-B read-back sizes the sort.
//    Only those bits are sorted: they are gathered ("compacted", an order-preserving bit gather of at
//    most 4 runs of bits) into a 32-bit key when they fit (int keys of pks below 2^30 vary in
//    6 + 24 bits) and expanded back to the full 64-bit key on the last pass's store.
// 2. k_sort_hist   one read of the keys: the digit histograms of EVERY pass (digits of up to 9 bits), run-
//                  length counted per thread over 16 consecutive keys, LDS atomics, one global add
//                  per (block, pass, digit).  k_sort_scan turns them into each digit's global base.
// 3. k_sort_pass   one launch per digit pass, one tile of NT*IPT keys per workgroup, tiles taken in
//                  order from an atomic counter (every earlier tile is resident or done):
//      a. load the tile (wave-striped, so (wave, item, lane) order is input order: stable);
//      b. early counts: the tile's digit histogram (LDS atomics) is published at once, so the
//         tiles after it rarely wait for it in their look-back;
//      c. rank: per wave and item, the lanes holding the same digit (one ballot per digit bit), a
//         per-(digit, wave) LDS counter bumped by the group's lowest lane; one block scan over the
//         [digit][wave] counters gives every (digit, wave) its start inside the tile;
//      d. reorder the tile in LDS by digit, look back over earlier tiles' published counts for
//         this tile's global offset per digit (decoupled look-back, a window of earlier tiles per
//         round trip, epoch-tagged 8-B agent-scope words: no per-pass clearing);
//      e. scatter from LDS in digit order: a digit's run of the tile is written to consecutive
//         addresses (coalesced), the last pass stores full keys + the original index.
// 4. k_gather_oid  OIDs permuted by the order (sorted k reads row order[k]; git-order leaves of one
//                  64-entry leaf tree stay within ~1.3 KB, so the reads are near-coalesced).
#include "kd_internal.h"
#include "kd_walkkey.h"

namespace kd {

#ifndef KD_RS_RB
#define KD_RS_RB 9
#endif
constexpr int RS_RB = KD_RS_RB;      // digit bits per pass (at most)
constexpr int RS_RD = 1 << RS_RB;    // digits
constexpr int RS_MAXRUNS = 4;        // compaction runs (more are merged, taking the constant gap bits)
constexpr int RS_HIST_NT = 256, RS_HIST_IPT = 16;
#ifndef KD_RS_NT
#define KD_RS_NT 512
#endif
#ifndef KD_RS_IPT32
#define KD_RS_IPT32 16
#endif
#ifndef KD_RS_IPT64
#define KD_RS_IPT64 8
#endif
constexpr int RS_NT = KD_RS_NT;

// which bits vary, and how they are gathered into the compact key
struct SortPlan {
    u64 kconst;                 // key bits outside the runs (equal in every key)
    u64 mask[RS_MAXRUNS];       // run r: (key >> lo[r]) & mask[r] -> compact bits at pos[r]
    u32 lo[RS_MAXRUNS], pos[RS_MAXRUNS];
    u32 nruns, bits;            // runs, compact key width
    u64 out_xor;                // the last pass stores rs_expand(key) ^ out_xor (signed pks: the sign bit)
};

template <typename CK>
__device__ __forceinline__ CK rs_compact(u64 k, const SortPlan& p) {
    u64 c = 0;
#pragma unroll
    for (int r = 0; r < RS_MAXRUNS; r++)
        if (r < (int)p.nruns) c |= ((k >> p.lo[r]) & p.mask[r]) << p.pos[r];
    return (CK)c;
}

__device__ __forceinline__ u64 rs_expand(u64 c, const SortPlan& p) {
    u64 k = p.kconst;
#pragma unroll
    for (int r = 0; r < RS_MAXRUNS; r++)
        if (r < (int)p.nruns) k |= ((c >> p.pos[r]) & p.mask[r]) << p.lo[r];
    return k;
}

// lanes of the wave holding the same digit as this lane
__device__ __forceinline__ u64 digit_peers(u32 d, bool valid) {
    u64 m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < RS_RB; b++) {
        const u64 v = __ballot(valid && ((d >> b) & 1));
        m &= ((d >> b) & 1) ? v : ~v;
    }
    return m;
}

__device__ __forceinline__ u32 lanes_below(u64 m) {
    return __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0));
}

// exclusive scan of one u32 per thread over the workgroup; *total <- the workgroup's sum
template <int NT>
__device__ __forceinline__ u32 block_scan_u32(u32 v, u32* s_wave, u32* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u32 x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_wave[wv] = x;
    __syncthreads();
    u32 pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const u32 s = s_wave[w];
        pre += w < wv ? s : 0u;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return pre + x - v;
}

// varying bits of the keys: OR of (key ^ key[0]) over all keys (16-B loads, four in flight per lane)
__global__ __launch_bounds__(256) void k_rs_bits(const u64* __restrict__ key, u64 n, u64* __restrict__ out) {
    const u64 k0 = key[0];
    u64 x = 0;
    const u64 tid = (u64)blockIdx.x * 256 + threadIdx.x, nt = (u64)gridDim.x * 256;
    u64 done = 0;
    if (((uintptr_t)key & 15) == 0) {
        const u64x2* p = (const u64x2*)key;
        const u64 n2 = n / 2;
        u64 i = tid;
        for (; i + 3 * nt < n2; i += 4 * nt) {
            const u64x2 a = p[i], b = p[i + nt], c = p[i + 2 * nt], d = p[i + 3 * nt];
            x |= (a.x ^ k0) | (a.y ^ k0) | (b.x ^ k0) | (b.y ^ k0) | (c.x ^ k0) | (c.y ^ k0) | (d.x ^ k0) | (d.y ^ k0);
        }
        for (; i < n2; i += nt) x |= (p[i].x ^ k0) | (p[i].y ^ k0);
        done = 2 * n2;
    }
    for (u64 i = done + tid; i < n; i += nt) x |= key[i] ^ k0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, 64);
    if ((threadIdx.x & 63) == 0 && x) atomicOr((unsigned long long*)out, (unsigned long long)x);
}

// ---- all passes' digit histograms in one read of the keys ----
// s_h holds digit d of a pass at d + d / 16 (KD_RS_HPAD): a thread counts 16 consecutive keys, so in
// walk order lane l adds digit ~16 l + j at step j, and unpadded lanes l, l + 4, l + 8, ... met in one
// bank (16-way); with the pad lane l lands in bank (17 l + j) mod 64
#ifndef KD_RS_HPAD
#define KD_RS_HPAD 1
#endif
constexpr int RS_HSTRIDE = KD_RS_HPAD ? RS_RD + RS_RD / 16 : RS_RD;
__device__ __forceinline__ u32 rs_hi(u32 d) { return KD_RS_HPAD ? d + (d >> 4) : d; }
template <typename CK>
__global__ __launch_bounds__(RS_HIST_NT) void k_sort_hist(const u64* __restrict__ key, u64 ncap, const u64* __restrict__ dn,
                                                           int npass, int width, SortPlan plan, u32* __restrict__ hist) {
    __shared__ u32 s_h[8 * RS_HSTRIDE];
    const int tid = threadIdx.x;
    const u64 n = dn ? min(*dn, ncap) : ncap;
    for (int i = tid; i < npass * RS_HSTRIDE; i += RS_HIST_NT) s_h[i] = 0;
    __syncthreads();
    const u32 dmask = (1u << width) - 1;
    const bool al16 = ((uintptr_t)key & 15) == 0;
    constexpr u64 CH = (u64)RS_HIST_NT * RS_HIST_IPT;
    for (u64 base = (u64)blockIdx.x * CH; base < n; base += (u64)gridDim.x * CH) {
        const u64 i0 = base + (u64)tid * RS_HIST_IPT;  // 16 consecutive keys per thread: runs of equal digits
        const int cnt = i0 < n ? (int)min<u64>(RS_HIST_IPT, n - i0) : 0;
        CK c[RS_HIST_IPT];
        if (cnt == RS_HIST_IPT && al16) {
            const u64x2* p = (const u64x2*)(key + i0);
#pragma unroll
            for (int j = 0; j < RS_HIST_IPT / 2; j++) {
                const u64x2 v = p[j];
                c[2 * j] = rs_compact<CK>(v.x, plan);
                c[2 * j + 1] = rs_compact<CK>(v.y, plan);
            }
        } else {
#pragma unroll
            for (int j = 0; j < RS_HIST_IPT; j++) c[j] = j < cnt ? rs_compact<CK>(key[i0 + j], plan) : 0;
        }
        for (int p = 0; p < npass; p++) {
            const int sh = p * width;
            u32 cur = (u32)(c[0] >> sh) & dmask, run = 0;
#pragma unroll
            for (int j = 0; j < RS_HIST_IPT; j++) {
                if (j < cnt) {
                    const u32 d = (u32)(c[j] >> sh) & dmask;
                    if (d != cur) {
                        atomicAdd(&s_h[p * RS_HSTRIDE + rs_hi(cur)], run);
                        cur = d;
                        run = 0;
                    }
                    run++;
                }
            }
            if (run) atomicAdd(&s_h[p * RS_HSTRIDE + rs_hi(cur)], run);
        }
    }
    __syncthreads();
    for (int i = tid; i < npass * RS_RD; i += RS_HIST_NT) {
        const u32 x = s_h[(i / RS_RD) * RS_HSTRIDE + rs_hi(i % RS_RD)];
        if (x) atomicAdd(&hist[i], x);
    }
}

// one block: hist[p][d] -> exclusive scan over d (each digit's first output position in pass p)
__global__ __launch_bounds__(RS_RD) void k_sort_scan(const u32* __restrict__ hist, int npass, u32* __restrict__ gbase) {
    __shared__ u32 s_w[RS_RD / 64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int p = 0; p < npass; p++) {
        const u32 x = hist[p * RS_RD + tid];
        u32 s = x;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
        if (lane == 63) s_w[wv] = s;
        __syncthreads();
        u32 pre = 0;
#pragma unroll
        for (int w = 0; w < RS_RD / 64; w++)
            if (w < wv) pre += s_w[w];
        gbase[p * RS_RD + tid] = pre + s - x;
        __syncthreads();
    }
}

// look-back words: flag << 62 | epoch << 40 | count; a word of another epoch is "not yet"
constexpr u64 RS_AGG = 1ull << 62, RS_INC = 2ull << 62, RS_CNT = (1ull << 40) - 1;
constexpr u32 RS_EPOCHS = 1u << 22;
#ifndef KD_RS_LBW
#define KD_RS_LBW 4
#endif
constexpr int RS_LBW = KD_RS_LBW;  // look-back words per round trip
#ifndef KD_RS_SWZ
#define KD_RS_SWZ 1
#endif
// k_sort_pass's per-(digit, wave) u16 counters: [wave][digit] (KD_RS_SWZ) puts a wave's digits in
// consecutive halfwords, so lanes of different digits spread over all 64 banks (two digits per
// dword); [digit][wave] with 8 waves gave digit d the bank (4d + wave / 2) mod 64: 16 banks for a
// wave's 64 lanes, and the block scan's reads of 8 consecutive counters per thread 4-way conflicts
template <int NW>
__device__ __forceinline__ u32 rs_ci(u32 d, u32 w) {
    return KD_RS_SWZ ? w * (u32)RS_RD + d : d * (u32)NW + w;
}
__device__ __forceinline__ void rs_store(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ u64 rs_load(const u64* p) {
    return __hip_atomic_load((u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One digit pass.  FIRST: value = the input index; IN64: the input keys are the caller's 64-bit
// keys (compacted on load), else compact keys already.  LAST: output = full 64-bit keys (expanded,
// ^ plan.out_xor) + the values.  The grid is persistent: workgroups take tiles in order from an
// atomic counter until the count (*dn when the caller's count lives on the device) is covered.
template <typename CK, int NT, int IPT, bool FIRST, bool LAST, bool IN64>
__global__ __launch_bounds__(NT) void k_sort_pass(const void* __restrict__ kin, const u32* __restrict__ vin,
                                                  void* __restrict__ kout, u32* __restrict__ vout, u64 ncap,
                                                  const u64* __restrict__ dn, int shift, u32 dmask,
                                                  const u32* __restrict__ gbase, u64* __restrict__ status, u32 epoch,
                                                  u32* __restrict__ tile_ctr, SortPlan plan) {
    constexpr int NW = NT / 64, TILE = NT * IPT, CPT = RS_RD * NW / NT;
    static_assert(NT >= RS_RD && (RS_RD * NW) % NT == 0, "tile shape");
    static_assert(TILE <= 65535, "s_cnt holds tile-local starts in 16 bits");
    __shared__ u16 s_cnt[RS_RD * NW];  // (digit, wave) at rs_ci: item counts, then (after the scan) starts (<= TILE)
    __shared__ u32 s_hist[RS_RD];      // the tile's digit counts (early: published before the ranking)
    __shared__ CK s_key[TILE];
    __shared__ u32 s_val[TILE];
    __shared__ u32 s_goff[RS_RD];      // global position of the digit's tile-local position 0
    __shared__ u32 s_wsum[NW];
    __shared__ u32 s_tile;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const u64 n = dn ? min(*dn, ncap) : ncap;
    const u64 ntiles = (n + TILE - 1) / TILE;
    while (true) {
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
    for (int i = tid; i < RS_RD * NW; i += NT) s_cnt[i] = 0;
    for (int i = tid; i < RS_RD; i += NT) s_hist[i] = 0;
    __syncthreads();
    const u32 tile = s_tile;
    if ((u64)tile >= ntiles) break;
    const u64 t0 = (u64)tile * TILE;
    const u32 valid = (u32)min<u64>((u64)TILE, n - t0);
    const u64 wbase = t0 + (u64)wv * 64 * IPT + lane;
    // ---- a. load ----
    CK c[IPT];
    u32 v[IPT], rk[IPT];
#pragma unroll
    for (int i = 0; i < IPT; i++) {
        const u64 idx = wbase + (u64)i * 64;
        const bool ok = idx < n;
        if (IN64) c[i] = ok ? rs_compact<CK>(((const u64*)kin)[idx], plan) : (CK)0;
        else c[i] = ok ? ((const CK*)kin)[idx] : (CK)0;
        if (FIRST) v[i] = (u32)idx;
        else v[i] = ok ? vin[idx] : 0;
    }
    // ---- b. early counts: the tile's digit histogram, published before the ranking so that later
    //         tiles' look-backs find this tile's aggregate as early as possible ----
#pragma unroll
    for (int i = 0; i < IPT; i++)
        if (wbase + (u64)i * 64 < n) atomicAdd(&s_hist[(u32)(c[i] >> shift) & dmask], 1u);
    __syncthreads();
    u32 dcnt = 0;
    u64* st = status + (u64)tile * RS_RD + tid;
    if (tid < RS_RD) {
        dcnt = s_hist[tid];
        rs_store(st, (tile == 0 ? RS_INC : RS_AGG) | ((u64)epoch << 40) | dcnt);
    }
    // ---- c. rank within the wave, then a block scan of the [digit][wave] counters ----
#pragma unroll
    for (int i = 0; i < IPT; i++) {
        const bool ok = wbase + (u64)i * 64 < n;
        const u32 d = (u32)(c[i] >> shift) & dmask;
        const u64 m = digit_peers(d, ok);
        const u32 below = lanes_below(m);
        u16* ctr = &s_cnt[rs_ci<NW>(d, wv)];
        const u32 pre = *ctr;  // read by every lane of the group before its lowest lane moves it
        __builtin_amdgcn_wave_barrier();
        if (ok && below == 0) *ctr = (u16)(pre + (u32)__popcll(m));
        __builtin_amdgcn_wave_barrier();
        rk[i] = pre + below;
    }
    __syncthreads();
    {
        u32 x[CPT], s = 0;
#pragma unroll
        for (int j = 0; j < CPT; j++) {
            const u32 L = (u32)(tid * CPT + j);  // (digit, wave) in digit-major scan order
            x[j] = s_cnt[rs_ci<NW>(L / NW, L % NW)];
            s += x[j];
        }
        u32 inc = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) s_wsum[wv] = inc;
        __syncthreads();
        u32 ex = inc - s;
#pragma unroll
        for (int w = 0; w < NW; w++)
            if (w < wv) ex += s_wsum[w];
#pragma unroll
        for (int j = 0; j < CPT; j++) {
            const u32 L = (u32)(tid * CPT + j);
            s_cnt[rs_ci<NW>(L / NW, L % NW)] = (u16)ex;
            ex += x[j];
        }
    }
    __syncthreads();
    // ---- d. reorder in LDS, look back ----
    const u32 dstart = tid < RS_RD ? (u32)s_cnt[rs_ci<NW>(tid, 0)] : 0;
#pragma unroll
    for (int i = 0; i < IPT; i++) {
        if (wbase + (u64)i * 64 < n) {
            const u32 d = (u32)(c[i] >> shift) & dmask;
            const u32 p = s_cnt[rs_ci<NW>(d, wv)] + rk[i];
            s_key[p] = c[i];
            s_val[p] = v[i];
        }
    }
    if (tid < RS_RD) {
        u64 ex = 0;
#ifdef KD_RS_PROBE_NOLB
        if (false) {  // probe: no look-back wait (wrong offsets, in bounds: times the rest)
#else
        if (tile > 0) {
#endif
            // RS_LBW earlier tiles' words per round trip (t-1, t-2, ...): their counts add up to the
            // first inclusive prefix; a word not yet published stops the round, and the next round
            // starts at it.  Tile 0 always publishes an inclusive prefix, so the walk ends there.
            // (Every earlier tile's ticket belongs to a running workgroup: the wait always ends.)
            i64 t = (i64)tile - 1;
            while (true) {
                u64 w[RS_LBW];
#pragma unroll
                for (int k = 0; k < RS_LBW; k++) w[k] = t - k >= 0 ? rs_load(status + (u64)(t - k) * RS_RD + tid) : RS_INC;
                int used = 0;
                bool done = false;
#pragma unroll
                for (int k = 0; k < RS_LBW; k++) {
                    if (done || used < k) continue;  // stopped earlier in this round
                    const u64 x = w[k];
                    const bool ready = (x >> 62) != 0 && ((u32)((x >> 40) & (RS_EPOCHS - 1)) == epoch || t - k < 0);
                    if (!ready) continue;
                    ex += x & RS_CNT;
                    used = k + 1;
                    done = (x >> 62) == 2;
                }
                if (done) break;
                t -= used;
                if (used < RS_LBW) __builtin_amdgcn_s_sleep(1);  // a predecessor has not published yet
            }
            rs_store(st, RS_INC | ((u64)epoch << 40) | (ex + dcnt));
        }
        s_goff[tid] = gbase[tid] + (u32)ex - dstart;
    }
    __syncthreads();
    // ---- e. scatter in digit order ----
    for (u32 j = tid; j < valid; j += NT) {
        const CK k = s_key[j];
        const u32 x = s_val[j];
        const u32 dst = s_goff[(u32)(k >> shift) & dmask] + j;
        if (LAST) ((u64*)kout)[dst] = rs_expand((u64)k, plan) ^ plan.out_xor;
        else ((CK*)kout)[dst] = k;
        vout[dst] = x;
    }
    __syncthreads();  // the next tile reuses the LDS arrays
    }
}

// rows of 20 bytes gathered by the sort order: out[k] = in[order[k]].  One wave per 64 rows: each
// lane loads its row (5 dwords; rows of one git leaf tree lie within ~1.3 KB), the wave's 1280 B
// go through LDS and leave as 80 coalesced 16-B stores.
__global__ __launch_bounds__(256) void k_gather_oid(const u8* __restrict__ in, const u32* __restrict__ order, u64 n,
                                                    u8* __restrict__ out) {
    typedef const __attribute__((address_space(1))) u32* gp32;
    __shared__ __attribute__((aligned(16))) u32 s_rows[4][64 * 5];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u32* R = s_rows[wv];
    const bool al16 = ((uintptr_t)out & 15) == 0;
    for (u64 r0 = ((u64)blockIdx.x * 4 + wv) * 64; r0 < n; r0 += (u64)gridDim.x * 256) {
        const u64 k = r0 + lane;
        const u32 m = (u32)min<u64>(64, n - r0);
        if (k < n) {
            const gp32 s = (gp32)(in + 20ull * order[k]);  // 20-B rows: 4-B aligned
            const u32 a = s[0], b = s[1], c = s[2], e = s[3], f = s[4];
            R[5 * lane] = a; R[5 * lane + 1] = b; R[5 * lane + 2] = c; R[5 * lane + 3] = e; R[5 * lane + 4] = f;
        }
        __builtin_amdgcn_wave_barrier();
        u32* d = (u32*)(out + 20ull * r0);
        if (m == 64 && al16) {
            const u32x4* S = (const u32x4*)R;
            ((u32x4*)d)[lane] = S[lane];
            if (lane < 16) ((u32x4*)d)[64 + lane] = S[64 + lane];
        } else {
            for (u32 j = lane; j < 5 * m; j += 64) d[j] = R[j];
        }
        __builtin_amdgcn_wave_barrier();  // the next chunk's LDS writes after this chunk's reads
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

// ---- deltas into pk order (DeltaDiff.sorted_items) ----
// pk of each delta record (base key's, or the target key's for an insert), as a sortable unsigned
// key (sign bit flipped), compacted by the plan; all passes' digit histograms.  n = *dn.
template <typename CK>
__global__ __launch_bounds__(RS_HIST_NT) void k_dpk_keys(const uint2* __restrict__ rec, u64 ncap, const u64* __restrict__ dn,
                                                          const u64* __restrict__ kA, const u64* __restrict__ kB,
                                                          const u64* __restrict__ rkey,
                                                          int npass, int width, SortPlan plan, CK* __restrict__ out,
                                                          u32* __restrict__ hist) {
    __shared__ u32 s_h[8 * RS_RD];
    const int tid = threadIdx.x;
    for (int i = tid; i < npass * RS_RD; i += RS_HIST_NT) s_h[i] = 0;
    __syncthreads();
    const u64 n = min(*dn, ncap);
    const u32 dmask = (1u << width) - 1;
    for (u64 r = (u64)blockIdx.x * RS_HIST_NT + tid; r < n; r += (u64)gridDim.x * RS_HIST_NT) {
        u64 key;
        if (rkey) key = rkey[r];  // the join wrote the records' keys beside them
        else {
            const uint2 d = rec[r];
            key = d.x != KD_NONE ? kA[d.x] : kB[d.y];
        }
        const u64 sk = (u64)wk::int_key_pk(key) ^ (1ull << 63);
        const CK c = rs_compact<CK>(sk, plan);
        out[r] = c;
        for (int p = 0; p < npass; p++) atomicAdd(&s_h[p * RS_RD + ((u32)(c >> (p * width)) & dmask)], 1u);
    }
    __syncthreads();
    for (int i = tid; i < npass * RS_RD; i += RS_HIST_NT)
        if (s_h[i]) atomicAdd(&hist[i], s_h[i]);
}

// ---- deltas into pk order by bitmap placement (a bounded pk range) ----
// Every pk occurs at most once in a record list, so the records of one 64-pk block [64b, 64b + 64)
// are exactly the set bits of a 64-bit mask: a record's rank in pk order is the number of records
// in earlier blocks (an exclusive scan of the masks' popcounts) plus the set bits below its own in
// its block's mask.  Three streaming kernels instead of a radix sort's passes.
//   k_pkm_mark   pk of each record (saved), its bit OR-ed into its block's mask: records of one
//                leaf tree are adjacent in walk order, so a wave first ORs runs of equal blocks
//                together (segmented shuffle reduction) and only each run's head lane does the atomic
//   k_pkm_scan   per chunk of PKM_CH masks: the popcounts' exclusive prefix (u32) + the chunk total
//   k_pkm_cscan  one block: exclusive prefix of the chunk totals
//   k_pkm_place  record -> its rank: chunk prefix + in-chunk prefix + popcount(mask below its bit)
#ifndef KD_PKM_IPT
#define KD_PKM_IPT 16  // masks per scan thread (r4pk, C3: 2 / 4 / 8 / 16 -> scan 0.111 / 0.074 / 0.052 / 0.038 ms)
#endif
constexpr int PKM_NT = 256, PKM_IPT = KD_PKM_IPT, PKM_CH = PKM_NT * PKM_IPT;

__global__ __launch_bounds__(PKM_NT) void k_pkm_mark(const uint2* __restrict__ rec, u64 ncap, const u64* __restrict__ dn,
                                                     const u64* __restrict__ kA, const u64* __restrict__ kB,
                                                     const u64* __restrict__ rkey, i64 lo_block, u64 nb,
                                                     u64* __restrict__ masks, i64* __restrict__ pk_out) {
    const u64 n = min(*dn, ncap);
    const int lane = threadIdx.x & 63;
    const u64 stride = (u64)gridDim.x * PKM_NT;
    for (u64 base = (u64)blockIdx.x * PKM_NT + (threadIdx.x & ~63); base < n; base += stride) {
        const u64 r = base + lane;
        const bool ok = r < n;
        i64 pk = 0;
        if (ok) {
            u64 key;
            if (rkey) key = rkey[r];  // the join wrote the records' keys beside them
            else {
                const uint2 d = rec[r];
                key = d.x != KD_NONE ? kA[d.x] : kB[d.y];
            }
            pk = wk::int_key_pk(key);
            if (!rkey) pk_out[r] = pk;  // (with the record keys, k_pkm_place recomputes it: no write)
        }
        const u64 b = (u64)((pk >> 6) - lo_block);
        const bool inb = ok && b < nb;  // (a pk outside the caller's bounds is dropped, never written out of range)
        u64 bit = inb ? 1ull << (pk & 63) : 0;
        // runs of equal blocks among the wave's lanes: OR each run into its head lane
        const u64 bprev = __shfl_up(b, 1, 64);
        const bool head = inb && (lane == 0 || bprev != b);
        const u64 heads = __ballot(head);
        const u64 later = lane == 63 ? 0 : heads & (~0ull << (lane + 1));
        const int seg_end = later ? __ffsll((long long)later) - 1 : 64;  // first lane of the next run
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u64 v = __shfl_down(bit, o, 64);
            if (lane + o < seg_end) bit |= v;
        }
        if (head) atomicOr((unsigned long long*)(masks + b), (unsigned long long)bit);
    }
}

// (masks and local prefixes moved 16 B per access; each thread's PKM_IPT masks are one 128-B line)
static_assert(PKM_IPT % 4 == 0, "k_pkm_scan: 16-B loads and stores");
// (zero: the other mask buffer, cleared here for the next call — no fill launch per call)
__global__ __launch_bounds__(PKM_NT) void k_pkm_scan(const u64* __restrict__ masks, u64 nb, u32* __restrict__ local,
                                                     u32* __restrict__ chunk_tot, u64* __restrict__ zero) {
    __shared__ u32 s_wave[PKM_NT / 64];
    const int tid = threadIdx.x;
    const u64 c0 = (u64)blockIdx.x * PKM_CH + (u64)tid * PKM_IPT;
    u32 cnt[PKM_IPT], sum = 0;
    if (c0 + PKM_IPT <= nb) {
        const u32x4* m4 = (const u32x4*)(masks + c0);
#pragma unroll
        for (int j = 0; j < PKM_IPT / 2; j++) {
            const u32x4 v = m4[j];
            cnt[2 * j] = (u32)__popc(v.x) + (u32)__popc(v.y);
            cnt[2 * j + 1] = (u32)__popc(v.z) + (u32)__popc(v.w);
        }
        u32x4* z4 = (u32x4*)(zero + c0);
#pragma unroll
        for (int j = 0; j < PKM_IPT / 2; j++) z4[j] = u32x4{0u, 0u, 0u, 0u};
    } else {
#pragma unroll
        for (int j = 0; j < PKM_IPT; j++) {
            cnt[j] = c0 + j < nb ? (u32)__popcll(masks[c0 + j]) : 0u;
            if (c0 + j < nb) zero[c0 + j] = 0;
        }
    }
#pragma unroll
    for (int j = 0; j < PKM_IPT; j++) sum += cnt[j];
    u32 tot;
    u32 ex = block_scan_u32<PKM_NT>(sum, s_wave, &tot);
    if (c0 + PKM_IPT <= nb) {
        u32x4* l4 = (u32x4*)(local + c0);
#pragma unroll
        for (int j = 0; j < PKM_IPT / 4; j++) {
            u32x4 o;
            o.x = ex; ex += cnt[4 * j];
            o.y = ex; ex += cnt[4 * j + 1];
            o.z = ex; ex += cnt[4 * j + 2];
            o.w = ex; ex += cnt[4 * j + 3];
            l4[j] = o;
        }
    } else {
#pragma unroll
        for (int j = 0; j < PKM_IPT; j++) {
            if (c0 + j < nb) local[c0 + j] = ex;
            ex += cnt[j];
        }
    }
    if (tid == 0) chunk_tot[blockIdx.x] = tot;
}

// one block: exclusive scan of the chunk totals (a kernel of its own: the launch boundary orders it
// after every chunk's total, where a last-block-done hand-off cost each block an agent-scope fence —
// an L2 write-back — and made the scan 37 us at C3's 415 chunks)
constexpr int PKC_PT = 8;
__global__ __launch_bounds__(1024) void k_pkm_cscan(const u32* __restrict__ chunk_tot, u32 nch, u32* __restrict__ chunk_pre) {
    __shared__ u32 s_wave[1024 / 64];
    const int tid = threadIdx.x;
    u32 carry = 0;
    for (u32 base = 0; base < nch; base += 1024 * PKC_PT) {  // (one pass up to 8192 chunks = 2^31 blocks)
        const u32 k0 = base + (u32)tid * PKC_PT;
        u32 v[PKC_PT], sum = 0;
#pragma unroll
        for (int j = 0; j < PKC_PT; j++) {
            v[j] = k0 + j < nch ? chunk_tot[k0 + j] : 0u;
            sum += v[j];
        }
        u32 t2;
        u32 e = block_scan_u32<1024>(sum, s_wave, &t2);
#pragma unroll
        for (int j = 0; j < PKC_PT; j++) {
            if (k0 + j < nch) chunk_pre[k0 + j] = carry + e;
            e += v[j];
        }
        carry += t2;
        __syncthreads();
    }
}

__global__ __launch_bounds__(PKM_NT) void k_pkm_place(const i64* __restrict__ pks, const u64* __restrict__ rkey, u64 ncap,
                                                      const u64* __restrict__ dn, i64 lo_block, u64 nb,
                                                      const u64* __restrict__ masks, const u32* __restrict__ local,
                                                      const u32* __restrict__ chunk_pre, i64* __restrict__ out_pk,
                                                      u32* __restrict__ out_perm) {
    const u64 n = min(*dn, ncap);
    for (u64 r = (u64)blockIdx.x * PKM_NT + threadIdx.x; r < n; r += (u64)gridDim.x * PKM_NT) {
        const i64 pk = rkey ? wk::int_key_pk(rkey[r]) : pks[r];
        const u64 b = (u64)((pk >> 6) - lo_block);
        if (b >= nb) continue;
        const u64 below = masks[b] & ((1ull << (pk & 63)) - 1);
        const u32 pos = chunk_pre[b / PKM_CH] + local[b] + (u32)__popcll(below);
        out_pk[pos] = pk;
        out_perm[pos] = (u32)r;
    }
}

// ---- segmented sort: keys ascending in their top bits (a side in walk order: the leaf tree's bucket)
// ordered by the whole key inside each run of equal top bits.  One workgroup per tile of SEG_T
// entries: the tile's keys plus SEG_H = RS_SEG_MAX on each side go to LDS in one coalesced pass (so
// every run of at most RS_SEG_MAX entries that touches the tile lies inside); the runs' bounds come
// from a block-wide max-scan of the run heads and a min-scan of the next heads; each entry's place
// = its run's start + the number of smaller keys in the run, counted with independent LDS reads (the
// lanes of one run read the same word: a broadcast).  err |= 1: a duplicate key or descending top
// bits; 4: a run longer than RS_SEG_MAX (the caller sorts with kd_sort_side_into instead).
// (Round 4's form scanned each entry's neighbours one dependent LDS read at a time: 0.33 ms per 50M
// C4 side of ~3-entry leaf trees, but 4.2 ms per 100M C3 side of ~64-entry ones.)
constexpr int RS_SEG_MAX = 512;
// halo SEG_H: RS_SEG_MAX, or 128 when the caller knows every run is at most that long (C4's ~3-entry
// leaf trees: 0.34 vs 0.46 ms per 50M side; C3's ~64-entry ones likewise)
#ifndef KD_SEG_IPT
#define KD_SEG_IPT 8
#endif
constexpr int SEG_NT = 256, SEG_IPT = KD_SEG_IPT, SEG_T = SEG_NT * SEG_IPT, SEG_HS = 128;

// block-wide inclusive scan (op = max or min) of one u32 per thread, in thread order
template <bool MAX>
__device__ __forceinline__ u32 seg_block_scan(u32 v, u32* s_w, bool reverse) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int NW = SEG_NT / 64;
    u32 x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = reverse ? __shfl_down(x, o, 64) : __shfl_up(x, o, 64);
        const bool in = reverse ? lane + o < 64 : lane >= o;
        if (in) x = MAX ? (y > x ? y : x) : (y < x ? y : x);
    }
    if (lane == (reverse ? 0 : 63)) s_w[wv] = x;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const u32 y = s_w[w];
        if (reverse ? w > wv : w < wv) x = MAX ? (y > x ? y : x) : (y < x ? y : x);
    }
    __syncthreads();
    return x;
}

// BM (runs of up to 64 keys that differ only in their low 6 bits — an int-PK leaf tree of one 2^30
// wrap, C3's fallback): each run's keys set their bit in a 64-bit map (at slot head / 2: heads of
// runs of two or more entries are at least two apart), and an entry's rank is the popcount of the
// bits below its own — O(1) per entry instead of a scan of its run.  A run whose map does not hold
// one bit per entry (a key differing above bit 5, or a duplicate) is scanned as before.
template <int SEG_H, bool BM>
__global__ __launch_bounds__(SEG_NT) void k_seg_sort(const u64* __restrict__ key, u64 n, int shift, u64* __restrict__ kout,
                                                     u32* __restrict__ order, u32* __restrict__ err) {
    constexpr int SEG_E = SEG_T + 2 * SEG_H, SEG_EPT = SEG_E / SEG_NT;  // staged entries, per thread (contiguous)
    static_assert(SEG_E % SEG_NT == 0 && SEG_E < 65536, "segmented-sort tile shape");
    __shared__ u64 s_k[SEG_E];
    __shared__ u64 s_bm[BM ? SEG_E / 2 : 1];
    __shared__ u16 s_st[SEG_E];  // start of the entry's run (LDS index)
    __shared__ u16 s_en[SEG_E];  // end (exclusive; SEG_E fits 16 bits)
    __shared__ u32 s_w[SEG_NT / 64];
    __shared__ u32 s_inc[SEG_NT];
    const int tid = threadIdx.x;
    const u64 ntiles = (n + SEG_T - 1) / SEG_T;
    // Persistent grid: tile t + gridDim.x's keys are loaded into registers (all SEG_EPT loads in
    // flight together, clamped rows masked when staged) while tile t is ranked and written.  (A
    // guarded load-then-store staging loop compiled to one HBM round trip per entry a thread stages.)
    auto geo = [&](u64 t, i64& g0, int& vlo, int& vhi) {
        g0 = (i64)(t * SEG_T) - SEG_H;  // global index of s_k[0]
        vlo = g0 < 0 ? (int)(-g0) : 0;  // valid LDS entries: [vlo, vhi)
        vhi = (int)min<i64>((i64)SEG_E, (i64)n - g0);
    };
    // Addresses are a uniform tile base (SGPRs) + a 32-bit byte offset per lane (LDS-index-sized), so
    // no lane does 64-bit address arithmetic: the kernel is VALU-bound (r5 counters on C4: ~1,200
    // VALU instructions per wave and tile, ~5 waves per SIMD each ~18 % VALU-active)
    u64 v[SEG_EPT];
    auto fetch = [&](u64 t) {
        i64 g0;
        int vlo, vhi;
        geo(t, g0, vlo, vhi);
        const char* kt = (const char*)(key + g0);  // (tile 0: below key; every lane's index is >= vlo)
#pragma unroll
        for (int j = 0; j < SEG_EPT; j++) {
            const int x = tid + j * SEG_NT;
            const u32 xc = (u32)(x < vlo ? vlo : (x >= vhi ? vhi - 1 : x));
            v[j] = *(const u64*)(kt + 8u * xc);
        }
    };
    u64 tile = blockIdx.x;
    if (tile < ntiles) fetch(tile);
    u32 bad = 0;
    for (; tile < ntiles; tile += gridDim.x) {  // block-uniform
        i64 g0;
        int vlo, vhi;
        geo(tile, g0, vlo, vhi);
#pragma unroll
        for (int j = 0; j < SEG_EPT; j++) {
            const int x = tid + j * SEG_NT;
            s_k[x] = (x >= vlo && x < vhi) ? v[j] : 0;
        }
        __syncthreads();
        if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);
        // run heads: an entry whose top bits differ from its predecessor's (or the first valid entry);
        // invalid entries are runs of their own.  Starts: the last head at or before the entry (a
        // max-scan of head index + 1, 0 = none yet); ends: the first head after it (a min-scan from
        // the right)
        // (the thread's SEG_EPT contiguous keys and its predecessor's read once; heads kept as bits)
        static_assert(SEG_EPT <= 32, "head bits");
        const int x0 = tid * SEG_EPT;
        u64 kk[SEG_EPT + 1];
        kk[0] = x0 > 0 ? s_k[x0 - 1] : 0;
#pragma unroll
        for (int j = 0; j < SEG_EPT; j++) kk[j + 1] = s_k[x0 + j];
        u32 hm = 0;
#pragma unroll
        for (int j = 0; j < SEG_EPT; j++) {
            const int x = x0 + j;
            const bool valid = x >= vlo && x < vhi;
            const bool head = !valid || x == vlo || ((kk[j + 1] ^ kk[j]) >> shift) != 0;
            hm |= head ? 1u << j : 0u;
            // descending top bits: checked at the heads of the tile's own range (each boundary once)
            if (head && valid && x > vlo && x >= SEG_H && x < SEG_H + SEG_T && (kk[j + 1] >> shift) < (kk[j] >> shift))
                bad |= 1u;
        }
        u32 st_loc[SEG_EPT], en_loc[SEG_EPT];
        u32 runp1 = 0;
#pragma unroll
        for (int j = 0; j < SEG_EPT; j++) {
            if ((hm >> j) & 1u) runp1 = (u32)(x0 + j) + 1;
            st_loc[j] = runp1;
        }
        u32 nxt = SEG_E;
#pragma unroll
        for (int j = SEG_EPT - 1; j >= 0; j--) {
            en_loc[j] = nxt;
            if ((hm >> j) & 1u) nxt = (u32)(x0 + j);
        }
        const u32 fwd = seg_block_scan<true>(runp1, s_w, false);
        s_inc[tid] = fwd;
        __syncthreads();
        const u32 before = tid ? s_inc[tid - 1] : 0u;  // the last head before this thread's chunk (+1)
        __syncthreads();
        const u32 bwd = seg_block_scan<false>(nxt, s_w, true);
        s_inc[tid] = bwd;
        __syncthreads();
        const u32 after = tid + 1 < SEG_NT ? s_inc[tid + 1] : (u32)SEG_E;  // the first head after the chunk
#pragma unroll
        for (int j = 0; j < SEG_EPT; j++) {
            s_st[x0 + j] = (u16)((st_loc[j] ? st_loc[j] : before) - 1);
            s_en[x0 + j] = (u16)(en_loc[j] != (u32)SEG_E ? en_loc[j] : after);
        }
        __syncthreads();
        if (BM) {  // the runs' bit maps: cleared by the heads, then every entry of the run sets its bit
#pragma unroll
            for (int j = 0; j < SEG_EPT; j++) {
                const int x = x0 + j;
                const u32 s0 = s_st[x], len = s_en[x] - s0;
                if (x >= vlo && x < vhi && (u32)x == s0 && len >= 2 && len <= 64) s_bm[x >> 1] = 0;
            }
            __syncthreads();
            // a thread's entries are contiguous, so its bits are OR'd per run in a register and each
            // (thread, run) pair does one LDS atomic: ~1.3 per thread instead of one per entry, the
            // ~7 threads of a 64-entry run contending instead of its 64 entries
            u64 acc = 0;
            u32 cur = 0;
#pragma unroll
            for (int j = 0; j < SEG_EPT; j++) {
                const int x = x0 + j;
                const u32 s0 = s_st[x], len = s_en[x] - s0;
                if (s0 != cur) {
                    if (acc) atomicOr((unsigned long long*)&s_bm[cur >> 1], acc);
                    acc = 0;
                    cur = s0;
                }
                if (x >= vlo && x < vhi && len >= 2 && len <= 64) {
                    const u64 k = s_k[x], hk = s_k[s0];
                    if (((k ^ hk) >> 6) == 0) acc |= 1ull << (k & 63);
                }
            }
            if (acc) atomicOr((unsigned long long*)&s_bm[cur >> 1], acc);
            __syncthreads();
        }
        // ranks of the tile's own entries; an entry's place = tile base + its LDS-index destination
        char* const ko = (char*)(kout + g0);
        char* const oo = (char*)(order + g0);
        const u32 og = (u32)g0;  // (mod 2^32: g0 + x of a real entry is in [0, n))
        const bool lo_open = g0 > 0, hi_open = g0 + SEG_E < (i64)n;  // block-uniform
#pragma unroll 2
        for (int j = 0; j < SEG_IPT; j++) {
            const int x = SEG_H + j * SEG_NT + tid;  // consecutive lanes: consecutive entries
            if (x >= vhi) break;
            const u64 k = s_k[x];
            const u32 s0 = s_st[x], e0 = s_en[x];
            if ((s0 == 0 && lo_open) || (e0 == (u32)SEG_E && hi_open) || e0 - s0 > (u32)RS_SEG_MAX) {
                bad |= 4u;  // a run longer than RS_SEG_MAX (or reaching past the halo)
                continue;
            }
            if (BM && e0 - s0 >= 2 && e0 - s0 <= 64) {
                const u64 bm = s_bm[s0 >> 1];
                if ((u32)__popcll(bm) == e0 - s0) {  // one bit per entry: distinct keys, ranked by the map
                    const u32 dl = s0 + (u32)__popcll(bm & ((1ull << (k & 63)) - 1));
                    *(u64*)(ko + 8u * dl) = k;
                    *(u32*)(oo + 4u * dl) = og + (u32)x;
                    continue;
                }
            }
            u32 rank = 0, dup = 0;
            u32 y = s0;
            for (; y + 4 <= e0; y += 4) {
                const u64 a = s_k[y], b = s_k[y + 1], c = s_k[y + 2], d = s_k[y + 3];
                rank += (a < k) + (b < k) + (c < k) + (d < k);
                dup += (a == k) + (b == k) + (c == k) + (d == k);
            }
            for (; y < e0; y++) {
                const u64 a = s_k[y];
                rank += a < k;
                dup += a == k;
            }
            bad |= dup > 1 ? 1u : 0u;
            const u32 dl = s0 + rank;
            *(u64*)(ko + 8u * dl) = k;
            *(u32*)(oo + 4u * dl) = og + (u32)x;
        }
        __syncthreads();  // s_k / s_st / s_en are restaged for the next tile
    }
    if (__ballot(bad != 0) && bad) atomicOr(err, bad);
}

// ---------------------------------------------------------------------------------------------
// host side
// the varying-bit mask -> compaction runs (at most RS_MAXRUNS: the narrowest gaps are absorbed)
static SortPlan make_plan(u64 vary, u64 k0) {
    SortPlan p{};
    u32 lo[32], hi[32], nr = 0;  // runs [lo, hi)
    for (u32 b = 0; b < 64;) {
        if (!((vary >> b) & 1)) { b++; continue; }
        u32 e = b;
        while (e < 64 && ((vary >> e) & 1)) e++;
        lo[nr] = b;
        hi[nr] = e;
        nr++;
        b = e;
    }
    while (nr > (u32)RS_MAXRUNS) {  // merge the pair of neighbouring runs with the narrowest gap
        u32 best = 0;
        for (u32 r = 1; r + 1 < nr; r++)
            if (lo[r + 1] - hi[r] < lo[best + 1] - hi[best]) best = r;
        hi[best] = hi[best + 1];
        for (u32 r = best + 1; r + 1 < nr; r++) { lo[r] = lo[r + 1]; hi[r] = hi[r + 1]; }
        nr--;
    }
    u64 used = 0;
    u32 pos = 0;
    for (u32 r = 0; r < nr; r++) {
        const u32 len = hi[r] - lo[r];
        const u64 m = len >= 64 ? ~0ull : ((1ull << len) - 1);
        p.mask[r] = m;
        p.lo[r] = lo[r];
        p.pos[r] = pos;
        used |= m << lo[r];
        pos += len;
    }
    p.nruns = nr;
    p.bits = pos;
    p.kconst = k0 & ~used;
    return p;
}

struct SortState {
    u64* status = nullptr;
    u32* tctr = nullptr;
    u32* hist = nullptr;
    u32* gbase = nullptr;
};

static int rs_epoch(kd_ctx* ctx, u64 status_bytes, SortState& S, u32* ep) {
    const size_t before = ctx->bufs["rs.status"].bytes;
    void* p;
    int rc = ensure(ctx, "rs.status", status_bytes, &p);
    if (rc) return rc;
    S.status = (u64*)p;
    const size_t after = ctx->bufs["rs.status"].bytes;
    if (after != before || ctx->rs_epoch + 1 >= RS_EPOCHS) {  // fresh memory, or the epochs wrapped
        KD_HIP(hipMemsetAsync(p, 0, after, ctx->stream));
        ctx->rs_epoch = 0;
    }
    *ep = ++ctx->rs_epoch;
    return KD_OK;
}

// resident k_sort_pass workgroups per CU (persistent grid when the count lives on the device)
template <typename CK, bool FIRST, bool LAST, bool IN64>
static int rs_occupancy(kd_ctx* ctx) {
    constexpr int IPT = sizeof(CK) == 4 ? KD_RS_IPT32 : KD_RS_IPT64;
    return occupancy(ctx, (const void*)k_sort_pass<CK, RS_NT, IPT, FIRST, LAST, IN64>, RS_NT, 0);
}

template <typename CK, bool FIRST, bool LAST, bool IN64>
static int rs_launch_pass(kd_ctx* ctx, SortState& S, const void* kin, const u32* vin, void* kout, u32* vout, u64 ncap,
                          const u64* dn, int pass, int shift, int width, const SortPlan& plan) {
    constexpr int IPT = sizeof(CK) == 4 ? KD_RS_IPT32 : KD_RS_IPT64;
    constexpr u64 TILE = (u64)RS_NT * IPT;
    const u64 ntiles = (ncap + TILE - 1) / TILE;
    // host count: one workgroup per tile; device count: at most the resident workgroups, each
    // taking tiles until the count is covered
    const u64 grid = dn ? std::min<u64>(ntiles, (u64)ctx->n_cu * rs_occupancy<CK, FIRST, LAST, IN64>(ctx)) : ntiles;
    if (grid == 0) return KD_OK;
    u32 ep;
    int rc = rs_epoch(ctx, ntiles * RS_RD * 8, S, &ep);
    if (rc) return rc;
    const u32* gb = S.gbase + pass * RS_RD;
    u32* tc = S.tctr + pass;
    u64* status = S.status;
    return launch(ctx, "k_sort_pass", [&] {
        hipLaunchKernelGGL((k_sort_pass<CK, RS_NT, IPT, FIRST, LAST, IN64>), dim3((unsigned)grid), dim3(RS_NT), 0,
                           ctx->stream, kin, vin, kout, vout, ncap, dn, shift, (u32)((1u << width) - 1), gb, status, ep, tc,
                           plan);
    });
}

// the digit passes: key_in = the caller's 64-bit keys (in64) or compact keys (the first pass's values
// are then the input indices either way); the last pass writes 64-bit keys and the values
template <typename CK>
static int rs_passes(kd_ctx* ctx, SortState& S, const void* key_in, bool in64, u64* key_out, u32* order, u64 ncap,
                     const u64* dn, int npass, int width, const SortPlan& plan) {
    int rc;
    void *kb[2], *vb[2];
    if (npass > 1) {
        if ((rc = ensure(ctx, "rs.k0", ncap * sizeof(CK), &kb[0]))) return rc;
        if ((rc = ensure(ctx, "rs.v0", ncap * 4, &vb[0]))) return rc;
    }
    if (npass > 2) {
        if ((rc = ensure(ctx, "rs.k1", ncap * sizeof(CK), &kb[1]))) return rc;
        if ((rc = ensure(ctx, "rs.v1", ncap * 4, &vb[1]))) return rc;
    }
    for (int p = 0; p < npass; p++) {
        const bool first = p == 0, last = p == npass - 1;
        const void* kin = first ? key_in : kb[(p - 1) & 1];
        const u32* vin = first ? nullptr : (const u32*)vb[(p - 1) & 1];
        void* kout = last ? (void*)key_out : kb[p & 1];
        u32* vout = last ? order : (u32*)vb[p & 1];
        const int sh = p * width;
#define KD_RSP(F, L, I) rs_launch_pass<CK, F, L, I>(ctx, S, kin, vin, kout, vout, ncap, dn, p, sh, width, plan)
        if (first && in64) rc = last ? KD_RSP(true, true, true) : KD_RSP(true, false, true);
        else if (first) rc = last ? KD_RSP(true, true, false) : KD_RSP(true, false, false);
        else rc = last ? KD_RSP(false, true, false) : KD_RSP(false, false, false);
#undef KD_RSP
        if (rc) return rc;
    }
    return KD_OK;
}

static int rs_state(kd_ctx* ctx, int npass, SortState& S) {
    void *tc, *hist, *gb;
    int rc;
    if ((rc = ensure(ctx, "rs.tctr", 64, &tc))) return rc;
    if ((rc = ensure(ctx, "rs.hist", 8 * RS_RD * 4, &hist))) return rc;
    if ((rc = ensure(ctx, "rs.gbase", 8 * RS_RD * 4, &gb))) return rc;
    S.tctr = (u32*)tc;
    S.hist = (u32*)hist;
    S.gbase = (u32*)gb;
    KD_HIP(hipMemsetAsync(tc, 0, 64, ctx->stream));
    KD_HIP(hipMemsetAsync(hist, 0, (size_t)npass * RS_RD * 4, ctx->stream));
    return KD_OK;
}

static void plan_passes(const SortPlan& plan, int* npass, int* width) {
    *npass = (int)((plan.bits + RS_RB - 1) / RS_RB);
    *width = *npass ? (int)((plan.bits + *npass - 1) / *npass) : 0;  // the bits spread evenly over the passes
}

// keys: key_in -> key_out (sorted), order[k] = input index of sorted entry k.  info (host, may be
// NULL): which key bits vary (kd_keys_scan); without it one 16-byte read-back finds them.
static int sort_keys(kd_ctx* ctx, const u64* key_in, u64* key_out, u32* order, u64 n, bool inplace,
                     const kd_keys_info* info) {
    int rc;
    const unsigned gs = (unsigned)std::max<u64>(1, std::min<u64>((n + 255) / 256, (u64)ctx->n_cu * 8));
    u64 vary, k0;
    if (info) {
        vary = info->vary;
        k0 = info->key0;
    } else {
        void* bits;
        if ((rc = ensure(ctx, "rs.bits", 16, &bits))) return rc;
        KD_HIP(hipMemsetAsync(bits, 0, 16, ctx->stream));
        rc = launch(ctx, "k_rs_bits", [&] {
            hipLaunchKernelGGL(k_rs_bits, dim3(gs), dim3(256), 0, ctx->stream, key_in, n, (u64*)bits);
        });
        if (rc) return rc;
        u64 hv[2] = {0, 0};
        KD_HIP(hipMemcpyAsync(hv, bits, 8, hipMemcpyDeviceToHost, ctx->stream));
        KD_HIP(hipMemcpyAsync(hv + 1, key_in, 8, hipMemcpyDeviceToHost, ctx->stream));
        KD_HIP(hipStreamSynchronize(ctx->stream));
        vary = hv[0];
        k0 = hv[1];
    }
    if (vary == 0) {  // every key equal (n == 1, or duplicates): identity order
        if (key_out != key_in) KD_HIP(hipMemcpyAsync(key_out, key_in, n * 8, hipMemcpyDeviceToDevice, ctx->stream));
        return launch(ctx, "k_iota", [&] {
            hipLaunchKernelGGL(k_iota_u32, dim3(gs), dim3(256), 0, ctx->stream, order, n);
        });
    }
    const SortPlan plan = make_plan(vary, k0);
    int npass, width;
    plan_passes(plan, &npass, &width);
    if (inplace && npass == 1) {  // the single pass would read and write the caller's array
        void* tmp;
        if ((rc = ensure(ctx, "rs.kin", n * 8, &tmp))) return rc;
        KD_HIP(hipMemcpyAsync(tmp, key_in, n * 8, hipMemcpyDeviceToDevice, ctx->stream));
        key_in = (const u64*)tmp;
    }
    SortState S;
    if ((rc = rs_state(ctx, npass, S))) return rc;
    const bool narrow = plan.bits <= 32;
    constexpr u64 HCH = (u64)RS_HIST_NT * RS_HIST_IPT;
    const unsigned hg = (unsigned)std::max<u64>(1, std::min<u64>((n + HCH - 1) / HCH, (u64)ctx->n_cu * 2));
    rc = launch(ctx, "k_sort_hist", [&] {
        if (narrow)
            hipLaunchKernelGGL(k_sort_hist<u32>, dim3(hg), dim3(RS_HIST_NT), 0, ctx->stream, key_in, n, (const u64*)nullptr,
                               npass, width, plan, S.hist);
        else
            hipLaunchKernelGGL(k_sort_hist<u64>, dim3(hg), dim3(RS_HIST_NT), 0, ctx->stream, key_in, n, (const u64*)nullptr,
                               npass, width, plan, S.hist);
    });
    if (rc) return rc;
    rc = launch(ctx, "k_sort_scan", [&] {
        hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(RS_RD), 0, ctx->stream, (const u32*)S.hist, npass, S.gbase);
    });
    if (rc) return rc;
    return narrow ? rs_passes<u32>(ctx, S, key_in, true, key_out, order, n, nullptr, npass, width, plan)
                  : rs_passes<u64>(ctx, S, key_in, true, key_out, order, n, nullptr, npass, width, plan);
}

static int gather_and_check(kd_ctx* ctx, const u8* oid_in, u8* oid_out, const u32* order, const u64* key_sorted, u64 n,
                            u32* d_dup) {
    const unsigned gs = (unsigned)std::max<u64>(1, std::min<u64>((n + 255) / 256, (u64)ctx->n_cu * 8));
    int rc;
    if (oid_in) {
        if ((rc = launch(ctx, "k_gather_oid", [&] {
                 hipLaunchKernelGGL(k_gather_oid, dim3(gs), dim3(256), 0, ctx->stream, oid_in, order, n, oid_out);
             })))
            return rc;
    }
    if (d_dup) {
        KD_HIP(hipMemsetAsync(d_dup, 0, 4, ctx->stream));
        if ((rc = launch(ctx, "k_check_sorted", [&] {
                 hipLaunchKernelGGL(k_check_sorted, dim3(gs), dim3(256), 0, ctx->stream, key_sorted, n, d_dup);
             })))
            return rc;
    }
    return KD_OK;
}

// the plan of a pk sort: every pk lies in [lo, hi], so the sortable keys share the bits above the
// highest bit in which lo and hi differ
static SortPlan pk_plan(i64 lo, i64 hi) {
    const u64 a = (u64)lo ^ (1ull << 63), b = (u64)hi ^ (1ull << 63);
    const u64 d = a ^ b;
    const u64 vary = d ? (d >> 63 ? ~0ull : ((1ull << (64 - __builtin_clzll(d))) - 1)) : 0;
    SortPlan p = make_plan(vary, a);
    p.out_xor = 1ull << 63;
    return p;
}

}  // namespace kd

using namespace kd;

extern "C" int kd_sort_side_into(kd_ctx* ctx, const uint64_t* d_key_in, const uint8_t* d_oid_in, uint64_t* d_key_out,
                                 uint8_t* d_oid_out, uint32_t* d_order, uint64_t n, uint32_t* d_dup,
                                 const kd_keys_info* info) {
    KD_CHECK(ctx && (n == 0 || (d_key_in && d_key_out && d_order)), "kd_sort_side_into: NULL");
    KD_CHECK(!d_oid_in == !d_oid_out, "kd_sort_side_into: OID input and output go together");
    KD_CHECK(n < 0xFFFFFFFFull, "kd_sort_side_into: side too large for uint32 indices");
    KD_CHECK(n == 0 || ((const void*)d_key_in != (const void*)d_key_out &&
                        (!d_oid_in || (const void*)d_oid_in != (const void*)d_oid_out)),
             "kd_sort_side_into: outputs must not alias the inputs (kd_sort_side sorts in place)");
    KD_HIP(hipSetDevice(ctx->device));
    if (n == 0) {
        if (d_dup) KD_HIP(hipMemsetAsync(d_dup, 0, 4, ctx->stream));
        return KD_OK;
    }
    int rc = sort_keys(ctx, d_key_in, d_key_out, d_order, n, false, info);
    if (rc) return rc;
    return gather_and_check(ctx, d_oid_in, d_oid_out, d_order, d_key_out, n, d_dup);
}

extern "C" int kd_sort_side(kd_ctx* ctx, uint64_t* d_key, uint8_t* d_oid, uint32_t* d_order, uint64_t n,
                            uint32_t* h_dup) {
    KD_CHECK(ctx && (n == 0 || (d_key && d_order)), "kd_sort_side: NULL");
    KD_CHECK(n < 0xFFFFFFFFull, "kd_sort_side: side too large for uint32 indices");
    KD_HIP(hipSetDevice(ctx->device));
    if (h_dup) *h_dup = 0;
    if (n == 0) return KD_OK;
    int rc = sort_keys(ctx, d_key, d_key, d_order, n, true, nullptr);
    if (rc) return rc;
    void *o2 = nullptr, *dup = nullptr;
    if (d_oid && (rc = ensure(ctx, "rs.oid", n * 20, &o2))) return rc;
    if (h_dup && (rc = ensure(ctx, "rs.dup", 16, &dup))) return rc;
    if ((rc = gather_and_check(ctx, d_oid, (u8*)o2, d_order, d_key, n, (u32*)dup))) return rc;
    if (d_oid) KD_HIP(hipMemcpyAsync(d_oid, o2, n * 20, hipMemcpyDeviceToDevice, ctx->stream));  // in place
    if (h_dup) {
        KD_HIP(hipMemcpyAsync(h_dup, dup, 4, hipMemcpyDeviceToHost, ctx->stream));
        KD_HIP(hipStreamSynchronize(ctx->stream));
    }
    return KD_OK;
}

extern "C" int kd_sort_segmented_into(kd_ctx* ctx, const uint64_t* d_key_in, uint64_t* d_key_out, uint32_t* d_order,
                                      uint64_t n, int seg_bits, int max_seg, uint32_t* d_err) {
    KD_CHECK(ctx && d_err && (n == 0 || (d_key_in && d_key_out && d_order)), "kd_sort_segmented_into: NULL");
    KD_CHECK(n < 0xFFFFFFFFull, "kd_sort_segmented_into: side too large for uint32 indices");
    KD_CHECK(seg_bits > 0 && seg_bits < 64, "kd_sort_segmented_into: seg_bits %d", seg_bits);
    KD_CHECK(n == 0 || (const void*)d_key_in != (const void*)d_key_out, "kd_sort_segmented_into: output aliases input");
    KD_HIP(hipSetDevice(ctx->device));
    if (n == 0) return KD_OK;
    const u64 ntiles = (n + SEG_T - 1) / SEG_T;
    const bool small = max_seg > 0 && max_seg <= SEG_HS;
    // the bit-map ranks for leaf trees of more than 16 entries (int-PK leaf trees hold up to 64; a
    // hash-PK bucket's few entries differ above bit 5 and are scanned)
    const bool bm = small && max_seg > 16;
    // one workgroup per tile (the kernel also walks tiles grid-stride with the next tile's keys
    // prefetched, but a resident grid of occupancy x CUs measured slower: 0.272 vs 0.250 ms per 50M
    // C4 side, r5e)
    const unsigned grid = (unsigned)ntiles;
    return launch(ctx, "k_seg_sort", [&] {
        if (small && bm)
            hipLaunchKernelGGL((k_seg_sort<SEG_HS, true>), dim3(grid), dim3(SEG_NT), 0, ctx->stream, d_key_in, n,
                               64 - seg_bits, d_key_out, d_order, d_err);
        else if (small)
            hipLaunchKernelGGL((k_seg_sort<SEG_HS, false>), dim3(grid), dim3(SEG_NT), 0, ctx->stream, d_key_in, n,
                               64 - seg_bits, d_key_out, d_order, d_err);
        else
            hipLaunchKernelGGL((k_seg_sort<RS_SEG_MAX, false>), dim3(grid), dim3(SEG_NT), 0, ctx->stream, d_key_in, n,
                               64 - seg_bits, d_key_out, d_order, d_err);
    });
}

extern "C" int kd_delta_pk_order(kd_ctx* ctx, const kd_side* base, const kd_side* target, const uint32_t* d_delta,
                                 const uint64_t* d_keys, uint64_t cap, const uint64_t* d_n, int64_t pk_lo, int64_t pk_hi,
                                 int64_t* d_pk, uint32_t* d_perm) {
    KD_CHECK(ctx && base && target && d_n && d_pk && d_perm && (cap == 0 || d_delta || d_keys), "kd_delta_pk_order: NULL");
    KD_CHECK(base->key_mode == KD_KEY_INT && target->key_mode == KD_KEY_INT, "kd_delta_pk_order: KD_KEY_INT sides only");
    KD_CHECK(base->mem == KD_MEM_DEVICE && target->mem == KD_MEM_DEVICE, "kd_delta_pk_order: sides must be device memory");
    KD_CHECK(pk_lo <= pk_hi, "kd_delta_pk_order: pk_lo > pk_hi");
    KD_CHECK(cap < 0xFFFFFFFFull, "kd_delta_pk_order: too many deltas for uint32 indices");
    KD_HIP(hipSetDevice(ctx->device));
    if (cap == 0) return KD_OK;
    int rc;
    void* dz;
    if ((rc = device_zeros(ctx, &dz))) return rc;
    const u64* kA = base->n ? base->key : (const u64*)dz;
    const u64* kB = target->n ? target->key : (const u64*)dz;
    // a bounded pk range: bitmap placement (one mask per 64-pk block)
    const i64 lo_block = pk_lo >> 6, hi_block = pk_hi >> 6;
    const u64 nb = (u64)hi_block - (u64)lo_block + 1;
    const u64 pkm_max = ctx->opt.pkm_max_blocks;  // (tests force the radix path with 0)
    if (nb <= pkm_max && nb / PKM_CH < 0xFFFFFFFFull) {
        void *mbuf[2], *local, *ctot, *cpre, *tpk;
        const u64 nch = (nb + PKM_CH - 1) / PKM_CH;
        if ((rc = ensure(ctx, "pkm.masks0", nb * 8, &mbuf[0]))) return rc;
        if ((rc = ensure(ctx, "pkm.masks1", nb * 8, &mbuf[1]))) return rc;
        const int cur = ctx->pkm_cur & 1;
        void* const masks = mbuf[cur];
        void* const other = mbuf[cur ^ 1];
        if ((rc = ensure(ctx, "pkm.local", nb * 4, &local))) return rc;
        if ((rc = ensure(ctx, "pkm.ctot", nch * 4, &ctot))) return rc;
        if ((rc = ensure(ctx, "pkm.cpre", nch * 4, &cpre))) return rc;
        if ((rc = ensure(ctx, "pkm.pk", cap * 8, &tpk))) return rc;
        // this call's masks must be zero for [0, nb): cleared by the previous call's scan, else here
        ctx->pkm_zero_nb[cur ^ 1] = 0;  // (until this call's scan has cleared it)
        if (ctx->pkm_zero_ptr[cur] != masks || ctx->pkm_zero_nb[cur] < nb) {
            ctx->pkm_zero_nb[cur] = 0;
            KD_HIP(hipMemsetAsync(masks, 0, nb * 8, ctx->stream));
        }
        ctx->pkm_zero_nb[cur] = 0;  // marked below
        const unsigned g1 = (unsigned)std::max<u64>(1, std::min<u64>((cap + PKM_NT - 1) / PKM_NT, (u64)ctx->n_cu * 8));
        rc = launch(ctx, "k_pkm_mark", [&] {
            hipLaunchKernelGGL(k_pkm_mark, dim3(g1), dim3(PKM_NT), 0, ctx->stream, (const uint2*)d_delta, cap, d_n, kA,
                               kB, d_keys, lo_block, nb, (u64*)masks, (i64*)tpk);
        });
        if (rc) return rc;
        rc = launch(ctx, "k_pkm_scan", [&] {
            hipLaunchKernelGGL(k_pkm_scan, dim3((unsigned)nch), dim3(PKM_NT), 0, ctx->stream, (const u64*)masks, nb,
                               (u32*)local, (u32*)ctot, (u64*)other);
        });
        if (rc) return rc;
        ctx->pkm_zero_ptr[cur ^ 1] = other;  // zero for [0, nb) once the scan has run (stream order)
        ctx->pkm_zero_nb[cur ^ 1] = nb;
        ctx->pkm_cur = cur ^ 1;
        rc = launch(ctx, "k_pkm_cscan", [&] {
            hipLaunchKernelGGL(k_pkm_cscan, dim3(1), dim3(1024), 0, ctx->stream, (const u32*)ctot, (u32)nch, (u32*)cpre);
        });
        if (rc) return rc;
        return launch(ctx, "k_pkm_place", [&] {
            hipLaunchKernelGGL(k_pkm_place, dim3(g1), dim3(PKM_NT), 0, ctx->stream, (const i64*)tpk, d_keys, cap, d_n,
                               lo_block, nb, (const u64*)masks, (const u32*)local, (const u32*)cpre, d_pk, d_perm);
        });
    }
    SortPlan plan = pk_plan(pk_lo, pk_hi);
    int npass, width;
    plan_passes(plan, &npass, &width);
    if (npass == 0) {  // a single pk value: at most one delta, in place already
        plan.nruns = 1; plan.mask[0] = 1; plan.lo[0] = 0; plan.pos[0] = 0; plan.bits = 1;
        plan.kconst = ((u64)pk_lo ^ (1ull << 63)) & ~1ull;
        npass = width = 1;
    }
    const bool narrow = plan.bits <= 32;
    void* ck;
    if ((rc = ensure(ctx, "dpk.keys", cap * (narrow ? 4 : 8), &ck))) return rc;
    SortState S;
    if ((rc = rs_state(ctx, npass, S))) return rc;
    const unsigned hg = (unsigned)std::max<u64>(1, std::min<u64>((cap + RS_HIST_NT - 1) / RS_HIST_NT, (u64)ctx->n_cu * 4));
    rc = launch(ctx, "k_dpk_keys", [&] {
        if (narrow)
            hipLaunchKernelGGL(k_dpk_keys<u32>, dim3(hg), dim3(RS_HIST_NT), 0, ctx->stream, (const uint2*)d_delta, cap, d_n,
                               kA, kB, d_keys, npass, width, plan, (u32*)ck, S.hist);
        else
            hipLaunchKernelGGL(k_dpk_keys<u64>, dim3(hg), dim3(RS_HIST_NT), 0, ctx->stream, (const uint2*)d_delta, cap, d_n,
                               kA, kB, d_keys, npass, width, plan, (u64*)ck, S.hist);
    });
    if (rc) return rc;
    rc = launch(ctx, "k_sort_scan", [&] {
        hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(RS_RD), 0, ctx->stream, (const u32*)S.hist, npass, S.gbase);
    });
    if (rc) return rc;
    return narrow ? rs_passes<u32>(ctx, S, ck, false, (u64*)d_pk, d_perm, cap, d_n, npass, width, plan)
                  : rs_passes<u64>(ctx, S, ck, false, (u64*)d_pk, d_perm, cap, d_n, npass, width, plan);
}
