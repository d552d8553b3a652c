// kd_classify2.hip — classify2: the two-way tree diff as one single-pass HIP kernel on gfx950.
//
// Replaces libgit2's tree-to-tree diff as consumed by RichBaseDataset.diff_feature
// (/root/reference/kart/rich_base_dataset.py:205-300): both commits' feature leaves arrive as
// strictly ascending join keys + 20-byte blob OIDs; a key on one side only is an insert/delete, a
// key on both sides with different OIDs is an update (GIT_DELTA_ADDED/DELETED/MODIFIED).
//
//   k_partition2  merge-path split points of the union sequence: 8 lanes per tile boundary,
//                 8-ary search (8 dependent HBM round trips instead of ~24 for binary search)
//   k_join2       per 2048-item tile (256 threads x 8 items):
//                   0. the tile's key ranges (both sides) -> LDS as 16-B chunks, every load issued
//                      before any use
//                   A. per-thread merge path over 8 items in LDS; each item's outcome (kind, local
//                      indices) kept in a register record
//                   B. OID compare of matched pairs: 20-B OIDs loaded in batches straight from HBM
//                   C. block scan of the tile's delta/update counts; records written key-ordered
//                      into a tile-local staging slot (ordered) or appended per tile (unordered)
//   k_place2      one tile per block: output offset from 64-tile group sums (accumulated by the
//                 join) + the earlier tiles of its group; staged records -> final key-ordered
//                 positions; totals from the last block.
// Inputs are read once; the staging round trip costs 16 B per delta.
#include "kd_join.h"

namespace kd {

// ---- merge-path partition: PW lanes per tile boundary, PW-ary search ------------------------------
// part[t] = number of A items among the first min(t*TILE, nA+nB) union items (ties: A first).
// A binary search is ~24 dependent HBM round trips at 10M keys; a 64-ary one needs 4 but fetches
// 128 random lines per round per boundary.  PW = 8 lanes: 8 round trips, 16 lines per round.
constexpr int PW = 8;
constexpr u64 C2_GROUP = 64;  // tiles per group sum (k_place2 offsets)
#ifndef KD_C2_STAGE_PAD
#define KD_C2_STAGE_PAD 32
#endif
// staging slot stride in records: one tile plus a pad, so the slots' hot first lines do not all
// fall on the same HBM channels (a 16 KB power-of-two stride would)
constexpr u64 C2_STAGE = C2_TILE + KD_C2_STAGE_PAD;
#ifndef KD_PLACE_NT
#define KD_PLACE_NT 64  // one wave per tile: up to 32 staged records per lane, all loads in flight
#endif

__global__ __launch_bounds__(256) void k_partition2(const u64* __restrict__ A, u64 nA, const u64* __restrict__ B,
                                                    u64 nB, u64 ntiles, u64* __restrict__ part,
                                                    u64* __restrict__ zero_counts, u32* __restrict__ zero_err,
                                                    u64* __restrict__ zero_gsum, u64 n_gsum) {
    // the join's counters start at zero: cleared here (stream-ordered before k_join2) instead of
    // by separate memset launches
    if (blockIdx.x == 0 && threadIdx.x < 4) zero_counts[threadIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 4) *zero_err = 0;
    for (u64 k = (u64)blockIdx.x * 256 + threadIdx.x; k < n_gsum; k += (u64)gridDim.x * 256) zero_gsum[k] = 0;
    const u64 t = ((u64)blockIdx.x * 256 + threadIdx.x) / PW;
    const int sub = threadIdx.x % PW;
    const int lane = threadIdx.x & 63;
    const int grp = lane / PW;  // group within the wave
    if (t > ntiles) return;  // whole groups exit together (group = PW consecutive lanes)
    const u64 total = nA + nB;
    u64 d = t * (u64)C2_TILE;
    if (d > total) d = total;
    // smallest i in [lo, hi] with pred(i) = (i == hi) || A[i] > B[d-1-i]
    u64 lo = d > nB ? d - nB : 0, hi = d < nA ? d : nA;
    while (hi > lo) {
        const u64 step = (hi - lo + PW - 1) / PW;  // lane s probes lo + step*(s+1) - 1
        const u64 probe = lo + step * (u64)(sub + 1) - 1;
        bool p = true;
        if (probe < hi) p = A[probe] > B[d - 1 - probe];
        const unsigned long long bal = (__ballot(p) >> (grp * PW)) & ((1ull << PW) - 1);
        if (bal == 0) { lo = hi; break; }  // all probes (the last is hi-1) false -> answer is hi
        const int f = __ffsll(bal) - 1;
        const u64 nh = lo + step * (u64)(f + 1) - 1;
        lo = lo + step * (u64)f;
        hi = nh < hi ? nh : hi;
        if (step == 1) { lo = hi; break; }
    }
    if (sub == 0) part[t] = lo;
}

struct Join2Args {
    const u64* A;
    const u8* oidA;
    u64 nA;
    const u64* B;
    const u8* oidB;
    u64 nB;
    const u64* part;
    const u8* nameA;
    const u64* nameOffA;
    const u8* nameB;
    const u64* nameOffB;
    int hash_mode;
    const u8* dummy;     // >= 64 readable device bytes (target of masked-off lanes' loads)
    uint2* stage_delta;  // ordered mode: tile-local slots of TILE records
    uint2* stage_upd;
    u32* tile_cnt;       // ordered mode: [ntiles*4] inserts, updates, deletes, deltas
    u64* gsum;           // ordered mode: [2*ngroups] per C2_GROUP tiles: deltas | updates<<32, inserts | deletes<<32
    uint2* out_delta;    // unordered mode: final lists, appended per tile
    uint2* out_upd;
    u64* counts;         // unordered mode: [4] inserts, updates, deletes, deltas (atomic)
    u32* err;
};

// The tile's four input byte ranges (A keys, B keys, A OIDs, B OIDs) are copied to LDS as
// 16-byte chunks of their 16-byte-aligned *absolute* addresses: a 16-byte-aligned chunk holding
// any valid byte lies inside one mapped page, so the over-read at either end can never fault, and
// every chunk load is a full-width, fully used global_load_dwordx4 issued before any use.
struct Range {
    u64 base;  // aligned-down absolute address
    u32 nch;   // 16-byte chunks
    u32 skew;  // byte offset of the first element inside chunk 0
};

__device__ __forceinline__ Range mk_range(const void* p, u64 first_byte, u64 end_byte) {
    Range r;
    const u64 a0 = (u64)p + first_byte, a1 = (u64)p + end_byte;
    r.base = a0 & ~(u64)15;
    r.skew = (u32)(a0 - r.base);
    r.nch = end_byte > first_byte ? (u32)((a1 - r.base + 15) >> 4) : 0;
    return r;
}

template <int NT, int IPT>
struct Join2Lds {
    static constexpr int TILE = NT * IPT;
    static constexpr int CH = TILE / 2 + 4;  // 16-B chunks holding the 8-B keys of both ranges
    static constexpr int UNR = (CH + NT - 1) / NT;
    static constexpr int KB = (TILE + NT - 1) / NT;  // A items per thread in the OID phase
};

// UNORD: each tile reserves its output ranges with one atomic add per counter and writes its
// (key-ordered) records straight to the final lists — tiles land in completion order, no staging,
// no scan, no scatter.  Ordered (default): tile-local staging + k_scan_tiles + k_scatter2.
template <int NT, int IPT, bool UNORD>
__global__ __launch_bounds__(NT) void k_join2(Join2Args g) {
    using LD = Join2Lds<NT, IPT>;
    constexpr int TILE = LD::TILE;
    static_assert(TILE <= 4095, "per-item records hold 12-bit local indices");
    constexpr u16 NOP = 0xFFFF;
    __shared__ u32x4 s_ch[LD::CH];
    __shared__ u16 s_partner[TILE];
    __shared__ u8 s_chg[TILE];
    __shared__ u32 s_wave[NT / 64];
    __shared__ u64 s_base[2];

    const int tid = threadIdx.x;
    const u64 tile = blockIdx.x;
    const u64 total = g.nA + g.nB;
    const u64 d0 = tile * (u64)TILE;
    const u64 d1 = d0 + TILE < total ? d0 + TILE : total;
    u64 i0 = g.part[tile], i1 = g.part[tile + 1];
    if (i1 < i0 || d1 - i1 < d0 - i0 || i1 - i0 > d1 - d0) {  // only on unsorted input
        if (tid == 0) {
            atomicOr(g.err, 1u);
            if (!UNORD) {
                u32* c = g.tile_cnt + 4 * tile;
                c[0] = c[1] = c[2] = c[3] = 0;
            }
        }
        return;
    }
    const u64 j0 = d0 - i0, j1 = d1 - i1;
    const int na = (int)(i1 - i0), nb = (int)(j1 - j0);

    // ---- the tile's keys (both ranges) -> LDS as 16-B chunks, all loads in flight together --------
    const Range rka = mk_range(g.A, 8 * i0, 8 * i1), rkb = mk_range(g.B, 8 * j0, 8 * j1);
    const u32 c1 = rka.nch, c2 = c1 + rkb.nch;
    {
        // branch-free issue (out-of-range lanes re-load chunk 0), then the LDS stores
        u32x4 v[LD::UNR];
#pragma unroll
        for (int k = 0; k < LD::UNR; k++) {
            const u32 c0 = tid + k * NT;
            const u32 c = c0 < c2 ? c0 : 0;
            const u64 addr = c < c1 ? rka.base + 16ull * c : rkb.base + 16ull * (c - c1);
            v[k] = *(const __attribute__((address_space(1))) u32x4*)addr;  // global_, not flat_
        }
#pragma unroll
        for (int k = 0; k < LD::UNR; k++) {
            const u32 c = tid + k * NT;
            if (c < c2) s_ch[c] = v[k];
        }
    }
    // lookbehind / lookahead keys (tiny, scalar)
    const bool has_lbA = i0 > 0, has_lbB = j0 > 0, has_la = j1 < g.nB;
    const u64 lbA = has_lbA ? g.A[i0 - 1] : 0;
    const u64 lbB = has_lbB ? g.B[j0 - 1] : 0;
    const u64 la = has_la ? g.B[j1] : 0;
    __syncthreads();
    const u64* sA = (const u64*)((const u8*)s_ch + rka.skew);
    const u64* sB = (const u64*)((const u8*)(s_ch + c1) + rkb.skew);

    // ---- A: per-thread merge path over IPT items (one walk); each item's outcome is kept in a
    //         register: rec = kind << 25 | changed << 24 | jb << 12 | ia  (local 12-bit indices; jb
    //         may be nb = the lookahead B[j1])
    enum : u32 { R_NONE = 0, R_DEL = 1, R_MATCH = 2, R_INS = 3 };
    const int nitems = na + nb;
    const int dd = tid * IPT < nitems ? tid * IPT : nitems;
    const int cnt = (dd + IPT < nitems ? dd + IPT : nitems) - dd;
    int lo = dd - nb > 0 ? dd - nb : 0, hi = dd < na ? dd : na;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (sA[mid] <= sB[dd - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    u32 rec[IPT];
    bool bad = false;
    {
        int ia = lo, jb = dd - lo;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            rec[k] = R_NONE << 25;
            if (k < cnt) {
                if (jb >= nb || (ia < na && sA[ia] <= sB[jb])) {
                    const u64 ka = sA[ia];
                    if (ia > 0 ? sA[ia - 1] >= ka : (has_lbA && lbA >= ka)) bad = true;
                    const bool hb = jb < nb ? true : has_la;
                    const u64 kb = jb < nb ? sB[jb] : la;
                    const bool m = hb && kb == ka;
                    s_partner[ia] = m ? (u16)jb : NOP;
                    rec[k] = ((m ? R_MATCH : R_DEL) << 25) | ((u32)jb << 12) | (u32)ia;
                    ia++;
                } else {
                    const u64 kb = sB[jb];
                    if (jb > 0 ? sB[jb - 1] >= kb : (has_lbB && lbB >= kb)) bad = true;
                    const bool partner = ia > 0 ? sA[ia - 1] == kb : (has_lbA && lbA == kb);
                    rec[k] = ((partner ? R_NONE : R_INS) << 25) | ((u32)jb << 12) | (u32)ia;
                    jb++;
                }
            }
        }
    }
    if (bad) atomicOr(g.err, 1u);
    __syncthreads();

    // ---- B: OID compare of matched pairs.  Lane l takes A items l, l+NT, ...: consecutive lanes
    //         read consecutive 20-B records of both sides (every fetched line fully used); all of a
    //         batch's loads are issued branch-free before the compares ------------------------------
    typedef const __attribute__((address_space(1))) u32* gp32;
    constexpr int BATCH = 4;
#pragma unroll
    for (int k0 = 0; k0 < LD::KB; k0 += BATCH) {
        u32 xa[BATCH][5], xb[BATCH][5];
        bool m[BATCH];
#pragma unroll
        for (int k = 0; k < BATCH; k++) {
            const int a = tid + (k0 + k) * NT;
            const bool in = a < na;
            const u16 p = in ? s_partner[a] : NOP;
            m[k] = p != NOP;
            gp32 pa = in ? (gp32)(g.oidA + 20 * (i0 + a)) : (gp32)g.dummy;
            gp32 pb = m[k] ? (gp32)(g.oidB + 20 * (j0 + p)) : pa;
#pragma unroll
            for (int w = 0; w < 5; w++) { xa[k][w] = pa[w]; xb[k][w] = pb[w]; }
        }
#pragma unroll
        for (int k = 0; k < BATCH; k++) {
            const int a = tid + (k0 + k) * NT;
            if (a < na) {
                u32 d = 0;
#pragma unroll
                for (int w = 0; w < 5; w++) d |= xa[k][w] ^ xb[k][w];
                s_chg[a] = (m[k] && d) ? 1 : 0;
                if (m[k] && g.hash_mode &&
                    !names_eq(g.nameA, g.nameOffA, i0 + a, g.nameB, g.nameOffB, j0 + s_partner[a]))
                    atomicOr(g.err, 2u);
            }
        }
    }
    __syncthreads();

    // ---- C: counts from the registers, block scan, ordered writes ----------------------------------
    u32 nd = 0, nu = 0, ndel = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u32 kind = rec[k] >> 25, ia = rec[k] & 0xFFF;
        if (kind == R_MATCH) {
            if (s_chg[ia]) { nd++; nu++; rec[k] |= 1u << 24; }  // bit 24: OIDs differ
        } else if (kind == R_DEL) { nd++; ndel++; }
        else if (kind == R_INS) nd++;
    }
    u32 tot_packed;
    const u32 off_packed = block_excl_scan<NT>(nd | (nu << 16), s_wave, &tot_packed);
    const u32 tot_del = block_sum<NT>(ndel, s_wave);
    const u32 tnd = tot_packed & 0xFFFF, tnu = tot_packed >> 16;
    u32 od = off_packed & 0xFFFF, ou = off_packed >> 16;
    uint2* sd;
    uint2* su;
    if (UNORD) {
        // four lanes of wave 0 reserve in parallel: deltas, updates (offsets) + inserts, deletes
        if (tid < 4) {
            const u64 v = tid == 0 ? tnd : tid == 1 ? tnu : tid == 2 ? tnd - tnu - tot_del : tot_del;
            const int slot = tid == 0 ? 3 : tid == 1 ? 1 : tid == 2 ? 0 : 2;
            const u64 old = v ? atomicAdd((unsigned long long*)(g.counts + slot), (unsigned long long)v) : 0;
            if (tid < 2) s_base[tid] = old;
        }
        __syncthreads();
        sd = g.out_delta + s_base[0];
        su = g.out_upd ? g.out_upd + s_base[1] : nullptr;
    } else {
        sd = g.stage_delta + tile * (u64)C2_STAGE;
        su = g.stage_upd + tile * (u64)C2_STAGE;
    }
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u32 kind = rec[k] >> 25, ia = rec[k] & 0xFFF, jb = (rec[k] >> 12) & 0xFFF;
        if (kind == R_DEL) sd[od++] = make_uint2((u32)(i0 + ia), KD_NONE);
        else if (kind == R_INS) sd[od++] = make_uint2(KD_NONE, (u32)(j0 + jb));
        else if (kind == R_MATCH && ((rec[k] >> 24) & 1)) {
            const uint2 v = make_uint2((u32)(i0 + ia), (u32)(j0 + jb));
            sd[od++] = v;
            if (su) su[ou++] = v;
        }
    }
    if (!UNORD && tid == 0) {
        u32* c = g.tile_cnt + 4 * tile;
        const u32 tins = tnd - tnu - tot_del;
        c[0] = tins;
        c[1] = tnu;
        c[2] = tot_del;
        c[3] = tnd;
        // group sums (<= 64 tiles x 2048 per 32-bit half: no carry between halves); a handful of
        // atomics per address
        u64* gs = g.gsum + 2 * (tile / C2_GROUP);
        atomicAdd((unsigned long long*)gs, (unsigned long long)(tnd | (u64)tnu << 32));
        atomicAdd((unsigned long long*)gs + 1, (unsigned long long)(tins | (u64)tot_del << 32));
    }
}

// Tile-local staging -> final key-ordered positions; one tile per block.  The tile's output
// offset = the group sums of all earlier C2_GROUP-tile groups + the counts of the earlier tiles of
// its own group (at most ngroups + C2_GROUP - 1 loads, issued together); the last block also
// writes the totals.  Work per block is bounded by one tile, so insert-dense regions do not
// serialise.
template <int NT>
__global__ __launch_bounds__(NT) void k_place2(const uint2* __restrict__ stage_delta, const uint2* __restrict__ stage_upd,
                                               const u32* __restrict__ tile_cnt, const u64* __restrict__ gsum,
                                               u64 ntiles, int tile_items, uint2* __restrict__ out_delta,
                                               uint2* __restrict__ out_upd, u64* __restrict__ counts) {
    __shared__ u64 s_red[4][NT / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const u64 t = blockIdx.x;
    const u64 grp = t / C2_GROUP, ngroups = (ntiles + C2_GROUP - 1) / C2_GROUP;
    const bool last = t == ntiles - 1;
    const u64 g_end = last ? ngroups : grp;  // the last block sums every group for the totals
    u64 pd = 0, pu = 0, si = 0, sx = 0;
    for (u64 k = tid; k < g_end; k += NT) {
        const u64 a = gsum[2 * k];
        if (k < grp) { pd += a & 0xFFFFFFFFu; pu += a >> 32; }
        if (last) {
            const u64 b = gsum[2 * k + 1];
            si += b & 0xFFFFFFFFu; sx += b >> 32;
            if (k >= grp) { pd += a & 0xFFFFFFFFu; pu += a >> 32; }  // totals: all groups
        }
    }
    // counts of the earlier tiles of this group (the last block already has them in the totals)
    const u64 t_lo = grp * C2_GROUP;
    if (!last && tid < (int)(t - t_lo)) {
        const uint4 c = *(const uint4*)(tile_cnt + 4 * (t_lo + tid));
        pd += c.w;
        pu += c.y;
    }
    const uint4 own = *(const uint4*)(tile_cnt + 4 * t);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        pd += __shfl_xor(pd, o, 64); pu += __shfl_xor(pu, o, 64);
        si += __shfl_xor(si, o, 64); sx += __shfl_xor(sx, o, 64);
    }
    if (lane == 0) { s_red[0][wid] = pd; s_red[1][wid] = pu; s_red[2][wid] = si; s_red[3][wid] = sx; }
    __syncthreads();
    pd = pu = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) { pd += s_red[0][w]; pu += s_red[1][w]; }
    if (last) {
        // pd/pu are the totals here; this tile's records start at total - own count
        if (tid == 0) {
            u64 ti = 0, tx = 0;
#pragma unroll
            for (int w = 0; w < NT / 64; w++) { ti += s_red[2][w]; tx += s_red[3][w]; }
            counts[0] = ti;
            counts[1] = pu;
            counts[2] = tx;
            counts[3] = pd;
        }
        pd -= own.w;
        pu -= own.y;
    }
    const uint2* sdp = stage_delta + t * (u64)tile_items;
    const uint2* sup = stage_upd + t * (u64)tile_items;
    // C2_TILE / NT records per thread at most: every load before any store
    constexpr int UC = C2_TILE / NT;
    uint2 v[UC];
#pragma unroll
    for (int j = 0; j < UC; j++) {
        const u32 r = j * NT + tid;
        if (r < own.w) v[j] = sdp[r];
    }
#pragma unroll
    for (int j = 0; j < UC; j++) {
        const u32 r = j * NT + tid;
        if (r < own.w) out_delta[pd + r] = v[j];
    }
    if (out_upd) {
#pragma unroll
        for (int j = 0; j < UC; j++) {
            const u32 r = j * NT + tid;
            if (r < own.y) v[j] = sup[r];
        }
#pragma unroll
        for (int j = 0; j < UC; j++) {
            const u32 r = j * NT + tid;
            if (r < own.y) out_upd[pu + r] = v[j];
        }
    }
}

int diff2_device(kd_ctx* ctx, const kd_side* A, const kd_side* B, u32 flags, u32* d_delta, u32* d_upd,
                 u64* d_counts, u32* d_err) {
    const bool unord = (flags & KD_DIFF_UNORDERED) != 0;
    const u64 nA = A->n, nB = B->n, total = nA + nB;
    KD_CHECK(nA < 0xFFFFFFFFull && nB < 0xFFFFFFFFull, "diff2: side too large for uint32 indices");
    const bool hash = A->key_mode == KD_KEY_HASH || B->key_mode == KD_KEY_HASH;
    KD_CHECK(A->key_mode == B->key_mode, "diff2: key modes differ");
    if (hash) KD_CHECK((nA == 0 || (A->name && A->name_off)) && (nB == 0 || (B->name && B->name_off)),
                       "diff2: KD_KEY_HASH needs filenames");
    const u64 ntiles = (total + C2_TILE - 1) / C2_TILE;
    if (ntiles == 0) {
        KD_HIP(hipMemsetAsync(d_err, 0, sizeof(u32), ctx->stream));
        KD_HIP(hipMemsetAsync(d_counts, 0, 4 * sizeof(u64), ctx->stream));
        return KD_OK;
    }
    void *part, *tcnt, *sdel, *supd, *gsum = nullptr;
    const u64 n_gsum = unord ? 0 : 2 * ((ntiles + C2_GROUP - 1) / C2_GROUP);
    int rc;
    if ((rc = ensure(ctx, "c2.part", (ntiles + 1) * sizeof(u64), &part))) return rc;
    if ((rc = ensure(ctx, "c2.tcnt", ntiles * 4 * sizeof(u32), &tcnt))) return rc;
    if (n_gsum && (rc = ensure(ctx, "c2.gsum", n_gsum * sizeof(u64), &gsum))) return rc;
    if (!unord) {
        if ((rc = ensure(ctx, "c2.sdel", ntiles * C2_STAGE * sizeof(uint2), &sdel))) return rc;
        if ((rc = ensure(ctx, "c2.supd", ntiles * C2_STAGE * sizeof(uint2), &supd))) return rc;
    } else {
        sdel = supd = nullptr;
    }
    void* dz;
    if ((rc = device_zeros(ctx, &dz))) return rc;
    const u64* kA = nA ? A->key : (const u64*)dz;  // an empty side points at device zeros
    const u64* kB = nB ? B->key : (const u64*)dz;
    const u8* empty_oid = (const u8*)dz;
    rc = launch(ctx, "k_partition2", [&] {
        unsigned nb = (unsigned)(((ntiles + 1) * PW + 255) / 256);
        hipLaunchKernelGGL(k_partition2, dim3(nb), dim3(256), 0, ctx->stream, kA, nA, kB, nB, ntiles, (u64*)part,
                           d_counts, d_err, (u64*)gsum, n_gsum);
    });
    if (rc) return rc;
    Join2Args g;
    g.A = kA; g.oidA = nA ? A->oid : empty_oid; g.nA = nA;
    g.B = kB; g.oidB = nB ? B->oid : empty_oid; g.nB = nB;
    g.part = (const u64*)part;
    g.nameA = A->name; g.nameOffA = A->name_off; g.nameB = B->name; g.nameOffB = B->name_off;
    g.hash_mode = hash ? 1 : 0;
    g.dummy = (const u8*)dz;
    g.stage_delta = (uint2*)sdel; g.stage_upd = (uint2*)supd;
    g.tile_cnt = (u32*)tcnt; g.gsum = (u64*)gsum; g.err = d_err;
    g.out_delta = (uint2*)d_delta; g.out_upd = (uint2*)d_upd; g.counts = d_counts;
    if (unord) {
        return launch(ctx, "k_join2", [&] {
            hipLaunchKernelGGL((k_join2<C2_NT, C2_IPT, true>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, g);
        });
    }
    rc = launch(ctx, "k_join2", [&] {
        hipLaunchKernelGGL((k_join2<C2_NT, C2_IPT, false>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, g);
    });
    if (rc) return rc;
    rc = launch(ctx, "k_place2", [&] {
        hipLaunchKernelGGL((k_place2<KD_PLACE_NT>), dim3((unsigned)ntiles), dim3(KD_PLACE_NT), 0, ctx->stream, (const uint2*)sdel,
                           (const uint2*)supd, (const u32*)tcnt, (const u64*)gsum, ntiles, C2_STAGE, (uint2*)d_delta,
                           (uint2*)d_upd, d_counts);
    });
    return rc;
}

}  // namespace kd
