// kd_classify2.hip — classify2: the two-way tree diff as one single-pass HIP kernel on gfx950.
//
// Replaces libgit2's tree-to-tree diff as consumed by RichBaseDataset.diff_feature
// (/root/reference/kart/rich_base_dataset.py:205-300): both commits' feature leaves arrive as
// strictly ascending join keys + 20-byte blob OIDs; a key on one side only is an insert/delete, a
// key on both sides with different OIDs is an update (GIT_DELTA_ADDED/DELETED/MODIFIED).
//
//   k_partition2  merge-path split points of the union sequence: 8 lanes per tile boundary,
//                 8-ary search (8 dependent HBM round trips instead of ~24 for binary search)
//   k_join2       per 1024-item tile (256 threads x 4 items):
//                   0. the tile's keys AND OIDs (both sides) -> LDS by LDS-DMA 16-B chunks, every
//                      load issued before any use: one HBM round trip per tile
//                   A. per-thread merge path over 4 items in LDS; matched pairs' OIDs compared
//                      from LDS; each item's outcome (kind, local indices) kept in a register
//                   B. block scan of the tile's delta/update counts; records written key-ordered
//                      into a tile-local staging slot (ordered) or appended per tile (unordered)
//   k_place2      one tile per block: output offset from 64-tile group sums (accumulated by the
//                 join) + the earlier tiles of its group; staged records -> final key-ordered
//                 positions; totals from the last block.
// Inputs are read once; the staging round trip costs 16 B per delta.
#include "kd_join.h"

namespace kd {

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

// One merge-path split by a group of PW consecutive lanes (PW-ary search, all PW lanes call it
// together): smallest i in [lo, hi] with i == hi || A[i] > B[d-1-i]  (ties: A first).
template <int PW>
__device__ __forceinline__ u64 mp_search(const u64* __restrict__ A, const u64* __restrict__ B, u64 d, u64 lo, u64 hi) {
    const int lane = threadIdx.x & 63, sub = lane % PW, grp = lane / PW;
    while (hi > lo) {
        const u64 step = (hi - lo + PW - 1) / PW;  // lane s probes lo + step*(s+1) - 1
        const u64 probe = lo + step * (u64)(sub + 1) - 1;
        bool p = true;
        if (probe < hi) p = A[probe] > B[d - 1 - probe];
        const unsigned long long bal = (__ballot(p) >> (grp * PW)) & ((PW == 64) ? ~0ull : ((1ull << PW) - 1));
        if (bal == 0) return hi;  // all probes (the last is hi-1) false -> answer is hi
        const int f = __ffsll(bal) - 1;
        const u64 nh = lo + step * (u64)(f + 1) - 1;
        lo = lo + step * (u64)f;
        hi = nh < hi ? nh : hi;
        if (step == 1) return hi;
    }
    return lo;
}

// Merge-path split points part[t] (A items among the first min(t*TILE, nA+nB) union items), two
// levels: one block per group of C2_PG tiles.  The group's two end splits are searched over the
// whole arrays (16 lanes each, 16-ary: ~6 rounds of random HBM reads); every inner split then lies
// inside the box the end splits span (i and d-i are both monotone in d), at most C2_PG tiles wide,
// and is found there by 8 lanes (8-ary) whose probes land in that small, cache-warm region.  This
// replaced one full-array 8-ary search per tile (~8 rounds x 16 random lines for every boundary).
constexpr int C2_PG = 32;
__global__ __launch_bounds__(256) void k_partition2(const u64* __restrict__ A, u64 nA, const u64* __restrict__ B,
                                                    u64 nB, u64 ntiles, u64* __restrict__ part,
                                                    u64* __restrict__ zero_counts, u32* __restrict__ zero_err,
                                                    u64* __restrict__ zero_gsum, u64 n_gsum) {
    // the join's counters start at zero: cleared here (stream-ordered before k_join2) instead of
    // by separate memset launches
    if (blockIdx.x == 0 && threadIdx.x < 4) zero_counts[threadIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 4) *zero_err = 0;
    for (u64 k = (u64)blockIdx.x * 256 + threadIdx.x; k < n_gsum; k += (u64)gridDim.x * 256) zero_gsum[k] = 0;
    __shared__ u64 s_end[2];
    const int tid = threadIdx.x;
    const u64 total = nA + nB;
    const u64 t0 = (u64)blockIdx.x * C2_PG, t1 = t0 + C2_PG < ntiles ? t0 + C2_PG : ntiles;
    if (tid < 32) {  // wave 0: lanes 0-15 -> split t0, lanes 16-31 -> split t1
        const u64 t = tid < 16 ? t0 : t1;
        u64 d = t * (u64)C2_TILE;
        if (d > total) d = total;
        const u64 i = mp_search<16>(A, B, d, d > nB ? d - nB : 0, d < nA ? d : nA);
        if ((tid & 15) == 0) s_end[tid >> 4] = i;
    }
    __syncthreads();
    const u64 i0 = s_end[0], i1 = s_end[1];
    const u64 d0 = t0 * (u64)C2_TILE, d1 = t1 * (u64)C2_TILE < total ? t1 * (u64)C2_TILE : total;
    const u64 j0 = d0 - i0, j1 = d1 - i1;
    if (tid == 0) part[t0] = i0;
    if (tid == 1 && t1 == ntiles) part[ntiles] = i1;
    const u64 t = t0 + 1 + (u64)(tid / 8);  // 8 lanes per inner split
    if (t < t1) {
        const u64 d = t * (u64)C2_TILE;
        const u64 lo = (d > j1 && d - j1 > i0) ? d - j1 : i0, hi = i1 < d - j0 ? i1 : d - j0;
        const u64 i = mp_search<8>(A, B, d, lo, hi);
        if ((tid & 7) == 0) part[t] = i;
    }
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
    uint2* stage_delta;  // ordered mode: tile-local slots of TILE records
    uint2* stage_upd;
    u32* tile_cnt;       // ordered mode: [ntiles*4] inserts, updates, deletes, deltas
    u64* gsum;           // ordered mode: [2*ngroups] per C2_GROUP tiles: deltas | updates<<32, inserts | deletes<<32
    uint2* out_delta;    // unordered mode: final lists, appended per tile
    uint2* out_upd;
    u64* counts;         // unordered mode: [4] inserts, updates, deletes, deltas (atomic)
    u32* err;
};

// A byte range of one input array, copied to LDS as 16-byte chunks of its 16-byte-aligned
// *absolute* addresses: an aligned 16-byte chunk that holds any valid byte lies inside one mapped
// page, so the over-read at either end can never fault, and every chunk is one full-width load.
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
    // na + nb <= TILE items; keys 8 B and OIDs 20 B per item, +1 lookahead entry on B, and at most
    // two extra (partial) chunks per range
    static constexpr int CH = (28 * (TILE + 1) + 15) / 16 + 8;
    static constexpr int ROUNDS = (CH + NT - 1) / NT;
    // 4-ary search rounds until a width of TILE shrinks to 0 (w -> ceil(w/4) - 1)
    static constexpr int rounds(int w) { return w <= 0 ? 0 : 1 + rounds((w + 3) / 4 - 1); }
    static constexpr int SEARCH_ROUNDS = rounds(TILE);
};

#ifndef KD_J_EXP
#define KD_J_EXP 0  // profiling builds only: 1 = DMA staging only, 9 = per-phase clock64 printf
#endif
typedef __attribute__((address_space(3))) void* lds_vp;
typedef const __attribute__((address_space(1))) void* glb_vp;

// The tile (merge-path items [d0, d1): A entries [i0, i1), B entries [j0, j1)) is staged in ONE
// HBM round trip: keys and OIDs of both sides, plus the B entry after the tile (a tile's last A
// item may match it), go global -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR staging, 16 B
// per lane, the wave's 64 chunks land contiguously), all issued before any use.  Everything after
// that — merge path, OID compare, compaction — reads LDS.
//
// UNORD: each tile reserves its output ranges with one atomic add per counter and writes its
// (key-ordered) records straight to the final lists.  Ordered (default): tile-local staging +
// k_place2.
template <int NT, int IPT, bool UNORD>
__global__ __launch_bounds__(NT) void k_join2(Join2Args g) {
    using LD = Join2Lds<NT, IPT>;
    constexpr int TILE = LD::TILE;
    static_assert(TILE <= 4095, "per-item records hold 12-bit local indices");
    __shared__ u32x4 s_ch[LD::CH];  // lanes past the tile's chunks are masked off
    __shared__ u32 s_wave[3 * NT / 64];
    __shared__ u64 s_base[2];

    const int tid = threadIdx.x;
    const u64 tile = blockIdx.x;
#if KD_J_EXP == 9
    const u64 T0 = clock64();
    u64 T1 = 0, T2 = 0, T3 = 0;
#endif
    const u64 total = g.nA + g.nB;
    const u64 d0 = tile * (u64)TILE;
    const u64 d1 = d0 + TILE < total ? d0 + TILE : total;
    const u64 i0 = g.part[tile], i1 = g.part[tile + 1];
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
    const u64 j1e = j1 < g.nB ? j1 + 1 : j1;  // + the lookahead entry B[j1]
    const int na = (int)(i1 - i0), nb = (int)(j1 - j0);

    // ---- stage: four byte ranges -> LDS, chunk c at LDS byte 16c ------------------------------------
    const Range rka = mk_range(g.A, 8 * i0, 8 * i1), rkb = mk_range(g.B, 8 * j0, 8 * j1e);
    const Range roa = mk_range(g.oidA, 20 * i0, 20 * i1), rob = mk_range(g.oidB, 20 * j0, 20 * j1e);
    const u32 c1 = rka.nch, c2 = c1 + rkb.nch, c3 = c2 + roa.nch;
    // 64-chunk pieces (one wave-instruction each: wave-uniform source base and LDS base, lane l takes
    // chunk 64p + l), dealt round-robin to the waves across the four ranges: scalar address math
    {
        constexpr int NW = NT / 64;
        const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
        u32 q0 = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const Range& R = r == 0 ? rka : r == 1 ? rkb : r == 2 ? roa : rob;
            const u32 off = r == 0 ? 0 : r == 1 ? c1 : r == 2 ? c2 : c3;
            const u32 np = (R.nch + 63) >> 6;
            for (u32 p = (u32)(wid + NW - (int)(q0 % NW)) % NW; p < np; p += NW) {
                const u32 c = 64 * p + lane;
                if (c < R.nch)
                    __builtin_amdgcn_global_load_lds((glb_vp)(R.base + 16ull * c), (lds_vp)(s_ch + off + 64 * p), 16, 0, 0);
            }
            q0 += np;
        }
    }
    // lookbehind keys (tiny, scalar; in flight with the DMA)
    const bool has_lbA = i0 > 0, has_lbB = j0 > 0, has_la = j1 < g.nB;
    const u64 lbA = has_lbA ? g.A[i0 - 1] : 0;
    const u64 lbB = has_lbB ? g.B[j0 - 1] : 0;
    __syncthreads();  // vmcnt(0) + barrier: the DMA has landed
#if KD_J_EXP == 9
    T1 = clock64();
#endif
    const u64* sA = (const u64*)((const u8*)s_ch + rka.skew);
    const u64* sB = (const u64*)((const u8*)(s_ch + c1) + rkb.skew);
    const u32* oA = (const u32*)((const u8*)(s_ch + c2) + roa.skew);  // 4-B aligned: 20*i is
    const u32* oB = (const u32*)((const u8*)(s_ch + c3) + rob.skew);  // and allocations are
#if KD_J_EXP == 1  // staging only (profiling builds)
    if (tid == 0 && !UNORD) {
        u32* c = g.tile_cnt + 4 * tile;
        c[0] = c[1] = c[2] = c[3] = ((const u32*)s_ch)[tid] == 0x12345678u ? (u32)(lbA ^ lbB) : 0;
    }
    return;
#endif

    // ---- merge path, branch-free (selects instead of divergent branches: SALU exec-mask traffic was
    //      the join's largest instruction stream).  4-ary search for the thread's split: 3 independent
    //      probes per round, a fixed round count (5 for a 1024-item tile); then a walk over IPT items with
    //      the current and previous keys in registers (one LDS round trip per item; the strictly-
    //      ascending check compares registers).  Outcome per item in a register:
    //      rec = kind << 25 | changed << 24 | jb << 12 | ia
    enum : u32 { R_NONE = 0, R_DEL = 1, R_MATCH = 2, R_INS = 3 };
    const int nitems = na + nb;
    const int nbx = nb + (has_la ? 1 : 0);  // B keys in LDS, including the lookahead
    const int dd = tid * IPT < nitems ? tid * IPT : nitems;
    const int cnt = (dd + IPT < nitems ? dd + IPT : nitems) - dd;
    int lo = dd - nb > 0 ? dd - nb : 0, hi = dd < na ? dd : na;
    // first i in [lo, hi] with i == hi || sA[i] > sB[dd-1-i]  (ties: A first)
#pragma unroll
    for (int r = 0; r < LD::SEARCH_ROUNDS; r++) {
        const int w = hi - lo;
        const int s = (w + 3) >> 2;
        const int p1 = lo + s - 1, p2 = p1 + s, p3 = p2 + s;
        const int hm = w > 0 ? hi - 1 : lo;
        const int q1 = p1 > lo ? p1 : lo, q2 = p2 < hm ? p2 : hm, q3 = p3 < hm ? p3 : hm;
        const u64 a1 = sA[q1], v1 = sB[dd - 1 - q1], a2 = sA[q2], v2 = sB[dd - 1 - q2];
        const u64 a3 = sA[q3], v3 = sB[dd - 1 - q3];  // all six reads issued together
        const bool b1 = a1 > v1;
        const bool b2 = (p2 >= hi) | (a2 > v2);
        const bool b3 = (p3 >= hi) | (a3 > v3);
        const int m2 = p2 < hi ? p2 : hi, m3 = p3 < hi ? p3 : hi;
        int nlo = p3 + 1, nhi = hi;  // select chain (the nested form compiled to branches)
        nlo = b3 ? p2 + 1 : nlo;
        nhi = b3 ? m3 : nhi;
        nlo = b2 ? p1 + 1 : nlo;
        nhi = b2 ? m2 : nhi;
        nlo = b1 ? lo : nlo;
        nhi = b1 ? p1 : nhi;
        lo = w > 0 ? nlo : lo;
        hi = w > 0 ? nhi : hi;
    }
    u32 rec[IPT];
    bool bad = false;
    {
        int ia = lo, jb = dd - lo;
        const int amax = na > 0 ? na - 1 : 0, bmax = nbx > 0 ? nbx - 1 : 0;
        u64 ka = sA[ia < amax ? ia : amax], kb = sB[jb < bmax ? jb : bmax];
        bool ap_ok = ia > 0 || has_lbA, bp_ok = jb > 0 || has_lbB;
        u64 ap = ia > 0 ? sA[ia - 1] : lbA;  // the A / B keys before the walk position
        u64 bp = jb > 0 ? sB[jb - 1] : lbB;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            const bool act = k < cnt;
            const bool ta = jb >= nb || (ia < na && ka <= kb);
            const bool m = jb < nbx && kb == ka;  // sB[nb] = the lookahead entry
            const bool partner = ap_ok && ap == kb;
            const u32 kind = !act ? R_NONE : ta ? (m ? R_MATCH : R_DEL) : (partner ? R_NONE : R_INS);
            rec[k] = (kind << 25) | ((u32)jb << 12) | (u32)ia;
            bad |= act && (ta ? (ap_ok && ap >= ka) : (bp_ok && bp >= kb));
            const bool sa = act && ta, sb = act && !ta;
            ap = sa ? ka : ap;
            bp = sb ? kb : bp;
            ap_ok |= sa;
            bp_ok |= sb;
            ia += sa;
            jb += sb;
            ka = sA[ia < amax ? ia : amax];
            kb = sB[jb < bmax ? jb : bmax];
        }
    }
    // ---- OID compare of the matched pairs: every LDS read issued before any compare ------------------
    {
        u32 x[IPT][5], y[IPT][5];
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            const bool m = (rec[k] >> 25) == R_MATCH;
            const u32 ia = m ? rec[k] & 0xFFF : 0, jb = m ? (rec[k] >> 12) & 0xFFF : 0;
#pragma unroll
            for (int w = 0; w < 5; w++) { x[k][w] = oA[5 * ia + w]; y[k][w] = oB[5 * jb + w]; }
        }
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            u32 d = 0;
#pragma unroll
            for (int w = 0; w < 5; w++) d |= x[k][w] ^ y[k][w];
            if ((rec[k] >> 25) == R_MATCH && d) rec[k] |= 1u << 24;
        }
    }
    if (g.hash_mode) {
#pragma unroll
        for (int k = 0; k < IPT; k++)
            if ((rec[k] >> 25) == R_MATCH &&
                !names_eq(g.nameA, g.nameOffA, i0 + (rec[k] & 0xFFF), g.nameB, g.nameOffB, j0 + ((rec[k] >> 12) & 0xFFF)))
                atomicOr(g.err, 2u);
    }
    if (bad) atomicOr(g.err, 1u);
#if KD_J_EXP == 9
    T2 = clock64();
#endif

    // ---- compaction: per item-slot ballots give the wave-local exclusive offsets (thread-major item
    //      order) with mbcnt — no LDS round trips; one barrier for the wave totals ---------------------
    const int lane = tid & 63, wid = tid >> 6;
    u32 od = 0, ou = 0, wd = 0, wu = 0, wx = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u32 kind = rec[k] >> 25;
        const bool chg = (rec[k] >> 24) & 1;
        const u64 bd = __ballot(kind == R_DEL || kind == R_INS || (kind == R_MATCH && chg));
        const u64 bu = __ballot(kind == R_MATCH && chg);
        const u64 bx = __ballot(kind == R_DEL);
        od += __builtin_amdgcn_mbcnt_hi((u32)(bd >> 32), __builtin_amdgcn_mbcnt_lo((u32)bd, 0));
        ou += __builtin_amdgcn_mbcnt_hi((u32)(bu >> 32), __builtin_amdgcn_mbcnt_lo((u32)bu, 0));
        wd += __popcll(bd);
        wu += __popcll(bu);
        wx += __popcll(bx);
    }
    if (lane == 0) { s_wave[wid] = wd; s_wave[NT / 64 + wid] = wu; s_wave[2 * NT / 64 + wid] = wx; }
    __syncthreads();
    u32 tnd = 0, tnu = 0, tot_del = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const u32 a = s_wave[w], b = s_wave[NT / 64 + w];
        if (w < wid) { od += a; ou += b; }
        tnd += a;
        tnu += b;
        tot_del += s_wave[2 * NT / 64 + w];
    }
#if KD_J_EXP == 9
    T3 = clock64();
#endif
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
        const bool upd = kind == R_MATCH && ((rec[k] >> 24) & 1);
        const bool del = kind == R_DEL, ins = kind == R_INS;
        const uint2 v = make_uint2(ins ? KD_NONE : (u32)(i0 + ia), del ? KD_NONE : (u32)(j0 + jb));
        if (del | ins | upd) sd[od] = v;
        od += del | ins | upd;
        if (su && upd) su[ou] = v;
        ou += upd;
    }
    if (!UNORD && tid == 0) {
        u32* c = g.tile_cnt + 4 * tile;
        const u32 tins = tnd - tnu - tot_del;
        c[0] = tins;
        c[1] = tnu;
        c[2] = tot_del;
        c[3] = tnd;
        // group sums (<= 64 tiles x TILE per 32-bit half: no carry between halves); a handful of
        // atomics per address
        u64* gs = g.gsum + 2 * (tile / C2_GROUP);
        atomicAdd((unsigned long long*)gs, (unsigned long long)(tnd | (u64)tnu << 32));
        atomicAdd((unsigned long long*)gs + 1, (unsigned long long)(tins | (u64)tot_del << 32));
    }
#if KD_J_EXP == 9
    if (tid == 0 && tile % 1009 == 0) {
        const u64 T4 = clock64();
        printf("JT tile %llu stage %llu merge %llu scan %llu write %llu total %llu\n", (unsigned long long)tile,
               (unsigned long long)(T1 - T0), (unsigned long long)(T2 - T1), (unsigned long long)(T3 - T2),
               (unsigned long long)(T4 - T3), (unsigned long long)(T4 - T0));
    }
#endif
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
        unsigned nb = (unsigned)((ntiles + C2_PG - 1) / C2_PG);
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
