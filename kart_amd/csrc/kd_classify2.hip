// kd_classify2.hip — classify2: the two-way tree diff on gfx950.
//
// Replaces libgit2's tree-to-tree diff as consumed by RichBaseDataset.diff_feature
// (/root/reference/kart/rich_base_dataset.py:205-300): both commits' feature leaves arrive as
// strictly ascending join keys + 20-byte blob OIDs; a key on one side only is an insert/delete, a
// key on both sides with different OIDs is an update (GIT_DELTA_ADDED/DELETED/MODIFIED).
//
// The key union is cut into 1024-item merge-path tiles (k_partition2, guided two-level search).
// Default (key-ordered) path, KD_C2_MODE 1:
//   k_join2    one tile per 256-thread workgroup: keys by LDS-DMA into LDS, branch-free 4-ary split
//              search + register walk, OIDs of matched pairs compared straight from HBM, ballot
//              compaction into the tile's staging slot + tile counts + 64-tile group sums;
//   k_place2   one wave per tile: earlier groups' sums + earlier tiles of its group -> offset, staged
//              records -> final key-ordered positions; the last tile writes the totals.
// KD_DIFF_UNORDERED: k_join2 appends each tile's records at an atomically reserved offset (tiles in
// completion order, key order inside each tile); no k_place2.
// Profiling builds (KD_C2_MODE): 0 = persistent register-prefetched k_join2p + k_place2;
// 2 = k_join2p with a decoupled look-back (slow: ~1000 tiles in flight -> long look-back walks);
// 3 = run merge k_join2r (persistent, per-wave run rounds, see its comment) + k_place2 over wave
// slots.  Measurements of each are in DESIGN.md §3.1.
#include "kd_join.h"

namespace kd {

constexpr u64 C2_GROUP = 64;  // tiles per group sum (staged path: k_place2 offsets)
#ifndef KD_C2_STAGE_PAD
#define KD_C2_STAGE_PAD 32
#endif
// staging slot stride in records: one tile plus a pad, so the slots' hot first lines do not all
// fall on the same HBM channels (a power-of-two stride would)
constexpr u64 C2_STAGE = C2_TILE + KD_C2_STAGE_PAD;
#ifndef KD_PLACE_NT
#define KD_PLACE_NT 64  // one wave per tile: up to 16 staged records per lane, all loads in flight
#endif
#ifndef KD_C2_MODE
#define KD_C2_MODE 1  // ordered path: 1 per-tile k_join2 + k_place2, 0 persistent k_join2p + k_place2, 2 look-back
#endif
#ifndef KD_J_CLOCK
#define KD_J_CLOCK 0  // profiling builds: run-merge phase stamps in the staging pad + one report line
#endif
#ifndef KD_J_EXP
#define KD_J_EXP 0  // profiling builds only: 1 = staging only (k_join2)
#endif
#ifndef KD_J_OIDG
#define KD_J_OIDG 1  // k_join2: keys-only LDS image, OIDs compared straight from HBM (more tiles per CU)
#endif
#ifndef KD_J2P_WAVES
#define KD_J2P_WAVES 4  // k_join2p waves per SIMD to fit (VGPR cap): 4 four-wave workgroups per CU, no spills
#endif

// ---------------------------------------------------------------------------------------------
// merge-path partition
// ---------------------------------------------------------------------------------------------

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

// The same split, starting from a guess: one round of PW probes spaced `step` apart around `guess`
// brackets the answer (or cuts the range down to one side of the probes), then mp_search finishes
// inside the bracket.  A 1 %-edit diff keeps each split within a few hundred entries of the
// proportional guess, so the first round almost always brackets it: ~3 dependent rounds instead of
// ~6 over the whole arrays.  Correct for any guess (the predicate is monotone; probes are clamped).
template <int PW>
__device__ __forceinline__ u64 mp_search_guided(const u64* __restrict__ A, const u64* __restrict__ B, u64 d, u64 lo,
                                                u64 hi, u64 guess, u64 step) {
    if (hi <= lo) return lo;
    const int lane = threadIdx.x & 63, sub = lane % PW, grp = lane / PW;
    const u64 span = step * (PW / 2);
    const u64 g0 = guess > lo + span ? guess - span : lo;  // probe k at g0 + k*step, clamped to [lo, hi]
    u64 probe = g0 + step * (u64)sub;
    if (probe > hi) probe = hi;
    bool p = true;
    if (probe < hi) p = A[probe] > B[d - 1 - probe];
    const unsigned long long bal = (__ballot(p) >> (grp * PW)) & ((PW == 64) ? ~0ull : ((1ull << PW) - 1));
    const int f = bal ? __ffsll(bal) - 1 : PW;  // first true probe (PW: none)
    const u64 pf = f < PW ? (g0 + step * (u64)f < hi ? g0 + step * (u64)f : hi) : hi;
    const u64 pl = f > 0 ? (g0 + step * (u64)(f - 1) < hi ? g0 + step * (u64)(f - 1) : hi) : lo;
    const u64 nlo = f > 0 ? pl + 1 : lo, nhi = pf;
    return mp_search<PW>(A, B, d, nlo < nhi ? nlo : nhi, nhi);
}

// Merge-path split points part[t] (A items among the first min(t*TILE, nA+nB) union items), two
// levels: one block per group of C2_PG tiles.  The group's two end splits are searched over the
// whole arrays (16 lanes each, 16-ary: ~6 rounds of random HBM reads); every inner split then lies
// inside the box the end splits span (i and d-i are both monotone in d), at most C2_PG tiles wide,
// and is found there by 8 lanes (8-ary) whose probes land in that small, cache-warm region.
// The kernel also clears the counters and look-back descriptors the join needs (stream-ordered
// before it), instead of separate memset launches.
#ifndef KD_PTOP
#define KD_PTOP 16  // lanes per top-level split search
#endif
constexpr int C2_PG = 32, C2_PNT = 256;  // tiles per group; threads (8 lanes per inner split)
__global__ __launch_bounds__(C2_PNT) void k_partition2(const u64* __restrict__ A, u64 nA, const u64* __restrict__ B,
                                                       u64 nB, u64 ntiles, u64* __restrict__ part,
                                                       u64* __restrict__ zero_counts, u32* __restrict__ zero_err,
                                                       u64* __restrict__ zero_buf, u64 n_zero) {
    if (blockIdx.x == 0 && threadIdx.x < 4) zero_counts[threadIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 4) *zero_err = 0;
    for (u64 k = (u64)blockIdx.x * C2_PNT + threadIdx.x; k < n_zero; k += (u64)gridDim.x * C2_PNT) zero_buf[k] = 0;
    __shared__ u64 s_end[2];
    const int tid = threadIdx.x;
    const u64 total = nA + nB;
    const u64 t0 = (u64)blockIdx.x * C2_PG, t1 = t0 + C2_PG < ntiles ? t0 + C2_PG : ntiles;
    if (tid < 2 * KD_PTOP) {  // wave 0: the group's end splits t0 and t1 (guided: ~3 rounds)
        const u64 t = tid < KD_PTOP ? t0 : t1;
        u64 d = t * (u64)C2_TILE;
        if (d > total) d = total;
        const u64 guess = (u64)((double)d * (double)nA / (double)(total ? total : 1));
        const u64 i = mp_search_guided<KD_PTOP>(A, B, d, d > nB ? d - nB : 0, d < nA ? d : nA, guess, 2048 / KD_PTOP);
        if ((tid & (KD_PTOP - 1)) == 0) s_end[tid / KD_PTOP] = i;
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
        // proportional guess inside the group's box
        const u64 guess = d1 > d0 ? i0 + (u64)((double)(d - d0) * (double)(i1 - i0) / (double)(d1 - d0)) : lo;
        const u64 i = mp_search_guided<8>(A, B, d, lo, hi, guess, 16);
        if ((tid & 7) == 0) part[t] = i;
    }
}

// ---------------------------------------------------------------------------------------------
// shared tile machinery
// ---------------------------------------------------------------------------------------------
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
    const u8* dummy;     // >= 16 readable device bytes: source of masked-off chunk loads
    uint2* stage_delta;  // staged path: tile-local slots of TILE records
    uint2* stage_upd;
    u32* tile_cnt;       // staged path: [ntiles*4] inserts, updates, deletes, deltas
    u64* gsum;           // staged path: [2*ngroups] deltas | updates<<32, inserts | deletes<<32
    uint2* out_delta;    // final lists
    uint2* out_upd;
    u64* counts;         // [4] inserts, updates, deletes, deltas
    u32* err;
    u64* desc;           // persistent path: [2*ntiles] look-back descriptors
    u64 ntiles;
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
    // na + nb <= TILE items; keys 8 B and OIDs 20 B per item, +1 lookahead entry on B, +1 lookbehind
    // key per side, and at most two extra (partial) chunks per range
    static constexpr int CH = (28 * (TILE + 1) + 16 + 15) / 16 + 8;  // + the two lookbehind keys
    static constexpr int ROUNDS = (CH + NT - 1) / NT;
    // 4-ary search rounds until a width of TILE shrinks to 0 (w -> ceil(w/4) - 1)
    static constexpr int rounds(int w) { return w <= 0 ? 0 : 1 + rounds((w + 3) / 4 - 1); }
    static constexpr int SEARCH_ROUNDS = rounds(TILE);
};

typedef __attribute__((address_space(3))) void* lds_vp;
typedef const __attribute__((address_space(1))) void* glb_vp;
typedef const __attribute__((address_space(1))) u32x4* gp_x4;

// Tile t's place in both sides: merge-path items [d0, d1), A entries [i0, i1), B entries [j0, j1)
// (+ the lookahead B[j1] when it exists), and the keys just before it on each side.
struct TileGeo {
    u64 i0, i1, j0, j1, j1e, lbA, lbB;
    int na, nb;
    bool ok, has_lbA, has_lbB, has_la;
};

// wave-uniform 64-bit value into SGPRs: the tile geometry is loaded through the vector path (the
// compiler cannot prove part[] read-only for s_load), and without this every derived address would
// sit in VGPRs — for the current AND the prefetched tile
__device__ __forceinline__ u64 uni64(u64 x) {
    // (readfirstlane returns int: widen through u32, or bit 31 of the low half would sign-extend)
    return (u64)(u32)__builtin_amdgcn_readfirstlane((u32)x) | (u64)(u32)__builtin_amdgcn_readfirstlane((u32)(x >> 32)) << 32;
}

// geometry of tile t from its two split points (p0 = part[t], p1 = part[t + 1])
__device__ __forceinline__ TileGeo tile_geo_from(const Join2Args& g, u64 t, int TILE, u64 p0, u64 p1) {
    TileGeo q;
    const u64 total = g.nA + g.nB;
    const u64 d0 = t * (u64)TILE, d1 = d0 + TILE < total ? d0 + TILE : total;
    q.i0 = uni64(p0);
    q.i1 = uni64(p1);
    q.ok = !(q.i1 < q.i0 || d1 - q.i1 < d0 - q.i0 || q.i1 - q.i0 > d1 - d0);  // fails only on unsorted input
    if (!q.ok) q.i1 = q.i0 = d0 < g.nA ? d0 : g.nA;
    q.j0 = d0 - q.i0;
    q.j1 = q.ok ? d1 - q.i1 : q.j0;
    if (q.j1 > g.nB) q.j1 = q.j0 = g.nB;
    q.j1e = q.j1 < g.nB ? q.j1 + 1 : q.j1;
    q.na = (int)(q.i1 - q.i0);
    q.nb = (int)(q.j1 - q.j0);
    q.has_lbA = q.i0 > 0;
    q.has_lbB = q.j0 > 0;
    q.has_la = q.j1 < g.nB;
    q.lbA = q.lbB = 0;  // read from LDS: the key ranges start one entry early (the lookbehind keys)
    return q;
}

__device__ __forceinline__ TileGeo tile_geo(const Join2Args& g, u64 t, int TILE) {
    return tile_geo_from(g, t, TILE, g.part[t], g.part[t + 1]);
}

struct TileRanges {
    Range ka, kb, oa, ob;
    u32 c1, c2, c3, c4;  // chunk offsets of the four ranges in the LDS image
};

__device__ __forceinline__ TileRanges tile_ranges(const Join2Args& g, const TileGeo& q) {
    TileRanges r;
    r.ka = mk_range(g.A, 8 * (q.i0 - q.has_lbA), 8 * q.i1);  // + A[i0-1], B[j0-1]: the lookbehind keys
    r.kb = mk_range(g.B, 8 * (q.j0 - q.has_lbB), 8 * q.j1e);
    r.oa = mk_range(g.oidA, 20 * q.i0, 20 * q.i1);
    r.ob = mk_range(g.oidB, 20 * q.j0, 20 * q.j1e);
    r.c1 = r.ka.nch;
    r.c2 = r.c1 + r.kb.nch;
    r.c3 = r.c2 + r.oa.nch;
    r.c4 = r.c3 + r.ob.nch;
    return r;
}

enum : u32 { R_NONE = 0, R_DEL = 1, R_MATCH = 2, R_INS = 3 };

// Merge path of one tile out of LDS, branch-free (selects instead of divergent branches: SALU
// exec-mask traffic was the join's largest instruction stream).  4-ary search for the thread's
// split — 3 independent probes per round, a fixed round count (5 for a 1024-item tile) — then a
// walk over IPT items with the current and previous keys in registers (one LDS round trip per item;
// the strictly-ascending check compares registers), then the OID compare of the matched pairs with
// every LDS read issued before any compare.  Outcome per item:
//   rec = kind << 25 | changed << 24 | jb << 12 | ia          (tile-local indices)
template <int NT, int IPT>
__device__ __forceinline__ void tile_walk(const u64* sA, const u64* sB, const TileGeo& q, u32 rec[IPT], bool& bad) {
    using LD = Join2Lds<NT, IPT>;
    const int tid = threadIdx.x, na = q.na, nb = q.nb;
    const int nitems = na + nb;
    const int nbx = nb + (q.has_la ? 1 : 0);  // B keys in LDS, including the lookahead
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
    {
        int ia = lo, jb = dd - lo;
        const int amax = na > 0 ? na - 1 : 0, bmax = nbx > 0 ? nbx - 1 : 0;
        u64 ka = sA[ia < amax ? ia : amax], kb = sB[jb < bmax ? jb : bmax];
        bool ap_ok = ia > 0 || q.has_lbA, bp_ok = jb > 0 || q.has_lbB;
        u64 ap = sA[ia - 1];  // the A / B keys before the walk position (sA[-1] / sB[-1]: the
        u64 bp = sB[jb - 1];  // lookbehind keys, staged with the tile; garbage when absent, unused)
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
}

// OID compare of the matched pairs out of the tile's LDS image, in batches of OB items: every LDS read
// of a batch issued before its compares (OB bounds the registers held while the persistent kernel
// also carries the next tile's prefetch)
template <int IPT, typename P = const u32*>
__device__ __forceinline__ void tile_oid_lds(P oA, P oB, u32 rec[IPT]) {
    constexpr int OB = IPT < 2 ? IPT : 2;
#pragma unroll
    for (int k0 = 0; k0 < IPT; k0 += OB) {
        u32 x[OB][5], y[OB][5];
#pragma unroll
        for (int k = 0; k < OB; k++) {
            const bool m = (rec[k0 + k] >> 25) == R_MATCH;
            const u32 ia = m ? rec[k0 + k] & 0xFFF : 0, jb = m ? (rec[k0 + k] >> 12) & 0xFFF : 0;
#pragma unroll
            for (int w = 0; w < 5; w++) { x[k][w] = oA[5 * ia + w]; y[k][w] = oB[5 * jb + w]; }
        }
#pragma unroll
        for (int k = 0; k < OB; k++) {
            u32 d = 0;
#pragma unroll
            for (int w = 0; w < 5; w++) d |= x[k][w] ^ y[k][w];
            if ((rec[k0 + k] >> 25) == R_MATCH && d) rec[k0 + k] |= 1u << 24;
        }
    }
}

// OID compare straight from HBM (keys-only LDS image): each thread loads the two 20-B OIDs of its own
// matched pairs (consecutive items -> neighbouring entries across lanes), all loads issued before any
// compare
template <int IPT>
__device__ __forceinline__ void tile_oid_global(const Join2Args& g, const TileGeo& q, u32 rec[IPT]) {
    typedef const __attribute__((address_space(1))) u32* gp32;
    u32 x[IPT][5], y[IPT][5];
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const bool m = (rec[k] >> 25) == R_MATCH;
        const gp32 pa = m ? (gp32)(g.oidA + 20 * (q.i0 + (rec[k] & 0xFFF))) : (gp32)g.dummy;
        const gp32 pb = m ? (gp32)(g.oidB + 20 * (q.j0 + ((rec[k] >> 12) & 0xFFF))) : (gp32)g.dummy;
#pragma unroll
        for (int w = 0; w < 5; w++) { x[k][w] = pa[w]; y[k][w] = pb[w]; }
    }
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        u32 d = 0;
#pragma unroll
        for (int w = 0; w < 5; w++) d |= x[k][w] ^ y[k][w];
        if ((rec[k] >> 25) == R_MATCH && d) rec[k] |= 1u << 24;
    }
}

template <int NT, int IPT>
__device__ __forceinline__ void tile_merge(const u64* sA, const u64* sB, const u32* oA, const u32* oB, const TileGeo& q,
                                           u32 rec[IPT], bool& bad) {
    tile_walk<NT, IPT>(sA, sB, q, rec, bad);
    tile_oid_lds<IPT>(oA, oB, rec);
}

// KD_KEY_HASH: a matched key must also match the full filename (a 64-bit key collision between two
// different names would otherwise be read as an update)
template <int IPT>
__device__ __forceinline__ void tile_names(const Join2Args& g, const TileGeo& q, const u32 rec[IPT]) {
    u32 ia[IPT], jb[IPT], act = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        ia[k] = (u32)q.i0 + (rec[k] & 0xFFF);
        jb[k] = (u32)q.j0 + ((rec[k] >> 12) & 0xFFF);
        act |= (u32)((rec[k] >> 25) == R_MATCH) << k;
    }
    if (names_ne_batch<IPT, 8>(g.nameA, g.nameOffA, ia, g.nameB, g.nameOffB, jb, act)) atomicOr(g.err, 2u);
}

// Per-item flag bits (bitwise, not short-circuit: no exec-mask branches), then per item-slot ballots:
// the wave-local exclusive offsets in thread-major item order come from mbcnt — no LDS round trips —
// and one barrier exchanges the wave totals.
struct TileCounts {
    u32 fd, fu;          // item k is a delta / an update
    u32 od, ou;          // this thread's first delta / update slot inside the tile
    u32 tnd, tnu, tdel;  // tile totals: deltas, updates, deletes
};

template <int NT, int IPT>
__device__ __forceinline__ TileCounts tile_counts(const u32 rec[IPT], u32* s_wave) {
    TileCounts c;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    u32 fd = 0, fu = 0, fx = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u32 kind = rec[k] >> 25, chg = (rec[k] >> 24) & 1;
        const u32 isx = (u32)(kind == R_DEL), isi = (u32)(kind == R_INS), isu = (u32)(kind == R_MATCH) & chg;
        fd |= (isx | isi | isu) << k;
        fu |= isu << k;
        fx |= isx << k;
    }
    u32 od = 0, ou = 0, wd = 0, wu = 0, wx = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u64 bd = __ballot((fd >> k) & 1);
        const u64 bu = __ballot((fu >> k) & 1);
        const u64 bx = __ballot((fx >> k) & 1);
        od += __builtin_amdgcn_mbcnt_hi((u32)(bd >> 32), __builtin_amdgcn_mbcnt_lo((u32)bd, 0));
        ou += __builtin_amdgcn_mbcnt_hi((u32)(bu >> 32), __builtin_amdgcn_mbcnt_lo((u32)bu, 0));
        wd += __popcll(bd);
        wu += __popcll(bu);
        wx += __popcll(bx);
    }
    if (lane == 0) { s_wave[wid] = wd; s_wave[NT / 64 + wid] = wu; s_wave[2 * NT / 64 + wid] = wx; }
    __syncthreads();
    u32 tnd = 0, tnu = 0, tdel = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const u32 a = s_wave[w], b = s_wave[NT / 64 + w];
        if (w < wid) { od += a; ou += b; }
        tnd += a;
        tnu += b;
        tdel += s_wave[2 * NT / 64 + w];
    }
    c.fd = fd; c.fu = fu; c.od = od; c.ou = ou; c.tnd = tnd; c.tnu = tnu; c.tdel = tdel;
    return c;
}

template <int IPT>
__device__ __forceinline__ void tile_write(const u32 rec[IPT], const TileCounts& c, u64 i0, u64 j0,
                                           uint2* __restrict__ sd, uint2* __restrict__ su) {
    u32 od = c.od, ou = c.ou;
    const u32 has_su = su != nullptr;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u32 kind = rec[k] >> 25, ia = rec[k] & 0xFFF, jb = (rec[k] >> 12) & 0xFFF;
        const u32 isd = (c.fd >> k) & 1, isu = (c.fu >> k) & 1;
        const uint2 v = make_uint2(kind == R_INS ? KD_NONE : (u32)(i0 + ia), kind == R_DEL ? KD_NONE : (u32)(j0 + jb));
        if (isd) sd[od] = v;
        od += isd;
        if (isu & has_su) su[ou] = v;
        ou += isu;
    }
}

// ---------------------------------------------------------------------------------------------
// k_join2: one tile per workgroup (unordered appends, or the staged ordered path)
// ---------------------------------------------------------------------------------------------
// The tile is staged in ONE HBM round trip: keys and OIDs of both sides go global -> LDS by LDS-DMA
// (global_load_lds_dwordx4: 16 B per lane, the wave's 64 chunks land contiguously), all issued
// before any use.
template <int NT, int IPT, bool UNORD, bool HASH>
__global__ __launch_bounds__(NT) void k_join2(Join2Args g) {
    // (HASH: filename checks compiled in; the int-key instantiation carries none of their registers)
    using LD = Join2Lds<NT, IPT>;
    static_assert(LD::TILE <= 4095, "per-item records hold 12-bit local indices");
    constexpr int NRANGE = KD_J_OIDG ? 2 : 4;  // keys only, or keys + OIDs
    constexpr int CHK = (8 * (LD::TILE + 1) + 16 + 15) / 16 + 4;  // chunks of the two key ranges
    __shared__ u32x4 s_ch[KD_J_OIDG ? CHK : LD::CH];  // lanes past the tile's chunks are masked off
    __shared__ u32 s_wave[3 * NT / 64];
    __shared__ u64 s_base[2];
    const int tid = threadIdx.x;
    const u64 tile = blockIdx.x;
    const TileGeo q = tile_geo(g, tile, LD::TILE);
    if (!q.ok && tid == 0) atomicOr(g.err, 1u);
    const TileRanges r = tile_ranges(g, q);
    // 64-chunk pieces (one wave-instruction each: wave-uniform source base and LDS base, lane l takes
    // chunk 64p + l), dealt round-robin to the waves across the four ranges: scalar address math
    {
        constexpr int NW = NT / 64;
        const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
        u32 q0 = 0;
#pragma unroll
        for (int k = 0; k < NRANGE; k++) {
            const Range& R = k == 0 ? r.ka : k == 1 ? r.kb : k == 2 ? r.oa : r.ob;
            const u32 off = k == 0 ? 0 : k == 1 ? r.c1 : k == 2 ? r.c2 : r.c3;
            const u32 np = (R.nch + 63) >> 6;
            for (u32 p = (u32)(wid + NW - (int)(q0 % NW)) % NW; p < np; p += NW) {
                const u32 c = 64 * p + lane;
                if (c < R.nch)
                    __builtin_amdgcn_global_load_lds((glb_vp)(R.base + 16ull * c), (lds_vp)(s_ch + off + 64 * p), 16, 0, 0);
            }
            q0 += np;
        }
    }
    __syncthreads();  // vmcnt(0) + barrier: the DMA has landed
    const u64* sA = (const u64*)((const u8*)s_ch + r.ka.skew) + q.has_lbA;
    const u64* sB = (const u64*)((const u8*)(s_ch + r.c1) + r.kb.skew) + q.has_lbB;
    const u32* oA = (const u32*)((const u8*)(s_ch + r.c2) + r.oa.skew);  // 4-B aligned: 20*i is
    const u32* oB = (const u32*)((const u8*)(s_ch + r.c3) + r.ob.skew);  // and allocations are
#if KD_J_EXP == 1
    if (tid == 0 && !UNORD) {
        u32* c = g.tile_cnt + 4 * tile;
        c[0] = c[1] = c[2] = c[3] = ((const u32*)s_ch)[tid] == 0x12345678u ? 1u : 0u;
    }
    return;
#endif
    u32 rec[IPT];
    bool bad = false;
#if KD_J_EXP == 2  // profiling: no merge path (records from the item index), OID loads kept
#pragma unroll
    for (int k = 0; k < IPT; k++) rec[k] = (R_MATCH << 25) | ((u32)((tid * IPT + k) / 2) << 12) | (u32)((tid * IPT + k) / 2);
    bad = sA[tid] == 0x123456789ull && sB[tid] == 7;
#else
    tile_walk<NT, IPT>(sA, sB, q, rec, bad);
#endif
    // complete order check: the walk only compares the keys it consumes, and on unsorted input the
    // per-thread merge-path splits can skip keys, so every adjacent pair of the tile's two ranges
    // (the first against the lookbehind key) is checked here as well
    for (int x = tid; x < q.na; x += NT) bad |= (x > 0 || q.has_lbA) && sA[x - 1] >= sA[x];
    for (int x = tid; x < q.nb; x += NT) bad |= (x > 0 || q.has_lbB) && sB[x - 1] >= sB[x];
#if KD_J_EXP != 3  // 3: profiling, no OID compare
    if (KD_J_OIDG) tile_oid_global<IPT>(g, q, rec);
    else tile_oid_lds<IPT>(oA, oB, rec);
#endif
    if (HASH) tile_names<IPT>(g, q, rec);
    if (bad) atomicOr(g.err, 1u);
    const TileCounts c = tile_counts<NT, IPT>(rec, s_wave);
    uint2 *sd, *su;
    if (UNORD) {
        // four lanes of wave 0 reserve in parallel: deltas, updates (offsets) + inserts, deletes
        if (tid < 4) {
            const u64 v = tid == 0 ? c.tnd : tid == 1 ? c.tnu : tid == 2 ? c.tnd - c.tnu - c.tdel : c.tdel;
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
    tile_write<IPT>(rec, c, q.i0, q.j0, sd, su);
    if (!UNORD && tid == 0) {
        u32* cc = g.tile_cnt + 4 * tile;
        const u32 tins = c.tnd - c.tnu - c.tdel;
        cc[0] = tins;
        cc[1] = c.tnu;
        cc[2] = c.tdel;
        cc[3] = c.tnd;
        // group sums (<= 64 tiles x TILE per 32-bit half: no carry between halves)
        u64* gs = g.gsum + 2 * (tile / C2_GROUP);
        atomicAdd((unsigned long long*)gs, (unsigned long long)(c.tnd | (u64)c.tnu << 32));
        atomicAdd((unsigned long long*)gs + 1, (unsigned long long)(tins | (u64)c.tdel << 32));
    }
}

// ---------------------------------------------------------------------------------------------
// k_join2r: run merge — one tile per workgroup, each wave walks its own 256-item stretch in runs
// ---------------------------------------------------------------------------------------------
// The merge path of a diff is almost all matched pairs, broken by short runs of inserts or deletes.
// A wave therefore does not search a split for every lane: it walks its stretch in rounds, lane l
// looking at A[a+l] and B[b+l] at once —
//   pair round: the leading lanes with equal keys are matched pairs (OIDs compared from LDS, changed
//               ones emitted), a and b advance by that count;
//   run round:  (first keys differ) the leading lanes of A below B[b] are deletes, or of B below A[a]
//               inserts, emitted and skipped in one step.
// A 1 %-edit stretch of 256 items takes ~6 rounds of one LDS read pair + ballots each.  A stretch
// still unfinished after RMAX rounds (dense interleaved edits) is finished by the per-lane merge path
// (search + walk) restricted to what is left.  Records go to the wave's own slot (256 records) of the
// tile's staging area, in key order; k_place2 concatenates the four slots.
constexpr int RW = 64 * C2_IPT;  // merge-path items per wave stretch (one tile: NT/64 stretches)
#ifndef KD_RMAX
#define KD_RMAX 24        // run rounds before the per-lane fallback
#endif

// 64-lane 64-ary merge-path search over the tile's LDS keys (2 rounds for a 1024-item tile)
__device__ __forceinline__ int mp_search_lds64(const u64* sA, const u64* sB, int d, int lo, int hi) {
    const int lane = threadIdx.x & 63;
    while (hi > lo) {
        const int step = (hi - lo + 63) >> 6;
        const int probe = lo + step * (lane + 1) - 1;
        const int pc = probe < hi ? probe : hi - 1;
        const bool p = probe >= hi || sA[pc] > sB[d - 1 - pc];
        const u64 bal = __ballot(p);
        if (bal == 0) return hi;
        const int f = __ffsll((long long)bal) - 1;
        const int nh = lo + step * (f + 1) - 1;
        lo = lo + step * f;
        hi = nh < hi ? nh : hi;
        if (step == 1) return hi;
    }
    return lo;
}

// Per-lane merge path (search + register walk) over what is left of a wave's stretch:
// A [a, ae), B [b, be) (tile-local; B keys readable up to nbx, the tile's lookahead included).
// Item outcome records as in tile_walk.
template <int IPT>
__device__ __forceinline__ void wave_walk(const u64* sA, const u64* sB, int a, int ae, int b, int be, int nbx,
                                          bool has_lbA, u32 rec[IPT]) {
    const int lane = threadIdx.x & 63;
    const int na = ae - a, nb = be - b, nitems = na + nb;
    const int dd = lane * IPT < nitems ? lane * IPT : nitems;
    const int cnt = (dd + IPT < nitems ? dd + IPT : nitems) - dd;
    int lo = dd - nb > 0 ? dd - nb : 0, hi = dd < na ? dd : na;
    while (lo < hi) {  // binary search: this path only runs for dense-edit stretches
        const int mid = (lo + hi) >> 1;
        if (sA[a + mid] <= sB[b + dd - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    int ia = a + lo, jb = b + dd - lo;
    const bool ap_ok0 = ia > 0 || has_lbA;
    u64 ap = sA[ia - 1];
    bool ap_ok = ap_ok0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        rec[k] = R_NONE << 25;
        if (k < cnt) {
            const u64 ka = ia < ae ? sA[ia] : ~0ull, kb = jb < nbx ? sB[jb] : ~0ull;
            if (jb >= be || (ia < ae && ka <= kb)) {
                const bool m = jb < nbx && kb == ka;
                rec[k] = ((m ? R_MATCH : R_DEL) << 25) | ((u32)jb << 12) | (u32)ia;
                ap = ka;
                ap_ok = true;
                ia++;
            } else {
                const bool partner = ap_ok && ap == kb;
                rec[k] = ((partner ? R_NONE : R_INS) << 25) | ((u32)jb << 12) | (u32)ia;
                jb++;
            }
        }
    }
}

// Run-merge LDS image: keys and OIDs in separate arrays (distinct alias scopes: the waitcnt pass then
// knows a key read cannot overlap an OID LDS-DMA still in flight, and inserts no vmcnt wait for it)
template <int NT>
struct RunLds {
    static constexpr int TILE = NT * C2_IPT;
    static constexpr int CHK = (8 * (TILE + 3) + 15) / 16 + 4;   // A + lookbehind, B + lookbehind + lookahead
    static constexpr int CHO = (20 * (TILE + 1) + 15) / 16 + 4;  // A, B + lookahead
};

// LDS-DMA staging of one tile: wave 0 issues the key pieces (then waits for them alone), waves 1.. the
// OID pieces, dealt round-robin.  Issue only.
template <int NT>
__device__ __forceinline__ void run_stage(const TileRanges& r, u32x4* s_key, u32x4* s_oid) {
    constexpr int NW = NT / 64;
    static_assert(NW >= 2, "one key wave + at least one OID wave");
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w == 0) {
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const Range& R = k == 0 ? r.ka : r.kb;
            u32x4* dst = s_key + (k == 0 ? 0 : r.c1);
            for (u32 p = 0; 64 * p < R.nch; p++) {
                const u32 c = 64 * p + lane;
                if (c < R.nch) __builtin_amdgcn_global_load_lds((glb_vp)(R.base + 16ull * c), (lds_vp)(dst + 64 * p), 16, 0, 0);
            }
        }
    } else {
        const u32 npa = (r.oa.nch + 63) >> 6, np = npa + ((r.ob.nch + 63) >> 6);
        for (u32 p = (u32)(w - 1); p < np; p += NW - 1) {
            const bool onA = p < npa;
            const Range& R = onA ? r.oa : r.ob;
            const u32 pp = onA ? p : p - npa;
            u32x4* dst = s_oid + (onA ? 0 : r.c3 - r.c2) + 64 * pp;
            const u32 c = 64 * pp + lane;
            if (c < R.nch) __builtin_amdgcn_global_load_lds((glb_vp)(R.base + 16ull * c), (lds_vp)dst, 16, 0, 0);
        }
    }
}

// workgroup barrier that waits for LDS traffic only: an LDS-DMA still in flight stays in flight
// across it (__syncthreads would also drain vmcnt)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// 64-bit value of lane 0 (wave-uniform: SGPRs)
__device__ __forceinline__ u64 lane0_64(u64 x) {
    return (u64)(u32)__builtin_amdgcn_readlane((u32)x, 0) | (u64)(u32)__builtin_amdgcn_readlane((u32)(x >> 32), 0) << 32;
}

// run descriptor: kind << 30 | length << 23 | a << 11 | b   (tile-local a, b < 2048; length <= 64)
enum : u32 { RUN_PAIR = 0, RUN_DEL = 1, RUN_INS = 2 };
static_assert(C2_TILE <= 2048, "run descriptors hold 11-bit tile-local indices");

// Run merge of one tile, in two phases so that the OIDs land while the keys are walked.
//   phase 1 (keys only — wave 0 waited for its key DMA, the OID DMA is still in flight): key order
//     check, per-wave stretch splits, then the run rounds: lane l looks at A[a+l] and B[b+l]; the
//     leading equal lanes are matched pairs, or (first keys differ) the leading A below B[b] are
//     deletes or the leading B below A[a] inserts.  A round only records its run (one descriptor per
//     round, in lane `round` of a VGPR); the walk state stays in SGPRs (scalar branches only).
//   phase 2 (after the OID DMA has landed): the runs in order — OIDs of each pair run compared out of
//     LDS, changed pairs, deletes and inserts written to the wave's slot in key order.
// A stretch still unfinished after RMAX rounds (dense interleaved edits) is finished by the per-lane
// merge path (search + walk) over what is left.
template <int NT, bool HASH, typename LandOids>
__device__ __forceinline__ void run_tile(const Join2Args& g, const TileGeo& q, const TileRanges& r, const u32x4* s_key,
                                         const u32x4* s_oid, int* s_split, u32 (*s_cnt)[4], u64 tile,
                                         LandOids land_oids) {
    constexpr int NW = NT / 64, TILE = NW * RW, IPL = RW / 64;  // IPL: items per lane (fallback walk)
    static_assert(KD_RMAX <= 64, "one run descriptor per lane");
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const u64* sA = (const u64*)((const u8*)s_key + r.ka.skew) + q.has_lbA;
    const u64* sB = (const u64*)((const u8*)(s_key + r.c1) + r.kb.skew) + q.has_lbB;
    // address space 3 + volatile: single ds_read_b32s (merged ds_read2s lose the alias scope)
    typedef const volatile __attribute__((address_space(3))) u32* lds_vu32;
    const lds_vu32 oA = (lds_vu32)((const u8*)s_oid + r.oa.skew);
    const lds_vu32 oB = (lds_vu32)((const u8*)(s_oid + (r.c3 - r.c2)) + r.ob.skew);
    const int na = q.na, nb = q.nb, nitems = na + nb, nbx = nb + (q.has_la ? 1 : 0);
#if KD_J_CLOCK
    u64* clk = (u64*)(g.stage_delta + tile * (u64)C2_STAGE + TILE);
#endif

    // ---- strictly ascending keys: item c of the tile checks its key against the one before it ----
    bool bad = false;
#pragma unroll
    for (int k = 0; k < TILE / NT; k++) {
        const int c = k * NT + tid;
        const bool onA = c < na;
        const int ci = onA ? c : c - na;
        const bool chk = (c < nitems) & (ci > 0 || (onA ? q.has_lbA : q.has_lbB));
        const u64* s = onA ? sA : sB;
        const int cc = chk ? ci : 1;
        const u64 k0 = s[cc - 1], k1 = s[cc];
        bad |= chk & (k0 >= k1);
    }
    if (__ballot(bad) && lane == 0) atomicOr(g.err, 1u);
#if KD_J_CLOCK
    if (tid == 0) clk[2] = wall_clock64();
#endif

    // ---- the stretch splits: wave w >= 1 finds the split at item w*RW ----
    if (tid == 0) { s_split[0] = 0; s_split[NW] = na; }
    if (wid >= 1) {
        const int d = wid * RW < nitems ? wid * RW : nitems;
        const int sp = mp_search_lds64(sA, sB, d, d - nb > 0 ? d - nb : 0, d < na ? d : na);
        if (lane == 0) s_split[wid] = sp;
    }
    lds_barrier();
#if KD_J_CLOCK
    if (tid == 0) clk[3] = wall_clock64();
#endif
    int a = __builtin_amdgcn_readfirstlane(s_split[wid]);
    const int ae = __builtin_amdgcn_readfirstlane(s_split[wid + 1]);
    const int d0 = wid * RW < nitems ? wid * RW : nitems, d1 = (wid + 1) * RW < nitems ? (wid + 1) * RW : nitems;
    int b = __builtin_amdgcn_readfirstlane(d0 - a);
    const int be = __builtin_amdgcn_readfirstlane(d1 - ae);
    // the stretch's first B may be the partner of the A just before it (matched there)
    if (b < be && (a > 0 || q.has_lbA) && uni64(sA[a - 1]) == uni64(sB[b])) b++;

    // ---- phase 1: the run rounds over the keys ----
    const int amax = na > 0 ? na - 1 : 0, bmax = nbx > 0 ? nbx - 1 : 0;
    u32 runs = 0;  // lane k: descriptor of round k
    int nr = 0;
    for (; nr < KD_RMAX && a + b < ae + be; nr++) {
        const int la = a + lane, lb = b + lane;
        const u64 ka = sA[la < amax ? la : amax], kb = sB[lb < bmax ? lb : bmax];
        const bool ina = la < ae;
        const u64 ne = __ballot(!(ina && lb < nbx && ka == kb));
        const int f = ne ? __ffsll((long long)ne) - 1 : 64;  // leading matched pairs
        u32 desc;
        if (f > 0) {
            desc = RUN_PAIR << 30 | (u32)f << 23 | (u32)a << 11 | (u32)b;
            a += f;
            b += f;
        } else {
            // lane 0 holds A[a] and B[b] (B[be] is the lookahead: an A below it is a delete)
            const u64 ka0 = a < ae ? lane0_64(ka) : ~0ull, kb0 = b < nbx ? lane0_64(kb) : ~0ull;
            if (ka0 < kb0) {
                const u64 nd = __ballot(!(ina && ka < kb0));
                const int run = nd ? __ffsll((long long)nd) - 1 : 64;
                desc = RUN_DEL << 30 | (u32)run << 23 | (u32)a << 11 | (u32)b;
                a += run;
            } else {
                const u64 ni = __ballot(!(lb < be && kb < ka0));
                const int run = ni ? __ffsll((long long)ni) - 1 : 64;
                desc = RUN_INS << 30 | (u32)run << 23 | (u32)a << 11 | (u32)b;
                b += run;
            }
        }
        runs = lane == nr ? desc : runs;
    }
#if KD_J_CLOCK
    if (lane == 0) { clk[4 + wid] = wall_clock64(); clk[8 + wid] = nr + ((a < ae || b < be) ? 1000 : 0); }
#endif

    // ---- the OIDs land in LDS (and a barrier publishes them) ----
    land_oids();
#if KD_J_CLOCK
    if (tid == 0) clk[14] = wall_clock64();
#endif

    // ---- phase 2: the runs in key order ----
    uint2* sd = g.stage_delta + tile * (u64)C2_STAGE + wid * RW;
    uint2* su = g.stage_upd + tile * (u64)C2_STAGE + wid * RW;
    const u32 i0 = (u32)q.i0, j0 = (u32)q.j0;
    const u64 lt = (1ull << lane) - 1;  // lanes below this one
    u32 cd = 0, cu = 0, cx = 0, ci = 0;
    for (int k = 0; k < nr; k++) {
        const u32 desc = __builtin_amdgcn_readlane(runs, k);
        const u32 kind = desc >> 30, len = (desc >> 23) & 127, ra = (desc >> 11) & 2047, rb = desc & 2047;
        const u32 la = ra + lane, lb = rb + lane;
        if (kind == RUN_PAIR) {
            const u32 ia = lane < len ? la : ra, jb = lane < len ? lb : rb;
            u32 d = 0;
#pragma unroll
            for (int w = 0; w < 5; w++) d |= oA[5 * ia + w] ^ oB[5 * jb + w];
            if (HASH && lane < len && !names_eq(g.nameA, g.nameOffA, q.i0 + la, g.nameB, g.nameOffB, q.j0 + lb))
                atomicOr(g.err, 2u);
            const bool chg = (lane < len) & (d != 0);
            const u64 bc = __ballot(chg);
            if (bc) {
                if (chg) {
                    const u32 pos = (u32)__popcll(bc & lt);
                    const uint2 v = make_uint2(i0 + la, j0 + lb);
                    sd[cd + pos] = v;
                    su[cu + pos] = v;
                }
                cd += (u32)__popcll(bc);
                cu += (u32)__popcll(bc);
            }
        } else {
            const bool del = kind == RUN_DEL;
            if (lane < len) sd[cd + lane] = del ? make_uint2(i0 + la, KD_NONE) : make_uint2(KD_NONE, j0 + lb);
            cd += len;
            if (del) cx += len;
            else ci += len;
        }
    }
    if (a < ae || b < be) {  // dense edits: the per-lane merge path finishes the stretch
        if (b > be) b = be;    // (only on unsorted input, already flagged: keeps the walk in bounds)
        u32 rec[IPL];
        wave_walk<IPL>(sA, sB, a, ae, b, be, nbx, q.has_lbA, rec);
        tile_oid_lds<IPL, lds_vu32>(oA, oB, rec);
        if (HASH) tile_names<IPL>(g, q, rec);
        TileCounts c;
        c.fd = c.fu = 0;
        u32 fx = 0, fi = 0;
#pragma unroll
        for (int k = 0; k < IPL; k++) {
            const u32 kind = rec[k] >> 25, chg = (rec[k] >> 24) & 1;
            const u32 isx = (u32)(kind == R_DEL), isi = (u32)(kind == R_INS), isu = (u32)(kind == R_MATCH) & chg;
            c.fd |= (isx | isi | isu) << k;
            c.fu |= isu << k;
            fx |= isx << k;
            fi |= isi << k;
        }
        // thread-major item order: this lane's records follow every record of the lanes below it
        u32 od = 0, ou = 0, wd = 0, wu = 0;
#pragma unroll
        for (int k = 0; k < IPL; k++) {
            const u64 bd = __ballot((c.fd >> k) & 1), bu = __ballot((c.fu >> k) & 1);
            od += (u32)__popcll(bd & lt);
            ou += (u32)__popcll(bu & lt);
            wd += (u32)__popcll(bd);
            wu += (u32)__popcll(bu);
            cx += (u32)__popcll(__ballot((fx >> k) & 1));
            ci += (u32)__popcll(__ballot((fi >> k) & 1));
        }
        c.od = cd + od;
        c.ou = cu + ou;
        tile_write<IPL>(rec, c, i0, j0, sd, su);
        cd += wd;
        cu += wu;
    }
#if KD_J_CLOCK
    if (lane == 0) clk[16 + wid] = wall_clock64();
#endif
    if (lane == 0) { s_cnt[wid][0] = cd; s_cnt[wid][1] = cu; s_cnt[wid][2] = cx; s_cnt[wid][3] = ci; }
    lds_barrier();
#if KD_J_CLOCK
    if (tid == 0) clk[12] = wall_clock64();
#endif
    if (tid == 0) {
        static_assert(NW <= 4, "tile_cnt packs at most four wave slots");
        u32 td = 0, tu = 0, tx = 0, tn = 0, packed[4] = {0, 0, 0, 0};
#pragma unroll
        for (int w = 0; w < NW; w++) {
            td += s_cnt[w][0]; tu += s_cnt[w][1]; tx += s_cnt[w][2]; tn += s_cnt[w][3];
            packed[w] = s_cnt[w][0] | s_cnt[w][1] << 16;
        }
        *(uint4*)(g.tile_cnt + 4 * tile) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
        u64* gs = g.gsum + 2 * (tile / C2_GROUP);
        atomicAdd((unsigned long long*)gs, (unsigned long long)(td | (u64)tu << 32));
        atomicAdd((unsigned long long*)gs + 1, (unsigned long long)(tn | (u64)tx << 32));
    }
}

#if KD_J_CLOCK
// stamps per tile (u64, in the staging pad): 13 before staging, 0 keys landed, 2 after the key check,
// 3 after the split barrier, 4+w wave w's rounds done, 8+w its rounds (+1000 = fell back), 14 OIDs
// landed, 16+w its records written, 12 after the final barrier
__global__ void k_jclk_report(const uint2* stage, u64 ntiles) {
    constexpr int NS = 11;
    __shared__ double s_sum[NS][256];
    double sm[NS] = {};
    for (u64 t = threadIdx.x; t < ntiles; t += 256) {
        const u64* p = (const u64*)(stage + t * (u64)C2_STAGE + C2_TILE);
        double r = 0, fb = 0, wr = 0, wl = 0;
        for (int w = 0; w < C2_NT / 64; w++) {
            r += (double)(p[8 + w] % 1000); fb += p[8 + w] >= 1000;
            wr += (double)(p[4 + w] - p[3]); wl += (double)(p[16 + w] - p[14]);
            sm[10] += (double)(p[20 + w] - p[4 + w]) / (C2_NT / 64);
        }
        const double nw = C2_NT / 64;
        sm[0] += (double)(p[0] - p[13]); sm[1] += (double)(p[2] - p[0]); sm[2] += (double)(p[3] - p[2]);
        sm[3] += wr / nw; sm[4] += (double)(p[14] - p[3]); sm[5] += wl / nw; sm[6] += (double)(p[12] - p[14]);
        sm[7] += r / nw; sm[8] += fb; sm[9] += (double)(p[12] - p[13]);
    }
    for (int k = 0; k < NS; k++) s_sum[k][threadIdx.x] = sm[k];
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 256; i++)
            for (int k = 0; k < NS; k++) sm[k] += s_sum[k][i];
        const double n = (double)ntiles, us = 0.01 / n;
        printf("JCLK tiles %llu mean_us keys %.3f check %.3f split %.3f rounds %.3f oids_landed %.3f emit %.3f "
               "tail %.3f total %.3f | rounds/wave %.2f fallbacks %.0f own_oid_wait %.3f\n",
               (unsigned long long)ntiles, sm[0] * us, sm[1] * us, sm[2] * us, sm[3] * us, sm[4] * us, sm[5] * us,
               sm[6] * us, sm[9] * us, sm[7] / n, sm[8], sm[10] * us);
    }
}
#endif

// Register staging of one tile: every thread loads a fixed number of 16-byte chunks of the key ranges
// (KP) and of the OID ranges (OP) — all loads issued up front, lanes past a range reload its first chunk
// (fixed counts: the compiler's vmcnt waits stay exact) — the keys are written to LDS at once, the OIDs
// only after the key phase (their loads stay in flight meanwhile).  Plain loads, not LDS-DMA: DMA
// writes into LDS lose arbitration to the co-resident workgroups' ds_reads and landed several µs late.
template <int NT>
struct RunRegs {
    static constexpr int KP = (RunLds<NT>::CHK + NT - 1) / NT, OP = (RunLds<NT>::CHO + NT - 1) / NT;
    u32x4 k[KP], o[OP];
};

template <int NT>
__device__ __forceinline__ void run_load(const TileRanges& r, RunRegs<NT>& v) {
    typedef const __attribute__((address_space(1))) u32x4* gx4;
    const u32 tid = threadIdx.x, nk = r.c2, no = r.c4 - r.c2;
#pragma unroll
    for (int k = 0; k < RunRegs<NT>::KP; k++) {
        const u32 c = k * NT + tid;
        const bool onA = c < r.c1;
        const Range& R = onA ? r.ka : r.kb;
        const u32 cc = c < nk ? (onA ? c : c - r.c1) : 0;
        v.k[k] = *(gx4)(R.base + 16ull * cc);
    }
#pragma unroll
    for (int k = 0; k < RunRegs<NT>::OP; k++) {
        const u32 c = k * NT + tid;
        const bool onA = c < r.c3 - r.c2;
        const Range& R = onA ? r.oa : r.ob;
        const u32 cc = c < no ? (onA ? c : c - (r.c3 - r.c2)) : 0;
        v.o[k] = *(gx4)(R.base + 16ull * cc);
    }
}

template <int NT>
__device__ __forceinline__ void run_put_keys(const TileRanges& r, const RunRegs<NT>& v, u32x4* s_key) {
#pragma unroll
    for (int k = 0; k < RunRegs<NT>::KP; k++) {
        const u32 c = k * NT + threadIdx.x;
        if (c < r.c2) s_key[c] = v.k[k];
    }
}

template <int NT>
__device__ __forceinline__ void run_put_oids(const TileRanges& r, const RunRegs<NT>& v, u32x4* s_oid) {
#pragma unroll
    for (int k = 0; k < RunRegs<NT>::OP; k++) {
        const u32 c = k * NT + threadIdx.x;
        if (c < r.c4 - r.c2) s_oid[c] = v.o[k];
    }
}

// Persistent and software-pipelined: workgroup b merges tiles b, b + G, b + 2G, ... (G = the grid,
// sized so that every workgroup is resident).  As soon as a tile's OIDs are in LDS (after its key
// phase), the loads of the next tile are issued into the same registers: they fly during the current
// tile's emit phase, and the next tile's split points one tile further ahead.
template <int NT, bool HASH>
__global__ __launch_bounds__(NT) void k_join2r(Join2Args g) {
    using LD = RunLds<NT>;
    static_assert(LD::TILE == (NT / 64) * RW, "one RW-item stretch per wave");
    __shared__ u32x4 s_key[LD::CHK];
    __shared__ u32x4 s_oid[LD::CHO];
    __shared__ int s_split[NT / 64 + 1];
    __shared__ u32 s_cnt[NT / 64][4];  // per wave: deltas, updates, deletes, inserts
    u64 tile = blockIdx.x;
    if (tile >= g.ntiles) return;
    TileGeo q = tile_geo(g, tile, LD::TILE);
    if (!q.ok && threadIdx.x == 0) atomicOr(g.err, 1u);
    TileRanges r = tile_ranges(g, q);
    RunRegs<NT> v;
    run_load<NT>(r, v);
    u64 tn = tile + gridDim.x, p0 = 0, p1 = 0;
    if (tn < g.ntiles) { p0 = g.part[tn]; p1 = g.part[tn + 1]; }
    run_put_keys<NT>(r, v, s_key);
    lds_barrier();
    for (;;) {
#if KD_J_CLOCK
        if (threadIdx.x == 0) {
            u64* clk = (u64*)(g.stage_delta + tile * (u64)C2_STAGE + LD::TILE);
            clk[0] = clk[13] = wall_clock64();
        }
#endif
        const bool more = tn < g.ntiles;
        TileGeo qn = q;
        TileRanges rn = r;
        u64 tnn = tn;
        run_tile<NT, HASH>(g, q, r, s_key, s_oid, s_split, s_cnt, tile, [&] {
#if KD_J_CLOCK
            vm_drain();
            if ((threadIdx.x & 63) == 0)
                ((u64*)(g.stage_delta + tile * (u64)C2_STAGE + LD::TILE))[20 + (threadIdx.x >> 6)] = wall_clock64();
#endif
            run_put_oids<NT>(r, v, s_oid);
            lds_barrier();
            if (more) {  // the next tile's loads fly during this tile's emit phase
                qn = tile_geo_from(g, tn, LD::TILE, p0, p1);
                if (!qn.ok && threadIdx.x == 0) atomicOr(g.err, 1u);
                rn = tile_ranges(g, qn);
                run_load<NT>(rn, v);
                tnn = tn + gridDim.x;
                if (tnn < g.ntiles) { p0 = g.part[tnn]; p1 = g.part[tnn + 1]; }
            }
        });  // ends with a barrier: LDS free for the next tile
        if (!more) break;
        run_put_keys<NT>(rn, v, s_key);
        lds_barrier();
        tile = tn;
        q = qn;
        r = rn;
        tn = tnn;
    }
}

// Staged path: tile-local staging -> final key-ordered positions; one tile per block.  The tile's
// output offset = the group sums of all earlier C2_GROUP-tile groups + the counts of the earlier
// tiles of its own group; the last block also writes the totals.
// WS (k_join2r): a tile's records sit in NW wave slots of RW records, tile_cnt holds per wave
// deltas | updates << 16; otherwise one contiguous slot and tile_cnt = inserts, updates, deletes, deltas.
template <bool WS>
__device__ __forceinline__ uint2 tile_du(const uint4 c) {  // (deltas, updates) of one tile
    if (!WS) return make_uint2(c.w, c.y);
    const u32 s = c.x + c.y + c.z + c.w;  // <= 1024 per half: no carry
    return make_uint2(s & 0xFFFF, s >> 16);
}

template <int NT, bool WS>
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
    const u64 t_lo = grp * C2_GROUP;
    if (!last && tid < (int)(t - t_lo)) {
        const uint2 c = tile_du<WS>(*(const uint4*)(tile_cnt + 4 * (t_lo + tid)));
        pd += c.x;
        pu += c.y;
    }
    const uint4 ownc = *(const uint4*)(tile_cnt + 4 * t);
    const uint2 own = tile_du<WS>(ownc);
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
        if (tid == 0) {
            u64 ti = 0, tx = 0;
#pragma unroll
            for (int w = 0; w < NT / 64; w++) { ti += s_red[2][w]; tx += s_red[3][w]; }
            counts[0] = ti;
            counts[1] = pu;
            counts[2] = tx;
            counts[3] = pd;
        }
        pd -= own.x;
        pu -= own.y;
    }
    const uint2* sdp = stage_delta + t * (u64)tile_items;
    const uint2* sup = stage_upd + t * (u64)tile_items;
    // record r of the tile -> its staging slot (WS: the wave slot holding it)
    u32 d1 = 0, d2 = 0, d3 = 0, u1 = 0, u2 = 0, u3 = 0;
    if (WS) {
        d1 = ownc.x & 0xFFFF; d2 = d1 + (ownc.y & 0xFFFF); d3 = d2 + (ownc.z & 0xFFFF);
        u1 = ownc.x >> 16; u2 = u1 + (ownc.y >> 16); u3 = u2 + (ownc.z >> 16);
    }
    auto slot = [&](u32 r, u32 p1, u32 p2, u32 p3) -> u32 {
        if (!WS) return r;
        const u32 w = (u32)(r >= p1) + (u32)(r >= p2) + (u32)(r >= p3);
        const u32 base = w == 0 ? 0 : w == 1 ? p1 : w == 2 ? p2 : p3;
        return w * RW + (r - base);
    };
    constexpr int UC = C2_TILE / NT;
    uint2 v[UC];
#pragma unroll
    for (int j = 0; j < UC; j++) {
        const u32 r = j * NT + tid;
        if (r < own.x) v[j] = sdp[slot(r, d1, d2, d3)];
    }
#pragma unroll
    for (int j = 0; j < UC; j++) {
        const u32 r = j * NT + tid;
        if (r < own.x) out_delta[pd + r] = v[j];
    }
    if (out_upd) {
#pragma unroll
        for (int j = 0; j < UC; j++) {
            const u32 r = j * NT + tid;
            if (r < own.y) v[j] = sup[slot(r, u1, u2, u3)];
        }
#pragma unroll
        for (int j = 0; j < UC; j++) {
            const u32 r = j * NT + tid;
            if (r < own.y) out_upd[pu + r] = v[j];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// k_join2p: persistent, register-prefetched tiles, decoupled look-back
// ---------------------------------------------------------------------------------------------
// (look-back descriptors and lookback(): kd_join.h)

template <int NT, int IPT, bool LOOKBACK>
__global__ __launch_bounds__(NT, KD_J2P_WAVES) void k_join2p(Join2Args g) {
    using LD = Join2Lds<NT, IPT>;
    static_assert(LD::TILE <= 4095, "per-item records hold 12-bit local indices");
    constexpr int R = LD::ROUNDS;
    __shared__ u32x4 s_ch[LD::CH];
    __shared__ u32 s_wave[3 * NT / 64];
    __shared__ u64 s_excl[2];
    const int tid = threadIdx.x;
    const u64 ntiles = g.ntiles, stride = gridDim.x;
    u64 t = blockIdx.x;
    if (t >= ntiles) return;

    // chunk k*NT + tid of the tile's LDS image -> its source address (per-range origin by selects)
    u32x4 v[R];
    auto issue = [&](const TileRanges& r) {
        const u64 ob = r.kb.base - 16ull * r.c1, oa2 = r.oa.base - 16ull * r.c2, ob2 = r.ob.base - 16ull * r.c3;
#pragma unroll
        for (int k = 0; k < R; k++) {
            const u32 c = k * NT + tid;
            const u64 org = c < r.c1 ? r.ka.base : c < r.c2 ? ob : c < r.c3 ? oa2 : ob2;
            const u64 src = c < r.c4 ? org + 16ull * c : (u64)g.dummy;
            v[k] = *(gp_x4)src;
        }
    };
    auto land = [&](const TileRanges& r) {
#pragma unroll
        for (int k = 0; k < R; k++) {
            const u32 c = k * NT + tid;
            if (c < r.c4) s_ch[c] = v[k];
        }
    };
    TileGeo q = tile_geo(g, t, LD::TILE);
    TileRanges r = tile_ranges(g, q);
    issue(r);
    land(r);
    __syncthreads();
    // split points of the tile after next: loaded one iteration early, consumed after a tile's work
    typedef const __attribute__((address_space(1))) u64* gp64;
    u64 pn0 = 0, pn1 = 0;
    if (t + stride < ntiles) { pn0 = ((gp64)g.part)[t + stride]; pn1 = ((gp64)g.part)[t + stride + 1]; }
    for (;;) {
        // ---- prefetch the next tile into registers (in flight during this tile's work) ----
        const u64 tn = t + stride;
        TileGeo qn = q;
        TileRanges rn = r;
        if (tn < ntiles) {
            qn = tile_geo_from(g, tn, LD::TILE, pn0, pn1);
            rn = tile_ranges(g, qn);
            issue(rn);
            const u64 tnn = tn + stride;
            if (tnn < ntiles) { pn0 = ((gp64)g.part)[tnn]; pn1 = ((gp64)g.part)[tnn + 1]; }
        }
        // ---- this tile, out of LDS ----
        const u64* sA = (const u64*)((const u8*)s_ch + r.ka.skew) + q.has_lbA;
        const u64* sB = (const u64*)((const u8*)(s_ch + r.c1) + r.kb.skew) + q.has_lbB;
        const u32* oA = (const u32*)((const u8*)(s_ch + r.c2) + r.oa.skew);
        const u32* oB = (const u32*)((const u8*)(s_ch + r.c3) + r.ob.skew);
        u32 rec[IPT];
        bool bad = !q.ok;
        tile_merge<NT, IPT>(sA, sB, oA, oB, q, rec, bad);
        if (g.hash_mode) tile_names<IPT>(g, q, rec);
        if (bad) atomicOr(g.err, 1u);
        const TileCounts c = tile_counts<NT, IPT>(rec, s_wave);
        if (LOOKBACK) {
            // ---- global offsets: decoupled look-back (wave 0) ----
            if (tid < 64) {
                const u64 ex = lookback(g.desc, ntiles, t, ((u64)c.tnd << 31) | c.tnu, (u64)c.tdel);
                if ((tid & 31) == 0) s_excl[tid >> 5] = ex;
                const u64 ex1 = __shfl(ex, 32, 64);
                if (t == ntiles - 1 && tid == 0) {  // the last tile knows the totals
                    const u64 nd = (ex >> 31) + c.tnd, nu = (ex & 0x7FFFFFFFull) + c.tnu, nx = ex1 + c.tdel;
                    g.counts[0] = nd - nu - nx;
                    g.counts[1] = nu;
                    g.counts[2] = nx;
                    g.counts[3] = nd;
                }
            }
            __syncthreads();
            const u64 e0 = s_excl[0];
            tile_write<IPT>(rec, c, q.i0, q.j0, g.out_delta + (e0 >> 31),
                            g.out_upd ? g.out_upd + (e0 & 0x7FFFFFFFull) : nullptr);
        } else {
            // ---- tile-local staging slots + counts; k_place2 moves them to their final positions ----
            tile_write<IPT>(rec, c, q.i0, q.j0, g.stage_delta + t * (u64)C2_STAGE, g.stage_upd + t * (u64)C2_STAGE);
            if (tid == 0) {
                u32* cc = g.tile_cnt + 4 * t;
                const u32 tins = c.tnd - c.tnu - c.tdel;
                cc[0] = tins;
                cc[1] = c.tnu;
                cc[2] = c.tdel;
                cc[3] = c.tnd;
                u64* gs = g.gsum + 2 * (t / C2_GROUP);
                atomicAdd((unsigned long long*)gs, (unsigned long long)(c.tnd | (u64)c.tnu << 32));
                atomicAdd((unsigned long long*)gs + 1, (unsigned long long)(tins | (u64)c.tdel << 32));
            }
        }
        if (tn >= ntiles) break;
        // ---- the prefetched tile -> LDS (after every wave is done with this one) ----
        __syncthreads();
        land(rn);
        __syncthreads();
        t = tn;
        q = qn;
        r = rn;
    }
}

int diff2_device(kd_ctx* ctx, const kd_side* A, const kd_side* B, u32 flags, u32* d_delta, u32* d_upd,
                 u64* d_counts, u32* d_err) {
    const bool unord = (flags & KD_DIFF_UNORDERED) != 0;
    const bool lookb = !unord && KD_C2_MODE == 2;  // persistent + decoupled look-back (profiling)
    const bool staged = !unord && !lookb;         // tile-local staging + k_place2 (default)
    const u64 nA = A->n, nB = B->n, total = nA + nB;
    KD_CHECK(nA < 0xFFFFFFFFull && nB < 0xFFFFFFFFull, "diff2: side too large for uint32 indices");
    KD_CHECK(!lookb || total < (1ull << 31), "diff2: look-back mode needs base.n + target.n < 2^31");
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
    void *part, *tcnt = nullptr, *sdel = nullptr, *supd = nullptr, *gsum = nullptr, *desc = nullptr;
    int rc;
    if ((rc = ensure(ctx, "c2.part", (ntiles + 1) * sizeof(u64), &part))) return rc;
    u64* zero = nullptr;
    u64 n_zero = 0;
    if (staged) {
        n_zero = 2 * ((ntiles + C2_GROUP - 1) / C2_GROUP);
        if ((rc = ensure(ctx, "c2.tcnt", ntiles * 4 * sizeof(u32), &tcnt))) return rc;
        if ((rc = ensure(ctx, "c2.gsum", n_zero * sizeof(u64), &gsum))) return rc;
        if ((rc = ensure(ctx, "c2.sdel", ntiles * C2_STAGE * sizeof(uint2), &sdel))) return rc;
        if ((rc = ensure(ctx, "c2.supd", ntiles * C2_STAGE * sizeof(uint2), &supd))) return rc;
        zero = (u64*)gsum;
    } else if (lookb) {
        n_zero = 2 * ntiles;
        if ((rc = ensure(ctx, "c2.desc", n_zero * sizeof(u64), &desc))) return rc;
        zero = (u64*)desc;
    }
    void* dz;
    if ((rc = device_zeros(ctx, &dz))) return rc;
    const u64* kA = nA ? A->key : (const u64*)dz;  // an empty side points at device zeros
    const u64* kB = nB ? B->key : (const u64*)dz;
    const u8* empty_oid = (const u8*)dz;
    rc = launch(ctx, "k_partition2", [&] {
        unsigned nb = (unsigned)((ntiles + C2_PG - 1) / C2_PG);
        hipLaunchKernelGGL(k_partition2, dim3(nb), dim3(C2_PNT), 0, ctx->stream, kA, nA, kB, nB, ntiles, (u64*)part,
                           d_counts, d_err, zero, n_zero);
    });
    if (rc) return rc;
    Join2Args g;
    g.A = kA; g.oidA = nA ? A->oid : empty_oid; g.nA = nA;
    g.B = kB; g.oidB = nB ? B->oid : empty_oid; g.nB = nB;
    g.part = (const u64*)part;
    // filename arenas of an empty side point at device zeros (the batched compare loads index 0 of
    // the offsets of lanes without a matched pair)
    g.nameA = nA && A->name ? A->name : (const u8*)dz;
    g.nameOffA = nA && A->name_off ? A->name_off : (const u64*)dz;
    g.nameB = nB && B->name ? B->name : (const u8*)dz;
    g.nameOffB = nB && B->name_off ? B->name_off : (const u64*)dz;
    g.hash_mode = hash ? 1 : 0;
    g.dummy = (const u8*)dz;
    g.stage_delta = (uint2*)sdel; g.stage_upd = (uint2*)supd;
    g.tile_cnt = (u32*)tcnt; g.gsum = (u64*)gsum; g.err = d_err;
    g.out_delta = (uint2*)d_delta; g.out_upd = (uint2*)d_upd; g.counts = d_counts;
    g.desc = (u64*)desc;
    g.ntiles = ntiles;
    if (unord) {
        return launch(ctx, "k_join2", [&] {
            if (hash)
                hipLaunchKernelGGL((k_join2<C2_NT, C2_IPT, true, true>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, g);
            else
                hipLaunchKernelGGL((k_join2<C2_NT, C2_IPT, true, false>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, g);
        });
    }
    const bool ws = KD_C2_MODE == 3;
    if (KD_C2_MODE == 3) {  // run merge, persistent, per-wave slots
        if (ctx->occ_join2r <= 0) {
            int nb = 0;
            KD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k_join2r<C2_NT, false>, C2_NT, 0));
            ctx->occ_join2r = nb > 0 ? nb : 1;
        }
        const u64 grid = std::min<u64>(ntiles, (u64)ctx->n_cu * (u64)ctx->occ_join2r);
        rc = launch(ctx, "k_join2", [&] {
            if (hash)
                hipLaunchKernelGGL((k_join2r<C2_NT, true>), dim3((unsigned)grid), dim3(C2_NT), 0, ctx->stream, g);
            else
                hipLaunchKernelGGL((k_join2r<C2_NT, false>), dim3((unsigned)grid), dim3(C2_NT), 0, ctx->stream, g);
        });
    } else if (KD_C2_MODE == 1) {  // one tile per workgroup, LDS-DMA staging
        rc = launch(ctx, "k_join2", [&] {
            if (hash)
                hipLaunchKernelGGL((k_join2<C2_NT, C2_IPT, false, true>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, g);
            else
                hipLaunchKernelGGL((k_join2<C2_NT, C2_IPT, false, false>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, g);
        });
    } else {
        // persistent: every workgroup resident at once (grid from the occupancy of this kernel)
        const void* kern = lookb ? (const void*)k_join2p<C2_NT, C2_IPT, true> : (const void*)k_join2p<C2_NT, C2_IPT, false>;
        if (ctx->occ_join2p <= 0) {
            int nb = 0;
            KD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, C2_NT, 0));
            ctx->occ_join2p = nb > 0 ? nb : 1;
        }
        const u64 grid = std::min<u64>(ntiles, (u64)ctx->n_cu * (u64)ctx->occ_join2p);
        rc = launch(ctx, "k_join2", [&] {
            if (lookb)
                hipLaunchKernelGGL((k_join2p<C2_NT, C2_IPT, true>), dim3((unsigned)grid), dim3(C2_NT), 0, ctx->stream, g);
            else
                hipLaunchKernelGGL((k_join2p<C2_NT, C2_IPT, false>), dim3((unsigned)grid), dim3(C2_NT), 0, ctx->stream, g);
        });
    }
    if (rc || lookb) return rc;
#if KD_J_CLOCK
    if (ws) hipLaunchKernelGGL(k_jclk_report, dim3(1), dim3(256), 0, ctx->stream, (const uint2*)sdel, ntiles);
#endif
    return launch(ctx, "k_place2", [&] {
        if (ws)
            hipLaunchKernelGGL((k_place2<KD_PLACE_NT, true>), dim3((unsigned)ntiles), dim3(KD_PLACE_NT), 0, ctx->stream,
                               (const uint2*)sdel, (const uint2*)supd, (const u32*)tcnt, (const u64*)gsum, ntiles,
                               (int)C2_STAGE, (uint2*)d_delta, (uint2*)d_upd, d_counts);
        else
            hipLaunchKernelGGL((k_place2<KD_PLACE_NT, false>), dim3((unsigned)ntiles), dim3(KD_PLACE_NT), 0, ctx->stream,
                               (const uint2*)sdel, (const uint2*)supd, (const u32*)tcnt, (const u64*)gsum, ntiles,
                               (int)C2_STAGE, (uint2*)d_delta, (uint2*)d_upd, d_counts);
    });
}

}  // namespace kd
