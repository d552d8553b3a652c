// kd_classify2.hip — classify2: the two-way tree diff on gfx950.
//
// Replaces libgit2's tree-to-tree diff as consumed by RichBaseDataset.diff_feature
// (/root/reference/kart/rich_base_dataset.py:205-300): both commits' feature leaves arrive as
// strictly ascending join keys + 20-byte blob OIDs; a key on one side only is an insert/delete, a
// key on both sides with different OIDs is an update (GIT_DELTA_ADDED/DELETED/MODIFIED).
//
// The key union is cut into 1024-item merge-path tiles (k_partition2, guided two-level search).
// Default (key-ordered) path:
//   k_join2    one tile per 256-thread workgroup: keys by LDS-DMA into LDS, branch-free 4-ary split
//              search + register walk, OIDs of matched pairs compared straight from HBM, ballot
//              compaction into the tile's staging slot + tile counts + 64-tile group sums;
//   k_gscan2   one block: exclusive prefix of the 64-tile group sums, and the totals
//   k_place2   one wave per tile: its group's prefix + earlier tiles of its group -> offset, staged
//              records -> final key-ordered positions.
// KD_DIFF_UNORDERED: k_join2 appends each tile's records at an atomically reserved offset (tiles in
// completion order, key order inside each tile); no k_place2.
// (Earlier variants — a persistent register-prefetched join, a decoupled look-back and a per-wave
// run merge — were measured slower and removed; their numbers are in DESIGN.md §3.1.)
#include <cstdlib>

#include "kd_join.h"

namespace kd {

constexpr u64 C2_GROUP = 64;  // tiles per group sum (staged path: k_place2 offsets)
#ifndef KD_C2_STAGE_PAD
#define KD_C2_STAGE_PAD 32
#endif
// staging slot stride in records: one tile plus a pad, so the slots' hot first lines do not all
// fall on the same HBM channels (a power-of-two stride would)
constexpr u64 C2_STAGE = C2_TILE + KD_C2_STAGE_PAD;
// PERM + KD_KEY_HASH: name rows staged beyond the tile's sorted range on each side (a per-bucket sort
// moves an entry less than its bucket's length)
#ifndef KD_J2_NAME_HALO
#define KD_J2_NAME_HALO 64
#endif
constexpr u64 J2_NAME_HALO = KD_J2_NAME_HALO;
#ifndef KD_PLACE_NT
#define KD_PLACE_NT 64  // one wave per tile: up to 16 staged records per lane, all loads in flight
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
// The kernel also clears the counters and group sums the join needs (stream-ordered
// before it), instead of separate memset launches.
#ifndef KD_PTOP
#define KD_PTOP 16  // lanes per top-level split search
#endif
constexpr int C2_PG = 32, C2_PNT = 256;  // tiles per group; threads (8 lanes per inner split)
template <int TILE>
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
        u64 d = t * (u64)TILE;
        if (d > total) d = total;
        const u64 guess = (u64)((double)d * (double)nA / (double)(total ? total : 1));
        const u64 i = mp_search_guided<KD_PTOP>(A, B, d, d > nB ? d - nB : 0, d < nA ? d : nA, guess, 2048 / KD_PTOP);
        if ((tid & (KD_PTOP - 1)) == 0) s_end[tid / KD_PTOP] = i;
    }
    __syncthreads();
    const u64 i0 = s_end[0], i1 = s_end[1];
    const u64 d0 = t0 * (u64)TILE, d1 = t1 * (u64)TILE < total ? t1 * (u64)TILE : total;
    const u64 j0 = d0 - i0, j1 = d1 - i1;
    if (tid == 0) part[t0] = i0;
    if (tid == 1 && t1 == ntiles) part[ntiles] = i1;
    const u64 t = t0 + 1 + (u64)(tid / 8);  // 8 lanes per inner split
    if (t < t1) {
        const u64 d = t * (u64)TILE;
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
    const u32* ordA;     // PERM: row of sorted entry i in the OID (and filename-offset) arrays
    const u32* ordB;
    uint2* stage_delta;  // staged path: tile-local slots of TILE records
    uint2* stage_upd;
    u32* tile_cnt;       // staged path: [ntiles*4] inserts, updates, deletes, deltas
    u64* gsum;           // staged path: [2*ngroups] deltas | updates<<32, inserts | deletes<<32
    uint2* out_delta;    // final lists
    uint2* out_upd;
    u64* stage_dkey;     // (optional) the join key of every staged delta / update record
    u64* stage_ukey;
    u64* out_dkey;       // (optional) the key of every delta / update, beside the final lists
    u64* out_ukey;
    u64* counts;         // [4] inserts, updates, deletes, deltas
    u32* err;
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
    // keys of both sides (8 B per item, +1 lookahead key on B, +1 lookbehind key per side) and at
    // most two extra (partial) chunks per range
    static constexpr int CHK = (8 * (TILE + 1) + 16 + 15) / 16 + 4;
    // KD_KEY_HASH: the tile's filename bytes of both sides (a tile whose names need more takes the
    // global compare); sized so four 256-thread blocks still fit a CU's LDS with the keys
#ifndef KD_J2_NAME_CH
#define KD_J2_NAME_CH 1900
#endif
    static constexpr int NMCH = KD_J2_NAME_CH;
    // the tile's OIDs of both sides (20 B per entry, the lookahead entry too) when staged in LDS
    static constexpr int OCH = (20 * (TILE + 1) + 32 + 15) / 16 + 4;
    // 4-ary search rounds until a width of TILE shrinks to 0 (w -> ceil(w/4) - 1)
    static constexpr int rounds(int w) { return w <= 0 ? 0 : 1 + rounds((w + 3) / 4 - 1); }
    static constexpr int SEARCH_ROUNDS = rounds(TILE);
};

typedef __attribute__((address_space(3))) void* lds_vp;
typedef const __attribute__((address_space(1))) void* glb_vp;

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
    Range ka, kb;
    u32 c1;  // chunk offset of the B key range in the LDS image
};

__device__ __forceinline__ TileRanges tile_ranges(const Join2Args& g, const TileGeo& q) {
    TileRanges r;
    r.ka = mk_range(g.A, 8 * (q.i0 - q.has_lbA), 8 * q.i1);  // + A[i0-1], B[j0-1]: the lookbehind keys
    r.kb = mk_range(g.B, 8 * (q.j0 - q.has_lbB), 8 * q.j1e);
    r.c1 = r.ka.nch;
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

// Rows of the tile's matched pairs in the OID (and filename-offset) arrays: the sorted indices, or
// (PERM: late materialisation after kd_sort_side_into / kd_sort_segmented_into without OIDs) the walk
// rows ord[i] — one more (coalesced) load round trip instead of a 44-B-per-entry OID gather per side.
template <int IPT, bool PERM>
__device__ __forceinline__ void tile_rows(const Join2Args& g, const TileGeo& q, const u32 rec[IPT], u32 ra[IPT],
                                          u32 rb[IPT]) {
    typedef const __attribute__((address_space(1))) u32* gp32;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        ra[k] = (u32)q.i0 + (rec[k] & 0xFFF);
        rb[k] = (u32)q.j0 + ((rec[k] >> 12) & 0xFFF);
    }
    if (PERM) {
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            const bool m = (rec[k] >> 25) == R_MATCH;
            const gp32 oa = m ? (gp32)(g.ordA + ra[k]) : (gp32)g.dummy;
            const gp32 ob = m ? (gp32)(g.ordB + rb[k]) : (gp32)g.dummy;
            ra[k] = *oa;
            rb[k] = *ob;
        }
    }
}

// OID compare straight from HBM (keys-only LDS image): each thread loads the two 20-B OIDs of its own
// matched pairs (consecutive items -> neighbouring entries across lanes), all loads issued before any
// compare.
template <int IPT>
__device__ __forceinline__ void tile_oid_cmp(const Join2Args& g, u32 rec[IPT], const u32 ra[IPT], const u32 rb[IPT]) {
    typedef const __attribute__((address_space(1))) u32* gp32;
    u32 x[IPT][5], y[IPT][5];
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const bool m = (rec[k] >> 25) == R_MATCH;
        const gp32 pa = m ? (gp32)(g.oidA + 20ull * ra[k]) : (gp32)g.dummy;
        const gp32 pb = m ? (gp32)(g.oidB + 20ull * rb[k]) : (gp32)g.dummy;
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

template <int IPT, bool PERM>
__device__ __forceinline__ void tile_oid_global(const Join2Args& g, const TileGeo& q, u32 rec[IPT], u32 ra[IPT],
                                                u32 rb[IPT]) {
    tile_rows<IPT, PERM>(g, q, rec, ra, rb);
    tile_oid_cmp<IPT>(g, rec, ra, rb);
}

// KD_KEY_HASH: a matched key must also match the full filename (a 64-bit key collision between two
// different names would otherwise be read as an update)
template <int IPT>
__device__ __forceinline__ void tile_names(const Join2Args& g, const u32 rec[IPT], const u32 ia[IPT], const u32 jb[IPT]) {
    u32 act = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) act |= (u32)((rec[k] >> 25) == R_MATCH) << k;
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

// a workgroup barrier for LDS only: waits for this wave's LDS operations, not for its global loads
// in flight (__syncthreads' release fence would drain those: the prefetch of a persistent kernel)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt at their maxima (no wait)
    __builtin_amdgcn_s_barrier();
}

template <int NT, int IPT, bool LB = false>
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
    if (LB) lds_barrier();
    else __syncthreads();
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
                                           uint2* __restrict__ sd, uint2* __restrict__ su, const u64* sA, const u64* sB,
                                           u64* __restrict__ kd, u64* __restrict__ ku) {
    u32 od = c.od, ou = c.ou;
    const u32 has_su = su != nullptr;
    const bool keys = kd != nullptr;  // (uniform)
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u32 kind = rec[k] >> 25, ia = rec[k] & 0xFFF, jb = (rec[k] >> 12) & 0xFFF;
        const u32 isd = (c.fd >> k) & 1, isu = (c.fu >> k) & 1;
        const uint2 v = make_uint2(kind == R_INS ? KD_NONE : (u32)(i0 + ia), kind == R_DEL ? KD_NONE : (u32)(j0 + jb));
        if (isd) sd[od] = v;
        if (keys && isd) {  // the record's key, from the tile's LDS image
            const u64 key = kind == R_INS ? sB[jb] : sA[ia];
            kd[od] = key;
            if ((isu & has_su) && ku) ku[ou] = key;
        }
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
template <int NT, int IPT, bool UNORD, bool HASH, bool PERM, bool OL = false>
__global__ __launch_bounds__(NT) void k_join2(Join2Args g) {
    // (HASH: filename checks compiled in; the int-key instantiation carries none of their registers)
    using LD = Join2Lds<NT, IPT>;
    static_assert(LD::TILE <= 4095, "per-item records hold 12-bit local indices");
    // filenames of matched pairs compared from LDS (KD_KEY_HASH).  PERM: the name arenas are in walk
    // order, and a per-bucket sort (kd_sort_segmented_into) moves an entry at most a bucket's length:
    // the staged rows are the tile's sorted range widened by J2_NAME_HALO on each side, and a pair whose
    // walk row falls outside them (a long bucket, or a full sort's order) is compared in HBM
    constexpr bool LNAMES = HASH;
    // OL (large int-key joins): the tile's OIDs by LDS-DMA with the keys, so the matched pairs
    // compare from LDS with no global round trip after the walk (20.6 KB more LDS: 5 blocks per CU
    // instead of 8, which costs more than it saves on small joins)
    constexpr bool LOIDS = OL && !HASH && !PERM;
    __shared__ u32x4 s_ch[LD::CHK];  // the two key ranges; lanes past the tile's chunks are masked off
    __shared__ u32x4 s_nm[LNAMES ? LD::NMCH : 1];
    __shared__ u32x4 s_oid[LOIDS ? LD::OCH : 1];
    __shared__ u32 s_wave[3 * NT / 64];
    __shared__ u64 s_base[2];
    const int tid = threadIdx.x;
    const u64 tile = blockIdx.x;
    const TileGeo q = tile_geo(g, tile, LD::TILE);
    if (!q.ok && tid == 0) atomicOr(g.err, 1u);
    const TileRanges r = tile_ranges(g, q);
    // the tile's filename byte ranges: A [off[i0], off[i1]), B [off[j0], off[j1e]) (the lookahead
    // entry's name too: a match may pair with it) — loaded with the key DMA
    u64 nmA0 = 0, nmA1 = 0, nmB0 = 0, nmB1 = 0;
    // staged name rows [rA0, rA1) / [rB0, rB1)
    const u64 rA0 = PERM ? (q.i0 > J2_NAME_HALO ? q.i0 - J2_NAME_HALO : 0) : q.i0;
    const u64 rA1 = PERM ? min(q.i1 + J2_NAME_HALO, g.nA) : q.i1;
    const u64 rB0 = PERM ? (q.j0 > J2_NAME_HALO ? q.j0 - J2_NAME_HALO : 0) : q.j0;
    const u64 rB1 = PERM ? min(q.j1e + J2_NAME_HALO, g.nB) : q.j1e;
    if (LNAMES) {
        nmA0 = g.nameOffA[rA0]; nmA1 = g.nameOffA[rA1];
        nmB0 = g.nameOffB[rB0]; nmB1 = g.nameOffB[rB1];
    }
    // 64-chunk pieces (one wave-instruction each: wave-uniform source base and LDS base, lane l takes
    // chunk 64p + l), dealt round-robin to the waves across the two ranges: scalar address math
    auto dma2 = [&](const Range& R0, const Range& R1, u32 c1, u32x4* dst) {
        constexpr int NW = NT / 64;
        const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
        u32 q0 = 0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const Range& R = k == 0 ? R0 : R1;
            const u32 off = k == 0 ? 0 : c1;
            const u32 np = (R.nch + 63) >> 6;
            for (u32 p = (u32)(wid + NW - (int)(q0 % NW)) % NW; p < np; p += NW) {
                const u32 c = 64 * p + lane;
                if (c < R.nch)
                    __builtin_amdgcn_global_load_lds((glb_vp)(R.base + 16ull * c), (lds_vp)(dst + off + 64 * p), 16, 0, 0);
            }
            q0 += np;
        }
    };
    dma2(r.ka, r.kb, r.c1, s_ch);
    Range roA{}, roB{};
    if (LOIDS) {
        roA = mk_range(g.oidA, 20 * q.i0, 20 * q.i1);
        roB = mk_range(g.oidB, 20 * q.j0, 20 * q.j1e);
        dma2(roA, roB, roA.nch, s_oid);
    }
    __syncthreads();  // vmcnt(0) + barrier: the DMA has landed
    // the names DMA runs under the walk and the OID loads
    Range rnA{}, rnB{};
    bool lnames = false;
    if (LNAMES) {
        nmA0 = uni64(nmA0); nmA1 = uni64(nmA1); nmB0 = uni64(nmB0); nmB1 = uni64(nmB1);
        rnA = mk_range(g.nameA, nmA0, nmA1);
        rnB = mk_range(g.nameB, nmB0, nmB1);
        lnames = nmA1 >= nmA0 && nmB1 >= nmB0 && (u64)rnA.nch + rnB.nch <= (u64)LD::NMCH;
        if (lnames) dma2(rnA, rnB, rnA.nch, s_nm);
    }
    const u64* sA = (const u64*)((const u8*)s_ch + r.ka.skew) + q.has_lbA;
    const u64* sB = (const u64*)((const u8*)(s_ch + r.c1) + r.kb.skew) + q.has_lbB;
    u32 rec[IPT];
    bool bad = false;
    tile_walk<NT, IPT>(sA, sB, q, rec, bad);
    // complete order check: the walk only compares the keys it consumes, and on unsorted input the
    // per-thread merge-path splits can skip keys, so every adjacent pair of the tile's two ranges
    // (the first against the lookbehind key) is checked here as well
    for (int x = tid; x < q.na; x += NT) bad |= (x > 0 || q.has_lbA) && sA[x - 1] >= sA[x];
    for (int x = tid; x < q.nb; x += NT) bad |= (x > 0 || q.has_lbB) && sB[x - 1] >= sB[x];
    u32 ra[IPT], rb[IPT];
    // the matched pairs' name offsets, issued with the OID loads: low words only (differences of
    // offsets inside one tile's names fit 32 bits, and modular arithmetic gives them exactly)
    u32 oa0[IPT], oa1[IPT], ob0[IPT], ob1[IPT];
    if (!LOIDS) tile_rows<IPT, PERM>(g, q, rec, ra, rb);
    if (LNAMES && lnames) {
        const u32* offA = (const u32*)g.nameOffA;
        const u32* offB = (const u32*)g.nameOffB;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            const bool m = (rec[k] >> 25) == R_MATCH;
            // unmatched items load nothing (a placeholder row could be the side's end: off[n + 1]
            // lies past the caller's n + 1 offsets)
            const u64 i = m ? ra[k] : 0, j = m ? rb[k] : 0;
            oa0[k] = m ? offA[2 * i] : 0u; oa1[k] = m ? offA[2 * i + 2] : 0u;
            ob0[k] = m ? offB[2 * j] : 0u; ob1[k] = m ? offB[2 * j + 2] : 0u;
        }
    }
    if (LOIDS) {  // matched pairs' OIDs from LDS (both tile ranges landed with the keys)
        typedef const __attribute__((address_space(3))) u32* l32;
        const u32 ob = (u32)(size_t)(const __attribute__((address_space(3))) u32x4*)s_oid;
        const u32 baseA = ob + roA.skew, baseB = ob + 16 * roA.nch + roB.skew;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            const bool m = (rec[k] >> 25) == R_MATCH;
            const u32 pa = baseA + 20 * (m ? (rec[k] & 0xFFF) : 0), pb = baseB + 20 * (m ? ((rec[k] >> 12) & 0xFFF) : 0);
            u32 d = 0;
#pragma unroll
            for (int w = 0; w < 5; w++) d |= *(l32)(size_t)(pa + 4 * w) ^ *(l32)(size_t)(pb + 4 * w);
            if (m && d) rec[k] |= 1u << 24;
        }
    } else {
        tile_oid_cmp<IPT>(g, rec, ra, rb);
    }
    if (LNAMES && lnames) {
        __syncthreads();  // vmcnt(0) + barrier: every wave's share of the names DMA has landed
        const u32 nm = (u32)(size_t)(const __attribute__((address_space(3))) u32x4*)s_nm;
        const u32 baseA = nm + rnA.skew, baseB = nm + 16 * rnA.nch + rnB.skew;
        bool ne = false;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            if ((rec[k] >> 25) != R_MATCH) continue;
            const u32 la = oa1[k] - oa0[k], lb = ob1[k] - ob0[k];
            if (PERM && (ra[k] < rA0 || ra[k] >= rA1 || rb[k] < rB0 || rb[k] >= rB1))  // a row outside the staged names
                ne |= !names_eq(g.nameA, g.nameOffA, ra[k], g.nameB, g.nameOffB, rb[k]);
            else
                ne |= la != lb || !lds_eq_bytes(baseA + (oa0[k] - (u32)nmA0), baseB + (ob0[k] - (u32)nmB0), la);
        }
        if (ne) atomicOr(g.err, 2u);
    } else if (HASH) {
        tile_names<IPT>(g, rec, ra, rb);
    }
    if (bad) atomicOr(g.err, 1u);
    const TileCounts c = tile_counts<NT, IPT>(rec, s_wave);
    uint2 *sd, *su;
    u64 *kd, *ku;
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
        kd = g.out_dkey ? g.out_dkey + s_base[0] : nullptr;
        ku = g.out_dkey && g.out_upd && g.out_ukey ? g.out_ukey + s_base[1] : nullptr;  // each key list optional
    } else {
        sd = g.stage_delta + tile * (u64)C2_STAGE;
        su = g.stage_upd + tile * (u64)C2_STAGE;
        kd = g.stage_dkey ? g.stage_dkey + tile * (u64)C2_STAGE : nullptr;
        ku = g.stage_dkey ? g.stage_ukey + tile * (u64)C2_STAGE : nullptr;
    }
    tile_write<IPT>(rec, c, q.i0, q.j0, sd, su, sA, sB, kd, ku);
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
// k_join2r: the large int-key join, persistent with the next tile prefetched into registers.
// A resident grid walks the tiles grid-stride; while tile t is walked, compared and written out
// from LDS, tile t+1's keys and OIDs (keys + OIDs of both sides, ~28 KB) are in flight as plain
// 16-B loads into registers (P per thread), and tile t+2's split points too.  After tile t the
// registers go to LDS.  The barriers inside a tile are LDS-only (lds_barrier), so nothing in the
// tile's own work waits for the prefetch — an LDS-DMA double buffer (tried in round 2) makes the
// compiler drain every load before each LDS read.
// ---------------------------------------------------------------------------------------------
template <int NT, int IPT>
struct J2RTile {
    TileGeo q;
    TileRanges r;
    Range oa, ob;
    u32 n0, n1, n2, n3;  // cumulative chunk counts: keys A, keys B, OIDs A, OIDs B
};

template <int NT, int IPT>
__device__ __forceinline__ void j2r_plan(const Join2Args& g, u64 tile, u64 p0, u64 p1, J2RTile<NT, IPT>& T) {
    using LD = Join2Lds<NT, IPT>;
    T.q = tile_geo_from(g, tile, LD::TILE, p0, p1);
    T.r = tile_ranges(g, T.q);
    T.oa = mk_range(g.oidA, 20 * T.q.i0, 20 * T.q.i1);
    T.ob = mk_range(g.oidB, 20 * T.q.j0, 20 * T.q.j1e);
    T.n0 = T.r.ka.nch;
    T.n1 = T.n0 + T.r.kb.nch;
    T.n2 = T.n1 + T.oa.nch;
    T.n3 = T.n2 + T.ob.nch;
}

template <int NT, int IPT>
__global__ __launch_bounds__(NT) void k_join2r(Join2Args g) {
    using LD = Join2Lds<NT, IPT>;
    static_assert(LD::TILE <= 4095, "per-item records hold 12-bit local indices");
    constexpr int P = (LD::CHK + LD::OCH + NT - 1) / NT;  // prefetched chunks per thread
    __shared__ u32x4 s_ch[LD::CHK];
    __shared__ u32x4 s_oid[LD::OCH];
    __shared__ u32 s_wave[3 * NT / 64];
    typedef __attribute__((address_space(3))) u32x4* l128;
    typedef const __attribute__((address_space(1))) u32x4* g128;
    const int tid = threadIdx.x;
    const u64 ntiles = g.ntiles;
    u64 tile = blockIdx.x;
    if (tile >= ntiles) return;
    J2RTile<NT, IPT> cur, nxt;
    u32x4 buf[P];
    auto fetch = [&](const J2RTile<NT, IPT>& T) {
#pragma unroll
        for (int p = 0; p < P; p++) {
            const u32 c = tid + NT * p;
            u64 src = 0;
            if (c < T.n0) src = T.r.ka.base + 16ull * c;
            else if (c < T.n1) src = T.r.kb.base + 16ull * (c - T.n0);
            else if (c < T.n2) src = T.oa.base + 16ull * (c - T.n1);
            else if (c < T.n3) src = T.ob.base + 16ull * (c - T.n2);
            if (c < T.n3) buf[p] = *(g128)src;
        }
    };
    auto deposit = [&](const J2RTile<NT, IPT>& T) {
#pragma unroll
        for (int p = 0; p < P; p++) {
            const u32 c = tid + NT * p;
            if (c < T.n0) *(l128)(s_ch + c) = buf[p];
            else if (c < T.n1) *(l128)(s_ch + T.r.c1 + (c - T.n0)) = buf[p];
            else if (c < T.n2) *(l128)(s_oid + (c - T.n1)) = buf[p];
            else if (c < T.n3) *(l128)(s_oid + T.oa.nch + (c - T.n2)) = buf[p];
        }
    };
    j2r_plan<NT, IPT>(g, tile, g.part[tile], g.part[tile + 1], cur);
    fetch(cur);
    deposit(cur);
    u64 nt = tile + gridDim.x;
    u64 np0 = 0, np1 = 0;
    if (nt < ntiles) { np0 = g.part[nt]; np1 = g.part[nt + 1]; }
    lds_barrier();
    for (;;) {
        const bool more = nt < ntiles;  // block-uniform
        if (more) {
            j2r_plan<NT, IPT>(g, nt, np0, np1, nxt);
            fetch(nxt);  // in flight under this tile's work
        }
        const u64 nn = nt + gridDim.x;
        u64 ap0 = 0, ap1 = 0;
        if (more && nn < ntiles) { ap0 = g.part[nn]; ap1 = g.part[nn + 1]; }
        // ---- tile `tile` from LDS ----
        const TileGeo& q = cur.q;
        if (!q.ok && tid == 0) atomicOr(g.err, 1u);
        const u64* sA = (const u64*)((const u8*)s_ch + cur.r.ka.skew) + q.has_lbA;
        const u64* sB = (const u64*)((const u8*)(s_ch + cur.r.c1) + cur.r.kb.skew) + q.has_lbB;
        u32 rec[IPT];
        bool bad = false;
        tile_walk<NT, IPT>(sA, sB, q, rec, bad);
        for (int x = tid; x < q.na; x += NT) bad |= (x > 0 || q.has_lbA) && sA[x - 1] >= sA[x];
        for (int x = tid; x < q.nb; x += NT) bad |= (x > 0 || q.has_lbB) && sB[x - 1] >= sB[x];
        {
            typedef const __attribute__((address_space(3))) u32* l32;
            const u32 ob = (u32)(size_t)(const __attribute__((address_space(3))) u32x4*)s_oid;
            const u32 baseA = ob + cur.oa.skew, baseB = ob + 16 * cur.oa.nch + cur.ob.skew;
#pragma unroll
            for (int k = 0; k < IPT; k++) {
                const bool m = (rec[k] >> 25) == R_MATCH;
                const u32 pa = baseA + 20 * (m ? (rec[k] & 0xFFF) : 0), pb = baseB + 20 * (m ? ((rec[k] >> 12) & 0xFFF) : 0);
                u32 d = 0;
#pragma unroll
                for (int w = 0; w < 5; w++) d |= *(l32)(size_t)(pa + 4 * w) ^ *(l32)(size_t)(pb + 4 * w);
                if (m && d) rec[k] |= 1u << 24;
            }
        }
        if (bad) atomicOr(g.err, 1u);
        const TileCounts c = tile_counts<NT, IPT, true>(rec, s_wave);
        uint2* sd = g.stage_delta + tile * (u64)C2_STAGE;
        uint2* su = g.stage_upd + tile * (u64)C2_STAGE;
        u64* kd = g.stage_dkey ? g.stage_dkey + tile * (u64)C2_STAGE : nullptr;
        u64* ku = g.stage_dkey ? g.stage_ukey + tile * (u64)C2_STAGE : nullptr;
        tile_write<IPT>(rec, c, q.i0, q.j0, sd, su, sA, sB, kd, ku);
        if (tid == 0) {
            u32* cc = g.tile_cnt + 4 * tile;
            const u32 tins = c.tnd - c.tnu - c.tdel;
            cc[0] = tins;
            cc[1] = c.tnu;
            cc[2] = c.tdel;
            cc[3] = c.tnd;
            u64* gs = g.gsum + 2 * (tile / C2_GROUP);
            atomicAdd((unsigned long long*)gs, (unsigned long long)(c.tnd | (u64)c.tnu << 32));
            atomicAdd((unsigned long long*)gs + 1, (unsigned long long)(tins | (u64)c.tdel << 32));
        }
        if (!more) break;
        lds_barrier();  // every thread is done with the tile's LDS (and s_wave)
        deposit(nxt);
        lds_barrier();
        cur = nxt;
        tile = nt;
        nt = nn;
        np0 = ap0;
        np1 = ap1;
    }
}

// Staged path, step 1: one block scans the C2_GROUP-tile group sums (exclusive prefix of deltas and
// updates per group) and writes the totals — so each k_place2 tile reads one prefix instead of
// summing every earlier group (which made k_place2 O(tiles x groups): 0.30 ms at C3's 195k tiles).
// layout 0 (classify2): counts = inserts, updates, deletes, deltas; layout 1 (k_join3, where the
// "deltas" are conflicts, the "updates" merge deltas and the "inserts" clean paths): counts = clean,
// conflicts, merge deltas, 0
// GSCAN_GPT groups per thread, contiguous, all loaded by one 16-B load each before any use: one pass
// (one HBM round trip) for up to 8192 groups = 524k tiles.  (The form with one group per thread walked
// 1024-group chunks, each behind the previous chunk's barrier: 44 us for C3's 3k groups, 58 for C4's.)
constexpr int GSCAN_GPT = 8;
__global__ __launch_bounds__(1024) void k_gscan2(const u64* __restrict__ gsum, u64 ngroups, u64* __restrict__ gpre,
                                                 u64* __restrict__ counts, int layout) {
    __shared__ u64 s_w[4][16];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const u32x4* g4 = (const u32x4*)gsum;  // group k: (deltas | updates << 32, inserts | deletes << 32)
    u32x4* p4 = (u32x4*)gpre;              // group k: (delta prefix, update prefix)
    u64 cd = 0, cu = 0, ci = 0, cx = 0;
    for (u64 base = 0; base < ngroups; base += 1024 * GSCAN_GPT) {  // (block-uniform; one pass up to 8192 groups)
        const u64 k0 = base + (u64)tid * GSCAN_GPT;
        u32x4 v[GSCAN_GPT];
#pragma unroll
        for (int j = 0; j < GSCAN_GPT; j++) v[j] = k0 + j < ngroups ? g4[k0 + j] : u32x4{0u, 0u, 0u, 0u};
        u64 td = 0, tu = 0, ti = 0, tx = 0;
#pragma unroll
        for (int j = 0; j < GSCAN_GPT; j++) {
            td += v[j].x; tu += v[j].y; ti += v[j].z; tx += v[j].w;
        }
        u64 sd = td, su = tu, si = ti, sx = tx;  // inclusive wave scans (d, u), sums (i, x)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u64 yd = __shfl_up(sd, o, 64), yu = __shfl_up(su, o, 64);
            if (lane >= o) { sd += yd; su += yu; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) { si += __shfl_xor(si, o, 64); sx += __shfl_xor(sx, o, 64); }
        if (lane == 63) { s_w[0][wid] = sd; s_w[1][wid] = su; }
        if (lane == 0) { s_w[2][wid] = si; s_w[3][wid] = sx; }
        __syncthreads();
        u64 wd = 0, wu = 0, Td = 0, Tu = 0, Ti = 0, Tx = 0;
#pragma unroll
        for (int w = 0; w < 16; w++) {
            if (w < wid) { wd += s_w[0][w]; wu += s_w[1][w]; }
            Td += s_w[0][w]; Tu += s_w[1][w]; Ti += s_w[2][w]; Tx += s_w[3][w];
        }
        u64 pd = cd + wd + sd - td, pu = cu + wu + su - tu;  // this thread's first group's prefixes
#pragma unroll
        for (int j = 0; j < GSCAN_GPT; j++) {
            if (k0 + j < ngroups) p4[k0 + j] = u32x4{(u32)pd, (u32)(pd >> 32), (u32)pu, (u32)(pu >> 32)};
            pd += v[j].x;
            pu += v[j].y;
        }
        cd += Td; cu += Tu; ci += Ti; cx += Tx;
        __syncthreads();
    }
    if (tid == 0) {
        counts[0] = ci;
        counts[1] = layout ? cd : cu;
        counts[2] = layout ? cu : cx;
        counts[3] = layout ? 0 : cd;
    }
}

// Staged path, step 2: tile-local staging -> final key-ordered positions; one tile per block.  The
// tile's output offset = its group's prefix (k_gscan2) + the counts of the earlier tiles of its own
// group.  tile_cnt = inserts, updates, deletes, deltas per tile.
template <int NT>
__global__ __launch_bounds__(NT) void k_place2(const uint2* __restrict__ stage_delta, const uint2* __restrict__ stage_upd,
                                               const u32* __restrict__ tile_cnt, const u64* __restrict__ gpre,
                                               int tile_items, uint2* __restrict__ out_delta, uint2* __restrict__ out_upd,
                                               const u64* __restrict__ stage_dkey, const u64* __restrict__ stage_ukey,
                                               u64* __restrict__ out_dkey, u64* __restrict__ out_ukey) {
    static_assert(NT == 64, "k_place2: one wave per tile");
    const int tid = threadIdx.x;
    const u64 t = blockIdx.x;
    const u64 grp = t / C2_GROUP;
    const u64 t_lo = grp * C2_GROUP;
    const uint2* sdp = stage_delta + t * (u64)tile_items;
    const uint2* sup = stage_upd + t * (u64)tile_items;
    // The first 64 staged records of both lists are loaded with the counts, before anything is known
    // about them (a tile's slot is always allocated whole; ~51 deltas and ~41 updates per tile at
    // 10 % edits): one memory round trip for most tiles instead of two
    const uint2 v0 = sdp[tid];
    const uint2 w0 = out_upd ? sup[tid] : make_uint2(0, 0);
    // (and the first 64 record keys of each list, when asked for: no second round trip for them)
    const u64* skd = out_dkey ? stage_dkey + t * (u64)tile_items : nullptr;
    const u64* sku = out_dkey && out_upd && out_ukey ? stage_ukey + t * (u64)tile_items : nullptr;
    const u64 kd0 = skd ? skd[tid] : 0, ku0 = sku ? sku[tid] : 0;
    u64 pd = 0, pu = 0;
    if (tid < (int)(t - t_lo)) {
        const uint4 c = *(const uint4*)(tile_cnt + 4 * (t_lo + tid));
        pd = c.w;
        pu = c.y;
    }
    const u64 gd = gpre[2 * grp], gu = gpre[2 * grp + 1];
    const uint4 ownc = *(const uint4*)(tile_cnt + 4 * t);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { pd += __shfl_xor(pd, o, 64); pu += __shfl_xor(pu, o, 64); }
    pd += gd;
    pu += gu;
    const uint2 own = make_uint2(ownc.w, ownc.y);  // (deltas, updates) of this tile
    constexpr int UC = C2_TILE / NT;
    uint2 v[UC];
#pragma unroll
    for (int j = 1; j < UC; j++) {
        const u32 r = j * NT + tid;
        if (r < own.x) v[j] = sdp[r];
    }
    if ((u32)tid < own.x) out_delta[pd + tid] = v0;
#pragma unroll
    for (int j = 1; j < UC; j++) {
        const u32 r = j * NT + tid;
        if (r < own.x) out_delta[pd + r] = v[j];
    }
    if (out_upd) {
#pragma unroll
        for (int j = 1; j < UC; j++) {
            const u32 r = j * NT + tid;
            if (r < own.y) v[j] = sup[r];
        }
        if ((u32)tid < own.y) out_upd[pu + tid] = w0;
#pragma unroll
        for (int j = 1; j < UC; j++) {
            const u32 r = j * NT + tid;
            if (r < own.y) out_upd[pu + r] = v[j];
        }
    }
    if (skd) {  // the records' keys, when the caller asked for them
        if ((u32)tid < own.x) out_dkey[pd + tid] = kd0;
        for (u32 r = tid + NT; r < own.x; r += NT) out_dkey[pd + r] = skd[r];
    }
    if (sku) {
        if ((u32)tid < own.y) out_ukey[pu + tid] = ku0;
        for (u32 r = tid + NT; r < own.y; r += NT) out_ukey[pu + r] = sku[r];
    }
}


// ---------------------------------------------------------------------------------------------
// k_join3: the three-way merge (libgit2 git_merge_trees, kart/merge.py:99-100) in one pass over
// the three sorted sides.  The O∪T key union is cut into k_join2's merge-path tiles; the ancestor
// entries of each tile's key range — [apart[t], apart[t+1]) plus one lookahead entry, apart[t] =
// lower_bound(ancestor, first key of tile t) (k_apart3) — are staged in LDS with the tile's keys.
// The tile walk pairs ours with theirs as k_join2 does; every path where they differ (one side only,
// or different OIDs) finds its ancestor entry by an LDS binary search, loads the (at most three)
// OIDs and applies the libgit2 rule: o == t -> clean; a == o -> theirs (merge delta); a == t ->
// ours (clean); else conflict.  Conflicts and merge deltas are staged per tile and placed in path
// order (k_gscan2 layout 1, k_place3).  The ancestor's keys are read once, in order, and its OIDs
// only where ours and theirs differ; the order checks of all three sides ride along.
// ---------------------------------------------------------------------------------------------
struct Join3Args {
    Join2Args j;          // A = ours, B = theirs (k_join2's two sides)
    const u64* K;         // the ancestor: keys, OIDs, filenames, walk rows (PERM)
    const u8* oidK;
    const u8* nameK;
    const u64* nameOffK;
    const u32* ordK;
    u64 nK;
    const u64* apart;     // [ntiles + 1]
    u32* stage_conf;      // per tile C2_STAGE slots of (a, o, t)
    uint2* stage_md;      // per tile C2_STAGE slots of (o, t)
    const u64* nsplit;    // (k_join3b, KD_KEY_HASH) [4 * (ntiles + 1)]: name offsets around each split
};
#ifndef KD_J3_ACAP
#define KD_J3_ACAP 1024   // ancestor keys of a tile staged in LDS (a longer range is searched in HBM)
#endif
constexpr int J3_ACAP = KD_J3_ACAP;
#ifndef KD_J3_IPT
#define KD_J3_IPT 3  // 768-item tiles: with the ancestor keys, four 256-thread blocks fit a CU's LDS
#endif
constexpr int J3_IPT = KD_J3_IPT;
constexpr int J3_TILE = C2_NT * J3_IPT;
#ifndef KD_J3_NAME_CH
#define KD_J3_NAME_CH 1425  // filename bytes of a tile in LDS (C4's 24-B names of a 768-item tile + halo: ~22 KB)
#endif

// smallest p in [lo, hi] with p == hi || K[p] >= key, by groups of PW lanes (PW-ary search)
template <int PW>
__device__ __forceinline__ u64 lb_search(const u64* __restrict__ K, u64 key, u64 lo, u64 hi) {
    const int lane = threadIdx.x & 63, sub = lane % PW, grp = lane / PW;
    while (hi > lo) {
        const u64 step = (hi - lo + PW - 1) / PW;
        const u64 probe = lo + step * (u64)(sub + 1) - 1;
        bool p = true;
        if (probe < hi) p = K[probe] >= key;
        const unsigned long long bal = (__ballot(p) >> (grp * PW)) & ((PW == 64) ? ~0ull : ((1ull << PW) - 1));
        if (bal == 0) return hi;
        const int f = __ffsll(bal) - 1;
        const u64 nh = lo + step * (u64)(f + 1) - 1;
        lo = lo + step * (u64)f;
        hi = nh < hi ? nh : hi;
        if (step == 1) return hi;
    }
    return lo;
}

// the same from a guess: PW probes `step` apart around it bracket the answer (or bound one side)
template <int PW>
__device__ __forceinline__ u64 lb_guided(const u64* __restrict__ K, u64 n, u64 key, u64 guess, u64 step) {
    const int lane = threadIdx.x & 63, sub = lane % PW, grp = lane / PW;
    const u64 span = step * (PW / 2);
    const u64 g0 = guess > span ? guess - span : 0;
    u64 probe = g0 + step * (u64)sub;
    if (probe > n) probe = n;
    const bool p = probe >= n || K[probe] >= key;
    const unsigned long long bal = (__ballot(p) >> (grp * PW)) & ((PW == 64) ? ~0ull : ((1ull << PW) - 1));
    const int f = bal ? __ffsll(bal) - 1 : PW;
    const u64 pf = f < PW ? (g0 + step * (u64)f < n ? g0 + step * (u64)f : n) : n;
    const u64 pl = f > 0 ? (g0 + step * (u64)(f - 1) < n ? g0 + step * (u64)(f - 1) : n) : 0;
    const u64 nlo = f > 0 ? pl + 1 : 0;
    return lb_search<PW>(K, key, nlo < pf ? nlo : pf, pf);
}

// apart[t] for t in [0, ntiles]: 8 lanes per split, guided by the proportional position
__global__ __launch_bounds__(256) void k_apart3(const u64* __restrict__ O, u64 nO, const u64* __restrict__ T, u64 nT,
                                                const u64* __restrict__ part, u64 ntiles, int tile_items,
                                                const u64* __restrict__ K, u64 nK, u64* __restrict__ apart) {
    const u64 t = ((u64)blockIdx.x * 256 + threadIdx.x) / 8;
    if (t > ntiles) return;  // (whole 8-lane groups)
    u64 r;
    if (t == 0) r = 0;
    else if (t == ntiles) r = nK;
    else {
        const u64 i = part[t], d = t * (u64)tile_items, j = d - i;
        const u64 a = i < nO ? O[i] : ~0ull, b = j < nT ? T[j] : ~0ull;
        const u64 key = a < b ? a : b;
        // ours is the ancestor with a few edits: its index i is the ancestor rank up to the edits'
        // running balance (a random walk of ~sqrt(edits) entries), so probes 256 apart around it
        // bracket the answer; without ours, the proportional position
        const u64 guess = nO ? (u64)((double)i / (double)nO * (double)nK) : (u64)((double)d / (double)(nO + nT) * (double)nK);
        r = lb_guided<8>(K, nK, key, guess < nK ? guess : nK, 256);
    }
    if ((threadIdx.x & 7) == 0) apart[t] = r;
}

// a byte range into LDS by LDS-DMA: 64-chunk pieces dealt round-robin to the waves, continuing the
// deal of earlier ranges (q0 = pieces dealt so far); returns the new count
template <int NT>
__device__ __forceinline__ u32 dma_range(const Range& R, u32x4* dst, u32 q0) {
    constexpr int NW = NT / 64;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const u32 np = (R.nch + 63) >> 6;
    for (u32 p = (u32)(wid + NW - (int)(q0 % NW)) % NW; p < np; p += NW) {
        const u32 c = 64 * p + lane;
        if (c < R.nch) __builtin_amdgcn_global_load_lds((glb_vp)(R.base + 16ull * c), (lds_vp)(dst + 64 * p), 16, 0, 0);
    }
    return q0 + np;
}

// SPLIT: every differing path is staged with its ancestor entry as a candidate (a, o, t) and the
// rule is applied by k_resolve3<HAVE_A> over the placed list (many paths per thread: the OID and
// filename loads of the few differing paths of a tile no longer hold the tile's LDS)
template <int NT, int IPT, bool HASH, bool PERM, bool SPLIT, bool OL = false>
__global__ __launch_bounds__(NT) void k_join3(Join3Args g3) {
    const Join2Args& g = g3.j;
    using LD = Join2Lds<NT, IPT>;
    // OL (A/B, sorted-form sides only): ours' and theirs' OIDs of the tile by LDS-DMA with the keys,
    // so the matched pairs compare from LDS (one HBM round trip less per tile, 15 KB more LDS)
    constexpr bool LOIDS = OL && !PERM;
    __shared__ u32x4 s_oid[LOIDS ? LD::OCH : 1];
    static_assert(LD::TILE <= 4095, "per-item records hold 12-bit local indices");
    constexpr int KCH = (8 * (J3_ACAP + 2) + 16 + 15) / 16 + 4;
    __shared__ u32x4 s_ch[LD::CHK];
    __shared__ u32x4 s_k[KCH];
    constexpr int NMCH = KD_J3_NAME_CH;
    __shared__ u32x4 s_nm[HASH ? NMCH : 1];
    // the tile's differing paths (their walk records) in path order: in hash mode the filename buffer
    // holds them (the names are compared before), else a buffer of their own
    __shared__ u32 s_drec_own[HASH ? 1 : LD::TILE];
    __shared__ u32 s_wave[3 * NT / 64];
    typedef const __attribute__((address_space(1))) u32* gp32;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const u64 tile = blockIdx.x;
    const TileGeo q = tile_geo(g, tile, LD::TILE);
    bool bad = !q.ok;
    const TileRanges r = tile_ranges(g, q);
    // the ancestor entries of the tile's key range [k0, k1) (+ the lookahead entry k1: a match of ours'
    // last entry with theirs' lookahead has the next tile's first key) and the lookbehind key
    const u64 k0 = uni64(g3.apart[tile]), kend = uni64(g3.apart[tile + 1]);
    const bool kok = kend >= k0 && kend <= g3.nK;
    bad |= !kok;
    const u64 k1 = kok ? kend : k0;
    const u64 k1e = k1 < g3.nK ? k1 + 1 : k1;
    const bool has_lbK = k0 > 0;
    const bool lk = k1e - k0 <= (u64)J3_ACAP;
    Range rk{};
    if (lk) rk = mk_range(g3.K, 8 * (k0 - has_lbK), 8 * k1e);
    u64 nmA0 = 0, nmA1 = 0, nmB0 = 0, nmB1 = 0;
    const u64 rA0 = PERM ? (q.i0 > J2_NAME_HALO ? q.i0 - J2_NAME_HALO : 0) : q.i0;
    const u64 rA1 = PERM ? min(q.i1 + J2_NAME_HALO, g.nA) : q.i1;
    const u64 rB0 = PERM ? (q.j0 > J2_NAME_HALO ? q.j0 - J2_NAME_HALO : 0) : q.j0;
    const u64 rB1 = PERM ? min(q.j1e + J2_NAME_HALO, g.nB) : q.j1e;
    if (HASH) {
        nmA0 = g.nameOffA[rA0]; nmA1 = g.nameOffA[rA1];
        nmB0 = g.nameOffB[rB0]; nmB1 = g.nameOffB[rB1];
    }
    u32 qq = dma_range<NT>(r.ka, s_ch, 0);
    qq = dma_range<NT>(r.kb, s_ch + r.c1, qq);
    if (lk) qq = dma_range<NT>(rk, s_k, qq);
    Range roA{}, roB{};
    if (LOIDS) {
        roA = mk_range(g.oidA, 20 * q.i0, 20 * q.i1);
        roB = mk_range(g.oidB, 20 * q.j0, 20 * q.j1e);
        qq = dma_range<NT>(roA, s_oid, qq);
        qq = dma_range<NT>(roB, s_oid + roA.nch, qq);
    }
    __syncthreads();  // vmcnt(0) + barrier: the keys have landed
    Range rnA{}, rnB{};
    bool lnames = false;
    if (HASH) {
        nmA0 = uni64(nmA0); nmA1 = uni64(nmA1); nmB0 = uni64(nmB0); nmB1 = uni64(nmB1);
        rnA = mk_range(g.nameA, nmA0, nmA1);
        rnB = mk_range(g.nameB, nmB0, nmB1);
        lnames = nmA1 >= nmA0 && nmB1 >= nmB0 && (u64)rnA.nch + rnB.nch <= (u64)NMCH;
        if (lnames) dma_range<NT>(rnB, s_nm + rnA.nch, dma_range<NT>(rnA, s_nm, 0));
    }
    const u64* sA = (const u64*)((const u8*)s_ch + r.ka.skew) + q.has_lbA;
    const u64* sB = (const u64*)((const u8*)(s_ch + r.c1) + r.kb.skew) + q.has_lbB;
    const u64* sK = (const u64*)((const u8*)s_k + rk.skew) + has_lbK;
    u32 rec[IPT];
    tile_walk<NT, IPT>(sA, sB, q, rec, bad);
    for (int x = tid; x < q.na; x += NT) bad |= (x > 0 || q.has_lbA) && sA[x - 1] >= sA[x];
    for (int x = tid; x < q.nb; x += NT) bad |= (x > 0 || q.has_lbB) && sB[x - 1] >= sB[x];
    // the ancestor strictly ascending: every adjacent pair (x-1, x) with x in [k0, k1) once over all tiles
    if (lk) {
        for (int x = tid; x < (int)(k1 - k0); x += NT) bad |= (x > 0 || has_lbK) && sK[x - 1] >= sK[x];
    } else {
        for (u64 x = k0 + tid; x < k1; x += NT) bad |= x > 0 && g3.K[x - 1] >= g3.K[x];
    }
    u32 ra[IPT], rb[IPT];
    u32 oa0[IPT], oa1[IPT], ob0[IPT], ob1[IPT];
    tile_rows<IPT, PERM>(g, q, rec, ra, rb);
    if (HASH && lnames) {
        const u32* offA = (const u32*)g.nameOffA;
        const u32* offB = (const u32*)g.nameOffB;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            const bool m = (rec[k] >> 25) == R_MATCH;
            // unmatched items load nothing (a placeholder row could be the side's end: off[n + 1]
            // lies past the caller's n + 1 offsets)
            const u64 i = m ? ra[k] : 0, j = m ? rb[k] : 0;
            oa0[k] = m ? offA[2 * i] : 0u; oa1[k] = m ? offA[2 * i + 2] : 0u;
            ob0[k] = m ? offB[2 * j] : 0u; ob1[k] = m ? offB[2 * j + 2] : 0u;
        }
    }
    if (LOIDS) {  // matched pairs' OIDs from LDS (both tile ranges landed with the keys)
        typedef const __attribute__((address_space(3))) u32* l32;
        const u32 ob = (u32)(size_t)(const __attribute__((address_space(3))) u32x4*)s_oid;
        const u32 baseA = ob + roA.skew, baseB = ob + 16 * roA.nch + roB.skew;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            const bool m = (rec[k] >> 25) == R_MATCH;
            const u32 pa = baseA + 20 * (m ? (rec[k] & 0xFFF) : 0), pb = baseB + 20 * (m ? ((rec[k] >> 12) & 0xFFF) : 0);
            u32 d = 0;
#pragma unroll
            for (int w = 0; w < 5; w++) d |= *(l32)(size_t)(pa + 4 * w) ^ *(l32)(size_t)(pb + 4 * w);
            if (m && d) rec[k] |= 1u << 24;
        }
    } else {
        tile_oid_cmp<IPT>(g, rec, ra, rb);
    }
    bool ne = false;
    if (HASH && lnames) {
        __syncthreads();  // vmcnt(0) + barrier: the names DMA has landed
        const u32 nm = (u32)(size_t)(const __attribute__((address_space(3))) u32x4*)s_nm;
        const u32 baseA = nm + rnA.skew, baseB = nm + 16 * rnA.nch + rnB.skew;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            if ((rec[k] >> 25) != R_MATCH) continue;
            const u32 la = oa1[k] - oa0[k], lb = ob1[k] - ob0[k];
            if (PERM && (ra[k] < rA0 || ra[k] >= rA1 || rb[k] < rB0 || rb[k] >= rB1))
                ne |= !names_eq(g.nameA, g.nameOffA, ra[k], g.nameB, g.nameOffB, rb[k]);
            else
                ne |= la != lb || !lds_eq_bytes(baseA + (oa0[k] - (u32)nmA0), baseB + (ob0[k] - (u32)nmB0), la);
        }
    } else if (HASH) {
        u32 act = 0;
#pragma unroll
        for (int k = 0; k < IPT; k++) act |= (u32)((rec[k] >> 25) == R_MATCH) << k;
        ne |= names_ne_batch<IPT, 8>(g.nameA, g.nameOffA, ra, g.nameB, g.nameOffB, rb, act) != 0;
    }
    if (bad) atomicOr(g.err, 1u);
    // ---- the paths where ours and theirs differ (one side only, or different OIDs): compacted into
    //      LDS in path order, then resolved one per thread — a few per tile, so the per-item arrays
    //      of the join do not carry ancestor state ----
    u32 dif = 0, clean = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u32 kind = rec[k] >> 25, chg = (rec[k] >> 24) & 1;
        dif |= (u32)(kind == R_DEL || kind == R_INS || (kind == R_MATCH && chg)) << k;
        clean += kind == R_MATCH && !chg;  // ours == theirs: clean, nothing to record
    }
    static_assert(!HASH || NMCH * 16 >= 4 * LD::TILE, "the differing paths fit the name buffer");
    u32* const s_drec = HASH ? (u32*)s_nm : s_drec_own;
    u32 od = 0, wd = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u64 bd = __ballot((dif >> k) & 1);
        od += __builtin_amdgcn_mbcnt_hi((u32)(bd >> 32), __builtin_amdgcn_mbcnt_lo((u32)bd, 0));
        wd += __popcll(bd);
    }
    if (lane == 0) s_wave[wid] = wd;
    __syncthreads();
    u32 ndif = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const u32 x = s_wave[w];
        if (w < wid) od += x;
        ndif += x;
    }
#pragma unroll
    for (int k = 0; k < IPT; k++)
        if ((dif >> k) & 1) s_drec[od++] = rec[k];
    __syncthreads();  // (s_wave reused below)
    const u64 nk = k1e - k0;
    const int rounds = nk ? 64 - __clzll((long long)nk) : 0;  // wave-uniform
    u32 tc = 0, tm = 0;  // running conflict / merge-delta counts of the tile
    u32* sc = g3.stage_conf + tile * (u64)C2_STAGE * 3;
    uint2* sm = g3.stage_md + tile * (u64)C2_STAGE;
    for (u32 c0 = 0; c0 < ndif; c0 += NT) {  // block-uniform
        const u32 x = c0 + tid;
        const bool act = x < ndif;
        const u32 r0 = act ? s_drec[x] : 0u;
        const u32 kind = r0 >> 25, ia = r0 & 0xFFF, jb = (r0 >> 12) & 0xFFF;
        const u64 key = kind == R_INS ? sB[jb] : sA[ia];
        // the ancestor entry: lower bound in the tile's range (LDS, or HBM for a long range)
        u64 lo = 0, hi = act ? nk : 0;
        for (int it = 0; it < rounds; it++) {
            const u64 m = (lo + hi) >> 1;
            const u64 mi = m < nk ? m : (nk ? nk - 1 : 0);
            const u64 v = lk ? sK[mi] : g3.K[k0 + mi];
            const bool on = lo < hi, lt = v < key;
            lo = on && lt ? m + 1 : lo;
            hi = on && !lt ? m : hi;
        }
        const bool found = act && lo < nk && (lk ? sK[lo] : g3.K[k0 + lo]) == key;
        const u32 ik = found ? (u32)(k0 + lo) : KD_NONE;
        const u32 io = act && kind != R_INS ? (u32)(q.i0 + ia) : KD_NONE;
        const u32 itt = act && kind != R_DEL ? (u32)(q.j0 + jb) : KD_NONE;
        bool md = false, cf = false;
        if constexpr (SPLIT) {
            cf = act;  // a candidate, resolved by k_resolve3
        } else {
        u32 rk3 = ik, ro = io, rt = itt;  // rows in the OID / filename arrays (PERM: through the orders)
        if (PERM) {
            rk3 = ik != KD_NONE ? *(gp32)(g3.ordK + ik) : KD_NONE;
            ro = io != KD_NONE ? *(gp32)(g.ordA + io) : KD_NONE;
            rt = itt != KD_NONE ? *(gp32)(g.ordB + itt) : KD_NONE;
        }
        const gp32 pk = rk3 != KD_NONE ? (gp32)(g3.oidK + 20ull * rk3) : (gp32)g.dummy;
        const gp32 po = ro != KD_NONE ? (gp32)(g.oidA + 20ull * ro) : (gp32)g.dummy;
        const gp32 pt = rt != KD_NONE ? (gp32)(g.oidB + 20ull * rt) : (gp32)g.dummy;
        u32 dko = 0, dkt = 0;
#pragma unroll
        for (int w = 0; w < 5; w++) {
            const u32 xk = pk[w];
            dko |= xk ^ po[w];
            dkt |= xk ^ pt[w];
        }
        if (HASH) {  // a matched ancestor path must carry the same filename (ours', else theirs')
            const u32 act_o = ik != KD_NONE && io != KD_NONE;
            const u32 act_t = ik != KD_NONE && itt != KD_NONE && io == KD_NONE;
            const u32 rr[1] = {rk3}, oo[1] = {ro}, tt[1] = {rt};
            if (__syncthreads_or((int)(act_o | act_t)))
                ne |= (names_ne_batch<1, 8>(g3.nameK, g3.nameOffK, rr, g.nameA, g.nameOffA, oo, act_o) |
                       names_ne_batch<1, 8>(g3.nameK, g3.nameOffK, rr, g.nameB, g.nameOffB, tt, act_t)) != 0;
        }
        // libgit2's rule where ours != theirs: a == o -> theirs (merge delta), a == t -> ours, else conflict
        const bool pa = ik != KD_NONE, pO = io != KD_NONE, pT = itt != KD_NONE;
        const bool a_eq_o = pa == pO && (!pa || dko == 0);
        const bool a_eq_t = pa == pT && (!pa || dkt == 0);
        md = act && a_eq_o;
        cf = act && !a_eq_o && !a_eq_t;
        clean += (act && !a_eq_o && a_eq_t && pO) || (md && pT);
        }
        u32 tot;
        const u32 off = block_excl_scan<NT>((u32)cf | (u32)md << 16, s_wave, &tot);
        if (cf) {
            u32* o = sc + 3 * (tc + (off & 0xFFFF));
            o[0] = ik; o[1] = io; o[2] = itt;
        }
        if (md) sm[tm + (off >> 16)] = make_uint2(io, itt);
        tc += tot & 0xFFFF;
        tm += tot >> 16;
    }
    if (ne) atomicOr(g.err, 2u);
    const u32 tcl = block_sum<NT>(clean, s_wave);
    if (tid == 0) {
        u32* cc = g.tile_cnt + 4 * tile;
        cc[0] = tcl; cc[1] = tm; cc[2] = 0; cc[3] = tc;
        u64* gs = g.gsum + 2 * (tile / C2_GROUP);
        atomicAdd((unsigned long long*)gs, (unsigned long long)(tc | (u64)tm << 32));
        atomicAdd((unsigned long long*)gs + 1, (unsigned long long)tcl);
    }
}

// staged conflicts / merge deltas -> final path-ordered positions; one wave per tile
__global__ __launch_bounds__(64) void k_place3(const u32* __restrict__ stage_conf, const uint2* __restrict__ stage_md,
                                               const u32* __restrict__ tile_cnt, const u64* __restrict__ gpre,
                                               u32* __restrict__ out_conf, uint2* __restrict__ out_md) {
    const int tid = threadIdx.x;
    const u64 t = blockIdx.x, grp = t / C2_GROUP, t_lo = grp * C2_GROUP;
    u64 pc = 0, pm = 0;
    if (tid < (int)(t - t_lo)) {
        const uint4 c = *(const uint4*)(tile_cnt + 4 * (t_lo + tid));
        pc = c.w;
        pm = c.y;
    }
    const uint4 own = *(const uint4*)(tile_cnt + 4 * t);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { pc += __shfl_xor(pc, o, 64); pm += __shfl_xor(pm, o, 64); }
    pc += gpre[2 * grp];
    pm += gpre[2 * grp + 1];
    const u32* scp = stage_conf + t * (u64)C2_STAGE * 3;
    const uint2* smp = stage_md + t * (u64)C2_STAGE;
    for (u32 x = tid; x < 3 * own.w; x += 64) out_conf[3 * pc + x] = scp[x];
    for (u32 x = tid; x < own.y; x += 64) out_md[pm + x] = smp[x];
}

// ---------------------------------------------------------------------------------------------
// k_join3b: the three-way join with every tile-sized range staged in one LDS-DMA round trip
// ---------------------------------------------------------------------------------------------
// k_join3 chains six to eight dependent memory round trips per tile (split points, then keys and
// name bounds, then names, walk rows, OIDs and name offsets, then the differing paths' ancestor
// rows, OIDs and names), and its 22-KB name buffer overflows on SURVEY's C4 names (12-24-character
// text pks: ~36-B paths), sending every filename compare to HBM.  k_join3b cuts the chain to five:
//   1. the tile's two split records (k_apart3b: merge-path split, ancestor lower bound and the name
//      arena offsets around the split, so no round trip waits on a split point to find its names);
//   2. ONE LDS-DMA batch: ours' / theirs' / the ancestor's keys, (PERM) the three walk-row ranges
//      of the tile's sorted entries, and ours' / theirs' filename bytes of the tile's rows (PERM: the
//      rows widened by a halo of J3B_HALO on each side — a per-leaf-tree sort moves an entry less than
//      its leaf tree's length; a row outside them is compared in HBM);
//   3. the matched pairs' OIDs and name offsets (rows from LDS), then OIDs and names compared;
//   4. per differing path (one per thread, after compaction; ancestor found by binary search in
//      LDS, its row from LDS): the three OIDs and the ancestor's / the path's name offsets;
//   5. the ancestor's filename (HBM window) against the path's name (LDS).
// Results are k_join3's (same staging, same k_place3).
// Where the time goes (C4, 50M rows, r5 timing probes KD_J3B_STOP / KD_J3B_PROBE_NONAMES, 2.67 ms
// in all): split records + the DMA batch 0.97 ms (~6.5 TB/s of staged bytes), + merge path and
// matched pairs 0.53 ms (0.2 of it the filename compare), + the differing paths 1.2 ms.  SQ counters
// put VALU at ~60 % of each SIMD's cycles with 4 waves per SIMD (LDS 35 KB and ~105 VGPRs per
// 256-thread block both allow 4), so cutting round trips alone does not pay: staging the ancestor's
// name offsets so its filename loads with the OIDs (one round trip less) measured 2.67 -> 2.70 ms,
// a resident grid prefetching the next tile's split records 2.83 -> 3.21, and the split form (join
// stages candidates, k_resolve3 resolves) 2.12 + 1.83 ms.  What paid: waves holding no differing
// path skip the resolve (most: ~30 per tile), a 32-bit ancestor search, and a cheaper compare.
#ifndef KD_J3B_IPT
#define KD_J3B_IPT 2
#endif
constexpr int J3B_IPT = KD_J3B_IPT;
// 192 threads x 2 items: 384-item tiles whose LDS (26.4 KB: C4's ~36-B names of a tile + halo in
// 16 KB) lets 6 blocks share a CU — 2.34 vs 2.56 ms for 256 x 2 (4 blocks per CU) on C4 (r5o;
// 128 x 4 / 192 x 3 / 128 x 3: 2.87 / 2.57 / 2.81; 192 x 2 with a 16-row halo, 27.2 KB, 5 blocks: 2.61)
#ifndef KD_J3B_NT
#define KD_J3B_NT 192
#endif
constexpr int J3B_NT = KD_J3B_NT;
constexpr int J3B_TILE = J3B_NT * J3B_IPT;
#ifndef KD_J3B_ACAP
#define KD_J3B_ACAP (J3B_TILE / 2 + 128)  // ancestor keys staged (a tile's range is ~half its items)
#endif
constexpr int J3B_ACAP = KD_J3B_ACAP;
#ifndef KD_J3B_NAME_CH
#define KD_J3B_NAME_CH (J3B_TILE == 384 ? 1000 : J3B_TILE * 11 / 4)  // 16 KB at 384 items (6 blocks per CU)
#endif
#ifndef KD_J3B_HALO
#define KD_J3B_HALO 8  // (a 16-row halo measured the same at 512-item tiles; C4's leaf trees hold ~3)
#endif
constexpr u64 J3B_HALO = KD_J3B_HALO;
#ifndef KD_J3B_PERSIST
#define KD_J3B_PERSIST 0  // 1: a resident grid walking the tiles, the next split records prefetched (slower)
#endif
constexpr bool J3B_PERSIST = KD_J3B_PERSIST;
#ifndef KD_J3B_STOP
#define KD_J3B_STOP 0
#endif
#ifndef KD_J3B_PROBE_NONAMES
#define KD_J3B_PROBE_NONAMES 0
#endif

// apart[t] and (nsplit) the name-arena offsets around split t: ours rows i_t -/+ halo, theirs rows
// j_t - halo and j_t + 1 + halo (clamped), j_t = min(t * tile, nO + nT) - i_t
__global__ __launch_bounds__(256) void k_apart3b(const u64* __restrict__ O, u64 nO, const u64* __restrict__ T, u64 nT,
                                                 const u64* __restrict__ part, u64 ntiles, int tile_items,
                                                 const u64* __restrict__ K, u64 nK, u64* __restrict__ apart,
                                                 const u64* __restrict__ offO, const u64* __restrict__ offT, u64 halo,
                                                 u64* __restrict__ nsplit) {
    const u64 t = ((u64)blockIdx.x * 256 + threadIdx.x) / 8;
    if (t > ntiles) return;  // (whole 8-lane groups)
    const int sub = threadIdx.x & 7;
    const u64 i = part[t];
    const u64 d = min(t * (u64)tile_items, nO + nT), j = d - i;
    if (nsplit && sub < 4) {
        u64 v;
        if (sub == 0) v = offO[i > halo ? i - halo : 0];
        else if (sub == 1) v = offO[min(i + halo, nO)];
        else if (sub == 2) v = offT[j > halo ? j - halo : 0];
        else v = offT[min(j + 1 + halo, nT)];
        nsplit[4 * t + sub] = v;
    }
    u64 r;
    if (t == 0) r = 0;
    else if (t == ntiles) r = nK;
    else {
        const u64 a = i < nO ? O[i] : ~0ull, b = j < nT ? T[j] : ~0ull;
        const u64 key = a < b ? a : b;
        const u64 guess = nO ? (u64)((double)i / (double)nO * (double)nK) : (u64)((double)d / (double)(nO + nT) * (double)nK);
        r = lb_guided<8>(K, nK, key, guess < nK ? guess : nK, 256);
    }
    if (sub == 0) apart[t] = r;
}

// a filename in HBM (bytes [a0, a0 + len)) against one in LDS (byte address lb)
__device__ __forceinline__ bool glb_lds_name_eq(const u8* __restrict__ na, u64 a0, u32 len, u32 lb) {
    typedef const __attribute__((address_space(3))) u32* l32;
    const u32 sa = (u32)(a0 & 3), sb = lb & 3;
    const u32* wa = (const u32*)(na + (a0 - sa));
    const u32 nwa = (sa + len + 3) >> 2;
    const u32 wb = lb - sb;
    if (nwa <= 16) {  // one window of 16 dwords, all loads issued together
        u32 x[17], y[17];
#pragma unroll
        for (int w = 0; w < 16; w++) x[w] = (u32)w < nwa ? wa[w] : 0u;
        x[16] = 0;
#pragma unroll
        for (int w = 0; w < 17; w++) y[w] = *(l32)(size_t)(wb + 4 * w);
        u32 diff = 0;
#pragma unroll
        for (int w = 0; w < 16; w++) {
            const u32 rem = len > 4u * w ? len - 4u * w : 0u;
            const u32 m = rem >= 4 ? 0xFFFFFFFFu : ((1u << (8 * rem)) - 1u);
            diff |= (__builtin_amdgcn_alignbyte(x[w + 1], x[w], sa) ^ __builtin_amdgcn_alignbyte(y[w + 1], y[w], sb)) & m;
        }
        return diff == 0;
    }
    typedef const __attribute__((address_space(3))) u8* l8;
    for (u32 k = 0; k < len; k++)
        if (na[a0 + k] != *(l8)(size_t)(lb + k)) return false;
    return true;
}

// SPLIT: the differing paths are staged as candidates (a, o, t) with the ancestor entry found in LDS
// (no OID or filename load in the tile) and k_resolve3<HAVE_A> applies the rule over the placed list
template <int NT, int IPT, bool HASH, bool PERM, bool SPLIT = false>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_join3b(Join3Args g3) {
    const Join2Args& g = g3.j;
    using LD = Join2Lds<NT, IPT>;
    constexpr int TILE = LD::TILE;
    static_assert(TILE <= 4095, "per-item records hold 12-bit local indices");
    constexpr int KCH = (8 * (J3B_ACAP + 2) + 16 + 15) / 16 + 4;
    // walk rows: ours [i0, i1) + theirs [j0, j1e) (<= TILE + 1 entries) and the ancestor's [k0, k1e)
    constexpr int ORDCH = PERM ? (4 * (TILE + 1) + 15) / 16 + 4 + (4 * (J3B_ACAP + 1) + 15) / 16 + 2 : 1;
    constexpr int NMCH = HASH ? KD_J3B_NAME_CH : 1;
    __shared__ u32x4 s_ch[LD::CHK];
    __shared__ u32x4 s_k[KCH];
    __shared__ u32x4 s_ord[ORDCH];
    __shared__ u32x4 s_nm[NMCH];
    __shared__ u32 s_drec[TILE];
    __shared__ u32 s_wave[3 * NT / 64];
    typedef const __attribute__((address_space(1))) u32* gp32;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const u64 ntiles = g.ntiles;
    u64 tile = blockIdx.x;
    if (tile >= ntiles) return;  // block-uniform
    // ---- 1. split records of both tile ends (later tiles': prefetched with the previous tile's DMA) ----
    u64 p0 = g.part[tile], p1 = g.part[tile + 1];
    u64 a0 = g3.apart[tile], a1 = g3.apart[tile + 1];
    u64 nmA0 = 0, nmA1 = 0, nmB0 = 0, nmB1 = 0;
    if (HASH) {
        nmA0 = g3.nsplit[4 * tile]; nmB0 = g3.nsplit[4 * tile + 2];
        nmA1 = g3.nsplit[4 * tile + 5]; nmB1 = g3.nsplit[4 * tile + 7];
    }
    u32 err = 0;
    for (;;) {  // persistent: tiles blockIdx.x, + gridDim.x, ...
    const u64 tnext = tile + gridDim.x;
    const bool more = J3B_PERSIST && tnext < ntiles;  // block-uniform
    const TileGeo q = tile_geo_from(g, tile, TILE, p0, p1);
    bool bad = !q.ok;
    const TileRanges r = tile_ranges(g, q);
    const u64 k0 = uni64(a0), kend = uni64(a1);
    const bool kok = kend >= k0 && kend <= g3.nK;
    bad |= !kok;
    const u64 k1 = kok ? kend : k0;
    const u64 k1e = k1 < g3.nK ? k1 + 1 : k1;
    const bool has_lbK = k0 > 0;
    const bool lk = k1e - k0 <= (u64)J3B_ACAP;
    // the staged name rows (PERM: the sorted ranges widened by the halo)
    const u64 H = PERM ? J3B_HALO : 0;
    const u64 rA0 = q.i0 > H ? q.i0 - H : 0, rA1 = min(q.i1 + H, g.nA);
    const u64 rB0 = q.j0 > H ? q.j0 - H : 0, rB1 = min(q.j1 + 1 + H, g.nB);
    // ---- 2. one DMA batch ----
    u32 qq = dma_range<NT>(r.ka, s_ch, 0);
    qq = dma_range<NT>(r.kb, s_ch + r.c1, qq);
    Range rk{};
    if (lk) {
        rk = mk_range(g3.K, 8 * (k0 - has_lbK), 8 * k1e);
        qq = dma_range<NT>(rk, s_k, qq);
    }
    Range roO{}, roT{}, roK{};
    if (PERM) {
        roO = mk_range(g.ordA, 4 * q.i0, 4 * q.i1);
        roT = mk_range(g.ordB, 4 * q.j0, 4 * q.j1e);
        qq = dma_range<NT>(roO, s_ord, qq);
        qq = dma_range<NT>(roT, s_ord + roO.nch, qq);
        if (lk) {
            roK = mk_range(g3.ordK, 4 * k0, 4 * k1e);
            qq = dma_range<NT>(roK, s_ord + roO.nch + roT.nch, qq);
        }
    }
    Range rnA{}, rnB{};
    bool lnames = false;
    if (HASH) {
        nmA0 = uni64(nmA0); nmA1 = uni64(nmA1); nmB0 = uni64(nmB0); nmB1 = uni64(nmB1);
        rnA = mk_range(g.nameA, nmA0, nmA1);
        rnB = mk_range(g.nameB, nmB0, nmB1);
        lnames = q.ok && nmA1 >= nmA0 && nmB1 >= nmB0 && (u64)rnA.nch + rnB.nch <= (u64)NMCH;
        if (lnames) {
            qq = dma_range<NT>(rnA, s_nm, qq);
            qq = dma_range<NT>(rnB, s_nm + rnA.nch, qq);
        }
    }
    // the next tile's split records, in flight with the batch (the name bounds in their own
    // registers: this tile's are read until its end)
    u64 xA0 = 0, xA1 = 0, xB0 = 0, xB1 = 0;
    if (more) {
        p0 = g.part[tnext]; p1 = g.part[tnext + 1];
        a0 = g3.apart[tnext]; a1 = g3.apart[tnext + 1];
        if (HASH) {
            xA0 = g3.nsplit[4 * tnext]; xB0 = g3.nsplit[4 * tnext + 2];
            xA1 = g3.nsplit[4 * tnext + 5]; xB1 = g3.nsplit[4 * tnext + 7];
        }
    }
    __syncthreads();  // vmcnt(0) + barrier: everything staged has landed
#if KD_J3B_STOP == 1  // timing probe only (results invalid): split records + the DMA batch
    if (tid == 0) { u32* cc = g.tile_cnt + 4 * tile; cc[0] = cc[1] = cc[2] = cc[3] = 0; }
    if (!more) break;
    tile = tnext; nmA0 = xA0; nmA1 = xA1; nmB0 = xB0; nmB1 = xB1;
    __syncthreads();
    continue;
#endif
    const u64* sA = (const u64*)((const u8*)s_ch + r.ka.skew) + q.has_lbA;
    const u64* sB = (const u64*)((const u8*)(s_ch + r.c1) + r.kb.skew) + q.has_lbB;
    const u64* sK = (const u64*)((const u8*)s_k + rk.skew) + has_lbK;
    const u32* sOrdO = (const u32*)((const u8*)s_ord + roO.skew);
    const u32* sOrdT = (const u32*)((const u8*)(s_ord + roO.nch) + roT.skew);
    const u32* sOrdK = (const u32*)((const u8*)(s_ord + roO.nch + roT.nch) + roK.skew);
    u32 rec[IPT];
    tile_walk<NT, IPT>(sA, sB, q, rec, bad);
    for (int x = tid; x < q.na; x += NT) bad |= (x > 0 || q.has_lbA) && sA[x - 1] >= sA[x];
    for (int x = tid; x < q.nb; x += NT) bad |= (x > 0 || q.has_lbB) && sB[x - 1] >= sB[x];
    if (lk) {
        for (int x = tid; x < (int)(k1 - k0); x += NT) bad |= (x > 0 || has_lbK) && sK[x - 1] >= sK[x];
    } else {
        for (u64 x = k0 + tid; x < k1; x += NT) bad |= x > 0 && g3.K[x - 1] >= g3.K[x];
    }
#if KD_J3B_STOP == 3  // timing probe only (results invalid): + the merge-path walk and order checks
    if (bad) err |= 1u;
    if ((rec[0] ^ rec[IPT - 1]) == 0x7FFFFFFFu) err |= 8u;
    __syncthreads();
    if (tid == 0) { u32* cc = g.tile_cnt + 4 * tile; cc[0] = cc[1] = cc[2] = cc[3] = 0; }
    if (!more) break;
    tile = tnext; nmA0 = xA0; nmA1 = xA1; nmB0 = xB0; nmB1 = xB1;
    continue;
#endif
    // ---- 3. matched pairs: rows from LDS, then OIDs and name offsets ----
    u32 ra[IPT], rb[IPT];
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const bool m = (rec[k] >> 25) == R_MATCH;
        const u32 ia = rec[k] & 0xFFF, jb = (rec[k] >> 12) & 0xFFF;
        ra[k] = PERM ? (m ? sOrdO[ia] : 0u) : (u32)q.i0 + ia;
        rb[k] = PERM ? (m ? sOrdT[jb] : 0u) : (u32)q.j0 + jb;
    }
    u32 oa0[IPT], oa1[IPT], ob0[IPT], ob1[IPT];
    if (HASH && lnames) {
        const u32* offA = (const u32*)g.nameOffA;
        const u32* offB = (const u32*)g.nameOffB;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            const bool m = (rec[k] >> 25) == R_MATCH;
            // unmatched items load nothing (a placeholder row could be the side's end: off[n + 1]
            // lies past the caller's n + 1 offsets)
            const u64 i = m ? ra[k] : 0, j = m ? rb[k] : 0;
            oa0[k] = m ? offA[2 * i] : 0u; oa1[k] = m ? offA[2 * i + 2] : 0u;
            ob0[k] = m ? offB[2 * j] : 0u; ob1[k] = m ? offB[2 * j + 2] : 0u;
        }
    }
    tile_oid_cmp<IPT>(g, rec, ra, rb);
    bool ne = false;
    if (HASH && lnames) {
        const u32 nm = (u32)(size_t)(const __attribute__((address_space(3))) u32x4*)s_nm;
        const u32 baseA = nm + rnA.skew, baseB = nm + 16 * rnA.nch + rnB.skew;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            if ((rec[k] >> 25) != R_MATCH) continue;
            const u32 la = oa1[k] - oa0[k], lb = ob1[k] - ob0[k];
            if (PERM && (ra[k] < rA0 || ra[k] >= rA1 || rb[k] < rB0 || rb[k] >= rB1))
                ne |= !names_eq(g.nameA, g.nameOffA, ra[k], g.nameB, g.nameOffB, rb[k]);
            else
#if KD_J3B_PROBE_NONAMES  // timing probe only (results invalid): the LDS name compare skipped
                ne |= la != lb || (baseA + oa0[k] == 7u && baseB + ob0[k] == 5u);
#else
                ne |= la != lb || !lds_eq_bytes(baseA + (oa0[k] - (u32)nmA0), baseB + (ob0[k] - (u32)nmB0), la);
#endif
        }
    } else if (HASH) {
        u32 act = 0;
#pragma unroll
        for (int k = 0; k < IPT; k++) act |= (u32)((rec[k] >> 25) == R_MATCH) << k;
        ne |= names_ne_batch<IPT, 8>(g.nameA, g.nameOffA, ra, g.nameB, g.nameOffB, rb, act) != 0;
    }
    if (bad) err |= 1u;
#if KD_J3B_STOP == 2  // timing probe only (results invalid): + the merge path and the matched pairs
    if (ne) err |= 2u;
    __syncthreads();
    if (tid == 0) { u32* cc = g.tile_cnt + 4 * tile; cc[0] = cc[1] = cc[2] = cc[3] = 0; }
    if (!more) break;
    tile = tnext; nmA0 = xA0; nmA1 = xA1; nmB0 = xB0; nmB1 = xB1;
    continue;
#endif
    // ---- the paths where ours and theirs differ, compacted in path order ----
    u32 dif = 0, clean = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u32 kind = rec[k] >> 25, chg = (rec[k] >> 24) & 1;
        dif |= (u32)(kind == R_DEL || kind == R_INS || (kind == R_MATCH && chg)) << k;
        clean += kind == R_MATCH && !chg;
    }
    u32 od = 0, wd = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const u64 bd = __ballot((dif >> k) & 1);
        od += __builtin_amdgcn_mbcnt_hi((u32)(bd >> 32), __builtin_amdgcn_mbcnt_lo((u32)bd, 0));
        wd += __popcll(bd);
    }
    if (lane == 0) s_wave[wid] = wd;
    __syncthreads();
    u32 ndif = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const u32 x = s_wave[w];
        if (w < wid) od += x;
        ndif += x;
    }
#pragma unroll
    for (int k = 0; k < IPT; k++)
        if ((dif >> k) & 1) s_drec[od++] = rec[k];
    __syncthreads();  // (s_wave reused below)
    const u64 nk = k1e - k0;
    // 4-ary lower bound: ceil(log4(nk + 1)) rounds of three independent LDS reads (wave-uniform)
    // (a round leaves at most max(q - 1, w - 3q) of w, q = ceil(w / 4): 5 rounds for 384 keys)
    int rounds = 0;
    for (u64 w = nk; w > 0; rounds++) {
        const u64 q = (w + 3) / 4;
        const u64 r = w > 3 * q ? w - 3 * q : 0;
        w = q - 1 > r ? q - 1 : r;
    }
    u32 tc = 0, tm = 0;
    u32* sc = g3.stage_conf + tile * (u64)C2_STAGE * 3;
    uint2* sm = g3.stage_md + tile * (u64)C2_STAGE;
    const u32 nmb = (u32)(size_t)(const __attribute__((address_space(3))) u32x4*)s_nm;
    for (u32 c0 = 0; c0 < ndif; c0 += NT) {  // block-uniform
        const u32 x = c0 + tid;
        const bool act = x < ndif;
        u32 ik = KD_NONE, io = KD_NONE, itt = KD_NONE;
        bool md = false, cf = false;
        // the join is VALU-bound (r5 SQ counters): waves holding no differing path (most of them —
        // C4 has ~30 per 512-item tile) skip straight to the scan
        if (c0 + 64u * (u32)wid < ndif) {  // wave-uniform
        const u32 r0 = act ? s_drec[x] : 0u;
        const u32 kind = r0 >> 25, ia = r0 & 0xFFF, jb = (r0 >> 12) & 0xFFF;
        const u64 key = kind == R_INS ? sB[jb] : sA[ia];
        const u32 nk32 = (u32)nk;
        // invariant: every index < lo holds a smaller key, every index >= hi a key >= key
        u32 lo = 0, hi = act ? nk32 : 0;
        const u32 last = nk32 ? nk32 - 1 : 0;
        for (int it = 0; it < rounds; it++) {
            const u32 st = (hi - lo + 3) >> 2;
            const u32 p1 = lo + st - 1, p2 = p1 + st, p3 = p2 + st;
            const u32 q1 = p1 < last ? p1 : last, q2 = p2 < last ? p2 : last, q3 = p3 < last ? p3 : last;
            const u64 v1 = lk ? sK[q1] : g3.K[k0 + q1], v2 = lk ? sK[q2] : g3.K[k0 + q2], v3 = lk ? sK[q3] : g3.K[k0 + q3];
            const bool on = lo < hi;
            const bool l1 = on && p1 < hi && v1 < key, l2 = on && p2 < hi && v2 < key, l3 = on && p3 < hi && v3 < key;
            const u32 nlo = l3 ? p3 + 1 : l2 ? p2 + 1 : l1 ? p1 + 1 : lo;
            const u32 nhi = !on ? hi : !l1 ? (p1 < hi ? p1 : hi) : !l2 ? (p2 < hi ? p2 : hi) : !l3 ? (p3 < hi ? p3 : hi) : hi;
            lo = nlo;
            hi = nhi;
        }
        const bool found = act && lo < nk32 && (lk ? sK[lo] : g3.K[k0 + lo]) == key;
        ik = found ? (u32)(k0 + lo) : KD_NONE;
        io = act && kind != R_INS ? (u32)(q.i0 + ia) : KD_NONE;
        itt = act && kind != R_DEL ? (u32)(q.j0 + jb) : KD_NONE;
        if constexpr (SPLIT) {
            cf = act;  // a candidate, resolved by k_resolve3
        } else {
        // ---- 4. rows (LDS), then the three OIDs and the name offsets ----
        u32 rk3 = ik, ro = io, rt = itt;
        if (PERM) {
            rk3 = ik != KD_NONE ? (lk ? sOrdK[lo] : *(gp32)(g3.ordK + ik)) : KD_NONE;
            ro = io != KD_NONE ? sOrdO[ia] : KD_NONE;
            rt = itt != KD_NONE ? sOrdT[jb] : KD_NONE;
        }
        const gp32 pk = rk3 != KD_NONE ? (gp32)(g3.oidK + 20ull * rk3) : (gp32)g.dummy;
        const gp32 po = ro != KD_NONE ? (gp32)(g.oidA + 20ull * ro) : (gp32)g.dummy;
        const gp32 pt = rt != KD_NONE ? (gp32)(g.oidB + 20ull * rt) : (gp32)g.dummy;
        // (HASH) a matched ancestor path must carry the same filename as ours' (else theirs')
        const bool chk = HASH && ik != KD_NONE && (io != KD_NONE || itt != KD_NONE);
        const bool side_o = io != KD_NONE;
        const u32 srow = side_o ? ro : rt;
        u64 kn0 = 0, kn1 = 0, sn0 = 0, sn1 = 0;
        if (HASH) {
            const u64* offS = side_o ? g.nameOffA : g.nameOffB;
            kn0 = g3.nameOffK[chk ? rk3 : 0]; kn1 = g3.nameOffK[chk ? rk3 + 1 : 0];
            sn0 = offS[chk ? srow : 0]; sn1 = offS[chk ? srow + 1 : 0];
        }
        u32 dko = 0, dkt = 0;
#pragma unroll
        for (int w = 0; w < 5; w++) {
            const u32 xk = pk[w];
            dko |= xk ^ po[w];
            dkt |= xk ^ pt[w];
        }
        // ---- 5. the ancestor's name against the path's (LDS, else HBM) ----
        if (HASH && chk) {
            const u32 len = (u32)(kn1 - kn0);
            if (len != (u32)(sn1 - sn0)) {
                ne = true;
            } else {
                const bool in_lds = lnames && (side_o ? (srow >= rA0 && srow < rA1) : (srow >= rB0 && srow < rB1));
                if (in_lds) {
                    const u32 sb = side_o ? nmb + rnA.skew + (u32)(sn0 - nmA0) : nmb + 16 * rnA.nch + rnB.skew + (u32)(sn0 - nmB0);
                    ne |= !glb_lds_name_eq(g3.nameK, kn0, len, sb);
                } else {
                    ne |= !names_eq(g3.nameK, g3.nameOffK, rk3, side_o ? g.nameA : g.nameB, side_o ? g.nameOffA : g.nameOffB,
                                    srow);
                }
            }
        }
        const bool pa = ik != KD_NONE, pO = io != KD_NONE, pT = itt != KD_NONE;
        const bool a_eq_o = pa == pO && (!pa || dko == 0);
        const bool a_eq_t = pa == pT && (!pa || dkt == 0);
        md = act && a_eq_o;
        cf = act && !a_eq_o && !a_eq_t;
        clean += (act && !a_eq_o && a_eq_t && pO) || (md && pT);
        }  // (!SPLIT)
        }  // (a wave with differing paths)
        // path-order places of the conflicts and merge deltas: ballots within the wave, the waves'
        // counts through LDS (one barrier pair; a shuffle scan chains six LDS-latency steps)
        const u64 bc = __ballot(cf), bm = __ballot(md);
        if (lane == 0) { s_wave[wid] = (u32)__popcll(bc); s_wave[NT / 64 + wid] = (u32)__popcll(bm); }
        __syncthreads();
        u32 pc = 0, pm = 0, nc = 0, nm = 0;
#pragma unroll
        for (int w = 0; w < NT / 64; w++) {
            const u32 xc = s_wave[w], xm = s_wave[NT / 64 + w];
            if (w < wid) { pc += xc; pm += xm; }
            nc += xc;
            nm += xm;
        }
        __syncthreads();  // (s_wave reused)
        if (cf) {
            u32* o = sc + 3 * (tc + pc + __builtin_amdgcn_mbcnt_hi((u32)(bc >> 32), __builtin_amdgcn_mbcnt_lo((u32)bc, 0)));
            o[0] = ik; o[1] = io; o[2] = itt;
        }
        if (md) sm[tm + pm + __builtin_amdgcn_mbcnt_hi((u32)(bm >> 32), __builtin_amdgcn_mbcnt_lo((u32)bm, 0))] = make_uint2(io, itt);
        tc += nc;
        tm += nm;
    }
    if (ne) err |= 2u;
    // the tile's clean count: per wave by bit-sliced ballots, summed by thread 0.  A thread counts at
    // most its IPT items plus one per compaction pass (at most ceil(ndif / NT) <= IPT passes), so
    // clean <= 2 IPT < 16: four slices
    static_assert(2 * IPT < 16, "k_join3b: the clean count's ballot slices");
    {
        const u32 wcl = (u32)__popcll(__ballot(clean & 1)) + 2u * (u32)__popcll(__ballot((clean >> 1) & 1)) +
                        4u * (u32)__popcll(__ballot((clean >> 2) & 1)) + 8u * (u32)__popcll(__ballot((clean >> 3) & 1));
        if (lane == 0) s_wave[2 * (NT / 64) + wid] = wcl;
    }
    __syncthreads();  // (also: every LDS read of this tile is done before the next tile's DMA)
    u32 tcl = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) tcl += s_wave[2 * (NT / 64) + w];
    if (tid == 0) {
        u32* cc = g.tile_cnt + 4 * tile;
        cc[0] = tcl; cc[1] = tm; cc[2] = 0; cc[3] = tc;
        u64* gs = g.gsum + 2 * (tile / C2_GROUP);
        atomicAdd((unsigned long long*)gs, (unsigned long long)(tc | (u64)tm << 32));
        atomicAdd((unsigned long long*)gs + 1, (unsigned long long)tcl);
    }
    if (!more) break;
    tile = tnext;
    nmA0 = xA0; nmA1 = xA1; nmB0 = xB0; nmB1 = xB1;
    }
    if (err) atomicOr(g.err, err);
}

// the three-way merge through k_join3 (sides device-resident; ord* non-null: late materialisation)
int merge3_join_device(kd_ctx* ctx, const kd_side& K, const kd_side& O, const kd_side& T, u32* d_conf, uint2* d_md,
                       u64* d_counts, u32* d_err, const u32* ordK, const u32* ordO, const u32* ordT) {
    const u64 nK = K.n, nO = O.n, nT = T.n, total = nO + nT;
    const bool hash = K.key_mode == KD_KEY_HASH;
    const bool perm = ordK || ordO || ordT;
    // merge3_split: the join stages candidates (a, o, t) and k_resolve3 applies the rule (C4, r4n:
    // 4.02 vs 3.78 ms from walk order, 2.37 vs 2.16 presorted — the default resolves in the join)
    const bool split = ctx->opt.merge3_split == 1;
    const bool j3_ol = ctx->opt.j3_ol == 1;  // (sorted-form sides' OIDs staged with the keys)
    const bool v2 = ctx->opt.j3_v != 0 && !(j3_ol && !perm);  // k_join3b
    const int TILE = v2 ? J3B_TILE : J3_TILE;
    if (hash) KD_CHECK((nK == 0 || (K.name && K.name_off)) && (nO == 0 || (O.name && O.name_off)) &&
                       (nT == 0 || (T.name && T.name_off)), "merge3: KD_KEY_HASH needs filenames");
    const u64 ntiles = (total + TILE - 1) / TILE;
    const u64 n_zero = 2 * ((ntiles + C2_GROUP - 1) / C2_GROUP);
    void *part, *apart, *tcnt, *gsum, *gpre, *sconf, *smd, *dz;
    int rc;
    if ((rc = ensure(ctx, "c2.part", (ntiles + 1) * sizeof(u64), &part))) return rc;
    if ((rc = ensure(ctx, "c3.apart", (ntiles + 1) * sizeof(u64), &apart))) return rc;
    if ((rc = ensure(ctx, "c2.tcnt", ntiles * 4 * sizeof(u32), &tcnt))) return rc;
    if ((rc = ensure(ctx, "c2.gsum", n_zero * sizeof(u64), &gsum))) return rc;
    if ((rc = ensure(ctx, "c2.gpre", n_zero * sizeof(u64), &gpre))) return rc;
    if ((rc = ensure(ctx, "c3.sconf", ntiles * C2_STAGE * 12, &sconf))) return rc;
    if ((rc = ensure(ctx, "c3.smd", ntiles * C2_STAGE * sizeof(uint2), &smd))) return rc;
    if ((rc = device_zeros(ctx, &dz))) return rc;
    auto P = [&](const void* p, u64 n) { return n && p ? p : (const void*)dz; };
    const u64* kO = (const u64*)P(O.key, nO);
    const u64* kT = (const u64*)P(T.key, nT);
    const u64* kK = (const u64*)P(K.key, nK);
    rc = launch(ctx, "k_partition2", [&] {
        unsigned nb = (unsigned)((ntiles + C2_PG - 1) / C2_PG);
        if (v2) hipLaunchKernelGGL(k_partition2<J3B_TILE>, dim3(nb), dim3(C2_PNT), 0, ctx->stream, kO, nO, kT, nT, ntiles,
                                   (u64*)part, d_counts, d_err, (u64*)gsum, n_zero);
        else hipLaunchKernelGGL(k_partition2<J3_TILE>, dim3(nb), dim3(C2_PNT), 0, ctx->stream, kO, nO, kT, nT, ntiles,
                                (u64*)part, d_counts, d_err, (u64*)gsum, n_zero);
    });
    if (rc) return rc;
    void* nsplit = nullptr;
    if (v2 && hash && (rc = ensure(ctx, "c3.nsplit", 4 * (ntiles + 1) * sizeof(u64), &nsplit))) return rc;
    rc = launch(ctx, "k_apart3", [&] {
        const u64 lanes = 8 * (ntiles + 1);
        if (v2)
            hipLaunchKernelGGL(k_apart3b, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, ctx->stream, kO, nO, kT, nT,
                               (const u64*)part, ntiles, TILE, kK, nK, (u64*)apart, (const u64*)P(O.name_off, nO),
                               (const u64*)P(T.name_off, nT), perm ? J3B_HALO : (u64)0, (u64*)nsplit);
        else
            hipLaunchKernelGGL(k_apart3, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, ctx->stream, kO, nO, kT, nT,
                               (const u64*)part, ntiles, TILE, kK, nK, (u64*)apart);
    });
    if (rc) return rc;
    Join3Args a;
    Join2Args& g = a.j;
    g.A = kO; g.oidA = (const u8*)P(O.oid, nO); g.nA = nO;
    g.B = kT; g.oidB = (const u8*)P(T.oid, nT); g.nB = nT;
    g.part = (const u64*)part;
    g.nameA = (const u8*)P(O.name, nO); g.nameOffA = (const u64*)P(O.name_off, nO);
    g.nameB = (const u8*)P(T.name, nT); g.nameOffB = (const u64*)P(T.name_off, nT);
    g.hash_mode = hash ? 1 : 0;
    g.dummy = (const u8*)dz;
    g.ordA = (const u32*)P(ordO, nO); g.ordB = (const u32*)P(ordT, nT);
    g.stage_delta = g.stage_upd = nullptr;
    g.tile_cnt = (u32*)tcnt; g.gsum = (u64*)gsum; g.err = d_err;
    g.out_delta = g.out_upd = nullptr; g.counts = d_counts;
    g.stage_dkey = g.stage_ukey = g.out_dkey = g.out_ukey = nullptr;
    g.ntiles = ntiles;
    a.K = kK; a.oidK = (const u8*)P(K.oid, nK); a.nameK = (const u8*)P(K.name, nK);
    a.nameOffK = (const u64*)P(K.name_off, nK); a.ordK = (const u32*)P(ordK, nK); a.nK = nK;
    a.apart = (const u64*)apart; a.stage_conf = (u32*)sconf; a.stage_md = (uint2*)smd;
    a.nsplit = (const u64*)nsplit;
    void *cand3 = nullptr, *c2 = nullptr;
    if (split) {
        if ((rc = ensure(ctx, "c3.cand3", (total + 1) * 12, &cand3))) return rc;
        if ((rc = ensure(ctx, "c3.c2j", 64, &c2))) return rc;
    }
    auto j3b_grid = [&](const void* kern) {
        if (!J3B_PERSIST) return (unsigned)ntiles;
        return (unsigned)std::max<u64>(1, std::min<u64>(ntiles, (u64)ctx->n_cu * (u64)occupancy(ctx, kern, J3B_NT, 0)));
    };
    rc = launch(ctx, "k_join3", [&] {
#define KD_J3(H, PM, S) hipLaunchKernelGGL((k_join3<C2_NT, J3_IPT, H, PM, S>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, a)
        if (v2) {
#define KD_J3B(H, PM, S) hipLaunchKernelGGL((k_join3b<J3B_NT, J3B_IPT, H, PM, S>), dim3(j3b_grid((const void*)k_join3b<J3B_NT, J3B_IPT, H, PM, S>)), dim3(J3B_NT), 0, ctx->stream, a)
            if (split) {
                if (hash) { if (perm) KD_J3B(true, true, true); else KD_J3B(true, false, true); }
                else { if (perm) KD_J3B(false, true, true); else KD_J3B(false, false, true); }
            } else {
                if (hash) { if (perm) KD_J3B(true, true, false); else KD_J3B(true, false, false); }
                else { if (perm) KD_J3B(false, true, false); else KD_J3B(false, false, false); }
            }
#undef KD_J3B
        } else if (split) {
            if (hash) { if (perm) KD_J3(true, true, true); else KD_J3(true, false, true); }
            else { if (perm) KD_J3(false, true, true); else KD_J3(false, false, true); }
        } else if (j3_ol && !perm) {
            if (hash) hipLaunchKernelGGL((k_join3<C2_NT, J3_IPT, true, false, false, true>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, a);
            else hipLaunchKernelGGL((k_join3<C2_NT, J3_IPT, false, false, false, true>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, a);
        } else {
            if (hash) { if (perm) KD_J3(true, true, false); else KD_J3(true, false, false); }
            else { if (perm) KD_J3(false, true, false); else KD_J3(false, false, false); }
        }
#undef KD_J3
    });
    if (rc) return rc;
    u64* jcounts = split ? (u64*)c2 : d_counts;
    rc = launch(ctx, "k_gscan2", [&] {
        hipLaunchKernelGGL(k_gscan2, dim3(1), dim3(1024), 0, ctx->stream, (const u64*)gsum, (u64)(n_zero / 2),
                           (u64*)gpre, jcounts, 1);
    });
    if (rc) return rc;
    rc = launch(ctx, "k_place3", [&] {
        hipLaunchKernelGGL(k_place3, dim3((unsigned)ntiles), dim3(64), 0, ctx->stream, (const u32*)sconf,
                           (const uint2*)smd, (const u32*)tcnt, (const u64*)gpre, split ? (u32*)cand3 : d_conf, d_md);
    });
    if (rc || !split) return rc;
    return resolve3_have_a(ctx, K, O, T, (const u32*)cand3, (const u64*)c2, d_conf, d_md, d_counts, d_err, ordK, ordO,
                           ordT);
}

int diff2_device(kd_ctx* ctx, const kd_side* A, const kd_side* B, u32 flags, u32* d_delta, u32* d_upd,
                 u64* d_counts, u32* d_err, const u32* ordA, const u32* ordB, u64* d_dkey, u64* d_ukey) {
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
    void *part, *tcnt = nullptr, *sdel = nullptr, *supd = nullptr, *gsum = nullptr, *gpre = nullptr;
    int rc;
    if ((rc = ensure(ctx, "c2.part", (ntiles + 1) * sizeof(u64), &part))) return rc;
    u64* zero = nullptr;
    u64 n_zero = 0;
    if (!unord) {
        n_zero = 2 * ((ntiles + C2_GROUP - 1) / C2_GROUP);
        if ((rc = ensure(ctx, "c2.tcnt", ntiles * 4 * sizeof(u32), &tcnt))) return rc;
        if ((rc = ensure(ctx, "c2.gsum", n_zero * sizeof(u64), &gsum))) return rc;
        if ((rc = ensure(ctx, "c2.gpre", n_zero * sizeof(u64), &gpre))) return rc;
        if ((rc = ensure(ctx, "c2.sdel", ntiles * C2_STAGE * sizeof(uint2), &sdel))) return rc;
        if ((rc = ensure(ctx, "c2.supd", ntiles * C2_STAGE * sizeof(uint2), &supd))) return rc;
        zero = (u64*)gsum;
    }
    void *skd = nullptr, *sku = nullptr;
    if (d_dkey && !unord) {
        if ((rc = ensure(ctx, "c2.skd", ntiles * C2_STAGE * sizeof(u64), &skd))) return rc;
        if ((rc = ensure(ctx, "c2.sku", ntiles * C2_STAGE * sizeof(u64), &sku))) return rc;
    }
    void* dz;
    if ((rc = device_zeros(ctx, &dz))) return rc;
    const u64* kA = nA ? A->key : (const u64*)dz;  // an empty side points at device zeros
    const u64* kB = nB ? B->key : (const u64*)dz;
    const u8* empty_oid = (const u8*)dz;
    rc = launch(ctx, "k_partition2", [&] {
        unsigned nb = (unsigned)((ntiles + C2_PG - 1) / C2_PG);
        hipLaunchKernelGGL(k_partition2<C2_TILE>, dim3(nb), dim3(C2_PNT), 0, ctx->stream, kA, nA, kB, nB, ntiles,
                           (u64*)part, d_counts, d_err, zero, n_zero);
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
    const bool perm = ordA != nullptr || ordB != nullptr;
    // OIDs staged in LDS from this many entries on (C3's 200M: k_join2 1.28 -> 1.20 ms; C2's 20M:
    // 0.131 -> 0.136, profiles/r03/join2_oid_lds_ab.jsonl); the j2_oidlds_min option overrides (tests)
    const bool oid_lds = nA + nB >= ctx->opt.j2_oidlds_min;
    // j2r: the persistent register-prefetched form of the large int-key join (C3, r4o: k_join2 1.93 vs
    // 1.18 ms — three resident tiles per CU prefetching hold fewer bytes in flight than five one-shot
    // tiles; one tile per workgroup stays the default)
    const bool j2r = ctx->opt.j2r == 1;
    const int j2r_occ = j2r ? occupancy(ctx, (const void*)k_join2r<C2_NT, C2_IPT>, C2_NT, 0) : 1;
    g.ordA = nA && ordA ? ordA : (const u32*)dz;
    g.ordB = nB && ordB ? ordB : (const u32*)dz;
    g.stage_delta = (uint2*)sdel; g.stage_upd = (uint2*)supd;
    g.tile_cnt = (u32*)tcnt; g.gsum = (u64*)gsum; g.err = d_err;
    g.out_delta = (uint2*)d_delta; g.out_upd = (uint2*)d_upd; g.counts = d_counts;
    g.stage_dkey = (u64*)skd; g.stage_ukey = (u64*)sku;
    g.out_dkey = d_dkey; g.out_ukey = d_upd ? d_ukey : nullptr;
    g.ntiles = ntiles;
    rc = launch(ctx, "k_join2", [&] {
#define KD_J2(U, H, P) hipLaunchKernelGGL((k_join2<C2_NT, C2_IPT, U, H, P>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, g)
#define KD_J2OL(U) hipLaunchKernelGGL((k_join2<C2_NT, C2_IPT, U, false, false, true>), dim3((unsigned)ntiles), dim3(C2_NT), 0, ctx->stream, g)
#define KD_J2R() hipLaunchKernelGGL((k_join2r<C2_NT, C2_IPT>), dim3((unsigned)std::min<u64>(ntiles, (u64)ctx->n_cu * j2r_occ)), dim3(C2_NT), 0, ctx->stream, g)
        if (perm) {
            if (unord) { if (hash) KD_J2(true, true, true); else KD_J2(true, false, true); }
            else { if (hash) KD_J2(false, true, true); else KD_J2(false, false, true); }
        } else if (!hash && oid_lds) {
            if (unord) KD_J2OL(true);
            else if (j2r) KD_J2R();
            else KD_J2OL(false);
        } else {
            if (unord) { if (hash) KD_J2(true, true, false); else KD_J2(true, false, false); }
            else { if (hash) KD_J2(false, true, false); else KD_J2(false, false, false); }
        }
#undef KD_J2
#undef KD_J2OL
#undef KD_J2R
    });
    if (rc || unord) return rc;
    rc = launch(ctx, "k_gscan2", [&] {
        hipLaunchKernelGGL(k_gscan2, dim3(1), dim3(1024), 0, ctx->stream, (const u64*)gsum, (u64)(n_zero / 2),
                           (u64*)gpre, d_counts, 0);
    });
    if (rc) return rc;
    return launch(ctx, "k_place2", [&] {
        hipLaunchKernelGGL((k_place2<KD_PLACE_NT>), dim3((unsigned)ntiles), dim3(KD_PLACE_NT), 0, ctx->stream,
                           (const uint2*)sdel, (const uint2*)supd, (const u32*)tcnt, (const u64*)gpre,
                           (int)C2_STAGE, (uint2*)d_delta, (uint2*)d_upd, (const u64*)skd, (const u64*)sku, d_dkey,
                           d_upd ? d_ukey : nullptr);
    });
}

}  // namespace kd
