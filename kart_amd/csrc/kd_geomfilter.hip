// kd_geomfilter.hip — the spatially filtered diff on the GPU: for every delta of a two-way diff,
// the geometry column is located inside the old and new feature blobs (msgpack), its GPKG header
// decoded (stored envelope, or the point WKB), tested against the filter envelope in FP64, and the
// deltas whose old or new value may match are compacted in key order; the new side's
// spatial-filter index envelope (EnvelopeEncoder) comes out of the same pass.
//
// Reference (file:line under /root/reference):
//   BaseDiffWriter.filtered_ds_feature_deltas ... kart/base_diff_writer.py:279-329
//       do_yield = old matches || new matches (a delta is kept when either side may match)
//   SpatialFilter.matches / matches_delta_value . kart/spatial_filter/__init__.py:534-605
//       None value -> NONEXISTENT; geometry None -> MATCHING; envelope (stored, else OGR's:
//       point (x,x,y,y), empty (0,0,0,0)) fails bbox_intersects_fast -> NON_MATCHING; else the
//       prepared filter's Intersects decides
//   Dataset3.get_feature ........................ kart/dataset3.py:185-223 (blob = msgpack
//       [legend hex, [non-pk values]]; the legend names the value positions, kart/schema.py:19-102)
//   index envelope ............................... kart/spatial_filter/index.py:485-579 (kd_geom.h)
//
// Per side the code is 0 NON_MATCHING, 1 CANDIDATE (bbox passes; the exact Intersects is the
// caller's), 2 MATCHING (null geometry, no geometry column, or — for a rectangular filter — the
// envelope inside the rectangle, where Intersects is certain), 3 FALLBACK (the host decides:
// unknown legend, nested values, envelope that needs OGR), 4 NONEXISTENT (no such side).  Empty
// geometries never match (Intersects(empty) is false), whatever their (0,0,0,0) envelope does.
//
// Layout: one lane per delta, 4096 deltas per workgroup (16 rounds of 256).  The fast path loads
// 112 bytes from each blob start (7 dwordx4, realigned with v_alignbyte) and decodes the common
// shape — [legend str8(40), fixarray|array16 values, geometry first as ext8/16/32 'G'] — from
// registers; anything else takes the byte-wise decoder on global memory.
#include <cstdlib>
#include <type_traits>

#include "kd_geom.h"

namespace kd {

constexpr int GF_NT = 256;
#ifndef KD_GF_ROUNDS
#define KD_GF_ROUNDS 16
#endif
constexpr int GF_ROUNDS = KD_GF_ROUNDS;  // (probe builds may change it)
constexpr int GF_TILE = GF_NT * GF_ROUNDS;
constexpr int GF_MAXLEG = 64;  // legends per side held in LDS

enum { GF_NON = 0, GF_CAND = 1, GF_MATCH = 2, GF_FALLBACK = 3, GF_NONE = 4 };

struct GfArgs {
    const u8* data[2];
    const u64* off[2];
    u64 nblob[2];
    const u8* leg_hex[2];  // [n_leg * 40]
    const i16* gidx[2];    // [n_leg]
    int n_leg[2];
    const u32* pairs;  // [2 * cap]
    u64 cap;
    const u64* d_n;  // device delta count (or null: cap)
    double f0, f1, f2, f3;
    int rect;
    int bits;
    u8* match;  // [2 * cap]
    u8* enc;    // [cap * bits/2] new side index envelope (optional)
    u8* enc_ok;
    u32* tile_cnt;  // [tiles]
};

struct GHit {
    int code;
    int r, pc;  // gpkg_env / point_env results (index envelope input)
    bool empty;
    double e[4], pe[4];
};

// ---- byte-wise msgpack walk (global memory) ----
__device__ __forceinline__ u32 be_n(const u8* p, int n) {
    u32 v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | p[i];
    return v;
}

// skip one msgpack value at p (end e), nested arrays / maps included (a count of values still
// to skip instead of recursion); false on truncation or an invalid byte
__device__ bool mp_skip(const u8*& p, const u8* e) {
    u64 pending = 1;
    while (pending) {
        if (p >= e || pending > (u64)(e - p)) return false;  // every value takes at least one byte
        const u8 c = *p++;
        pending--;
        u64 n = 0;
        if (c <= 0x7f || c >= 0xe0 || c == 0xc0 || c == 0xc2 || c == 0xc3) continue;
        if ((c & 0xe0) == 0xa0) n = c & 31;
        else if ((c & 0xf0) == 0x90) { pending += c & 15; continue; }
        else if ((c & 0xf0) == 0x80) { pending += 2 * (c & 15); continue; }
        else {
            switch (c) {
                case 0xcc: case 0xd0: n = 1; break;
                case 0xcd: case 0xd1: n = 2; break;
                case 0xce: case 0xd2: case 0xca: n = 4; break;
                case 0xcf: case 0xd3: case 0xcb: n = 8; break;
                case 0xd9: case 0xc4: if (p + 1 > e) return false; n = be_n(p, 1); p += 1; break;
                case 0xda: case 0xc5: if (p + 2 > e) return false; n = be_n(p, 2); p += 2; break;
                case 0xdb: case 0xc6: if (p + 4 > e) return false; n = be_n(p, 4); p += 4; break;
                case 0xd4: n = 2; break;
                case 0xd5: n = 3; break;
                case 0xd6: n = 5; break;
                case 0xd7: n = 9; break;
                case 0xd8: n = 17; break;
                case 0xc7: if (p + 1 > e) return false; n = be_n(p, 1) + 1; p += 1; break;
                case 0xc8: if (p + 2 > e) return false; n = be_n(p, 2) + 1; p += 2; break;
                case 0xc9: if (p + 4 > e) return false; n = (u64)be_n(p, 4) + 1; p += 4; break;
                case 0xdc: if (p + 2 > e) return false; pending += be_n(p, 2); p += 2; continue;
                case 0xdd: if (p + 4 > e) return false; pending += be_n(p, 4); p += 4; continue;
                case 0xde: if (p + 2 > e) return false; pending += 2ull * be_n(p, 2); p += 2; continue;
                case 0xdf: if (p + 4 > e) return false; pending += 2ull * be_n(p, 4); p += 4; continue;
                default: return false;  // 0xc1 (never used)
            }
        }
        if ((u64)(e - p) < n) return false;
        p += n;
    }
    return true;
}

// legend index of a 40-byte hex at p (LDS table), -1 if unknown
__device__ __forceinline__ int leg_lookup_bytes(const u8* p, const u32* s_leg, int n_leg) {
    for (int l = 0; l < n_leg; l++) {
        bool eq = true;
        for (int j = 0; j < 40 && eq; j++) eq = p[j] == (u8)(s_leg[l * 10 + (j >> 2)] >> (8 * (j & 3)));
        if (eq) return l;
    }
    return -1;
}

// geometry payload (GPKG bytes) of a feature blob, byte-wise: rc 1 found (offset, length in the
// blob), 0 null geometry / no geometry column (MATCHING), -1 fallback.  The rare path: kept out of
// line, its result returned in registers.
struct GeomLoc {
    int rc;
    u32 off;
    u64 len;
};
__device__ __noinline__ GeomLoc find_geom_slow(const u8* b, u64 len, const u32* s_leg, const i16* s_gidx, int n_leg) {
    const u8 *p = b, *e = b + len;
    if (len < 2 || *p++ != 0x92) return GeomLoc{-1, 0, 0};
    // legend hex: a 40-byte str
    u32 sl;
    const u8 c = *p++;
    if ((c & 0xe0) == 0xa0) sl = c & 31;
    else if (c == 0xd9 && p < e) sl = *p++;
    else if (c == 0xda && p + 2 <= e) { sl = be_n(p, 2); p += 2; }
    else return GeomLoc{-1, 0, 0};
    if (sl != 40 || p + 40 > e) return GeomLoc{-1, 0, 0};
    const int l = leg_lookup_bytes(p, s_leg, n_leg);
    if (l < 0) return GeomLoc{-1, 0, 0};
    p += 40;
    const int gi = s_gidx[l];
    if (gi < 0) return GeomLoc{0, 0, 0};
    if (p >= e) return GeomLoc{-1, 0, 0};
    u32 cnt;
    const u8 h = *p++;
    if ((h & 0xf0) == 0x90) cnt = h & 15;
    else if (h == 0xdc && p + 2 <= e) { cnt = be_n(p, 2); p += 2; }
    else if (h == 0xdd && p + 4 <= e) { cnt = be_n(p, 4); p += 4; }
    else return GeomLoc{-1, 0, 0};
    if ((u32)gi >= cnt) return GeomLoc{-1, 0, 0};
    for (int k = 0; k < gi; k++)
        if (!mp_skip(p, e)) return GeomLoc{-1, 0, 0};
    if (p >= e) return GeomLoc{-1, 0, 0};
    const u8 v = *p++;
    if (v == 0xc0) return GeomLoc{0, 0, 0};
    u64 n;
    switch (v) {
        case 0xd4: n = 1; break;
        case 0xd5: n = 2; break;
        case 0xd6: n = 4; break;
        case 0xd7: n = 8; break;
        case 0xd8: n = 16; break;
        case 0xc7: if (p + 1 > e) return GeomLoc{-1, 0, 0}; n = be_n(p, 1); p += 1; break;
        case 0xc8: if (p + 2 > e) return GeomLoc{-1, 0, 0}; n = be_n(p, 2); p += 2; break;
        case 0xc9: if (p + 4 > e) return GeomLoc{-1, 0, 0}; n = be_n(p, 4); p += 4; break;
        default: return GeomLoc{-1, 0, 0};  // not an ext value
    }
    if (p >= e || *p++ != 'G') return GeomLoc{-1, 0, 0};
    if ((u64)(e - p) < n) return GeomLoc{-1, 0, 0};
    return GeomLoc{1, (u32)(p - b), n};
}

// compile-time loop: f(integral_constant<I>) for I in [I0, N) — register-window indices stay
// constants from the first optimisation pass on, so the windows never spill to scratch
template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

// match code of one geometry given its decoded envelope state
__device__ __forceinline__ int geom_code(const GfArgs& a, GHit& h, u8 hflags) {
    h.empty = h.r >= 0 && (hflags & 0x10);
    double env[4];
    bool have = false;
    if (h.r == 1) {
        have = true;
    } else if (h.r >= 0) {
        if (h.empty || h.pc == 0) return GF_NON;  // empty geometry (or empty point): Intersects is false
        have = h.pc == 1;  // the point's envelope (decode_side moved it into e)
    }
    env[0] = h.e[0]; env[1] = h.e[1]; env[2] = h.e[2]; env[3] = h.e[3];
    if (!have) return GF_FALLBACK;
    int x = range_ov(a.f0, a.f1, env[0], env[1]);
    if (x > 0) x = range_ov(a.f2, a.f3, env[2], env[3]);
    if (x < 0) return GF_FALLBACK;  // inverted envelope: the reference raises
    if (x == 0) return GF_NON;
    if (a.rect && a.f0 <= env[0] && env[1] <= a.f1 && a.f2 <= env[2] && env[3] <= a.f3) return GF_MATCH;
    return GF_CAND;
}

// decode side s's blob `bi` for one lane
// (o, len): the blob's arena offset and length, loaded by the caller for both sides up front (the
// second side's offset loads are not serialised behind the first side's decode)
// LDSW: the blob's first 112 bytes come from its LDS image (k_gf_match's staged heads: 7 chunks
// from the blob's 16-B-aligned start at LDS byte address img) instead of 7 global loads
template <bool LDSW>
__device__ __forceinline__ void decode_side(const GfArgs& a, int s, u32 bi, u64 o, u64 len, u64 arena_end,
                                            const u32* s_leg, const i16* s_gidx, GHit& h, u32 img = 0) {
    typedef const __attribute__((address_space(1))) u32x4* gx4;
    h.r = -1;
    h.pc = -1;
    h.empty = false;
    if (bi == KD_NONE) { h.code = GF_NONE; return; }
    if ((u64)bi >= a.nblob[s]) { h.code = GF_FALLBACK; return; }
    const u8* b = a.data[s] + o;
    const int n_leg = a.n_leg[s];
    const u8* gp = nullptr;
    u64 glen = 0;
    u8 hflags = 0;
    bool fast = false, located = false;
    const u64 a0 = (u64)b, a4 = a0 & ~(u64)3;
    if (len >= 52 && a4 + 112 <= arena_end) {
        u32 w[28];
        if (LDSW) {  // words from a4 in the image (from a16 = a4 & ~15; the words past its 112 bytes
                     // are not among the bytes the fast path uses: those end at blob byte 95)
            typedef const __attribute__((address_space(3))) u32* l32;
            const u32 q = img + (u32)(a4 & 15);
            sfor<0, 28>([&](auto k) { w[k] = *(l32)(size_t)(q + 4 * k); });
        } else {
            sfor<0, 7>([&](auto k) {
                const u32x4 v = *(gx4)(a4 + 16 * k);
                w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
            });
        }
        const u32 sh = (u32)(a0 - a4);
        u32 rr[27];
        sfor<0, 27>([&](auto j) { rr[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh); });
        // [0x92, 0xd9, 40, hex x40, values header]
        if ((rr[0] & 0xFFFFFFu) == 0x28d992u) {
            u32 hx[10];
            sfor<0, 10>([&](auto j) { hx[j] = __builtin_amdgcn_alignbyte(rr[j + 1], rr[j], 3); });
            int l = -1;
            for (int q = 0; q < n_leg && l < 0; q++) {
                bool eq = true;
                sfor<0, 10>([&](auto j) { eq &= hx[j] == s_leg[q * 10 + j]; });
                if (eq) l = q;
            }
            const u32 ah = rr[10] >> 24;  // byte 43
            const int p = (ah & 0xf0) == 0x90 ? 44 : ah == 0xdc ? 46 : -1;
            if (l < 0) { h.code = GF_FALLBACK; return; }  // unknown legend: the reference raises KeyError
            const int gi = s_gidx[l];
            if (gi < 0) { h.code = GF_MATCH; return; }  // this legend has no geometry column: value None
            if (gi == 0 && p > 0) {
                const u32 w11 = rr[11];
                const u32 v = p == 44 ? (w11 & 0xff) : ((w11 >> 16) & 0xff);
                if (v == 0xc0) { h.code = GF_MATCH; return; }  // null geometry
                // ext header bytes p+1 .. p+5 (p = 44: bytes 45..49, p = 46: 47..51)
                const u32 x0 = p == 44 ? __builtin_amdgcn_alignbyte(rr[12], rr[11], 1)
                                       : __builtin_amdgcn_alignbyte(rr[12], rr[11], 3);
                const u32 x1 = p == 44 ? __builtin_amdgcn_alignbyte(rr[13], rr[12], 1)
                                       : __builtin_amdgcn_alignbyte(rr[13], rr[12], 3);
                int q = -1;
                u32 gl = 0, typ = 0;
                if (v == 0xc7) { gl = x0 & 0xff; typ = (x0 >> 8) & 0xff; q = p + 3; }
                else if (v == 0xc8) { gl = ((x0 & 0xff) << 8) | ((x0 >> 8) & 0xff); typ = (x0 >> 16) & 0xff; q = p + 4; }
                else if (v == 0xc9) { gl = __builtin_bswap32(x0); typ = x1 & 0xff; q = p + 6; }
                if (q > 0) {
                    if (typ != 'G' || (u64)q + gl > len) { h.code = GF_FALLBACK; return; }
                    located = true;
                    gp = b + q;
                    glen = gl;
                    // GPKG window: 11 dwords from byte q (q in 47..52: dwords 11..13 + j)
                    const int qd = q >> 2, qs = q & 3;  // qd in 11..13
                    u32 rq[11];
                    sfor<0, 11>([&](auto j) {
                        const u32 a11 = rr[11 + j], a12 = rr[12 + j], a13 = rr[13 + j], a14 = rr[14 + j];
                        const u32 lo = qd == 11 ? a11 : qd == 12 ? a12 : a13;
                        const u32 hi = qd == 11 ? a12 : qd == 12 ? a13 : a14;
                        rq[j] = __builtin_amdgcn_alignbyte(hi, lo, qs);
                    });
                    if (glen >= 8) {
                        fast = env_fast(rq, glen, h.r, h.e, h.pc, h.pe);
                        hflags = rq[0] >> 24;
                    }
                }
            }
        }
    }
    if (!located) {
        const GeomLoc f = find_geom_slow(b, len, s_leg, s_gidx, n_leg);
        if (f.rc < 0) { h.code = GF_FALLBACK; return; }
        if (f.rc == 0) { h.code = GF_MATCH; return; }
        gp = b + f.off;
        glen = f.len;
    }
    if (!fast) {  // byte-wise GPKG decode (short or unusual geometry headers)
        h.r = gpkg_env(gp, glen, h.e);
        h.pc = -1;
        if (h.r == 0 || h.r == 2) h.pc = point_env(gp, glen, h.pe);
        if (h.r >= 0) hflags = gp[3];
    }
    if (h.r != 1 && h.pc >= 0) {  // one envelope from here on: the point's (x, x, y, y)
        h.e[0] = h.pe[0]; h.e[1] = h.pe[1]; h.e[2] = h.pe[2]; h.e[3] = h.pe[3];
    }
    h.code = geom_code(a, h, hflags);
}

// STAGE: each round's blob heads are staged in LDS by LDS-DMA, one side at a time — chunk c of a
// wave's instruction k goes to owner lane c / 7, head chunk c % 7 — so a wave-instruction reads the
// heads of ~9 blobs, 7 consecutive chunks each, instead of one 16-B piece of 64 different blobs
// (per-lane scattered loads run at about half the request rate, scripts/probe/scatter_probe.hip)
#ifndef KD_GF_STAGE
#define KD_GF_STAGE 1
#endif
constexpr int GF_HCH = 7;  // head chunks per blob (112 B from the 16-B-aligned start: blob bytes >= 97)
template <bool STAGE>
__global__ __launch_bounds__(GF_NT) void k_gf_match(GfArgs a) {
    typedef __attribute__((address_space(3))) void* lvp;
    typedef const __attribute__((address_space(1))) void* gvp;
    __shared__ u32x4 s_img[STAGE ? GF_NT * GF_HCH : 1];
    __shared__ u32 s_leg[2][GF_MAXLEG * 10];
    __shared__ i16 s_gidx[2][GF_MAXLEG];
    __shared__ u8 s_enc[GF_NT * 16];
    __shared__ u8 s_ok[GF_NT];
    __shared__ u32 s_wc[GF_NT / 64];
    const int tid = threadIdx.x;
    // legend tables: hex as little-endian dwords (compared with the realigned blob words)
    for (int s = 0; s < 2; s++) {
        for (int i = tid; i < a.n_leg[s]; i += GF_NT) s_gidx[s][i] = a.gidx[s][i];
        for (int i = tid; i < a.n_leg[s] * 10; i += GF_NT) {
            const u8* p = a.leg_hex[s] + 4 * i;
            s_leg[s][i] = (u32)p[0] | (u32)p[1] << 8 | (u32)p[2] << 16 | (u32)p[3] << 24;
        }
    }
    __syncthreads();
    const u64 n = a.d_n ? *a.d_n : a.cap;
    const int nb = a.bits / 2;
    const double vmax = (double)((1ull << a.bits) - 1);
    const u64 t0 = (u64)blockIdx.x * GF_TILE;
    const u64 end0 = (u64)a.data[0] + a.off[0][a.nblob[0]], end1 = (u64)a.data[1] + a.off[1][a.nblob[1]];
    u32 kept = 0;
    for (int r = 0; r < GF_ROUNDS; r++) {
        const u64 d0 = t0 + (u64)r * GF_NT;
        if (d0 >= n) break;  // block-uniform
        const u64 d = d0 + tid;
        bool keep = false;
        u8 ok = 0;
        if (a.enc)
            for (int k = 0; k < nb; k++) s_enc[tid * nb + k] = 0;
        if (STAGE) {
            // both sides' heads through LDS, one side at a time (block-uniform: every lane stages
            // and waits, valid delta or not)
            u32 po = KD_NONE, pn = KD_NONE;
            u64 oo = 0, oe = 0, no = 0, ne = 0;
            if (d < n) {
                po = a.pairs[2 * d];
                pn = a.pairs[2 * d + 1];
                if ((u64)po < a.nblob[0]) { oo = a.off[0][po]; oe = a.off[0][po + 1]; }
                if ((u64)pn < a.nblob[1]) { no = a.off[1][pn]; ne = a.off[1][pn + 1]; }
            }
            const int lane = tid & 63, wv = tid >> 6;
            const u32 wimg = (u32)(size_t)(const __attribute__((address_space(3))) u32x4*)s_img + 16u * (u32)(wv * 64 * GF_HCH);
            int code[2];
            GHit h;
#pragma unroll
            for (int sd = 0; sd < 2; sd++) {
                const u32 bi = sd ? pn : po;
                const u64 o = sd ? no : oo, len = sd ? ne - no : oe - oo, aend = sd ? end1 : end0;
                const u64 a0 = (u64)a.data[sd] + o, a16 = a0 & ~(u64)15;
                // chunks of this lane's head that lie below the arena's end (a present, long-enough blob)
                const bool stage = d < n && bi != KD_NONE && (u64)bi < a.nblob[sd] && len >= 52;
                const u32 nch = stage ? (u32)min<u64>((aend - a16 + 15) >> 4, (u64)GF_HCH) : 0u;
#pragma unroll
                for (int k = 0; k < GF_HCH; k++) {
                    const int c = 64 * k + lane, ow = c / GF_HCH, ci = c - ow * GF_HCH;
                    const u64 src = __shfl(a16, ow);
                    const u32 cn = __shfl(nch, ow);
                    if ((u32)ci < cn)
                        __builtin_amdgcn_global_load_lds((gvp)(src + 16ull * ci), (lvp)(s_img + wv * 64 * GF_HCH + 64 * k), 16, 0, 0);
                }
                __syncthreads();  // vmcnt(0) + barrier: the heads have landed
                if (d < n)
                    decode_side<true>(a, sd, bi, o, len, aend, s_leg[sd], s_gidx[sd], h, wimg + 16u * (u32)(GF_HCH * lane));
                code[sd] = h.code;
                __syncthreads();  // the image is free for the other side
            }
            if (d < n) {
                const int co = code[0], cn = code[1];
                keep = (co >= 1 && co <= 3) || (cn >= 1 && cn <= 3);
                *(u16*)(a.match + 2 * d) = (u16)(co | cn << 8);
                if (a.enc && cn != GF_NONE && cn != GF_FALLBACK && h.r >= 0)
                    ok = index_env(h.r, h.pc, h.e, h.e, h.empty, a.bits, vmax, [&](int k, u8 v) { s_enc[tid * nb + k] = v; });
            }
        } else if (d < n) {
            const u32 po = a.pairs[2 * d], pn = a.pairs[2 * d + 1];
            const bool vo = (u64)po < a.nblob[0], vn = (u64)pn < a.nblob[1];
            const u64 oo = vo ? a.off[0][po] : 0, oe = vo ? a.off[0][po + 1] : 0;
            const u64 no = vn ? a.off[1][pn] : 0, ne = vn ? a.off[1][pn + 1] : 0;
            GHit h;
            decode_side<false>(a, 0, po, oo, oe - oo, end0, s_leg[0], s_gidx[0], h);
            const int co = h.code;
            decode_side<false>(a, 1, pn, no, ne - no, end1, s_leg[1], s_gidx[1], h);
            const int cn = h.code;
            keep = (co >= 1 && co <= 3) || (cn >= 1 && cn <= 3);
            *(u16*)(a.match + 2 * d) = (u16)(co | cn << 8);
            if (a.enc && cn != GF_NONE && cn != GF_FALLBACK && h.r >= 0)
                ok = index_env(h.r, h.pc, h.e, h.e, h.empty, a.bits, vmax, [&](int k, u8 v) { s_enc[tid * nb + k] = v; });
        }
        const u64 bal = __ballot(keep);
        kept += (u32)__popcll(bal);
        if (a.enc) {  // index envelopes through LDS: contiguous dword stores
            s_ok[tid] = ok;
            __syncthreads();
            const u32 cnt = (u32)(n - d0 < GF_NT ? n - d0 : GF_NT);
            u8* dst = a.enc + d0 * nb;
            const u32 bytes = cnt * nb;
            if ((((u64)dst) & 3) == 0) {
                const u32 nw = bytes >> 2;
                for (u32 k = tid; k < nw; k += GF_NT) ((u32*)dst)[k] = ((const u32*)s_enc)[k];
                for (u32 k = 4 * nw + tid; k < bytes; k += GF_NT) dst[k] = s_enc[k];
            } else {
                for (u32 k = tid; k < bytes; k += GF_NT) dst[k] = s_enc[k];
            }
            for (u32 k = tid; k < cnt; k += GF_NT) a.enc_ok[d0 + k] = s_ok[k];
            __syncthreads();
        }
    }
    if ((tid & 63) == 0) s_wc[tid >> 6] = kept;
    __syncthreads();
    if (tid == 0) {
        u32 t = 0;
        for (int w = 0; w < GF_NT / 64; w++) t += s_wc[w];
        a.tile_cnt[blockIdx.x] = t;
    }
}

// ---- the heads form: one 48-B geometry head per blob side (kd_geom_heads), no msgpack walk ----
struct GfHeadArgs {
    const kd_geom_head* head[2];
    u64 nhead[2];
    const u8* data[2];  // the arenas the heads came from (null: no slow path, such sides FALLBACK)
    const u64* off[2];
    const u8* zeros;    // >= 48 readable zero bytes: the source of an absent side's head loads
    const uint2* bpairs;  // (optional) the blob of each delta side in the arenas, when the heads are
                          // not indexed like the arenas (delta-order heads over per-entry arenas)
    u32* fb_list;         // (optional) deltas whose head needs its blob are listed here and left to
    u32* fb_count;        // k_gf_fb, so the streaming pass never waits on a byte-wise blob decode
    int dense;            // heads indexed by delta (slot d holds delta d's head; the pairs say only
                          // which sides are present): k_gf_dense, no pair -> head dependency
    int pres_only;        // (dense) the pairs are the deltas' blob rows (bpairs == pairs): a present
                          // side's head is at slot d
};

// (dense) the head slots of delta d's sides from its pair
__device__ __forceinline__ uint2 head_slots(const GfHeadArgs& g, uint2 p, u64 d) {
    if (!g.pres_only) return p;
    return make_uint2(p.x == KD_NONE ? KD_NONE : (u32)d, p.y == KD_NONE ? KD_NONE : (u32)d);
}

struct HeadLd {
    u32x4 v0, v1, v2;
};

// one side's head record (three 16-B loads; an absent side reads the zero block): unconditional,
// so no branch hides them from the wait counting of a pipelined caller
__device__ __forceinline__ HeadLd load_head(const GfHeadArgs& g, int s, u32 bi) {
    typedef const __attribute__((address_space(1))) u32x4* gx4;
    HeadLd L;
    const bool ok = bi != KD_NONE && (u64)bi < g.nhead[s];
    const u64 base = ok ? (u64)(g.head[s] + bi) : (u64)g.zeros;
    L.v0 = *(gx4)base;
    L.v1 = *(gx4)(base + 16);
    L.v2 = *(gx4)(base + 32);
    return L;
}

// returns false when the geometry needs its blob and the caller defers it (g.fb_list): code FALLBACK
__device__ __forceinline__ bool decode_head(const GfArgs& a, const GfHeadArgs& g, int s, u32 bi, const HeadLd& L,
                                            GHit& h, u64 d, bool defer) {
    h.r = -1;
    h.pc = -1;
    h.empty = false;
    if (bi == KD_NONE) { h.code = GF_NONE; return true; }
    if ((u64)bi >= g.nhead[s]) { h.code = GF_FALLBACK; return true; }
    const u32x4 v0 = L.v0, v1 = L.v1, v2 = L.v2;
    const u32 st = v2.w >> 24;
    if (st == KD_GH_NULL) { h.code = GF_MATCH; return true; }
    if (st != KD_GH_GEOM) { h.code = GF_FALLBACK; return true; }
    const u32 glen = v2.z;
    const u32 r[11] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, 0u};
    u8 hflags = (u8)(v0.x >> 24);
    const bool fast = env_fast(r, glen, h.r, h.e, h.pc, h.pe);
    if (!fast) {  // XYZ/XYM/XYZM envelope or a NaN one: the byte-wise decode on the blob
        if (!g.data[s]) { h.code = GF_FALLBACK; h.r = -1; return true; }
        if (defer) { h.code = GF_FALLBACK; h.r = -1; return false; }
        const u32 blob = g.bpairs ? (s ? g.bpairs[d].y : g.bpairs[d].x) : bi;
        if (blob == KD_NONE || (u64)blob >= a.nblob[s]) { h.code = GF_FALLBACK; h.r = -1; return true; }
        const u8* gp = g.data[s] + g.off[s][blob] + (v2.w & 0xFFFFFFu);
        h.r = gpkg_env(gp, glen, h.e);
        h.pc = -1;
        if (h.r == 0 || h.r == 2) h.pc = point_env(gp, glen, h.pe);
        if (h.r >= 0) hflags = gp[3];
    }
    if (h.r != 1 && h.pc >= 0) {
        h.e[0] = h.pe[0]; h.e[1] = h.pe[1]; h.e[2] = h.pe[2]; h.e[3] = h.pe[3];
    }
    h.code = geom_code(a, h, hflags);
    return true;
}

// k_gf_match over heads: the same tiles, codes, kept counts and index envelopes.
// Each wave works alone until the tile's kept count: its 64 deltas' index envelopes are staged in
// its own LDS slice and written out as contiguous dwords by the wave (no block barrier per round —
// a barrier's fence waits for every load in flight, prefetches included), and the loads run two
// rounds deep: round r+1's heads and round r+2's delta pair are in flight while round r decodes.
__global__ __launch_bounds__(GF_NT) void k_gf_heads(GfArgs a, GfHeadArgs g) {
    __shared__ u32 s_encw[GF_NT * 4];  // 16 B per lane: nb <= 16 index-envelope bytes
    __shared__ u32 s_wc[GF_NT / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const u64 n = a.d_n ? *a.d_n : a.cap;
    const int nb = a.bits / 2;
    const double vmax = (double)((1ull << a.bits) - 1);
    u8* const wenc = (u8*)(s_encw + 64 * 4 * wid);  // this wave's slice
    // persistent: the grid is the resident set, tiles taken grid-stride (no partial last wave of
    // blocks).  Every tile of the capacity is visited: k_gf_scan reads all their kept counts, and a
    // tile past the device count writes 0
    const u64 ntiles = (a.cap + GF_TILE - 1) / GF_TILE;
    for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const u64 t0 = tile * GF_TILE;
    u32 kept = 0;
    auto ld_pair = [&](u64 d) {  // (unconditional load, clamped index)
        const uint2 v = *(n ? (const uint2*)a.pairs + (d < n ? d : n - 1) : (const uint2*)g.zeros);
        return d < n ? v : make_uint2(KD_NONE, KD_NONE);
    };
    uint2 pr = ld_pair(t0 + tid);
    uint2 pr1 = GF_ROUNDS > 1 ? ld_pair(t0 + GF_NT + tid) : make_uint2(KD_NONE, KD_NONE);
    HeadLd L0 = load_head(g, 0, pr.x), L1 = load_head(g, 1, pr.y);
    for (int rd = 0; rd < GF_ROUNDS; rd++) {
        const u64 d0 = t0 + (u64)rd * GF_NT;
        if (d0 >= n) break;  // block-uniform
        const u64 d = d0 + tid;
        // issue order = wait order: the pair two rounds ahead, then the next round's heads (its
        // pair arrived a round ago), then this round's decode waits only for this round's heads
        const uint2 pr2 = rd + 2 < GF_ROUNDS ? ld_pair(d + 2 * GF_NT) : make_uint2(KD_NONE, KD_NONE);
        const HeadLd M0 = load_head(g, 0, pr1.x), M1 = load_head(g, 1, pr1.y);
        bool keep = false;
        u8 ok = 0;
        if (a.enc)
            for (int k = 0; k < nb; k++) wenc[lane * nb + k] = 0;
        bool deferred = false;
        if (d < n) {
            GHit h;
#ifdef KD_GF_PROBE_NODECODE  // profiling variant: the loads and stores alone
            const u32 x = L0.v0.x ^ L0.v1.y ^ L0.v2.w ^ L1.v0.z ^ L1.v1.w ^ L1.v2.x;
            const int co = (int)(x & 3), cn = (int)((x >> 2) & 3);
            h.r = -1;
            (void)g;
#else
            const bool defer = g.fb_list != nullptr;
            deferred = !decode_head(a, g, 0, pr.x, L0, h, d, defer);
            const int co = h.code;
            deferred |= !decode_head(a, g, 1, pr.y, L1, h, d, defer);
            const int cn = h.code;
#endif
            keep = (co >= 1 && co <= 3) || (cn >= 1 && cn <= 3);
            *(u16*)(a.match + 2 * d) = (u16)(co | cn << 8);
            if (a.enc && !deferred && cn != GF_NONE && cn != GF_FALLBACK && h.r >= 0)
                ok = index_env(h.r, h.pc, h.e, h.e, h.empty, a.bits, vmax, [&](int k, u8 v) { wenc[lane * nb + k] = v; });
            if (a.enc) a.enc_ok[d] = ok;
        }
        kept += (u32)__popcll(__ballot(keep));
        {  // deferred deltas: one atomic per wave, slots in lane order
            const u64 bd = __ballot(deferred);
            if (bd) {
                u32 base = 0;
                if (lane == 0) base = atomicAdd(g.fb_count, (u32)__popcll(bd));
                base = __shfl(base, 0);
                if (deferred)
                    g.fb_list[base + __builtin_amdgcn_mbcnt_hi((u32)(bd >> 32), __builtin_amdgcn_mbcnt_lo((u32)bd, 0))] = (u32)d;
            }
        }
        if (a.enc) {
            __builtin_amdgcn_wave_barrier();  // (one wave: its LDS operations stay in program order)
            const u64 w0 = d0 + 64ull * wid;
            const u32 cnt = w0 < n ? (u32)(n - w0 < 64 ? n - w0 : 64) : 0u;
            u8* dst = a.enc + w0 * nb;
            const u32 bytes = cnt * nb;
            if ((((u64)dst) & 3) == 0) {
                const u32 nw = bytes >> 2;
                for (u32 k = lane; k < nw; k += 64) ((u32*)dst)[k] = ((const u32*)wenc)[k];
                for (u32 k = 4 * nw + lane; k < bytes; k += 64) dst[k] = wenc[k];
            } else {
                for (u32 k = lane; k < bytes; k += 64) dst[k] = wenc[k];
            }
            __builtin_amdgcn_wave_barrier();  // read out before the next round's zeroing
        }
        L0 = M0;
        L1 = M1;
        pr = pr1;
        pr1 = pr2;
    }
    if (lane == 0) s_wc[wid] = kept;
    __syncthreads();
    if (tid == 0) {
        u32 t = 0;
        for (int w = 0; w < GF_NT / 64; w++) t += s_wc[w];
        a.tile_cnt[tile] = t;
    }
    __syncthreads();  // s_wc is rewritten by the next tile
    }
}

// k_gf_heads for dense heads (kd_geom_filter_deltas: the device gather put delta d's heads in
// slot d).  Head addresses follow from the delta index, so nothing waits on the pairs before its
// loads are issued.  Each wave owns 64-delta chunks (grid-stride over chunks, so the persistent
// grid ends within one chunk of balance) and keeps PF chunks of loads in flight beyond the one it
// decodes.  TR: a chunk's 2 x 3 KB of heads are read as lane-contiguous 16-B pieces (each load
// instruction one 1-KB run) and transposed through the wave's LDS slice; else three 16-B loads
// per lane and side at the 48-B head stride.  Kept counts go to the chunk's tile by one atomic per
// wave (tile_cnt zeroed before the launch).
struct DenseLd {
    u32x4 h[6];  // TR: pieces k of side s at [3s + k]; else side s head dwords at [3s + k]
    uint2 pr;
};

template <bool TR>
__device__ __forceinline__ DenseLd dense_load(const GfArgs& a, const GfHeadArgs& g, u64 c, u64 nchunk, u64 n, int lane) {
    typedef const __attribute__((address_space(1))) u32x4* gx4;
    DenseLd L;
    const u64 cc = c < nchunk ? c : (nchunk ? nchunk - 1 : 0);  // (past the end: a clamped, unused load)
    const u64 d = cc * 64 + lane;
    // (the slots are allocated in whole 64-delta chunks: every chunk below nchunk is readable)
    const u64 o = TR ? cc * 3072 + (u64)lane * 16 : d * 48;
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const u64 base = (u64)g.head[s] + o;
#pragma unroll
        for (int k = 0; k < 3; k++) L.h[3 * s + k] = *(gx4)(base + (TR ? 1024 : 16) * k);
    }
    const u64 dp = n ? (d < n ? d : n - 1) : 0;
    const uint2 v = *(n ? (const uint2*)a.pairs + dp : (const uint2*)g.zeros);
    L.pr = d < n ? head_slots(g, v, d) : make_uint2(KD_NONE, KD_NONE);
    return L;
}

// PP: the pairs run one chunk ahead of the heads, so a side the pair marks absent (an insert's old
// side, a delete's new side: ~20 % of C5's delta sides) is loaded from the zero block, not from its
// slot — those bytes never leave the cache
__device__ __forceinline__ uint2 dense_pair(const GfArgs& a, const GfHeadArgs& g, u64 c, u64 n, int lane) {
    const u64 d = c * 64 + lane;
    const u64 dp = n ? (d < n ? d : n - 1) : 0;
    const uint2 v = *(n ? (const uint2*)a.pairs + dp : (const uint2*)g.zeros);
    return d < n ? head_slots(g, v, d) : make_uint2(KD_NONE, KD_NONE);
}

__device__ __forceinline__ DenseLd dense_load_pp(const GfHeadArgs& g, u64 c, u64 nchunk, uint2 pr, int lane) {
    typedef const __attribute__((address_space(1))) u32x4* gx4;
    DenseLd L;
    const u64 cc = c < nchunk ? c : (nchunk ? nchunk - 1 : 0);
    const u64 o = (cc * 64 + lane) * 48;
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const bool pres = (s ? pr.y : pr.x) != KD_NONE;
        const u64 base = pres ? (u64)g.head[s] + o : (u64)g.zeros;
#pragma unroll
        for (int k = 0; k < 3; k++) L.h[3 * s + k] = *(gx4)(base + 16 * k);
    }
    L.pr = pr;
    return L;
}

#ifndef KD_GFD_PP
#define KD_GFD_PP 1
#endif
#ifndef KD_GFD_PF
#define KD_GFD_PF 1  // k_gf_dense prefetch depth (chunks ahead)
#endif
#ifndef KD_GFD_TR
#define KD_GFD_TR false  // k_gf_dense: heads loaded as lane-contiguous runs, transposed through LDS
#endif
#ifndef KD_GFD_ZW
#define KD_GFD_ZW 1  // C5: 0.317 -> 0.312 ms (r5m)
#endif
#ifndef KD_GFD_WAVES
#define KD_GFD_WAVES 4  // k_gf_dense<1, false>: waves per SIMD the register budget is cut for
#endif
template <int PF, bool TR>
__global__ __launch_bounds__(GF_NT) __attribute__((amdgpu_waves_per_eu(PF == 1 && !TR ? KD_GFD_WAVES : 3))) void k_gf_dense(GfArgs a, GfHeadArgs g) {
    static_assert(PF == 1 || PF == 2, "prefetch depth");
    __shared__ u32 s_encw[GF_NT * 4];  // 16 B per lane: nb <= 16 index-envelope bytes
    __shared__ u32x4 s_tr[TR ? (GF_NT / 64) * 6 * 64 : 1];  // 6 KB per wave
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const u64 n = a.d_n ? *a.d_n : a.cap;
    const u64 nchunk = (n + 63) / 64;
    const int nb = a.bits / 2;
    const double vmax = (double)((1ull << a.bits) - 1);
    u8* const wenc = (u8*)(s_encw + 64 * 4 * wid);
    u32x4* const wtr = s_tr + (TR ? wid * 6 * 64 : 0);
    const u64 wstride = (u64)gridDim.x * (GF_NT / 64);
    u64 c = (u64)blockIdx.x * (GF_NT / 64) + wid;
    constexpr bool PP = KD_GFD_PP && PF == 1 && !TR;
    uint2 pr1 = make_uint2(KD_NONE, KD_NONE);
    DenseLd A;
    if (PP) {
        A = dense_load_pp(g, c, nchunk, dense_pair(a, g, c, n, lane), lane);
        pr1 = dense_pair(a, g, c + wstride, n, lane);
    } else {
        A = dense_load<TR>(a, g, c, nchunk, n, lane);
    }
    DenseLd B;
    if (PF == 2) B = dense_load<TR>(a, g, c + wstride, nchunk, n, lane);
    for (; c < nchunk; c += wstride) {  // wave-uniform
        // the load PF chunks ahead first, so this chunk's wait leaves it in flight
        DenseLd Nx;
        if (PP) {
            const uint2 pr2 = dense_pair(a, g, c + 2 * wstride, n, lane);
            Nx = dense_load_pp(g, c + wstride, nchunk, pr1, lane);
            pr1 = pr2;
        } else {
            Nx = dense_load<TR>(a, g, c + PF * wstride, nchunk, n, lane);
        }
        const u64 d = c * 64 + lane;
        HeadLd L0, L1;
        if (TR) {
#pragma unroll
            for (int k = 0; k < 6; k++) wtr[k * 64 + lane] = A.h[k];  // piece (s, k) = index (3s + k) * 64 + lane
            __builtin_amdgcn_wave_barrier();
            // side s, head of this lane: bytes [lane * 48, +48) of the side's 3 KB = pieces lane*3 + j
            L0.v0 = wtr[lane * 3 + 0]; L0.v1 = wtr[lane * 3 + 1]; L0.v2 = wtr[lane * 3 + 2];
            L1.v0 = wtr[192 + lane * 3 + 0]; L1.v1 = wtr[192 + lane * 3 + 1]; L1.v2 = wtr[192 + lane * 3 + 2];
            __builtin_amdgcn_wave_barrier();
        } else {
            L0.v0 = A.h[0]; L0.v1 = A.h[1]; L0.v2 = A.h[2];
            L1.v0 = A.h[3]; L1.v1 = A.h[4]; L1.v2 = A.h[5];
        }
        const uint2 pr = A.pr;
        bool keep = false, deferred = false;
        u8 ok = 0;
#if KD_GFD_ZW  // the wave's slice zeroed as dwords (64 nb bytes = 16 nb dwords), not nb bytes per lane
        if (a.enc) {
            for (int k = lane; k < 16 * nb; k += 64) ((u32*)wenc)[k] = 0;
            __builtin_amdgcn_wave_barrier();
        }
#else
        if (a.enc)
            for (int k = 0; k < nb; k++) wenc[lane * nb + k] = 0;
#endif
        if (d < n) {
            GHit h;
#ifdef KD_GF_PROBE_NODECODE  // profiling variant: the loads and stores alone
            const u32 x = L0.v0.x ^ L0.v1.y ^ L0.v2.w ^ L1.v0.z ^ L1.v1.w ^ L1.v2.x ^ pr.x ^ pr.y;
            const int co = (int)(x & 3), cn = (int)((x >> 2) & 3);
            h.r = -1;
#else
            const bool defer = g.fb_list != nullptr;
            deferred = !decode_head(a, g, 0, pr.x, L0, h, d, defer);
            const int co = h.code;
            deferred |= !decode_head(a, g, 1, pr.y, L1, h, d, defer);
            const int cn = h.code;
#endif
            keep = (co >= 1 && co <= 3) || (cn >= 1 && cn <= 3);
            *(u16*)(a.match + 2 * d) = (u16)(co | cn << 8);
            if (a.enc && !deferred && cn != GF_NONE && cn != GF_FALLBACK && h.r >= 0)
                ok = index_env(h.r, h.pc, h.e, h.e, h.empty, a.bits, vmax, [&](int k, u8 v) { wenc[lane * nb + k] = v; });
            if (a.enc) a.enc_ok[d] = ok;
        }
        const u32 kept = (u32)__popcll(__ballot(keep));
        if (lane == 0 && kept) atomicAdd(a.tile_cnt + (c * 64) / GF_TILE, kept);
        {
            const u64 bd = __ballot(deferred);
            if (bd) {
                u32 base = 0;
                if (lane == 0) base = atomicAdd(g.fb_count, (u32)__popcll(bd));
                base = __shfl(base, 0);
                if (deferred)
                    g.fb_list[base + __builtin_amdgcn_mbcnt_hi((u32)(bd >> 32), __builtin_amdgcn_mbcnt_lo((u32)bd, 0))] = (u32)d;
            }
        }
        if (a.enc) {
            __builtin_amdgcn_wave_barrier();
            const u64 w0 = c * 64;
            const u32 cnt = (u32)(n - w0 < 64 ? n - w0 : 64);
            u8* dst = a.enc + w0 * nb;
            const u32 bytes = cnt * nb;
            if ((((u64)dst) & 3) == 0) {
                const u32 nw = bytes >> 2;
                for (u32 k = lane; k < nw; k += 64) ((u32*)dst)[k] = ((const u32*)wenc)[k];
                for (u32 k = 4 * nw + lane; k < bytes; k += 64) dst[k] = wenc[k];
            } else {
                for (u32 k = lane; k < bytes; k += 64) dst[k] = wenc[k];
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (PF == 2) {
            A = B;
            B = Nx;
        } else {
            A = Nx;
        }
    }
}

// The deferred deltas (a head that needs its blob: XYZ/XYM/XYZM or NaN envelopes): both sides decoded
// again with the blob path, codes and the index envelope rewritten, and the tile's kept count
// corrected — k_gf_heads counted them as kept (FALLBACK), the final codes may not be.
__global__ __launch_bounds__(256) void k_gf_fb(GfArgs a, GfHeadArgs g) {
    const u32 cnt = *g.fb_count;
    const int nb = a.bits / 2;
    const double vmax = (double)((1ull << a.bits) - 1);
    for (u32 x = blockIdx.x * 256 + threadIdx.x; x < cnt; x += gridDim.x * 256) {
        const u64 d = g.fb_list[x];
        const uint2 pr = head_slots(g, ((const uint2*)a.pairs)[d], d);
        const HeadLd L0 = load_head(g, 0, pr.x), L1 = load_head(g, 1, pr.y);
        GHit h;
        decode_head(a, g, 0, pr.x, L0, h, d, false);
        const int co = h.code;
        decode_head(a, g, 1, pr.y, L1, h, d, false);
        const int cn = h.code;
        const bool keep = (co >= 1 && co <= 3) || (cn >= 1 && cn <= 3);
        *(u16*)(a.match + 2 * d) = (u16)(co | cn << 8);
        if (a.enc) {
            u8* e = a.enc + d * nb;
            for (int k = 0; k < nb; k++) e[k] = 0;
            u8 ok = 0;
            if (cn != GF_NONE && cn != GF_FALLBACK && h.r >= 0)
                ok = index_env(h.r, h.pc, h.e, h.e, h.empty, a.bits, vmax, [&](int k, u8 v) { e[k] = v; });
            a.enc_ok[d] = ok;
        }
        if (!keep) atomicSub(a.tile_cnt + d / GF_TILE, 1u);
    }
}

// one block: exclusive scan of the tile counts in place, the total to *n_keep.  GF_SPT counts per
// thread, contiguous, loaded together (16-B loads where whole): one pass up to 8,192 tiles = 33.5M
// deltas, instead of 1,024-tile chunks each behind the previous chunk's barrier
constexpr int GF_SPT = 8;
__global__ __launch_bounds__(1024) void k_gf_scan(u32* __restrict__ cnt, u32 ntiles, u64* __restrict__ n_keep) {
    __shared__ u32 s_w[16];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    u32 carry = 0;
    for (u32 base = 0; base < ntiles; base += 1024 * GF_SPT) {  // (block-uniform)
        const u32 i0 = base + (u32)tid * GF_SPT;
        const bool whole = i0 + GF_SPT <= ntiles;
        u32 x[GF_SPT];
        if (whole) {
            const u32x4* c4 = (const u32x4*)(cnt + i0);
#pragma unroll
            for (int j = 0; j < GF_SPT / 4; j++) {
                const u32x4 v = c4[j];
                x[4 * j] = v.x; x[4 * j + 1] = v.y; x[4 * j + 2] = v.z; x[4 * j + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < GF_SPT; j++) x[j] = i0 + j < ntiles ? cnt[i0 + j] : 0u;
        }
        u32 t = 0;
#pragma unroll
        for (int j = 0; j < GF_SPT; j++) t += x[j];
        u32 s = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
        if (lane == 63) s_w[wid] = s;
        __syncthreads();
        u32 wp = 0, all = 0;
#pragma unroll
        for (int w = 0; w < 16; w++) {
            if (w < wid) wp += s_w[w];
            all += s_w[w];
        }
        u32 e = carry + wp + s - t;
        if (whole) {
            u32x4* c4 = (u32x4*)(cnt + i0);
#pragma unroll
            for (int j = 0; j < GF_SPT / 4; j++) {
                u32x4 o;
                o.x = e; e += x[4 * j];
                o.y = e; e += x[4 * j + 1];
                o.z = e; e += x[4 * j + 2];
                o.w = e; e += x[4 * j + 3];
                c4[j] = o;
            }
        } else {
#pragma unroll
            for (int j = 0; j < GF_SPT; j++) {
                if (i0 + j < ntiles) cnt[i0 + j] = e;
                e += x[j];
            }
        }
        carry += all;
        __syncthreads();
    }
    if (tid == 0) *n_keep = carry;
}

// kept delta indices in key order: tile base (scanned) + rank inside the tile
__global__ __launch_bounds__(GF_NT) void k_gf_place(const u8* __restrict__ match, u64 cap, const u64* __restrict__ d_n,
                                                    const u32* __restrict__ tile_base, u32* __restrict__ keep) {
    __shared__ u32 s_w[GF_NT / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const u64 n = d_n ? *d_n : cap;
    const u64 t0 = (u64)blockIdx.x * GF_TILE;
    u32 run = tile_base[blockIdx.x];
    for (int r = 0; r < GF_ROUNDS; r++) {
        const u64 d0 = t0 + (u64)r * GF_NT;
        if (d0 >= n) break;
        const u64 d = d0 + tid;
        bool k = false;
        if (d < n) {
            const u16 m = *(const u16*)(match + 2 * d);
            const u32 co = m & 0xff, cn = m >> 8;
            k = (co >= 1 && co <= 3) || (cn >= 1 && cn <= 3);
        }
        const u64 bal = __ballot(k);
        if (lane == 0) s_w[wid] = (u32)__popcll(bal);
        __syncthreads();
        u32 wp = 0, all = 0;
#pragma unroll
        for (int w = 0; w < GF_NT / 64; w++) {
            if (w < wid) wp += s_w[w];
            all += s_w[w];
        }
        if (k) keep[run + wp + __builtin_amdgcn_mbcnt_hi((u32)(bal >> 32), __builtin_amdgcn_mbcnt_lo((u32)bal, 0))] = (u32)d;
        run += all;
        __syncthreads();
    }
}


// Delta-order heads: delta d's old and new heads copied to slot d of two contiguous arrays (the
// layout the drop-in's blob reader hands over: it reads the deltas' blobs after classification), and
// its pair rewritten to (d | NONE, d | NONE).  One lane per delta, three 16-B loads and stores per side.
__global__ __launch_bounds__(256) void k_gh_gather(const kd_geom_head* __restrict__ ho, u64 no, const kd_geom_head* __restrict__ hn,
                                                   u64 nn, const uint2* __restrict__ pairs, u64 cap, const u64* __restrict__ d_n,
                                                   kd_geom_head* __restrict__ oo, kd_geom_head* __restrict__ on,
                                                   uint2* __restrict__ opairs) {
    const u64 n = d_n ? min(*d_n, cap) : cap;
    for (u64 d = (u64)blockIdx.x * 256 + threadIdx.x; d < n; d += (u64)gridDim.x * 256) {
        const uint2 p = pairs[d];
        const bool a = p.x != KD_NONE && (u64)p.x < no, b = p.y != KD_NONE && (u64)p.y < nn;
        if (a) {
            const u32x4* src = (const u32x4*)(ho + p.x);
            u32x4* dst = (u32x4*)(oo + d);
            const u32x4 x0 = src[0], x1 = src[1], x2 = src[2];
            dst[0] = x0; dst[1] = x1; dst[2] = x2;
        }
        if (b) {
            const u32x4* src = (const u32x4*)(hn + p.y);
            u32x4* dst = (u32x4*)(on + d);
            const u32x4 y0 = src[0], y1 = src[1], y2 = src[2];
            dst[0] = y0; dst[1] = y1; dst[2] = y2;
        }
        // a side without a head in range keeps an index past the heads: the filter's FALLBACK
        opairs[d] = make_uint2(p.x == KD_NONE ? KD_NONE : a ? (u32)d : 0xFFFFFFFEu,
                               p.y == KD_NONE ? KD_NONE : b ? (u32)d : 0xFFFFFFFEu);
    }
}

// the launches and result copies shared by kd_geom_filter (arenas) and kd_geom_filter_heads (heads)
static int gf_run(kd_ctx* ctx, GfArgs& a, const GfHeadArgs* g, const uint32_t* pairs, uint64_t n, const uint64_t* d_n,
                  uint32_t pairs_mem, const double filt_env[4], uint32_t flags, int bits, uint8_t* match, uint32_t* keep,
                  uint64_t* n_keep, uint8_t* enc, uint8_t* enc_ok, uint32_t out_mem) {
    int rc;
    const void* dp;
    if ((rc = stage_in(ctx, "gf.pairs", n ? (const void*)pairs : nullptr, n ? n * 8 : 0, pairs_mem, &dp))) return rc;
    const u64 tiles = (n + GF_TILE - 1) / GF_TILE;
    KD_CHECK(tiles < (1ull << 31), "kd_geom_filter: too many deltas");
    u8* dm = match;
    u32* dk = keep;
    u8 *de = enc, *dok = enc_ok;
    const int nb = bits / 2;
    void *t_cnt, *t_nk;
    if ((rc = ensure(ctx, "gf.tiles", (tiles + 1) * 4, &t_cnt)) || (rc = ensure(ctx, "gf.nk", 8, &t_nk))) return rc;
    if (out_mem == KD_MEM_HOST) {
        void *x, *y, *z = nullptr, *w = nullptr;
        if ((rc = ensure(ctx, "gf.match", 2 * n + 2, &x)) || (rc = ensure(ctx, "gf.keep", 4 * n + 4, &y))) return rc;
        if (enc && ((rc = ensure(ctx, "gf.enc", n * nb + 4, &z)) || (rc = ensure(ctx, "gf.encok", n + 4, &w)))) return rc;
        dm = (u8*)x; dk = (u32*)y; de = (u8*)z; dok = (u8*)w;
    }
    a.pairs = (const u32*)dp;
    a.cap = n;
    a.d_n = d_n;
    a.f0 = filt_env[0]; a.f1 = filt_env[1]; a.f2 = filt_env[2]; a.f3 = filt_env[3];
    a.rect = (flags & KD_GF_RECT) ? 1 : 0;
    a.bits = enc ? bits : 2;
    a.match = dm;
    a.enc = enc ? de : nullptr;
    a.enc_ok = enc ? dok : nullptr;
    a.tile_cnt = (u32*)t_cnt;
    // the kept count goes straight to the caller's device word (no copy after the scan); the scan
    // writes it whenever there are tiles, so only an empty call sets it here
    u64* const nk_dst = out_mem == KD_MEM_DEVICE ? n_keep : (u64*)t_nk;
    if (!tiles) KD_HIP(hipMemsetAsync(nk_dst, 0, 8, ctx->stream));
    GfHeadArgs gh{};
    if (g) {
        gh = *g;
        if (gh.pres_only) gh.bpairs = (const uint2*)dp;  // the blob of each side: the pairs themselves
        // with blob arenas, heads that need their blob are deferred to k_gf_fb
        if (gh.data[0] && gh.data[1] && n) {
            void *fl, *fc;
            if ((rc = ensure(ctx, "gf.fblist", n * 4 + 4, &fl)) || (rc = ensure(ctx, "gf.fbcnt", 16, &fc))) return rc;
            gh.fb_list = (u32*)fl;
            gh.fb_count = (u32*)fc;
            KD_HIP(hipMemsetAsync(fc, 0, 4, ctx->stream));
        }
    }
    if (tiles) {
        if (g && gh.dense) {
            // prefetch depth 1, strided loads (r4w on the C5 mix: 1-deep strided 0.320 ms, 2-deep 0.334,
            // 2-deep transposed through LDS 0.338, 1-deep transposed 0.346; k_gf_heads 0.355)
            KD_HIP(hipMemsetAsync(t_cnt, 0, tiles * 4, ctx->stream));
            const int occ = occupancy(ctx, (const void*)k_gf_dense<KD_GFD_PF, KD_GFD_TR>, GF_NT, 0);
            const u64 nchunk = (n + 63) / 64;
            const u64 grid = std::max<u64>(1, std::min<u64>((nchunk + 3) / 4, (u64)ctx->n_cu * (u64)occ));
            if ((rc = launch(ctx, "k_gf_heads", [&] {
                     hipLaunchKernelGGL((k_gf_dense<KD_GFD_PF, KD_GFD_TR>), dim3((unsigned)grid), dim3(GF_NT), 0, ctx->stream, a, gh);
                 })))
                return rc;
            if (gh.fb_list && (rc = launch(ctx, "k_gf_fb", [&] {
                                   const unsigned fgrid = (unsigned)std::max<u64>(1, std::min<u64>((n + 255) / 256, (u64)ctx->n_cu * 2));
                                   hipLaunchKernelGGL(k_gf_fb, dim3(fgrid), dim3(256), 0, ctx->stream, a, gh);
                               })))
                return rc;
        } else if (g) {
            const int occ_heads = occupancy(ctx, (const void*)k_gf_heads, GF_NT, 0);  // resident workgroups per CU
            const u64 hgrid = std::min<u64>(tiles, (u64)ctx->n_cu * (u64)occ_heads);  // (one block per tile: 0.345 vs 0.353 ms, r4v)
            if ((rc = launch(ctx, "k_gf_heads", [&] {
                     hipLaunchKernelGGL(k_gf_heads, dim3((unsigned)hgrid), dim3(GF_NT), 0, ctx->stream, a, gh);
                 })))
                return rc;
            if (gh.fb_list && (rc = launch(ctx, "k_gf_fb", [&] {
                                   const unsigned grid = (unsigned)std::max<u64>(1, std::min<u64>((n + 255) / 256, (u64)ctx->n_cu * 2));
                                   hipLaunchKernelGGL(k_gf_fb, dim3(grid), dim3(256), 0, ctx->stream, a, gh);
                               })))
                return rc;
        } else if ((rc = launch(ctx, "k_gf_match", [&] {
                        hipLaunchKernelGGL(k_gf_match<KD_GF_STAGE != 0>, dim3((unsigned)tiles), dim3(GF_NT), 0, ctx->stream, a);
                    })))
            return rc;
        if ((rc = launch(ctx, "k_gf_scan", [&] {
                 hipLaunchKernelGGL(k_gf_scan, dim3(1), dim3(1024), 0, ctx->stream, (u32*)t_cnt, (u32)tiles, nk_dst);
             })))
            return rc;
        if ((rc = launch(ctx, "k_gf_place", [&] {
                 hipLaunchKernelGGL(k_gf_place, dim3((unsigned)tiles), dim3(GF_NT), 0, ctx->stream, (const u8*)dm, n, d_n,
                                    (const u32*)t_cnt, dk);
             })))
            return rc;
    }
    if (out_mem == KD_MEM_DEVICE) return KD_OK;
    u64 nk = 0;
    KD_HIP(hipMemcpyAsync(&nk, t_nk, 8, hipMemcpyDeviceToHost, ctx->stream));
    KD_HIP(hipStreamSynchronize(ctx->stream));
    if (n) {
        KD_HIP(hipMemcpyAsync(match, dm, 2 * n, hipMemcpyDeviceToHost, ctx->stream));
        if (nk) KD_HIP(hipMemcpyAsync(keep, dk, 4 * nk, hipMemcpyDeviceToHost, ctx->stream));
        if (enc) {
            KD_HIP(hipMemcpyAsync(enc, de, n * nb, hipMemcpyDeviceToHost, ctx->stream));
            KD_HIP(hipMemcpyAsync(enc_ok, dok, n, hipMemcpyDeviceToHost, ctx->stream));
        }
    }
    KD_HIP(hipStreamSynchronize(ctx->stream));
    *n_keep = nk;
    return prof_flush(ctx);
}

}  // namespace kd

using namespace kd;

extern "C" int kd_geom_filter(kd_ctx* ctx, const kd_blobs* old_blobs, const kd_blobs* new_blobs, const uint32_t* pairs,
                              uint64_t n, const uint64_t* d_n, uint32_t pairs_mem, const kd_geom_cols* cols,
                              const double filt_env[4], uint32_t flags, int bits, uint8_t* match, uint32_t* keep,
                              uint64_t* n_keep, uint8_t* enc, uint8_t* enc_ok, uint32_t out_mem) {
    KD_CHECK(ctx && old_blobs && new_blobs && cols && filt_env && match && keep && n_keep, "kd_geom_filter: NULL argument");
    KD_CHECK(n == 0 || pairs, "kd_geom_filter: pairs NULL");
    KD_CHECK(d_n == nullptr || (out_mem == KD_MEM_DEVICE && pairs_mem == KD_MEM_DEVICE),
             "kd_geom_filter: a device count needs device pairs and outputs");
    KD_CHECK(filt_env[0] <= filt_env[1] && filt_env[2] <= filt_env[3], "kd_geom_filter: inverted filter envelope");
    KD_CHECK(!enc || (enc_ok && bits >= 2 && bits <= 32 && bits % 2 == 0), "kd_geom_filter: bits must be even and <= 32");
    KD_CHECK(cols->n_leg_old >= 0 && cols->n_leg_new >= 0, "kd_geom_filter: legend counts");
    if (cols->n_leg_old > GF_MAXLEG || cols->n_leg_new > GF_MAXLEG) {
        set_error("kd_geom_filter: more than %d legends on a side", GF_MAXLEG);
        return KD_EUNSUPPORTED;
    }
    KD_CHECK(old_blobs->mem == new_blobs->mem, "kd_geom_filter: both arenas in the same memory");
    KD_HIP(hipSetDevice(ctx->device));
    int rc;
    GfArgs a{};
    const kd_blobs* bl[2] = {old_blobs, new_blobs};
    const char* tag[2][2] = {{"gf.od", "gf.oo"}, {"gf.nd", "gf.no"}};
    for (int s = 0; s < 2; s++) {
        const kd_blobs* B = bl[s];
        const void *dd, *doff;
        const u64 bytes = B->mem == KD_MEM_HOST ? (B->n ? B->off[B->n] : 0) : 0;
        if ((rc = stage_in(ctx, tag[s][1], B->off, (B->n + 1) * 8, B->mem, &doff))) return rc;
        if ((rc = stage_in(ctx, tag[s][0], B->data, bytes ? bytes : 1, B->mem, &dd))) return rc;
        a.data[s] = (const u8*)dd;
        a.off[s] = (const u64*)doff;
        a.nblob[s] = B->n;
    }
    // legend tables (host memory, small)
    const int nl[2] = {cols->n_leg_old, cols->n_leg_new};
    const uint8_t* lh[2] = {cols->leg_old_hex, cols->leg_new_hex};
    const int16_t* gx[2] = {cols->gidx_old, cols->gidx_new};
    const char* ltag[2][2] = {{"gf.lo", "gf.go"}, {"gf.ln", "gf.gn"}};
    for (int s = 0; s < 2; s++) {
        KD_CHECK(nl[s] == 0 || (lh[s] && gx[s]), "kd_geom_filter: legend table NULL");
        const void *dl, *dg;
        static const u8 zero16[16] = {0};
        if ((rc = stage_in(ctx, ltag[s][0], nl[s] ? (const void*)lh[s] : zero16, nl[s] ? (size_t)nl[s] * 40 : 16,
                           KD_MEM_HOST, &dl)))
            return rc;
        if ((rc = stage_in(ctx, ltag[s][1], nl[s] ? (const void*)gx[s] : zero16, nl[s] ? (size_t)nl[s] * 2 : 16,
                           KD_MEM_HOST, &dg)))
            return rc;
        a.leg_hex[s] = (const u8*)dl;
        a.gidx[s] = (const i16*)dg;
        a.n_leg[s] = nl[s];
    }
    return gf_run(ctx, a, nullptr, pairs, n, d_n, pairs_mem, filt_env, flags, bits, match, keep, n_keep, enc, enc_ok,
                  out_mem);
}

extern "C" int kd_geom_filter_heads(kd_ctx* ctx, const kd_geom_head* heads_old, uint64_t n_old,
                                    const kd_geom_head* heads_new, uint64_t n_new, uint32_t heads_mem,
                                    const kd_blobs* old_blobs, const kd_blobs* new_blobs, const uint32_t* pairs,
                                    uint64_t n, const uint64_t* d_n, uint32_t pairs_mem, const double filt_env[4],
                                    uint32_t flags, int bits, uint8_t* match, uint32_t* keep, uint64_t* n_keep,
                                    uint8_t* enc, uint8_t* enc_ok, uint32_t out_mem) {
    KD_CHECK(ctx && filt_env && match && keep && n_keep, "kd_geom_filter_heads: NULL argument");
    KD_CHECK((n_old == 0 || heads_old) && (n_new == 0 || heads_new), "kd_geom_filter_heads: heads NULL");
    KD_CHECK(n == 0 || pairs, "kd_geom_filter_heads: pairs NULL");
    KD_CHECK(d_n == nullptr || (out_mem == KD_MEM_DEVICE && pairs_mem == KD_MEM_DEVICE),
             "kd_geom_filter_heads: a device count needs device pairs and outputs");
    KD_CHECK(filt_env[0] <= filt_env[1] && filt_env[2] <= filt_env[3], "kd_geom_filter_heads: inverted filter envelope");
    KD_CHECK(!enc || (enc_ok && bits >= 2 && bits <= 32 && bits % 2 == 0),
             "kd_geom_filter_heads: bits must be even and <= 32");
    KD_CHECK(!old_blobs == !new_blobs, "kd_geom_filter_heads: both arenas or neither");
    KD_HIP(hipSetDevice(ctx->device));
    static_assert(sizeof(kd_geom_head) == 48, "kd_geom_head is 48 bytes");
    int rc;
    GfArgs a{};
    GfHeadArgs g{};
    const kd_geom_head* hs[2] = {heads_old, heads_new};
    const u64 nh[2] = {n_old, n_new};
    const char* htag[2] = {"gh.o", "gh.n"};
    for (int s = 0; s < 2; s++) {
        const void* dh;
        if ((rc = stage_in(ctx, htag[s], nh[s] ? (const void*)hs[s] : nullptr, nh[s] * sizeof(kd_geom_head), heads_mem, &dh)))
            return rc;
        KD_CHECK(((u64)dh & 15) == 0, "kd_geom_filter_heads: heads must be 16-byte aligned");
        g.head[s] = (const kd_geom_head*)dh;
        g.nhead[s] = nh[s];
    }
    {
        void* dz;
        if ((rc = device_zeros(ctx, &dz))) return rc;  // 256 zero bytes
        g.zeros = (const u8*)dz;
    }
    const bool dh = (flags & KD_GF_DELTA_HEADS) != 0;
    if (dh) {  // heads in delta order: slot d is delta d's; the pairs give presence and the blobs
        const u64 slots = (n + 63) / 64 * 64;
        KD_CHECK(nh[0] >= slots && nh[1] >= slots, "kd_geom_filter_heads: KD_GF_DELTA_HEADS needs %llu head slots per side",
                 (unsigned long long)slots);
        g.dense = 1;
        g.pres_only = 1;
    }
    if (old_blobs) {
        const kd_blobs* bl[2] = {old_blobs, new_blobs};
        const char* tag[2][2] = {{"gf.od", "gf.oo"}, {"gf.nd", "gf.no"}};
        for (int s = 0; s < 2; s++) {
            const kd_blobs* B = bl[s];
            KD_CHECK(dh || B->n == nh[s], "kd_geom_filter_heads: arena %d holds %llu blobs, %llu heads", s,
                     (unsigned long long)B->n, (unsigned long long)nh[s]);
            const void *dd, *doff;
            const u64 bytes = B->mem == KD_MEM_HOST ? (B->n ? B->off[B->n] : 0) : 0;
            if ((rc = stage_in(ctx, tag[s][1], B->off, (B->n + 1) * 8, B->mem, &doff))) return rc;
            if ((rc = stage_in(ctx, tag[s][0], B->data, bytes ? bytes : 1, B->mem, &dd))) return rc;
            g.data[s] = (const u8*)dd;
            g.off[s] = (const u64*)doff;
        }
    }
    a.nblob[0] = dh && old_blobs ? old_blobs->n : n_old;
    a.nblob[1] = dh && new_blobs ? new_blobs->n : n_new;
    return gf_run(ctx, a, &g, pairs, n, d_n, pairs_mem, filt_env, flags, bits, match, keep, n_keep, enc, enc_ok, out_mem);
}

extern "C" int kd_geom_filter_deltas(kd_ctx* ctx, const kd_geom_head* heads_old, uint64_t n_old,
                                     const kd_geom_head* heads_new, uint64_t n_new, const kd_blobs* old_blobs,
                                     const kd_blobs* new_blobs, const uint32_t* pairs, uint64_t cap, const uint64_t* d_n,
                                     const double filt_env[4], uint32_t flags, int bits, uint8_t* match, uint32_t* keep,
                                     uint64_t* n_keep, uint8_t* enc, uint8_t* enc_ok) {
    KD_CHECK(ctx && filt_env && match && keep && n_keep && d_n && (cap == 0 || pairs), "kd_geom_filter_deltas: NULL argument");
    KD_CHECK((n_old == 0 || heads_old) && (n_new == 0 || heads_new), "kd_geom_filter_deltas: heads NULL");
    KD_CHECK(filt_env[0] <= filt_env[1] && filt_env[2] <= filt_env[3], "kd_geom_filter_deltas: inverted filter envelope");
    KD_CHECK(!enc || (enc_ok && bits >= 2 && bits <= 32 && bits % 2 == 0),
             "kd_geom_filter_deltas: bits must be even and <= 32");
    KD_CHECK(!old_blobs == !new_blobs, "kd_geom_filter_deltas: both arenas or neither");
    KD_CHECK(cap < 0xFFFFFFF0ull, "kd_geom_filter_deltas: too many deltas");
    KD_CHECK(((u64)heads_old & 15) == 0 && ((u64)heads_new & 15) == 0, "kd_geom_filter_deltas: heads must be 16-byte aligned");
    KD_HIP(hipSetDevice(ctx->device));
    static_assert(sizeof(kd_geom_head) == 48, "kd_geom_head is 48 bytes");
    int rc;
    void* dz;
    if ((rc = device_zeros(ctx, &dz))) return rc;
    GfArgs a{};
    GfHeadArgs g{};
    g.zeros = (const u8*)dz;
    g.dense = 1;
    const uint32_t* fpairs = pairs;  // the pairs the filter reads
    const u64 slots = (cap + 63) / 64 * 64;  // whole 64-delta chunks (k_gf_dense's loads)
    if (flags & KD_GF_DELTA_HEADS) {  // heads already in delta order (the blob reader's layout)
        KD_CHECK(n_old >= slots && n_new >= slots, "kd_geom_filter_deltas: KD_GF_DELTA_HEADS needs %llu head slots per side",
                 (unsigned long long)slots);
        g.head[0] = heads_old;
        g.head[1] = heads_new;
        g.nhead[0] = n_old;
        g.nhead[1] = n_new;
        g.pres_only = 1;  // (bpairs = the pairs, set by gf_run)
    } else {  // per-entry heads: gathered into delta order first (k_gh_gather)
        void *go, *gn, *gp;
        if ((rc = ensure(ctx, "gd.ho", (slots + 1) * sizeof(kd_geom_head), &go))) return rc;
        if ((rc = ensure(ctx, "gd.hn", (slots + 1) * sizeof(kd_geom_head), &gn))) return rc;
        if ((rc = ensure(ctx, "gd.pairs", (cap + 1) * 8, &gp))) return rc;
        if (cap) {
            const unsigned grid = (unsigned)std::max<u64>(1, std::min<u64>((cap + 255) / 256, (u64)ctx->n_cu * 16));
            rc = launch(ctx, "k_gh_gather", [&] {
                hipLaunchKernelGGL(k_gh_gather, dim3(grid), dim3(256), 0, ctx->stream, n_old ? heads_old : (const kd_geom_head*)dz,
                                   n_old, n_new ? heads_new : (const kd_geom_head*)dz, n_new, (const uint2*)pairs, cap, d_n,
                                   (kd_geom_head*)go, (kd_geom_head*)gn, (uint2*)gp);
            });
            if (rc) return rc;
        }
        g.head[0] = (const kd_geom_head*)go;
        g.head[1] = (const kd_geom_head*)gn;
        g.nhead[0] = g.nhead[1] = cap;
        g.bpairs = (const uint2*)pairs;
        fpairs = (const uint32_t*)gp;
    }
    if (old_blobs) {
        const kd_blobs* bl[2] = {old_blobs, new_blobs};
        for (int s = 0; s < 2; s++) {
            KD_CHECK(bl[s]->mem == KD_MEM_DEVICE, "kd_geom_filter_deltas: arenas must be device memory");
            g.data[s] = bl[s]->data;
            g.off[s] = bl[s]->off;
            a.nblob[s] = bl[s]->n;
        }
    }
    return gf_run(ctx, a, &g, fpairs, cap, d_n, KD_MEM_DEVICE, filt_env, flags, bits, match, keep, n_keep, enc, enc_ok,
                  KD_MEM_DEVICE);
}
