// kd_fielddiff.hip — per-update msgpack field decode + column compare with Python `==` semantics.
//
// Replaces, for every update delta, Dataset3.get_feature (kart/dataset3.py:185-223: msg_unpack
// of [legend_hex, [values]] + Legend.value_tuples_to_raw_dict, kart/schema.py:66-79) on both
// sides, Schema.feature_from_raw_dict (schema.py:288-293) and the field loop of
// TextDiffWriter.write_feature_delta (kart/text_diff_writer.py:135-145):
//     changed(k) = old.get(k, _NULL) != new.get(k, _NULL)   for k in old keys ∪ new-only keys.
// The host turns both schemas + every legend into per-legend maps (kartdiff.h kd_legend_maps);
// here one lane walks one update's two blobs.  Value semantics follow msgpack.unpackb(raw=False)
// with the ext hook of kart/serialise_util.py:26-31 and Python's ==:
// ints of any width by value, bool == int, exact int/float compare, IEEE float ==, str/bytes by
// payload, bin == ext 'G' payload, None only == None, empty ext 'G' -> None.
//
// Fast path: when the old and new legend maps are identical (the common case: no schema change)
// both blobs are walked in lockstep with no per-value storage.  Otherwise value offsets go to a
// small per-lane array and keys are resolved through the maps.
#include "kd_internal.h"

namespace kd {

// Blob bytes are read through address-space-qualified pointers: LDS-staged blobs as
// address_space(3) (ds_read, word-wide compares), blobs too large for a slot as address_space(1)
// (global loads).  A generic pointer would turn every byte access into a flat load.
typedef const __attribute__((address_space(3))) u8* lp8;
typedef const __attribute__((address_space(3))) u32* lp32;
typedef const __attribute__((address_space(3))) u32x4* lp128;
typedef const __attribute__((address_space(1))) u8* gp8;

enum : u8 { V_NIL = 0, V_INT = 1, V_FLOAT = 2, V_STR = 3, V_BYTES = 4, V_EXT = 5 };

template <class P>
struct DVal {
    u8 cls;
    u8 big;     // V_INT: value in [2^63, 2^64) held in bits as uint64
    i8 ext;
    u64 bits;   // V_INT: int64 (or uint64 if big); V_FLOAT: double bits
    P p;
    u32 len;
};

// big-endian W-byte integer: the W loads are independent (issued together)
template <int W, class P>
__device__ __forceinline__ u64 ld_be(P p) {
    u64 v = 0;
#pragma unroll
    for (int i = 0; i < W; i++) v = (v << 8) | p[i];
    return v;
}

template <class P>
__device__ __forceinline__ u64 ld_be_w(P p, int w) {
    switch (w) {
    case 1: return ld_be<1>(p);
    case 2: return ld_be<2>(p);
    case 4: return ld_be<4>(p);
    default: return ld_be<8>(p);
    }
}

// decode one value; returns bytes consumed, 0 on malformed / unsupported
template <class P>
__device__ __forceinline__ u32 dv_decode(P p, u32 avail, DVal<P>& v) {
    if (avail == 0) return 0;
    const u8 t = p[0];
    v.big = 0;
    if (t <= 0x7f) { v.cls = V_INT; v.bits = t; return 1; }
    if (t >= 0xe0) { v.cls = V_INT; v.bits = (u64)(i64)(int8_t)t; return 1; }
    if (t >= 0xa0 && t <= 0xbf) {
        u32 n = t & 31;
        if (1 + n > avail) return 0;
        v.cls = V_STR; v.p = p + 1; v.len = n; return 1 + n;
    }
    switch (t) {
    case 0xc0: v.cls = V_NIL; return 1;
    case 0xc2: v.cls = V_INT; v.bits = 0; return 1;
    case 0xc3: v.cls = V_INT; v.bits = 1; return 1;
    case 0xcc: case 0xcd: case 0xce: case 0xcf: {
        int w = 1 << (t - 0xcc);
        if ((u32)(1 + w) > avail) return 0;
        v.cls = V_INT; v.bits = ld_be_w(p + 1, w); v.big = (w == 8 && (v.bits >> 63)) ? 1 : 0;
        return 1 + w;
    }
    case 0xd0: case 0xd1: case 0xd2: case 0xd3: {
        int w = 1 << (t - 0xd0);
        if ((u32)(1 + w) > avail) return 0;
        int sh = 64 - 8 * w;
        v.cls = V_INT; v.bits = (u64)(((i64)(ld_be_w(p + 1, w) << sh)) >> sh);
        return 1 + w;
    }
    case 0xca: {
        if (5 > avail) return 0;
        u32 b = (u32)ld_be<4>(p + 1);
        v.cls = V_FLOAT; v.bits = (u64)__double_as_longlong((double)__uint_as_float(b));
        return 5;
    }
    case 0xcb: {
        if (9 > avail) return 0;
        v.cls = V_FLOAT; v.bits = ld_be<8>(p + 1);
        return 9;
    }
    case 0xd9: case 0xda: case 0xdb: case 0xc4: case 0xc5: case 0xc6: {
        int w = (t == 0xd9 || t == 0xc4) ? 1 : (t == 0xda || t == 0xc5) ? 2 : 4;
        if ((u32)(1 + w) > avail) return 0;
        u64 n = ld_be_w(p + 1, w);
        if ((u64)1 + w + n > avail) return 0;
        v.cls = t >= 0xd9 ? V_STR : V_BYTES; v.p = p + 1 + w; v.len = (u32)n;
        return 1 + w + (u32)n;
    }
    case 0xd4: case 0xd5: case 0xd6: case 0xd7: case 0xd8: case 0xc7: case 0xc8: case 0xc9: {
        u64 n;
        u32 hdr;
        if (t <= 0xd8 && t >= 0xd4) { n = 1u << (t - 0xd4); hdr = 2; }
        else {
            int w = 1 << (t - 0xc7);
            if ((u32)(2 + w) > avail) return 0;
            n = ld_be_w(p + 1, w); hdr = 2 + w;
        }
        if ((u64)hdr + n > avail) return 0;
        v.ext = (i8)p[hdr - 1]; v.p = p + hdr; v.len = (u32)n;
        if (v.ext == 'G') {
            if (n == 0) { v.cls = V_NIL; return hdr; }               // Geometry.of(b"") -> None
            if (n < 2 || v.p[0] != 'G' || v.p[1] != 'P') return 0;  // Geometry() raises
            v.cls = V_BYTES;
        } else {
            v.cls = V_EXT;
        }
        return hdr + (u32)n;
    }
    default: return 0;  // arrays / maps / 0xc1: not field values Kart writes
    }
}

// ---- LDS-staged blobs: branch-free header decode -------------------------------------------------
// Every msgpack type byte maps to one table entry (built at compile time, copied to LDS per block):
//   bits 0-2 class (7 = not a field value), 3-5 header bytes, 6-10 fixed payload bytes (numbers: their
//   width), 11-13 width of a big-endian length field, 14-17 number width (0 = immediate), 18 signed,
//   19 float32, 24-31 immediate value.
// A value is then decoded from one 12-byte window read (two ds_read2_b32 + v_alignbyte) with selects
// and shifts instead of a divergent switch: lanes holding different types (fixint vs uint16, fixstr vs
// str8) stay converged.
struct MpTab {
    u32 e[256];
    static constexpr u32 mk(u32 cls, u32 hdr, u32 plen, u32 lenw, u32 numw, u32 sgn, u32 f32, u32 imm) {
        return cls | hdr << 3 | plen << 6 | lenw << 11 | numw << 14 | sgn << 18 | f32 << 19 | imm << 24;
    }
    constexpr MpTab() : e() {
        for (u32 t = 0; t < 256; t++) {
            u32 v = mk(7, 1, 0, 0, 0, 0, 0, 0);
            if (t <= 0x7f) v = mk(V_INT, 1, 0, 0, 0, 0, 0, t);
            else if (t >= 0xe0) v = mk(V_INT, 1, 0, 0, 0, 1, 0, t);
            else if (t >= 0xa0 && t <= 0xbf) v = mk(V_STR, 1, t & 31, 0, 0, 0, 0, 0);
            else if (t == 0xc0) v = mk(V_NIL, 1, 0, 0, 0, 0, 0, 0);
            else if (t == 0xc2 || t == 0xc3) v = mk(V_INT, 1, 0, 0, 0, 0, 0, t & 1);
            else if (t >= 0xc4 && t <= 0xc6) { u32 w = 1u << (t - 0xc4); v = mk(V_BYTES, 1 + w, 0, w, 0, 0, 0, 0); }
            else if (t >= 0xc7 && t <= 0xc9) { u32 w = 1u << (t - 0xc7); v = mk(V_EXT, 2 + w, 0, w, 0, 0, 0, 0); }
            else if (t == 0xca) v = mk(V_FLOAT, 1, 4, 0, 4, 0, 1, 0);
            else if (t == 0xcb) v = mk(V_FLOAT, 1, 8, 0, 8, 0, 0, 0);
            else if (t >= 0xcc && t <= 0xcf) { u32 w = 1u << (t - 0xcc); v = mk(V_INT, 1, w, 0, w, 0, 0, 0); }
            else if (t >= 0xd0 && t <= 0xd3) { u32 w = 1u << (t - 0xd0); v = mk(V_INT, 1, w, 0, w, 1, 0, 0); }
            else if (t >= 0xd4 && t <= 0xd8) v = mk(V_EXT, 2, 1u << (t - 0xd4), 0, 0, 0, 0, 0);
            else if (t >= 0xd9 && t <= 0xdb) { u32 w = 1u << (t - 0xd9); v = mk(V_STR, 1 + w, 0, w, 0, 0, 0, 0); }
            e[t] = v;
        }
    }
};
__shared__ u32 s_mp[256];

__device__ __forceinline__ void mp_tab_to_lds() {
    constexpr MpTab T{};
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_mp[i] = T.e[i];
}

template <>
__device__ __forceinline__ u32 dv_decode<lp8>(lp8 p, u32 avail, DVal<lp8>& v) {
    const u32 s = (u32)(size_t)p & 3;
    const lp32 a = (lp32)(p - s);
    const u32 a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
    const u32 x0 = __builtin_amdgcn_alignbyte(a1, a0, s), x1 = __builtin_amdgcn_alignbyte(a2, a1, s),
              x2 = __builtin_amdgcn_alignbyte(a3, a2, s);
    const u64 lo = (u64)x0 | (u64)x1 << 32;
    const u32 t = x0 & 0xff;
    const u32 e = s_mp[t];
    u32 cls = e & 7;
    const u32 hdr = (e >> 3) & 7, plen = (e >> 6) & 31, lenw = (e >> 11) & 7, numw = (e >> 14) & 15;
    const u64 be = __builtin_bswap64((lo >> 8) | (u64)x2 << 56);  // bytes 1..8, big-endian
    const u64 lenv = lenw ? be >> (64 - 8 * lenw) : plen;
    u64 nv = numw ? be >> (64 - 8 * numw) : (u64)(e >> 24);
    const u32 sh = 64 - 8 * (numw ? numw : 1);
    if ((e >> 18) & 1) nv = (u64)((i64)(nv << sh) >> sh);
    if ((e >> 19) & 1) nv = (u64)__double_as_longlong((double)__uint_as_float((u32)nv));
    v.bits = nv;
    v.big = (cls == V_INT && !((e >> 18) & 1) && numw == 8 && (nv >> 63)) ? 1 : 0;
    const u32 et = (u32)(lo >> (8 * (hdr - 1))) & 0xff;  // ext type byte (hdr <= 6)
    v.ext = (i8)et;
    const u64 used = hdr + lenv;
    bool ok = cls != 7 && used <= avail;
    if (cls == V_EXT && et == 'G') {  // Geometry: b"" -> None; else must start "GP" (Geometry())
        const u32 g0 = (u32)(lo >> (8 * hdr)) & 0xff, g1 = (u32)(lo >> (8 * hdr + 8)) & 0xff;
        ok = ok && (lenv == 0 || (lenv >= 2 && g0 == 'G' && g1 == 'P'));
        cls = lenv == 0 ? V_NIL : V_BYTES;
    }
    v.cls = (u8)cls;
    v.p = p + hdr;
    v.len = (u32)lenv;
    return ok ? (u32)used : 0;
}

__device__ __forceinline__ bool int_eq_float(u8 big, u64 bits, double d) {
    if (!(d == d)) return false;
    if (floor(d) != d) return false;
    if (big) {
        // value in [2^63, 2^64)
        if (!(d >= 9223372036854775808.0 && d < 18446744073709551616.0)) return false;
        return (u64)d == bits;
    }
    if (!(d >= -9223372036854775808.0 && d < 9223372036854775808.0)) return false;
    return (i64)d == (i64)bits;
}

template <class P>
__device__ bool bytes_eq(P a, P b, u32 n) {
    for (u32 k = 0; k < n; k++)
        if (a[k] != b[k]) return false;
    return true;
}

// LDS: four bytes at a time from aligned words, realigned with v_alignbyte; the aligned reads
// may run up to 4 bytes past either range (still inside the workgroup's LDS allocation, or
// returning 0 past its end) and those bytes are masked off.
__device__ __forceinline__ u32 lds_word(lp32 w, u32 k, u32 s) {
    return __builtin_amdgcn_alignbyte(w[k + 1], w[k], s);
}

#ifndef KD_FD_EXP
#define KD_FD_EXP 0  // profiling builds only: 1 = no parse, 2 = no LDS byte-payload compare
#endif
#ifndef KD_FD_B128
#define KD_FD_B128 0  // 1: 32-B blocks from three 16-B LDS reads per side (measured 2x slower on C3)
#endif
// the 8 dwords starting at byte s (0..15) of a 48-B aligned window: dword shift by selects, byte
// shift by v_alignbyte
__device__ __forceinline__ void window8(const u32x4 w0, const u32x4 w1, const u32x4 w2, u32 s, u32 out[8]) {
    const u32 x[12] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x, w2.y, w2.z, w2.w};
    const u32 d = s >> 2, sb = s & 3;
    u32 t1[11], t2[9];
#pragma unroll
    for (int i = 0; i < 11; i++) t1[i] = (d & 1) ? x[i + 1] : x[i];
#pragma unroll
    for (int i = 0; i < 9; i++) t2[i] = (d & 2) ? t1[i + 2] : t1[i];
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = __builtin_amdgcn_alignbyte(t2[i + 1], t2[i], sb);
}

template <>
__device__ bool bytes_eq<lp8>(lp8 a, lp8 b, u32 n) {
#if KD_FD_EXP == 2
    return a[0] == b[0] || n > 0;
#endif
#if KD_FD_B128
    // 32-byte blocks, each side's 48-B aligned window read as three ds_read_b128 (a third of the
    // LDS instructions of dword reads); reads past the pool return 0 or stay in the allocation
    const u32 sa = (u32)(size_t)a & 15, sb = (u32)(size_t)b & 15;
    lp128 wa = (lp128)(a - sa), wb = (lp128)(b - sb);
    u32 rem = n, diff = 0;
    while (rem > 0 && diff == 0) {
        const u32x4 a0 = wa[0], a1 = wa[1], a2 = wa[2], b0 = wb[0], b1 = wb[1], b2 = wb[2];
        u32 xa[8], xb[8];
        window8(a0, a1, a2, sa, xa);
        window8(b0, b1, b2, sb, xb);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const u32 valid = rem >= 4u * j + 4 ? 0xFFFFFFFFu : rem > 4u * j ? (1u << (8 * (rem - 4 * j))) - 1 : 0u;
            diff |= (xa[j] ^ xb[j]) & valid;
        }
        wa += 2;
        wb += 2;
        rem = rem > 32 ? rem - 32 : 0;
    }
    return diff == 0;
#else
    // 32-byte blocks: the 9 aligned words of each side are read together (one LDS round trip per
    // block, no per-word early exit), realigned with v_alignbyte and compared; bytes past n masked
    const u32 sa = (u32)(size_t)a & 3, sb = (u32)(size_t)b & 3;
    lp32 wa = (lp32)(a - sa), wb = (lp32)(b - sb);
    u32 rem = n, diff = 0;
    while (rem > 0 && diff == 0) {
        u32 xa[9], xb[9];
#pragma unroll
        for (int j = 0; j < 9; j++) { xa[j] = wa[j]; xb[j] = wb[j]; }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const u32 d = __builtin_amdgcn_alignbyte(xa[j + 1], xa[j], sa) ^ __builtin_amdgcn_alignbyte(xb[j + 1], xb[j], sb);
            const u32 valid = rem >= 4u * j + 4 ? 0xFFFFFFFFu : rem > 4u * j ? (1u << (8 * (rem - 4 * j))) - 1 : 0u;
            diff |= d & valid;
        }
        wa += 8;
        wb += 8;
        rem = rem > 32 ? rem - 32 : 0;
    }
    return diff == 0;
#endif
}

template <class P>
__device__ __forceinline__ bool py_eq(const DVal<P>& a, const DVal<P>& b) {
    if (a.cls == V_NIL || b.cls == V_NIL) return a.cls == b.cls;
    if (a.cls == V_INT && b.cls == V_INT) return a.big == b.big && a.bits == b.bits;
    if (a.cls == V_FLOAT && b.cls == V_FLOAT) return __longlong_as_double((i64)a.bits) == __longlong_as_double((i64)b.bits);
    if (a.cls == V_INT && b.cls == V_FLOAT) return int_eq_float(a.big, a.bits, __longlong_as_double((i64)b.bits));
    if (a.cls == V_FLOAT && b.cls == V_INT) return int_eq_float(b.big, b.bits, __longlong_as_double((i64)a.bits));
    if (a.cls != b.cls) return false;
    if (a.cls == V_EXT && a.ext != b.ext) return false;
    return a.len == b.len && bytes_eq(a.p, b.p, a.len);
}

// LDS values: Python == with the scalar cases as selects; only a same-class, same-length byte
// payload pair reaches the (LDS) byte compare.  The branchy generic form cost most of the parse.
__device__ __forceinline__ bool int_eq_float_sel(u8 big, u64 bits, double d) {
    const bool whole = d == d && floor(d) == d;
    const bool in_big = d >= 9223372036854775808.0 && d < 18446744073709551616.0;
    const bool in_small = d >= -9223372036854775808.0 && d < 9223372036854775808.0;
    const double dc_b = in_big ? d : 9223372036854775808.0, dc_s = in_small ? d : 0.0;
    const bool eq_b = in_big && (u64)dc_b == bits, eq_s = in_small && (i64)dc_s == (i64)bits;
    return whole && (big ? eq_b : eq_s);
}

template <>
__device__ __forceinline__ bool py_eq<lp8>(const DVal<lp8>& a, const DVal<lp8>& b) {
    const bool an = a.cls == V_NIL, bn = b.cls == V_NIL;
    const bool ai = a.cls == V_INT, bi = b.cls == V_INT, af = a.cls == V_FLOAT, bf = b.cls == V_FLOAT;
    const double da = __longlong_as_double((i64)a.bits), db = __longlong_as_double((i64)b.bits);
    const bool ii = ai && bi, ff = af && bf, mixed = (ai && bf) || (af && bi);
    const bool r_ii = a.big == b.big && a.bits == b.bits;
    const bool r_ff = da == db;
    const bool r_mx = int_eq_float_sel(ai ? a.big : b.big, ai ? a.bits : b.bits, ai ? db : da);
    const bool num = (ai || af) && (bi || bf);
    const bool r_num = ii ? r_ii : ff ? r_ff : mixed && r_mx;
    const bool byt = !an && !bn && !(ai || af) && a.cls == b.cls && (a.cls != V_EXT || a.ext == b.ext) && a.len == b.len;
    bool eqb = false;
    if (byt) eqb = bytes_eq(a.p, b.p, a.len);
    return (an || bn) ? (an && bn) : num ? r_num : eqb;
}

// header: 0x92, str(40) legend hex, array header -> returns 0 ok
template <class P>
__device__ __forceinline__ int parse_header(P b, u32 n, u32* nvals, u32* off) {
    if (n < 3 || b[0] != 0x92) return 1;
    DVal<P> lv;
    u32 c = dv_decode(b + 1, n - 1, lv);
    if (!c || lv.cls != V_STR || lv.len != 40) return 1;
    u32 o = 1 + c;
    if (o >= n) return 1;
    u8 t = b[o];
    if (t >= 0x90 && t <= 0x9f) { *nvals = t & 15; o += 1; }
    else if (t == 0xdc) { if (o + 3 > n) return 1; *nvals = (u32)ld_be<2>(b + o + 1); o += 3; }
    else if (t == 0xdd) { if (o + 5 > n) return 1; *nvals = (u32)ld_be<4>(b + o + 1); o += 5; }
    else return 1;
    *off = o;
    return 0;
}

// device-side tables (built by the host per call)
// AS = -1: generic pointers into the device copy; AS = 3: the block's LDS copy (small tables)
template <int AS, class T>
struct ASP { typedef const __attribute__((address_space(AS))) T* type; };
template <class T>
struct ASP<-1, T> { typedef const T* type; };
template <int AS>
struct FdTabT {
    int n_keys, words, n_lo, n_ln, maxv;
    typename ASP<AS, u32>::type leg_o;       // [n_lo*10]: 40-byte legend hex strings as words
    typename ASP<AS, u32>::type leg_n;       // [n_ln*10]
    typename ASP<AS, i16>::type map_o;       // [n_lo*n_keys]
    typename ASP<AS, i16>::type map_n;       // [n_ln*n_keys]
    typename ASP<AS, u64>::type cmp;         // [words]
    typename ASP<AS, u8>::type aligned;      // [n_lo*n_ln]: maps identical on every compared key
    typename ASP<AS, i16>::type key_of_val;  // [n_lo*maxv]: union key of value v of legend lo (-1 none)
};
typedef FdTabT<-1> FdTab;
struct FdTabOff {  // byte offsets of the tables inside the packed upload (what an LDS copy rebases)
    u32 leg_o, leg_n, map_o, map_n, cmp, aligned, key_of_val, bytes;
};

// the 40 hex bytes at p (after the 3 header bytes 0x92 0xd9 0x28) as 10 little-endian words
template <class P>
__device__ __forceinline__ void hex_words(P p, u32 w[10]) {
#pragma unroll
    for (int i = 0; i < 10; i++)
        w[i] = (u32)p[4 * i] | (u32)p[4 * i + 1] << 8 | (u32)p[4 * i + 2] << 16 | (u32)p[4 * i + 3] << 24;
}
template <>
__device__ __forceinline__ void hex_words<lp8>(lp8 p, u32 w[10]) {
    const u32 s = (u32)(size_t)p & 3;
    const lp32 a = (lp32)(p - s);
    u32 x[11];
#pragma unroll
    for (int i = 0; i < 11; i++) x[i] = a[i];  // one LDS round trip
#pragma unroll
    for (int i = 0; i < 10; i++) w[i] = __builtin_amdgcn_alignbyte(x[i + 1], x[i], s);
}

template <class P, class TP>
__device__ __forceinline__ int find_legend(TP tab, int n, P hex) {
    u32 h[10];
    hex_words(hex, h);
    for (int l = 0; l < n; l++) {
        u32 x = 0;
#pragma unroll
        for (int i = 0; i < 10; i++) x |= tab[10 * l + i] ^ h[i];
        if (x == 0) return l;
    }
    return -1;
}

constexpr u32 FD_MAXV = 4096;  // oracle limit (status 3 above it)
constexpr int FD_NT = 64;      // one wave per block: each lane owns one update and two LDS slots

__device__ __forceinline__ void set_bit(u64 mk[4], u64* m, int k) {
    const u64 bit = 1ull << (k & 63);
    const int w = k >> 6;  // selects, not a dynamic index: mk stays in registers
    mk[0] |= w == 0 ? bit : 0;
    mk[1] |= w == 1 ? bit : 0;
    mk[2] |= w == 2 ? bit : 0;
    mk[3] |= w == 3 ? bit : 0;
    if (w >= 4) m[w] |= bit;
}

// Value `want` of a blob, walking forward from a cursor (idx, pos); a backward request restarts
// at the first value.  Maps are near-monotone, so a key loop costs about one walk per blob.
template <class P>
__device__ __forceinline__ bool seek_value(P b, u32 n, u32 first, u32 want, u32& idx, u32& pos, DVal<P>& out) {
    if (want < idx) { idx = 0; pos = first; }
    for (;;) {
        u32 c = dv_decode(b + pos, n - pos, out);
        if (!c) return false;
        if (idx == want) return true;
        pos += c;
        idx++;
    }
}

// one update: returns the status; mask bits (k < 256) in mk, the rest straight into m
#ifndef KD_FD_CLOCK
#define KD_FD_CLOCK 0  // profiling builds only: per-phase clock64 printf of sampled waves
#endif
#if KD_FD_CLOCK
__device__ u64 g_fd_dbg[4 * 8192 * 64];
#define FD_DBG(i) g_fd_dbg[4 * ((blockIdx.x % 8192) * 64 + threadIdx.x) + (i)]
#endif
template <class P, class TB>
__device__ __forceinline__ u8 diff_one(P ob, u32 on, P nb, u32 nn, const TB& tb, u64 mk[4], u64* m) {
#if KD_FD_CLOCK
    const u64 D0 = clock64();
    u64 tdec = 0, teq = 0;
#endif
    u32 cvo, cvn, po, pn;
    if (parse_header(ob, on, &cvo, &po) || parse_header(nb, nn, &cvn, &pn)) return 1;
    const int li_o = find_legend(tb.leg_o, tb.n_lo, ob + 3);
    const int li_n = find_legend(tb.leg_n, tb.n_ln, nb + 3);
    if (li_o < 0 || li_n < 0) return 2;
    if (cvo > FD_MAXV || cvn > FD_MAXV) return 3;
    const bool al = tb.aligned[li_o * tb.n_ln + li_n];
    if (al && cvo == cvn) {
        // ---- lockstep: value v of both blobs belongs to the same union key ----
        const auto kov = tb.key_of_val + (u64)li_o * tb.maxv;
        u32 pa = po, pb = pn;
#if KD_FD_CLOCK
        FD_DBG(0) = clock64() - D0;
#endif
        for (u32 v = 0; v < cvo; v++) {
            DVal<P> a, b;
#if KD_FD_CLOCK
            u64 E0 = clock64();
#endif
            const u32 ca = dv_decode(ob + pa, on - pa, a), cb = dv_decode(nb + pb, nn - pb, b);
            if (!ca || !cb) return 4;
            pa += ca;
            pb += cb;
            const int k = v < (u32)tb.maxv ? kov[v] : -1;
#if KD_FD_CLOCK
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            u64 E1 = clock64();
            tdec += E1 - E0;
#endif
            if (k >= 0 && !py_eq(a, b)) set_bit(mk, m, k);
#if KD_FD_CLOCK
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            teq += clock64() - E1;
#endif
        }
#if KD_FD_CLOCK
        FD_DBG(1) = tdec;
        FD_DBG(2) = teq;
        FD_DBG(3) = cvo;
#endif
        if (pa != on || pb != nn) return 4;  // trailing bytes: unpackb raises ExtraData
        return 0;
    }
    // ---- general: validate both blobs (msgpack.unpackb decodes everything first), then
    //      resolve each union key through both maps ----
    u32 p = po;
    for (u32 v = 0; v < cvo; v++) { DVal<P> x; u32 c = dv_decode(ob + p, on - p, x); if (!c) return 4; p += c; }
    if (p != on) return 4;
    p = pn;
    for (u32 v = 0; v < cvn; v++) { DVal<P> x; u32 c = dv_decode(nb + p, nn - p, x); if (!c) return 4; p += c; }
    if (p != nn) return 4;
    const auto mo = tb.map_o + (u64)li_o * tb.n_keys;
    const auto mn = tb.map_n + (u64)li_n * tb.n_keys;
    u32 io = 0, ipo = po, in = 0, ipn = pn;
    for (int k = 0; k < tb.n_keys; k++) {
        if (!((tb.cmp[k >> 6] >> (k & 63)) & 1)) continue;
        const int so = mo[k], sn = mn[k];
        bool changed;
        if (so == -1 || sn == -1) changed = !(so == -1 && sn == -1);
        else if (so == -3 || sn == -3) {
            if (so == -3 && sn == -3) changed = false;
            else return 4;
        } else {
            DVal<P> a, b;
            if (so == -2) a.cls = V_NIL;
            else if ((u32)so >= cvo) return 1;
            else seek_value(ob, on, po, (u32)so, io, ipo, a);
            if (sn == -2) b.cls = V_NIL;
            else if ((u32)sn >= cvn) return 1;
            else seek_value(nb, nn, pn, (u32)sn, in, ipn, b);
            changed = !py_eq(a, b);
        }
        if (changed) set_bit(mk, m, k);
    }
    return 0;
}

constexpr u32 FD_TAB_LDS_MAX = 16384;  // tables up to this size are copied into each block's LDS

// One wave per block, one update per lane.  Per round of 64 updates:
//   1. pair + blob offsets (coalesced pair loads; offset loads per lane);
//   2. cooperative staging: the 64 updates' 2x64 blobs are cut into 16-B chunks and dealt to the lanes
//      so that one wave-instruction reads consecutive chunks of a few blobs (a handful of cache lines)
//      instead of 64 scattered lines — per-lane staging of its own blobs made every load instruction
//      touch 64 lines and the staging dominated the kernel;
//   3. each lane walks its two blobs from LDS (table-driven decoder, tables in LDS).
typedef __attribute__((address_space(3))) void* fd_lds_vp;
typedef const __attribute__((address_space(1))) void* fd_glb_vp;

template <int POOL>
__global__ __launch_bounds__(FD_NT) void k_fielddiff(const u8* __restrict__ od, const u64* __restrict__ ooff,
                                                     const u8* __restrict__ nd, const u64* __restrict__ noff,
                                                     const uint2* __restrict__ pairs, u64 n_upd_host,
                                                     const u64* __restrict__ n_upd_dev, FdTab tg, FdTabOff to,
                                                     const u8* __restrict__ tab_base, u64* __restrict__ masks,
                                                     u8* __restrict__ status) {
    __shared__ u32x4 s_pool[POOL];  // the round's blobs, packed back to back in 16-B chunks
    extern __shared__ __attribute__((aligned(16))) u8 s_tab[];
    const int lane = threadIdx.x;
#if KD_FD_CLOCK
    const u64 WE = wall_clock64();
#endif
    // device count: n_upd_host is the capacity of pairs, so pairs[u] (u < capacity) is loaded
    // before the count arrives; capacity 0 = unknown -> wait for the count first
    const bool spec = n_upd_dev && n_upd_host;
    const u64 n_upd = n_upd_dev ? *n_upd_dev : n_upd_host;
    const u64 lim = spec ? n_upd_host : n_upd;
    // one round ahead: the next round's pair is loaded while this round stages, its blob offsets
    // while this round parses, so a round waits on one HBM latency (the staging) instead of three
    const u64 step = (u64)gridDim.x * FD_NT;
    auto load_pair = [&](u64 uu) {
        uint2 p = make_uint2((u32)uu, (u32)uu);
        if (pairs && uu < lim) p = pairs[uu];
        return p;
    };
    auto load_off = [&](uint2 p, bool a, u64& os_, u64& ns_, u32& on_, u32& nn_) {
        os_ = ns_ = 0;
        on_ = nn_ = 0;
        if (a) {
            os_ = ooff[p.x];
            ns_ = noff[p.y];
            on_ = (u32)(ooff[p.x + 1] - os_);
            nn_ = (u32)(noff[p.y + 1] - ns_);
        }
    };
    u64 u0 = (u64)blockIdx.x * FD_NT;
    u64 os = 0, ns = 0;
    u32 on = 0, nn = 0;
    // (the first round's pair and offsets are in flight while the tables are copied to LDS)
    if (u0 < lim) load_off(load_pair(u0 + lane), u0 + lane < n_upd, os, ns, on, nn);
    typedef const __attribute__((address_space(1))) u32x4* gp;
    for (u32 i = 16 * lane; i < to.bytes; i += 16 * FD_NT) *(u32x4*)(s_tab + i) = *(gp)(tab_base + i);
    mp_tab_to_lds();
    FdTabT<3> tb;
    tb.n_keys = tg.n_keys; tb.words = tg.words; tb.n_lo = tg.n_lo; tb.n_ln = tg.n_ln; tb.maxv = tg.maxv;
    typedef __attribute__((address_space(3))) u8* l8;
    const l8 lt = (l8)s_tab;
    tb.leg_o = (typename ASP<3, u32>::type)(lt + to.leg_o);
    tb.leg_n = (typename ASP<3, u32>::type)(lt + to.leg_n);
    tb.map_o = (typename ASP<3, i16>::type)(lt + to.map_o);
    tb.map_n = (typename ASP<3, i16>::type)(lt + to.map_n);
    tb.cmp = (typename ASP<3, u64>::type)(lt + to.cmp);
    tb.aligned = (typename ASP<3, u8>::type)(lt + to.aligned);
    tb.key_of_val = (typename ASP<3, i16>::type)(lt + to.key_of_val);
    __syncthreads();
    for (; u0 < lim; u0 += step) {
        const u64 u = u0 + lane;
#if KD_FD_CLOCK
        const u64 T0 = clock64(), W0 = wall_clock64();
#endif
        if (u0 >= n_upd) break;  // wave-uniform
        const bool act = u < n_upd;
        const u64 un = u + step;
        const uint2 pr_n = load_pair(un);
        // ---- pool allocation: exclusive wave scan of the lanes' chunk counts ----
        const u64 a0 = (u64)od + os, b0 = (u64)nd + ns;
        const u64 ab = a0 & ~(u64)15, bb = b0 & ~(u64)15;
        const u32 ad = (u32)(a0 - ab), bd = (u32)(b0 - bb);
        const u32 na = act ? (ad + on + 15) >> 4 : 0, nb = act ? (bd + nn + 15) >> 4 : 0;
        const u32 need = na + nb;
        u32 x = need;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        const u32 off = x - need;
        const bool fit = act && x <= (u32)POOL;  // lanes past the pool parse from global memory
        const u64 bal = __ballot(fit);
        const u32 used = bal ? __shfl(x, 63 - __clzll((long long)bal), 64) : 0;  // end of the last fitting lane
        (void)used;
#if KD_FD_CLOCK
        const u64 T1 = clock64();
#endif
        // ---- staging, global -> LDS directly (LDS-DMA): owner lane by owner lane (a wave-uniform
        //      loop, its descriptors read with readlane into SGPRs), lane l loads chunk c0 + l of the
        //      owner's two blobs into pool chunk off + c0 + l (wave-uniform LDS base + 16 l), so
        //      consecutive lanes read consecutive 16-B chunks and every load of the round is in
        //      flight at once, without registers and without LDS reads between the loads ----
        const u32 need_fit = fit ? need : 0u;
        for (int w = 0; w < FD_NT; w++) {
            const u32 need_w = (u32)__builtin_amdgcn_readlane((int)need_fit, w);
            if (need_w == 0) continue;
            const u32 off_w = (u32)__builtin_amdgcn_readlane((int)off, w);
            const u32 na_w = (u32)__builtin_amdgcn_readlane((int)na, w);
            const u64 ab_w = (u64)(u32)__builtin_amdgcn_readlane((int)(u32)ab, w) |
                             (u64)(u32)__builtin_amdgcn_readlane((int)(u32)(ab >> 32), w) << 32;
            const u64 bb_w = (u64)(u32)__builtin_amdgcn_readlane((int)(u32)bb, w) |
                             (u64)(u32)__builtin_amdgcn_readlane((int)(u32)(bb >> 32), w) << 32;
            for (u32 c0 = 0; c0 < need_w; c0 += FD_NT) {
                const u32 c = c0 + lane;
                if (c < need_w) {
                    const u64 src = c < na_w ? ab_w + 16ull * c : bb_w + 16ull * (c - na_w);
                    __builtin_amdgcn_global_load_lds((fd_glb_vp)src, (fd_lds_vp)(s_pool + off_w + c0), 16, 0, 0);
                }
            }
        }
        __syncthreads();
        u64 os_n, ns_n;
        u32 on_n, nn_n;
        load_off(pr_n, un < n_upd, os_n, ns_n, on_n, nn_n);
#if KD_FD_CLOCK
        const u64 T2 = clock64();
#endif
        if (act) {
            u64* m = masks + u * tb.words;
            u64 mk[4] = {0, 0, 0, 0};  // mask words kept in registers for <= 256 keys
            u8 st;
#if KD_FD_EXP == 1
            if (fit) st = ((const u8*)(s_pool + off))[ad] == 7 ? 9 : 0;
#else
            if (fit) st = diff_one((lp8)((const u8*)(s_pool + off) + ad), on, (lp8)((const u8*)(s_pool + off + na) + bd), nn, tb, mk, m);
#endif
            else st = diff_one((gp8)(od + os), on, (gp8)(nd + ns), nn, tb, mk, m);
            if (st) { mk[0] = mk[1] = mk[2] = mk[3] = 0; }
            for (int w = 0; w < tb.words; w++) {
                if (w < 4) m[w] = mk[w];
                else if (st) m[w] = 0;
            }
            status[u] = st;
        }
        __syncthreads();  // the pool is rewritten by the next round
        os = os_n; ns = ns_n; on = on_n; nn = nn_n;
#if KD_FD_CLOCK
        if (lane == 0) printf("FB %u %llu %llu\n", blockIdx.x, (unsigned long long)WE, (unsigned long long)wall_clock64());
        if (lane == 0 && blockIdx.x % 97 == 0) {
            const u64 T3 = clock64(), W3 = wall_clock64();
            printf("FD entry->start %llu entry->end %llu wall %llu (x10ns) start %llu | blk %u offsets %llu staging %llu parse %llu total %llu used %u | hdr %llu dec %llu eq %llu nv %llu\n",
                   (unsigned long long)(W0 - WE), (unsigned long long)(W3 - WE), (unsigned long long)(W3 - W0), (unsigned long long)W0 % 100000000, blockIdx.x, (unsigned long long)(T1 - T0), (unsigned long long)(T2 - T1), (unsigned long long)(T3 - T2),
                   (unsigned long long)(T3 - T0), used, (unsigned long long)FD_DBG(0), (unsigned long long)FD_DBG(1),
                   (unsigned long long)FD_DBG(2), (unsigned long long)FD_DBG(3));
        }
#endif
    }
}

// Fallback for blobs larger than the biggest slot or tables too large for LDS: one lane per update,
// blobs parsed straight from global memory.
__global__ __launch_bounds__(FD_NT) void k_fielddiff_g(const u8* __restrict__ od, const u64* __restrict__ ooff,
                                                       const u8* __restrict__ nd, const u64* __restrict__ noff,
                                                       const uint2* __restrict__ pairs, u64 n_upd_host,
                                                       const u64* __restrict__ n_upd_dev, FdTab tb,
                                                       u64* __restrict__ masks, u8* __restrict__ status) {
    const int lane = threadIdx.x;
    mp_tab_to_lds();
    __syncthreads();
    const bool spec = n_upd_dev && n_upd_host;
    const u64 n_upd = n_upd_dev ? *n_upd_dev : n_upd_host;
    const u64 lim = spec ? n_upd_host : n_upd;
    for (u64 u0 = (u64)blockIdx.x * FD_NT; u0 < lim; u0 += (u64)gridDim.x * FD_NT) {
        const u64 u = u0 + lane;
        uint2 pr = make_uint2((u32)u, (u32)u);
        if (pairs && u < lim) pr = pairs[u];
        if (u0 >= n_upd || u >= n_upd) break;
        const u64 os = ooff[pr.x], ns = noff[pr.y];
        const u32 on = (u32)(ooff[pr.x + 1] - os);
        const u32 nn = (u32)(noff[pr.y + 1] - ns);
        u64* m = masks + u * tb.words;
        u64 mk[4] = {0, 0, 0, 0};
        const u8 st = diff_one((gp8)(od + os), on, (gp8)(nd + ns), nn, tb, mk, m);
        if (st) { mk[0] = mk[1] = mk[2] = mk[3] = 0; }
        for (int w = 0; w < tb.words; w++) {
            if (w < 4) m[w] = mk[w];
            else if (st) m[w] = 0;
        }
        status[u] = st;
    }
}

}  // namespace kd

using namespace kd;

extern "C" int kd_fielddiff(kd_ctx* ctx, const kd_blobs* ob, const kd_blobs* nb, const uint32_t* pu, uint64_t n_upd,
                            const uint64_t* d_n_upd, uint32_t pairs_mem, const kd_legend_maps* mp, uint64_t* masks,
                            uint8_t* status, uint32_t out_mem) {
    KD_CHECK(ctx && ob && nb && mp && masks && status, "kd_fielddiff: NULL argument");
    KD_CHECK(mp->n_keys >= 0 && mp->words == (mp->n_keys + 63) / 64 && mp->words >= 1, "kd_fielddiff: bad words");
    KD_CHECK(mp->n_leg_old > 0 && mp->n_leg_new > 0 && mp->n_leg_old <= 4096 && mp->n_leg_new <= 4096,
             "kd_fielddiff: bad legend counts");
    KD_CHECK(d_n_upd == nullptr || out_mem == KD_MEM_DEVICE, "kd_fielddiff: device count needs device outputs");
    KD_HIP(hipSetDevice(ctx->device));
    int rc;
    // ---- host tables -> device ----
    const int nk = mp->n_keys, nlo = mp->n_leg_old, nln = mp->n_leg_new, W = mp->words;
    // value count per old legend = max value index + 1 over its map (non-pk columns)
    int maxv = 1;
    std::vector<u32> nvo(nlo, 0);
    for (int l = 0; l < nlo; l++)
        for (int k = 0; k < nk; k++) {
            int s = mp->map_old[(size_t)l * nk + k];
            if (s >= 0 && (u32)s + 1 > nvo[l]) nvo[l] = (u32)s + 1;
        }
    for (int l = 0; l < nlo; l++) maxv = std::max<int>(maxv, (int)nvo[l]);
    std::vector<u8> aligned((size_t)nlo * nln, 0);
    for (int a = 0; a < nlo; a++)
        for (int b = 0; b < nln; b++) {
            bool ok = true;
            for (int k = 0; k < nk && ok; k++) {
                if (!((mp->cmp_mask[k >> 6] >> (k & 63)) & 1)) continue;
                int so = mp->map_old[(size_t)a * nk + k], sn = mp->map_new[(size_t)b * nk + k];
                // identical map entries (value index, None or pk on both sides); a _NULL key
                // (absent from a schema) always compares changed, so it forces the general path
                ok = so == sn && so != -1;
            }
            aligned[(size_t)a * nln + b] = ok ? 1 : 0;
        }
    std::vector<i16> kov((size_t)nlo * maxv, -1);
    for (int l = 0; l < nlo; l++)
        for (int k = 0; k < nk; k++) {
            if (!((mp->cmp_mask[k >> 6] >> (k & 63)) & 1)) continue;
            int s = mp->map_old[(size_t)l * nk + k];
            if (s >= 0 && s < maxv) kov[(size_t)l * maxv + s] = (i16)k;
        }
    // one packed upload
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    size_t o_lo = 0, o_ln = al(o_lo + (size_t)nlo * 40), o_mo = al(o_ln + (size_t)nln * 40),
           o_mn = al(o_mo + (size_t)nlo * nk * 2), o_cmp = al(o_mn + (size_t)nln * nk * 2),
           o_al = al(o_cmp + (size_t)W * 8), o_kov = al(o_al + aligned.size()), o_nv = al(o_kov + kov.size() * 2),
           o_end = al(o_nv + (size_t)nlo * 4);
    std::vector<u8> h(o_end, 0);
    std::memcpy(&h[o_lo], mp->leg_old_hex, (size_t)nlo * 40);
    std::memcpy(&h[o_ln], mp->leg_new_hex, (size_t)nln * 40);
    std::memcpy(&h[o_mo], mp->map_old, (size_t)nlo * nk * 2);
    std::memcpy(&h[o_mn], mp->map_new, (size_t)nln * nk * 2);
    std::memcpy(&h[o_cmp], mp->cmp_mask, (size_t)W * 8);
    std::memcpy(&h[o_al], aligned.data(), aligned.size());
    if (!kov.empty()) std::memcpy(&h[o_kov], kov.data(), kov.size() * 2);
    std::memcpy(&h[o_nv], nvo.data(), (size_t)nlo * 4);
    void* dt;
    if ((rc = ensure(ctx, "fd.tab", o_end, &dt))) return rc;
    if (ctx->fd_tab != h) {
        ctx->fd_tab.swap(h);  // keep the source alive until the stream has consumed it
        KD_HIP(hipMemcpyAsync(dt, ctx->fd_tab.data(), o_end, hipMemcpyHostToDevice, ctx->stream));
    }
    FdTab tb;
    tb.n_keys = nk; tb.words = W; tb.n_lo = nlo; tb.n_ln = nln; tb.maxv = maxv;
    const u8* base = (const u8*)dt;
    tb.leg_o = (const u32*)(base + o_lo); tb.leg_n = (const u32*)(base + o_ln);
    tb.map_o = (const i16*)(base + o_mo); tb.map_n = (const i16*)(base + o_mn);
    tb.cmp = (const u64*)(base + o_cmp); tb.aligned = base + o_al;
    tb.key_of_val = (const i16*)(base + o_kov);

    // ---- inputs ----
    const void *d_od, *d_ooff, *d_nd, *d_noff, *d_pu = nullptr;
    u64 ob_bytes = 0, nb_bytes = 0;
    if (ob->mem == KD_MEM_HOST) ob_bytes = ob->off[ob->n];
    if (nb->mem == KD_MEM_HOST) nb_bytes = nb->off[nb->n];
    if ((rc = stage_in(ctx, "fd.ooff", ob->off, (ob->n + 1) * 8, ob->mem, &d_ooff))) return rc;
    if ((rc = stage_in(ctx, "fd.od", ob->data, ob_bytes ? ob_bytes : 1, ob->mem, &d_od))) return rc;
    if ((rc = stage_in(ctx, "fd.noff", nb->off, (nb->n + 1) * 8, nb->mem, &d_noff))) return rc;
    if ((rc = stage_in(ctx, "fd.nd", nb->data, nb_bytes ? nb_bytes : 1, nb->mem, &d_nd))) return rc;
    if (d_n_upd) {
        KD_CHECK(pu == nullptr || pairs_mem == KD_MEM_DEVICE, "kd_fielddiff: device count needs device pairs");
        d_pu = pu;  // device pairs with a device count; n_upd is then the capacity (0 = unknown)
    } else if (pu && n_upd) {
        if ((rc = stage_in(ctx, "fd.pu", pu, n_upd * 8, pairs_mem, &d_pu))) return rc;
    }
    u64 *d_masks = masks;
    u8* d_status = status;
    if (out_mem == KD_MEM_HOST && n_upd && !d_n_upd) {
        void *a, *b;
        if ((rc = ensure(ctx, "fd.masks", n_upd * W * 8, &a))) return rc;
        if ((rc = ensure(ctx, "fd.status", n_upd, &b))) return rc;
        d_masks = (u64*)a;
        d_status = (u8*)b;
    }
    if (n_upd == 0 && d_n_upd == nullptr) return KD_OK;
    // grid-stride: at most one resident wave per LDS-slot set (8 single-wave blocks per CU)
    u64 work = d_n_upd ? (n_upd ? n_upd : (u64)1 << 22) : n_upd;
    // typical blob size: kd_blobs.size_hint, or the mean of host arenas
    auto typical = [](const kd_blobs* b) -> u64 {
        if (b->size_hint) return b->size_hint;
        if (b->mem == KD_MEM_HOST && b->n) return (b->off[b->n] - b->off[0] + b->n - 1) / b->n;
        return 256;
    };
    const u64 typ = std::max(typical(ob), typical(nb));
    FdTabOff to;
    to.leg_o = (u32)o_lo; to.leg_n = (u32)o_ln; to.map_o = (u32)o_mo; to.map_n = (u32)o_mn; to.cmp = (u32)o_cmp;
    to.aligned = (u32)o_al; to.key_of_val = (u32)o_kov; to.bytes = (u32)o_end;
    const bool lds_tab = o_end <= FD_TAB_LDS_MAX;
    // LDS pool for one round of 64 updates: both blobs of every lane packed back to back, sized from
    // the typical (mean) blob — ~(len + 15) / 16 chunks with the 16-B alignment skew — with 10 %
    // headroom (1152 chunks: seven 64-update blocks per CU for ~110-B point features); a lane whose blobs do not fit the round's pool parses them from global memory.
    const u64 per_round = (u64)FD_NT * 2 * (typ + 15) / 16 * 110 / 100;
    int pool = !lds_tab ? 0 : per_round <= 1152 ? 1152 : per_round <= 1536 ? 1536 : per_round <= 2048 ? 2048
                   : per_round <= 3072 ? 3072 : per_round <= 4096 ? 4096 : 0;
#ifndef KD_FD_FORCE_G
#define KD_FD_FORCE_G 0  // profiling builds: 1 = always the global-memory kernel
#endif
#ifndef KD_FD_G_PER_CU
#define KD_FD_G_PER_CU 8  // resident single-wave blocks per CU for the global-memory kernel
#endif
    if (KD_FD_FORCE_G) pool = 0;
    const u64 lds_blk = pool ? (u64)pool * 16 + 1024 + o_end : 1024;
    const u64 per_cu = pool ? std::min<u64>(8, (160 * 1024) / lds_blk) : (u64)KD_FD_G_PER_CU;
    unsigned blocks = (unsigned)std::min<u64>((work + FD_NT - 1) / FD_NT, (u64)ctx->n_cu * per_cu);
    if (blocks == 0) blocks = 1;
    rc = launch(ctx, "k_fielddiff", [&] {
        auto args = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(FD_NT), o_end, ctx->stream, (const u8*)d_od, (const u64*)d_ooff,
                               (const u8*)d_nd, (const u64*)d_noff, (const uint2*)d_pu, n_upd, d_n_upd,
                               tb, to, (const u8*)dt, d_masks, d_status);
        };
        if (pool == 1152) args(k_fielddiff<1152>);
        else if (pool == 1536) args(k_fielddiff<1536>);
        else if (pool == 2048) args(k_fielddiff<2048>);
        else if (pool == 3072) args(k_fielddiff<3072>);
        else if (pool == 4096) args(k_fielddiff<4096>);
        else
            hipLaunchKernelGGL(k_fielddiff_g, dim3(blocks), dim3(FD_NT), 0, ctx->stream, (const u8*)d_od, (const u64*)d_ooff,
                               (const u8*)d_nd, (const u64*)d_noff, (const uint2*)d_pu, n_upd, d_n_upd, tb, d_masks,
                               d_status);
    });
    if (rc) return rc;
    if (out_mem == KD_MEM_HOST) {
        KD_HIP(hipMemcpyAsync(masks, d_masks, n_upd * W * 8, hipMemcpyDeviceToHost, ctx->stream));
        KD_HIP(hipMemcpyAsync(status, d_status, n_upd, hipMemcpyDeviceToHost, ctx->stream));
        KD_HIP(hipStreamSynchronize(ctx->stream));
        prof_flush(ctx);
    }
    return KD_OK;
}
