// kd_fielddiff.hip — per-update msgpack field decode + column compare with Python `==` semantics.
//
// Replaces, for every update delta, Dataset3.get_feature (kart/dataset3.py:185-223: msg_unpack
// of [legend_hex, [values]] + Legend.value_tuples_to_raw_dict, kart/schema.py:66-79) on both
// sides, Schema.feature_from_raw_dict (schema.py:288-293) and the field loop of
// TextDiffWriter.write_feature_delta (kart/text_diff_writer.py:135-145):
//     changed(k) = old.get(k, _NULL) != new.get(k, _NULL)   for k in old keys ∪ new-only keys.
// The host turns both schemas + every legend into per-legend maps (kartdiff.h kd_legend_maps).
// Value semantics follow msgpack.unpackb(raw=False) with the ext hook of
// kart/serialise_util.py:26-31 and Python's ==: ints of any width by value,
// bool == int, exact int/float compare, IEEE float ==, str/bytes by payload, bin == ext 'G'
// payload, None only == None, empty ext 'G' -> None.
//
// k_fielddiff (one wave per workgroup, UPR updates per round, one lane per update):
//   1. LDS windows.  Per blob only a head window (NH 16-B chunks from the blob's aligned start) and a
//      tail window (the NTL aligned chunks ending with the blob's last byte) are
//      copied to LDS by LDS-DMA — the msgpack headers, the legend, and the short values that follow
//      a long one.  Long payloads (geometries) never enter LDS: 17.3 KiB per 52-update round.
//   2. Parse: each lane walks its two blobs value by value from the windows (table-driven header
//      decode from a 12-byte window; bytes outside both windows come from global memory), compares
//      scalars and short payloads in registers or LDS, and queues every byte payload it cannot see
//      whole in LDS as a compare task (old address, new address, length, lane, key).
//   3. Tasks: the wave compares the queued payloads cooperatively, 16 lanes x 16 B per step straight
//      from HBM (coalesced; the new side realigned to the old side's byte offset with a funnel
//      shift), and ORs the changed keys into the owners' masks in LDS.
// Payloads of unequal length are "changed" without reading them.  Tables too large for LDS take
// k_fielddiff_g (one lane per update, everything from global memory).
#include <cstdlib>
#include <type_traits>

#include "kd_internal.h"

namespace kd {

typedef const __attribute__((address_space(3))) u32* lp32;
typedef const __attribute__((address_space(1))) u8* gp8;
typedef const __attribute__((address_space(1))) u32* gp32;
typedef const __attribute__((address_space(1))) u32x4* gp128;

enum : u8 { V_NIL = 0, V_INT = 1, V_FLOAT = 2, V_STR = 3, V_BYTES = 4, V_EXT = 5 };

// ================================================================================================
// generic decoder (global-memory pointers): the large-table fallback kernel k_fielddiff_g
// ================================================================================================
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

// header: 0x92, str(40) legend hex, array header -> returns 0 ok
template <class P>
__device__ __forceinline__ int parse_header(P b, u32 n, u32* nvals, u32* off, u32* lp) {
    if (n < 3 || b[0] != 0x92) return 1;
    DVal<P> lv;
    u32 c = dv_decode(b + 1, n - 1, lv);
    if (!c || lv.cls != V_STR || lv.len != 40) return 1;
    *lp = 1 + c - 40;
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

// ================================================================================================
// device-side tables (built by the host per call)
// ================================================================================================
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

template <class TP>
__device__ __forceinline__ int find_legend_w(TP tab, int n, const u32 h[10]) {
    for (int l = 0; l < n; l++) {
        u32 x = 0;
#pragma unroll
        for (int i = 0; i < 10; i++) x |= tab[10 * l + i] ^ h[i];
        if (x == 0) return l;
    }
    return -1;
}

template <class P, class TP>
__device__ __forceinline__ int find_legend(TP tab, int n, P hex) {
    u32 h[10];
    hex_words(hex, h);
    return find_legend_w(tab, n, h);
}

constexpr u32 FD_MAXV = 4096;  // oracle limit (status 3 above it)
constexpr int FD_NT = 64;      // one wave per block

// MR mask words live in registers (constant indices: selects, not a dynamic index, so mk stays in
// VGPRs); words >= MR are ORed in place
template <int MR = 4>
__device__ __forceinline__ void set_bit(u64 mk[4], u64* m, int k) {
    const u64 bit = 1ull << (k & 63);
    const int w = k >> 6;
#pragma unroll
    for (int i = 0; i < MR; i++) mk[i] |= w == i ? bit : 0;
    if (w >= MR) m[w] |= bit;
}

// the update's mask words: the first MR from registers, the rest were ORed in place and are cleared
// when the update failed
template <int MR = 4>
__device__ __forceinline__ void store_masks(u64* m, int words, const u64 mk[4], u8 st) {
    m[0] = mk[0];
#pragma unroll
    for (int i = 1; i < MR; i++)
        if (words > i) m[i] = mk[i];
    if (st)
        for (int w = MR; w < words; w++) m[w] = 0;
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

// one update from global memory (k_fielddiff_g): returns the status; mask bits (k < 256) in mk,
// the rest straight into m
template <class P, class TB>
__device__ __forceinline__ u8 diff_one(P ob, u32 on, P nb, u32 nn, const TB& tb, u64 mk[4], u64* m) {
    u32 cvo, cvn, po, pn, lpo, lpn;
    if (parse_header(ob, on, &cvo, &po, &lpo) || parse_header(nb, nn, &cvn, &pn, &lpn)) return 1;
    const int li_o = find_legend(tb.leg_o, tb.n_lo, ob + lpo);
    const int li_n = find_legend(tb.leg_n, tb.n_ln, nb + lpn);
    if (li_o < 0 || li_n < 0) return 2;
    if (cvo > FD_MAXV || cvn > FD_MAXV) return 3;
    const bool al = tb.aligned[li_o * tb.n_ln + li_n];
    if (al && cvo == cvn) {
        const auto kov = tb.key_of_val + (u64)li_o * tb.maxv;
        u32 pa = po, pb = pn;
        for (u32 v = 0; v < cvo; v++) {
            DVal<P> a, b;
            const u32 ca = dv_decode(ob + pa, on - pa, a), cb = dv_decode(nb + pb, nn - pb, b);
            if (!ca || !cb) return 4;
            pa += ca;
            pb += cb;
            const int k = v < (u32)tb.maxv ? kov[v] : -1;
            if (k >= 0 && !py_eq(a, b)) set_bit(mk, m, k);
        }
        if (pa != on || pb != nn) return 4;  // trailing bytes: unpackb raises ExtraData
        return 0;
    }
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

// ================================================================================================
// windowed decoder (k_fielddiff)
// ================================================================================================
// Every msgpack type byte maps to one table entry (built at compile time, copied to LDS per block):
//   bits 0-2 class (7 = not a field value), 3-5 header bytes, 6-10 fixed payload bytes (numbers: their
//   width), 11-13 width of a big-endian length field, 14-17 number width (0 = immediate), 18 signed,
//   19 float32, 24-31 immediate value.
// A value is decoded from one 12-byte window (three words) with selects and shifts instead of a
// divergent switch: lanes holding different types (fixint vs uint16, fixstr vs str8) stay converged.
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
__shared__ u32 s_mp[32];  // entries of 0xc0..0xdf; the fix ranges are computed (128 B of LDS, not 1 KiB)

__device__ __forceinline__ void mp_tab_to_lds() {
    constexpr MpTab T{};
    for (int i = threadIdx.x; i < 32; i += blockDim.x) s_mp[i] = T.e[0xc0 + i];
}

__device__ __forceinline__ u32 mp_entry(u32 t) {
    const u32 fix = t < 0x80 ? MpTab::mk(V_INT, 1, 0, 0, 0, 0, 0, 0) | t << 24          // positive fixint
                  : t >= 0xe0 ? MpTab::mk(V_INT, 1, 0, 0, 0, 1, 0, 0) | t << 24       // negative fixint
                  : t >= 0xa0 ? MpTab::mk(V_STR, 1, 0, 0, 0, 0, 0, 0) | (t & 31) << 6  // fixstr
                  : MpTab::mk(7, 1, 0, 0, 0, 0, 0, 0);                                  // fixmap / fixarray
    const u32 tab = s_mp[t & 31];
    return (t >> 5) == 6 ? tab : fix;
}

// One blob of one lane: its bytes in HBM, and the LDS image of its head and tail windows.
//   head: chunks [hb, hb + 16 NH)                      (hb = start rounded down to 16)
//   tail: chunks [tb, tb + 16 NTL), tb = last chunk - 16 (NTL - 1): the NTL chunks ending with the
//         chunk holding the last byte.  A read that starts inside it runs on into the next image
//         (or past the array); the bytes it needs lie inside, as no blob byte follows the window.
// Chunks holding no byte of the blob are not loaded: their LDS bytes are stale, and every decode
// is bounded by the blob length.
template <int NH, int NTL>
struct WBlob {
    static constexpr bool lds_only = false;
    u64 start;  // device address of byte 0
    u32 len;
    u32 s0;     // start - hb (0..15): blob position p is at offset x = p + s0 from hb
    int t0;     // tb - hb (negative for blobs shorter than the tail window)
    u32 img;    // LDS byte address of the image (head chunks, then tail chunks)
    // image offset of the bytes at hb offsets [x, x + n) when they lie in one window, else ~0u
    __device__ __forceinline__ u32 win(u32 x, u32 n) const {
        if (x + n <= 16 * NH) return x;
        const int y = (int)x - t0;
        // the tail window ends with the blob's last byte: a read starting inside it needs no byte
        // past it (what it reads beyond lands in the next image or past the array, and every
        // decoded byte is bounded by the blob length)
        if (y >= 0 && y < 16 * NTL) return 16 * NH + (u32)y;
        return ~0u;
    }
};

// One blob of one lane read straight from global memory (k_fdwalk): no LDS image.  Every read is
// one 16-B load at a byte address (gfx950 runs in unaligned mode: global_load_dwordx4 takes any
// address), so a decode window costs one load and no realignment.  GUARD: the blob lies within 16 B
// of its arena's end (`guard`) — loads then stop at `lim` (aligned dwords below it, realigned), so
// nothing is read past the caller's allocation; every other blob reads unguarded (up to 15 B past its
// end, inside the arena; callers bound every decoded byte by the blob length).
template <bool GUARD>
struct HBlobT {
    static constexpr bool lds_only = false;
    u64 start;
    u32 len;
    bool guard;  // GUARD: this blob's loads are bounded by lim (else unguarded)
    u64 lim;     // end of the arena's valid bytes
};
typedef u32x4 __attribute__((aligned(1))) u32x4_b;
typedef const __attribute__((address_space(1))) u32x4_b* gp128b;

template <bool GUARD>
__device__ __forceinline__ u32x4 h_ld16(const HBlobT<GUARD>& b, u32 p) {
    const u64 x = b.start + p;
    if (!GUARD || !b.guard || x + 16 <= b.lim) return *(gp128b)x;
    const u64 x4 = x & ~3ull;
    const u32 s = (u32)(x & 3);
    u32 w[5];
#pragma unroll
    for (int i = 0; i < 5; i++) w[i] = x4 + 4 * i < b.lim ? ((gp32)x4)[i] : 0u;
    u32x4 r;
    r.x = __builtin_amdgcn_alignbyte(w[1], w[0], s);
    r.y = __builtin_amdgcn_alignbyte(w[2], w[1], s);
    r.z = __builtin_amdgcn_alignbyte(w[3], w[2], s);
    r.w = __builtin_amdgcn_alignbyte(w[4], w[3], s);
    return r;
}

__device__ __forceinline__ u32 lds_u32(u32 addr) { return *(lp32)(size_t)addr; }

// bytes [p, p + 12) of a blob as three little-endian words (bytes past the blob: zero or garbage;
// callers bound every access by the blob length)
#ifndef KD_FD_LDSU
#define KD_FD_LDSU 0  // 1: LDS windows read by byte-addressed ds_read_b128 (measured ~2 % slower than aligned dwords + v_alignbyte)
#endif
typedef const __attribute__((address_space(3))) u32x4_b* lp128b;
__device__ __forceinline__ u32x4 lds_u128(u32 addr) { return *(lp128b)(size_t)addr; }

template <class BL>
__device__ __forceinline__ void rd12(const BL& b, u32 p, u32& x0, u32& x1, u32& x2) {
    const u32 x = p + b.s0, x4 = x & ~3u, s = x & 3;
    if (KD_FD_LDSU) {  // one 16-B read at the byte address (the 4 bytes past the 12 are not used)
        const u32 o = b.win(x, 12);
        if (BL::lds_only || o != ~0u) {
            const u32x4 v = lds_u128(b.img + o);
            x0 = v.x; x1 = v.y; x2 = v.z;
            return;
        }
    }
    u32 w0, w1, w2, w3;
    const u32 o = b.win(x4, 16);
    if (BL::lds_only || o != ~0u) {
        const u32 q = b.img + o;
        w0 = lds_u32(q); w1 = lds_u32(q + 4); w2 = lds_u32(q + 8); w3 = lds_u32(q + 12);
    } else {  // outside both windows: aligned dwords holding a blob byte, from global memory
        const u32 end = b.len + b.s0;
        const gp32 g = (gp32)(b.start - b.s0 + x4);
        w0 = x4 < end ? g[0] : 0;
        w1 = x4 + 4 < end ? g[1] : 0;
        w2 = x4 + 8 < end ? g[2] : 0;
        w3 = x4 + 12 < end ? g[3] : 0;
    }
    x0 = __builtin_amdgcn_alignbyte(w1, w0, s);
    x1 = __builtin_amdgcn_alignbyte(w2, w1, s);
    x2 = __builtin_amdgcn_alignbyte(w3, w2, s);
}

template <bool GUARD>
__device__ __forceinline__ void rd12(const HBlobT<GUARD>& b, u32 p, u32& x0, u32& x1, u32& x2) {
    const u32x4 v = h_ld16(b, p);
    x0 = v.x;
    x1 = v.y;
    x2 = v.z;
}

template <bool GUARD>
__device__ __forceinline__ void rd_legend(const HBlobT<GUARD>& b, u32 lp, u32 h[10]) {
    const u32x4 c0 = h_ld16(b, lp), c1 = h_ld16(b, lp + 16), c2 = h_ld16(b, lp + 32);
    h[0] = c0.x; h[1] = c0.y; h[2] = c0.z; h[3] = c0.w;
    h[4] = c1.x; h[5] = c1.y; h[6] = c1.z; h[7] = c1.w;
    h[8] = c2.x; h[9] = c2.y;
}

// the 40 legend hex bytes at blob position lp as 10 words
template <class BL>
__device__ __forceinline__ void rd_legend(const BL& b, u32 lp, u32 h[10]) {
    const u32 x = lp + b.s0, x4 = x & ~3u, s = x & 3;
    if (KD_FD_LDSU) {
        const u32 o = b.win(x, 40);
        if (BL::lds_only || o != ~0u) {
            const u32x4 c0 = lds_u128(b.img + o), c1 = lds_u128(b.img + o + 16), c2 = lds_u128(b.img + o + 32);
            h[0] = c0.x; h[1] = c0.y; h[2] = c0.z; h[3] = c0.w;
            h[4] = c1.x; h[5] = c1.y; h[6] = c1.z; h[7] = c1.w;
            h[8] = c2.x; h[9] = c2.y;
            return;
        }
    }
    u32 w[11];
    const u32 o = b.win(x4, 44);
    if (BL::lds_only || o != ~0u) {
#pragma unroll
        for (int i = 0; i < 11; i++) w[i] = lds_u32(b.img + o + 4 * i);
    } else {
        const u32 end = b.len + b.s0;
        const gp32 g = (gp32)(b.start - b.s0 + x4);
#pragma unroll
        for (int i = 0; i < 11; i++) w[i] = x4 + 4 * i < end ? g[i] : 0;
    }
#pragma unroll
    for (int i = 0; i < 10; i++) h[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], s);
}

// a decoded value: class, header size and length, and either the number's bits or (byte classes)
// the first 12 payload bytes as they sit in the decode window (short payloads compare from here)
struct WVal {
    u32 meta;  // cls | big << 3 | hdr << 4 | ext << 8
    u32 len;
    u64 bits;  // numbers: int64 (uint64 if big) / double bits; byte classes: payload bytes 0..7
    u32 hi;    // byte classes: payload bytes 8..11
    __device__ __forceinline__ u32 cls() const { return meta & 7; }
    __device__ __forceinline__ u32 big() const { return (meta >> 3) & 1; }
    __device__ __forceinline__ u32 hdr() const { return (meta >> 4) & 15; }
    __device__ __forceinline__ u32 ext() const { return meta >> 8; }
};

__device__ __forceinline__ u32 decode_w(u32 x0, u32 x1, u32 x2, u32 avail, WVal& v) {
    const u64 lo = (u64)x0 | (u64)x1 << 32;
    const u32 t = x0 & 0xff;
    const u32 e = mp_entry(t);
    u32 cls = e & 7;
    const u32 hdr = (e >> 3) & 7, plen = (e >> 6) & 31, lenw = (e >> 11) & 7, numw = (e >> 14) & 15;
    const u64 be = __builtin_bswap64((lo >> 8) | (u64)x2 << 56);  // bytes 1..8, big-endian
    const u64 lenv = lenw ? be >> (64 - 8 * lenw) : plen;
    u64 nv = numw ? be >> (64 - 8 * numw) : (u64)(e >> 24);
    const u32 sh = 64 - 8 * (numw ? numw : 1);
    if ((e >> 18) & 1) nv = (u64)((i64)(nv << sh) >> sh);
    if ((e >> 19) & 1) nv = (u64)__double_as_longlong((double)__uint_as_float((u32)nv));
    const u32 big = (cls == V_INT && !((e >> 18) & 1) && numw == 8 && (nv >> 63)) ? 1 : 0;
    const u32 et = (u32)(lo >> (8 * (hdr - 1))) & 0xff;  // ext type byte (hdr <= 6)
    const u64 used = hdr + lenv;
    bool ok = cls != 7 && used <= avail;
    if (cls == V_EXT && et == 'G') {  // Geometry: b"" -> None; else must start "GP" (Geometry())
        const u32 g0 = (u32)(lo >> (8 * hdr)) & 0xff, g1 = (u32)(lo >> (8 * hdr + 8)) & 0xff;
        ok = ok && (lenv == 0 || (lenv >= 2 && g0 == 'G' && g1 == 'P'));
        cls = lenv == 0 ? V_NIL : V_BYTES;
    }
    const bool num = cls == V_INT || cls == V_FLOAT;
    const unsigned __int128 w = ((unsigned __int128)lo | ((unsigned __int128)x2 << 64)) >> (8 * hdr);
    v.meta = cls | big << 3 | hdr << 4 | et << 8;
    v.len = (u32)lenv;
    v.bits = num ? nv : (u64)w;
    v.hi = (u32)(w >> 64);
    return ok ? (u32)used : 0;
}

// Python == of two decoded values without their payload bytes: 0 equal, 1 changed, 2 the byte
// payloads (same class, same ext code, same length >= 1) decide
__device__ __forceinline__ u32 scalar_eq(const WVal& a, const WVal& b) {
    const u32 ac = a.cls(), bc = b.cls();
    const bool an = ac == V_NIL, bn = bc == V_NIL;
    const bool ai = ac == V_INT, bi = bc == V_INT, af = ac == V_FLOAT, bf = bc == V_FLOAT;
    const double da = __longlong_as_double((i64)a.bits), db = __longlong_as_double((i64)b.bits);
    const bool ii = ai && bi, ff = af && bf, mixed = (ai && bf) || (af && bi);
    const bool r_ii = a.big() == b.big() && a.bits == b.bits;
    const bool r_ff = da == db;
    const bool num = (ai || af) && (bi || bf);
    bool r_num = ii ? r_ii : ff && r_ff;
    if (mixed) r_num = int_eq_float(ai ? a.big() : b.big(), ai ? a.bits : b.bits, ai ? db : da);  // rare
    const bool byt = !an && !bn && !(ai || af) && ac == bc && (ac != V_EXT || a.ext() == b.ext()) && a.len == b.len;
    if (an || bn) return (an && bn) ? 0u : 1u;
    if (num) return r_num ? 0u : 1u;
    if (!byt) return 1u;
    return a.len == 0 ? 0u : 2u;
}

// LDS byte compare: 32-byte blocks, the 9 aligned words of each side read together and realigned
// with v_alignbyte; bytes past n masked (the aligned reads may run up to 4 bytes past either range,
// still inside the block's LDS, or return 0 past its end)
__device__ bool lds_bytes_eq(u32 a, u32 b, u32 n) {
    const u32 sa = a & 3, sb = b & 3;
    u32 wa = a - sa, wb = b - sb;
    u32 rem = n, diff = 0;
    while (rem > 0 && diff == 0) {  // 16-byte blocks: 5 aligned words per side, read together
        u32 xa[5], xb[5];
#pragma unroll
        for (int j = 0; j < 5; j++) { xa[j] = lds_u32(wa + 4 * j); xb[j] = lds_u32(wb + 4 * j); }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const u32 d = __builtin_amdgcn_alignbyte(xa[j + 1], xa[j], sa) ^ __builtin_amdgcn_alignbyte(xb[j + 1], xb[j], sb);
            const u32 valid = rem >= 4u * j + 4 ? 0xFFFFFFFFu : rem > 4u * j ? (1u << (8 * (rem - 4 * j))) - 1 : 0u;
            diff |= d & valid;
        }
        wa += 16;
        wb += 16;
        rem = rem > 16 ? rem - 16 : 0;
    }
    return diff == 0;
}

// LDS byte compare by byte-addressed 16-B reads (the reads may run up to 15 bytes past either range,
// inside the block's LDS, or return 0 past its end; bytes past n are masked)
__device__ bool lds_bytes_eq_u(u32 a, u32 b, u32 n) {
    u32 diff = 0;
    for (u32 o = 0; o < n && diff == 0; o += 16) {
        const u32x4 x = lds_u128(a + o) ^ lds_u128(b + o);
        const u32 r = n - o;
        const u32 m0 = r >= 4 ? ~0u : (1u << (8 * r)) - 1;
        const u32 m1 = r >= 8 ? ~0u : r <= 4 ? 0u : (1u << (8 * (r - 4))) - 1;
        const u32 m2 = r >= 12 ? ~0u : r <= 8 ? 0u : (1u << (8 * (r - 8))) - 1;
        const u32 m3 = r >= 16 ? ~0u : r <= 12 ? 0u : (1u << (8 * (r - 12))) - 1;
        diff = (x.x & m0) | (x.y & m1) | (x.z & m2) | (x.w & m3);
    }
    return diff == 0;
}

// global byte compare by one lane (queue overflow, keys >= 256): aligned dword loads, realigned;
// a dword is loaded only when it holds a byte of its range
__device__ bool glb_bytes_eq(u64 a, u64 b, u32 n) {
    const u32 sa = (u32)(a & 3), sb = (u32)(b & 3);
    const u64 a4 = a - sa, b4 = b - sb, ae = a + n, bend = b + n;
    u32 pa = ((gp32)a4)[0], pb = ((gp32)b4)[0];
    for (u32 k = 0; 4 * k < n; k++) {
        const u64 na = a4 + 4 * (k + 1), nb = b4 + 4 * (k + 1);
        const u32 qa = na < ae ? ((gp32)na)[0] : 0, qb = nb < bend ? ((gp32)nb)[0] : 0;
        const u32 d = __builtin_amdgcn_alignbyte(qa, pa, sa) ^ __builtin_amdgcn_alignbyte(qb, pb, sb);
        const u32 r = n - 4 * k;
        const u32 valid = r >= 4 ? 0xFFFFFFFFu : (1u << (8 * r)) - 1;
        if (d & valid) return false;
        pa = qa;
        pb = qb;
    }
    return true;
}

#ifndef KD_FD_PROBE_NOPARSE
#define KD_FD_PROBE_NOPARSE 0
#endif
#ifndef KD_FD_PROBE_NOCMP
#define KD_FD_PROBE_NOCMP 0
#endif
#ifndef KD_FD_PROBE_NOLDSCMP
#define KD_FD_PROBE_NOLDSCMP 0  // timing probe only (results invalid): in-LDS payload compares skipped
#endif

#ifndef KD_FD_HEADF
#define KD_FD_HEADF 1  // windowed kernel: the fast header read (head_fast) before the general parse
#endif

// Per-round queue of payloads compared cooperatively after the parse (in LDS).
typedef __attribute__((address_space(3))) u64* lds_u64p;
typedef __attribute__((address_space(3))) u32* lds_u32p;
struct FdQueue {
    lds_u64p task;  // [2 * cap]: (old address | lane << 48 | key << 54, new address | len << 48)
    lds_u32p count;
    u32 cap;
};

// queue the compare of n bytes at a against n bytes at b (16 B per task: device addresses below 2^48,
// payloads of 16 B to 64 KiB, keys < 64); false when it does not fit (the caller compares alone)
__device__ __forceinline__ bool task_put(const FdQueue& q, u64 a, u64 b, u32 n, int key) {
    if (!q.cap || key >= 64 || n < 16 || n >= 65536 || ((a | b) >> 48)) return false;
    const u32 t = __hip_atomic_fetch_add(q.count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (t >= q.cap) return false;
    q.task[2 * t] = a | (u64)(threadIdx.x & 63) << 48 | (u64)key << 54;
    q.task[2 * t + 1] = b | (u64)n << 48;
    return true;
}

// bytes [pa, pa + n) of blob A against [pb, pb + n) of blob B: 0 equal, 1 changed, 3 queued for
// the cooperative compare (from the LDS windows when both ranges lie in one, else queued while the
// round's queue has room, else compared by this lane from HBM)
template <class BL>
__device__ __forceinline__ u32 range_eq(const BL& A, u32 pa, const BL& B, u32 pb, u32 n, int key, const FdQueue& q) {
    const u32 ya = pa + A.s0, yb = pb + B.s0;  // offsets from the head bases
    if (KD_FD_LDSU) {
        const u32 oa = A.win(ya, n), ob = B.win(yb, n);
        if (BL::lds_only || (oa != ~0u && ob != ~0u)) {
            if (KD_FD_PROBE_NOLDSCMP) return 0u;
            return lds_bytes_eq_u(A.img + oa, B.img + ob, n) ? 0u : 1u;
        }
    } else {
        const u32 oa = A.win(ya & ~3u, n + 8), ob = B.win(yb & ~3u, n + 8);
        if (BL::lds_only || (oa != ~0u && ob != ~0u)) {
            if (KD_FD_PROBE_NOLDSCMP) return 0u;
            return lds_bytes_eq(A.img + oa + (ya & 3), B.img + ob + (yb & 3), n) ? 0u : 1u;
        }
    }
    const u64 xa = A.start + pa, xb = B.start + pb;
    if (task_put(q, xa, xb, n, key)) return 3;
    return glb_bytes_eq(xa, xb, n) ? 0u : 1u;
}

#ifndef KD_FD_SPLIT
// windowed kernel, 1: a long payload's window parts compared from LDS, only its middle queued (C3v
// 1.49 -> 1.40 ms, but C3 1.30 -> 1.34: its attribute edits compare unchanged geometries either
// way); 2: the prefix only; 0 (default): the whole payload queued
#define KD_FD_SPLIT 0
#endif
// The windowed kernel's payload compare: the parts of the two ranges that lie in both blobs' head
// windows (a prefix) and in both tail windows (a suffix) compare from LDS first — a difference there
// settles the value without any HBM read (a moved vertex changes the GPKG envelope, in the head) —
// and only the middle, which no window holds, is queued for the cooperative compare.  The window
// lines are not fetched a second time after the L2 has turned over (round 5's 1.41x traffic).
template <int NH, int NTL>
__device__ __forceinline__ u32 range_eq(const WBlob<NH, NTL>& A, u32 pa, const WBlob<NH, NTL>& B, u32 pb, u32 n, int key,
                                        const FdQueue& q) {
    const u32 ya = pa + A.s0, yb = pb + B.s0;  // offsets from the head bases
    {
        const u32 oa = A.win(ya & ~3u, n + 8), ob = B.win(yb & ~3u, n + 8);
        if (oa != ~0u && ob != ~0u) {
            if (KD_FD_PROBE_NOLDSCMP) return 0u;
            return lds_bytes_eq(A.img + oa + (ya & 3), B.img + ob + (yb & 3), n) ? 0u : 1u;
        }
    }
    u32 pre = 0, suf = n;
    if (KD_FD_SPLIT) {
        // prefix: the aligned LDS compare of m bytes at y reads head bytes up to (y & ~3) + m + 8
        const int hp = min(16 * NH - 8 - (int)ya, 16 * NH - 8 - (int)yb);
        pre = hp > 0 ? min((u32)hp, n) : 0u;
        // suffix: from the first offset whose aligned start lies in both tail windows (reads past a
        // tail window's end are past its blob's last byte)
        const int ts = max(A.t0 + 3 - (int)ya, B.t0 + 3 - (int)yb);
        suf = KD_FD_SPLIT == 2 ? n : ts <= (int)pre ? pre : ts >= (int)n ? n : (u32)ts;  // 2: the prefix only
        if (pre >= 16 || suf + 16 <= n) {
            bool ne = false;
            if (pre) ne = !lds_bytes_eq(A.img + (ya & ~3u) + (ya & 3), B.img + (yb & ~3u) + (yb & 3), pre);
            if (!ne && suf < n) {
                const u32 za = ya + suf, zb = yb + suf;
                // (the whole suffix's extent: a head window holds it only if it ends inside)
                const u32 oa = A.win(za & ~3u, n - suf + 8), ob = B.win(zb & ~3u, n - suf + 8);
                ne = !lds_bytes_eq(A.img + oa + (za & 3), B.img + ob + (zb & 3), n - suf);
            }
            if (ne) return 1u;
        } else {
            pre = 0;  // too little in the windows to be worth it: the whole range below
            suf = n;
        }
    }
    const u32 m = suf - pre;
    if (m == 0) return 0u;
    const u64 xa = A.start + pa + pre, xb = B.start + pb + pre;
    if (task_put(q, xa, xb, m, key)) return 3;
    return glb_bytes_eq(xa, xb, m) ? 0u : 1u;
}

// bytes [p, p + 16) of a and b differ, counting only the first n (n >= 1)
__device__ __forceinline__ bool chunk_ne(const u32x4& a, const u32x4& b, u32 n) {
    const u32 m0 = n >= 4 ? ~0u : (1u << (8 * n)) - 1;
    const u32 m1 = n >= 8 ? ~0u : n <= 4 ? 0u : (1u << (8 * (n - 4))) - 1;
    const u32 m2 = n >= 12 ? ~0u : n <= 8 ? 0u : (1u << (8 * (n - 8))) - 1;
    const u32 m3 = n >= 16 ? ~0u : n <= 12 ? 0u : (1u << (8 * (n - 12))) - 1;
    return (((a.x ^ b.x) & m0) | ((a.y ^ b.y) & m1) | ((a.z ^ b.z) & m2) | ((a.w ^ b.w) & m3)) != 0;
}

// k_fdwalk's payload compare: up to FD_LOCAL bytes by this lane (every 16-B load of both ranges issued
// before the first compare), longer payloads queued for the wave's cooperative compare while the
// queue has room, else by this lane FD_LOCAL bytes at a time
constexpr u32 FD_LOCAL = 32;
template <bool GUARD>
__device__ __forceinline__ u32 range_eq(const HBlobT<GUARD>& A, u32 pa, const HBlobT<GUARD>& B, u32 pb, u32 n, int key,
                                        const FdQueue& q) {
    if (n > FD_LOCAL && task_put(q, A.start + pa, B.start + pb, n, key)) return 3;
    for (u32 o = 0; o < n; o += FD_LOCAL) {
        u32x4 a[FD_LOCAL / 16], b[FD_LOCAL / 16];
        const u32 r = n - o;
#pragma unroll
        for (int k = 0; k < (int)(FD_LOCAL / 16); k++)
            if (16u * k < r) {
                a[k] = h_ld16(A, pa + o + 16 * k);
                b[k] = h_ld16(B, pb + o + 16 * k);
            }
        bool ne = false;
#pragma unroll
        for (int k = 0; k < (int)(FD_LOCAL / 16); k++)
            if (16u * k < r) ne |= chunk_ne(a[k], b[k], r - 16 * k);
        if (ne) return 1u;
    }
    return 0u;
}

// byte payloads of a and b (same class, ext, length >= 1) at blob positions pa / pb:
// 0 equal, 1 changed, 3 queued
template <class BL>
__device__ __forceinline__ u32 payload_eq(const WVal& a, const BL& A, u32 pa, const WVal& b, const BL& B, u32 pb,
                                          int key, const FdQueue& q) {
    const u32 n = a.len;
    if (a.hdr() + n <= 12 && b.hdr() + n <= 12) {  // whole payload in the decode windows
        const u64 m0 = n >= 8 ? ~0ull : (1ull << (8 * n)) - 1;
        const u32 m1 = n <= 8 ? 0u : (1u << (8 * (n - 8))) - 1;
        return (((a.bits ^ b.bits) & m0) | ((a.hi ^ b.hi) & m1)) ? 1u : 0u;
    }
    return range_eq(A, pa + a.hdr(), B, pb + b.hdr(), n, key, q);
}

// ---- the lockstep fast path: a value's size and class from its type byte alone ----
// Two encodings of one msgpack type byte are equal values (Python ==) exactly when their bytes are
// equal — for nil, bool, every int width, str, bin and ext — except floats (NaN != NaN, -0.0 ==
// 0.0); and two byte-like values (str / bin / ext) of different payload lengths always differ.
// Those cases — nearly every column of every update — are settled from the raw bytes, without the
// number / payload extraction of decode_w; the rest (mixed type bytes: int vs float, str8 vs fixstr,
// ext8 vs bin8 of one length) take decode_w + scalar_eq.
struct FVal {
    u32 t;     // type byte
    u32 cls;   // MpTab class (7 = not a field value)
    u32 hdr;   // header bytes
    u32 len;   // payload length (numbers: their width)
    u32 used;  // hdr + len, 0 = invalid (nested value, truncated, or an ext 'G' that is no GeoPackage)
    u64 be;    // bytes 1..8 big-endian (float bits)
};

__device__ __forceinline__ FVal fast_decode(u32 x0, u32 x1, u32 x2, u32 avail) {
    FVal f;
    f.t = x0 & 0xff;
    const u32 e = mp_entry(f.t);
    f.cls = e & 7;
    f.hdr = (e >> 3) & 7;
    const u32 plen = (e >> 6) & 31, lenw = (e >> 11) & 7;
    const u64 lo = (u64)x0 | (u64)x1 << 32;
    f.be = __builtin_bswap64((lo >> 8) | (u64)x2 << 56);
    f.len = lenw ? (u32)(f.be >> (64 - 8 * lenw)) : plen;
    const u64 used = (u64)f.hdr + f.len;
    bool ok = f.cls != 7 && used <= avail;
    if (f.cls == V_EXT) {  // ext 'G': b"" -> None; else it must start "GP" (Geometry())
        const u32 et = (u32)(lo >> (8 * (f.hdr - 1))) & 0xff;
        const u32 g0 = (u32)(lo >> (8 * f.hdr)) & 0xff, g1 = (u32)(lo >> (8 * f.hdr + 8)) & 0xff;
        ok = ok && (et != 'G' || f.len == 0 || (f.len >= 2 && g0 == 'G' && g1 == 'P'));
    }
    f.used = ok ? (u32)used : 0u;
    return f;
}

// bytes [0, n) of two 12-byte windows differ (n <= 12)
__device__ __forceinline__ bool win_ne(u32 a0, u32 a1, u32 a2, u32 b0, u32 b1, u32 b2, u32 n) {
    const u32 m0 = n >= 4 ? ~0u : (1u << (8 * n)) - 1;
    const u32 m1 = n >= 8 ? ~0u : n <= 4 ? 0u : (1u << (8 * (n - 4))) - 1;
    const u32 m2 = n >= 12 ? ~0u : n <= 8 ? 0u : (1u << (8 * (n - 8))) - 1;
    return (((a0 ^ b0) & m0) | ((a1 ^ b1) & m1) | ((a2 ^ b2) & m2)) != 0;
}

// the fast comparison when it applies: 0 equal, 1 changed, 3 queued; 2 = not settled here
template <class BL>
__device__ __forceinline__ u32 fast_eq(const FVal& a, u32 a0, u32 a1, u32 a2, const BL& A, u32 pa, const FVal& b, u32 b0,
                                       u32 b1, u32 b2, const BL& B, u32 pb, int key, const FdQueue& q) {
    const bool byt_a = a.cls == V_STR || a.cls == V_BYTES || a.cls == V_EXT;
    const bool byt_b = b.cls == V_STR || b.cls == V_BYTES || b.cls == V_EXT;
    if (a.t != b.t) return byt_a && byt_b && a.len != b.len ? 1u : 2u;
    if (a.cls == V_FLOAT) {  // same width: equal bits and not NaN, or both zeros
        const u32 w = a.len;  // 4 or 8
        const u64 xa = a.be >> (64 - 8 * w), xb = b.be >> (64 - 8 * w);
        const u64 mag = w == 8 ? 0x7FFFFFFFFFFFFFFFull : 0x7FFFFFFFull;
        const u64 inf = w == 8 ? 0x7FF0000000000000ull : 0x7F800000ull;
        const bool nan = (xa & mag) > inf;
        return (xa == xb && !nan) || ((xa | xb) & mag) == 0 ? 0u : 1u;
    }
    if (byt_a && a.len != b.len) return 1u;
    if (a.used <= 12) return win_ne(a0, a1, a2, b0, b1, b2, a.used) ? 1u : 0u;
    // a long payload: the equal headers (type, length, ext code) are in the windows; the payloads
    if (win_ne(a0, a1, a2, b0, b1, b2, a.hdr)) return 1u;
    return range_eq(A, pa + a.hdr, B, pb + a.hdr, a.len, key, q);
}

template <class BL>
__device__ __forceinline__ u32 rd_decode(const BL& b, u32 p, WVal& v) {
    u32 x0, x1, x2;
    rd12(b, p, x0, x1, x2);
    return decode_w(x0, x1, x2, b.len - p, v);
}

// header of a windowed blob: 0x92, str(40) legend hex (str8, or a wider str header), array header
// -> 0 ok; *lp = position of the legend hex
template <class BL>
__device__ __forceinline__ int parse_header_w(const BL& b, u32* nvals, u32* off, u32* lp) {
    if (b.len < 44) return 1;
    u32 x0, x1, x2;
    rd12(b, 0, x0, x1, x2);
    if ((x0 & 0xff) != 0x92) return 1;
    const u32 t1 = (x0 >> 8) & 0xff;
    if (t1 == 0xd9 && (x0 >> 16 & 0xff) == 40) *lp = 3;                       // d9 28
    else if (t1 == 0xda && (x0 >> 16) == 0x2800) *lp = 4;                       // da 00 28
    else if (t1 == 0xdb && (x0 >> 16) == 0 && (x1 & 0xffff) == 0x2800) *lp = 6;  // db 00 00 00 28
    else return 1;
    u32 o = *lp + 40;
    if (o >= b.len) return 1;
    rd12(b, o, x0, x1, x2);
    const u32 t = x0 & 0xff;
    const u32 be2 = ((x0 >> 8) & 0xff) << 8 | ((x0 >> 16) & 0xff);
    const u32 be4 = ((x0 >> 8) & 0xff) << 24 | ((x0 >> 16) & 0xff) << 16 | (x0 >> 24) << 8 | (x1 & 0xff);
    if (t >= 0x90 && t <= 0x9f) { *nvals = t & 15; o += 1; }
    else if (t == 0xdc) { if (o + 3 > b.len) return 1; *nvals = be2; o += 3; }
    else if (t == 0xdd) { if (o + 5 > b.len) return 1; *nvals = be4; o += 5; }
    else return 1;
    *off = o;
    return 0;
}

template <class BL>
__device__ __forceinline__ bool seek_value_w(const BL& b, u32 first, u32 want, u32& idx, u32& pos, WVal& out) {
    if (want < idx) { idx = 0; pos = first; }
    for (;;) {
        const u32 c = rd_decode(b, pos, out);
        if (!c) return false;
        if (idx == want) return true;
        pos += c;
        idx++;
    }
}

// one update from its windows: returns the status; mask bits (k < 256) in mk, the rest straight into m
template <int MR, class BL, class TB>
__device__ __forceinline__ u8 diff_body(const BL& A, const BL& B, const TB& tb, u32 cvo, u32 po, u32 cvn, u32 pn,
                                        int li_o, int li_n, u64 mk[4], u64* m, const FdQueue& q);

template <int MR = 4, class BL, class TB>
__device__ __forceinline__ u8 diff_one_w(const BL& A, const BL& B, const TB& tb, u64 mk[4], u64* m, const FdQueue& q) {
    u32 cvo, cvn, po, pn, lpo, lpn;
    if (parse_header_w(A, &cvo, &po, &lpo) || parse_header_w(B, &cvn, &pn, &lpn)) return 1;
    u32 h[10];
    rd_legend(A, lpo, h);
    const int li_o = find_legend_w(tb.leg_o, tb.n_lo, h);
    rd_legend(B, lpn, h);
    const int li_n = find_legend_w(tb.leg_n, tb.n_ln, h);
    return diff_body<MR>(A, B, tb, cvo, po, cvn, pn, li_o, li_n, mk, m, q);
}

// The fast header read: bytes [0, 48) of the blob in one batch — 0x92, the canonical str8 legend
// header d9 28 (what msgpack writes for a 40-char str), the 40 legend bytes and the array header —
// -> 0 ok, 1 malformed (as parse_header_w), -1 another legend header form (the caller takes
// parse_header_w + rd_legend)
// the header checks of head_fast on bytes [0, 48) of a blob as 12 words
__device__ __forceinline__ int head_words(const u32 d[12], u32 len, u32* nvals, u32* off, u32 h[10]) {
    if ((d[0] & 0xff) != 0x92) return 1;
    if ((d[0] & 0xffffff) != 0x28d992) return -1;
#pragma unroll
    for (int i = 0; i < 10; i++) h[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], 3);  // bytes 3..42
    const u32 t = d[10] >> 24;  // byte 43: the array header
    const u32 b44 = d[11] & 0xff, b45 = (d[11] >> 8) & 0xff, b46 = (d[11] >> 16) & 0xff, b47 = d[11] >> 24;
    if (t >= 0x90 && t <= 0x9f) { *nvals = t & 15; *off = 44; return 0; }
    if (t == 0xdc) { if (46 > len) return 1; *nvals = b44 << 8 | b45; *off = 46; return 0; }
    if (t == 0xdd) { if (48 > len) return 1; *nvals = b44 << 24 | b45 << 16 | b46 << 8 | b47; *off = 48; return 0; }
    return 1;
}

// the same from a windowed blob's head window (it holds bytes [0, 48) whenever it spans 64 B: the
// blob starts at most 15 B into it): 13 aligned LDS words, realigned once
template <int NH, int NTL>
__device__ __forceinline__ int head_fast(const WBlob<NH, NTL>& b, u32* nvals, u32* off, u32 h[10]) {
    static_assert(16 * NH >= 64, "head window");
    if (b.len < 44) return 1;
    const u32 s = b.s0 & 3, q = b.img + (b.s0 & ~3u);
    u32 w[13], d[12];
#pragma unroll
    for (int i = 0; i < 13; i++) w[i] = lds_u32(q + 4 * i);
#pragma unroll
    for (int i = 0; i < 12; i++) d[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], s);
    return head_words(d, b.len, nvals, off, h);
}

template <bool GUARD>
__device__ __forceinline__ int head_fast(const HBlobT<GUARD>& b, u32* nvals, u32* off, u32 h[10]) {
    if (b.len < 44) return 1;
    const u32x4 c0 = h_ld16(b, 0), c1 = h_ld16(b, 16), c2 = h_ld16(b, 32);
    const u32 d[12] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w};
    return head_words(d, b.len, nvals, off, h);
}

// one update with the fast header read (head_fast), else as diff_one_w
template <int MR, class BL, class TB>
__device__ __forceinline__ u8 diff_one_f(const BL& A, const BL& B, const TB& tb, u64 mk[4], u64* m, const FdQueue& q) {
    u32 cvo = 0, cvn = 0, po = 0, pn = 0, lp, ha[10], hb[10];
    const int ra = head_fast(A, &cvo, &po, ha), rb = head_fast(B, &cvn, &pn, hb);
    if (ra == 1 || rb == 1) return 1;
    // a non-canonical legend header (str16 / str32): the general header parse
    if (ra < 0) {
        if (parse_header_w(A, &cvo, &po, &lp)) return 1;
        rd_legend(A, lp, ha);
    }
    if (rb < 0) {
        if (parse_header_w(B, &cvn, &pn, &lp)) return 1;
        rd_legend(B, lp, hb);
    }
    const int li_o = find_legend_w(tb.leg_o, tb.n_lo, ha);
    const int li_n = find_legend_w(tb.leg_n, tb.n_ln, hb);
    return diff_body<MR>(A, B, tb, cvo, po, cvn, pn, li_o, li_n, mk, m, q);
}

template <int MR, class BL, class TB>
__device__ __forceinline__ u8 diff_body(const BL& A, const BL& B, const TB& tb, u32 cvo, u32 po, u32 cvn, u32 pn,
                                        int li_o, int li_n, u64 mk[4], u64* m, const FdQueue& q) {
    if (li_o < 0 || li_n < 0) return 2;
    if (cvo > FD_MAXV || cvn > FD_MAXV) return 3;
    const bool al = tb.aligned[li_o * tb.n_ln + li_n];
    if (al && cvo == cvn) {
        // ---- lockstep: value v of both blobs belongs to the same union key ----
        const auto kov = tb.key_of_val + (u64)li_o * tb.maxv;
        u32 pa = po, pb = pn;
        for (u32 v = 0; v < cvo; v++) {
            u32 a0, a1, a2, b0, b1, b2;
            rd12(A, pa, a0, a1, a2);
            rd12(B, pb, b0, b1, b2);
            const FVal fa = fast_decode(a0, a1, a2, A.len - pa), fb = fast_decode(b0, b1, b2, B.len - pb);
            if (!fa.used || !fb.used) return 4;
            const int k = v < (u32)tb.maxv ? kov[v] : -1;
            if (k >= 0) {
                u32 r = fast_eq(fa, a0, a1, a2, A, pa, fb, b0, b1, b2, B, pb, k, q);
                if (r == 2) {  // mixed type bytes: the full decode
                    WVal a, b;
                    decode_w(a0, a1, a2, A.len - pa, a);
                    decode_w(b0, b1, b2, B.len - pb, b);
                    r = scalar_eq(a, b);
                    if (r == 2) r = payload_eq(a, A, pa, b, B, pb, k, q);
                }
                if (r == 1) set_bit<MR>(mk, m, k);
            }
            pa += fa.used;
            pb += fb.used;
        }
        if (pa != A.len || pb != B.len) return 4;  // trailing bytes: unpackb raises ExtraData
        return 0;
    }
    // ---- general: validate both blobs (msgpack.unpackb decodes everything first), then resolve
    //      each union key through both maps ----
    u32 p = po;
    for (u32 v = 0; v < cvo; v++) { WVal x; u32 c = rd_decode(A, p, x); if (!c) return 4; p += c; }
    if (p != A.len) return 4;
    p = pn;
    for (u32 v = 0; v < cvn; v++) { WVal x; u32 c = rd_decode(B, p, x); if (!c) return 4; p += c; }
    if (p != B.len) return 4;
    const auto mo = tb.map_o + (u64)li_o * tb.n_keys;
    const auto mn = tb.map_n + (u64)li_n * tb.n_keys;
    u32 io = 0, ipo = po, in = 0, ipn = pn;
    for (int k = 0; k < tb.n_keys; k++) {
        if (!((tb.cmp[k >> 6] >> (k & 63)) & 1)) continue;
        const int so = mo[k], sn = mn[k];
        u32 r;
        if (so == -1 || sn == -1) r = (so == -1 && sn == -1) ? 0u : 1u;
        else if (so == -3 || sn == -3) {
            if (so == -3 && sn == -3) r = 0;
            else return 4;
        } else {
            WVal a, b;
            a.meta = b.meta = V_NIL;
            a.len = b.len = 0;
            if (so != -2) {
                if ((u32)so >= cvo) return 1;
                seek_value_w(A, po, (u32)so, io, ipo, a);
            }
            if (sn != -2) {
                if ((u32)sn >= cvn) return 1;
                seek_value_w(B, pn, (u32)sn, in, ipn, b);
            }
            r = scalar_eq(a, b);
            if (r == 2) r = payload_eq(a, A, ipo, b, B, ipn, k, q);
        }
        if (r == 1) set_bit<MR>(mk, m, k);
    }
    return 0;
}

// Cooperative compare of M queued payloads by one 16-lane group: lane j of step s takes old chunk
// c = 16 s + j of each payload's aligned range and the matching 16 new bytes (two aligned chunks,
// funnel-shifted by the two sides' relative skew), every payload's loads issued before any compare.
// d[m] = "payload m differs", on every lane of the group.  A chunk is loaded only if it holds a
// byte of its payload (else zeros); an absent payload has n = 0.
template <int M, int G, int S>
__device__ __forceinline__ void coop_differs(const u64 (&a)[M], const u64 (&b)[M], const u32 (&n)[M], bool (&d)[M]) {
    const u32 j = threadIdx.x & (G - 1), grp = (threadIdx.x & 63) / G;
    u32 sa[M], sd[M], nch[M];
    u64 abase[M], ebase[M];
    u32 nmax = 0;
    bool diff[M];
#pragma unroll
    for (int m = 0; m < M; m++) {
        sa[m] = (u32)(a[m] & 15);
        abase[m] = a[m] - sa[m];
        const u64 e = b[m] - sa[m];
        ebase[m] = e & ~(u64)15;
        sd[m] = (u32)(e & 15);
        nch[m] = n[m] ? (n[m] + sa[m] + 15) >> 4 : 0;
        nmax = nch[m] > nmax ? nch[m] : nmax;
        diff[m] = false;
    }
    for (u32 c0 = 0; c0 < nmax; c0 += G * S) {
        u32x4 O[M][S], N0[M][S], N1[M][S];
#pragma unroll
        for (int m = 0; m < M; m++)
#pragma unroll
            for (int s = 0; s < S; s++) {
                const u32 c = c0 + G * s + j;
                const bool act = c < nch[m];
                const u64 oa = abase[m] + 16ull * c, na = ebase[m] + 16ull * c, bend = b[m] + n[m];
                const bool ok0 = act && na < bend && na + 16 > b[m];
                const bool ok1 = act && sd[m] != 0 && na + 16 < bend;
                const u32x4 z = {0, 0, 0, 0};
                O[m][s] = act ? *(gp128)oa : z;
                N0[m][s] = ok0 ? *(gp128)na : z;
                N1[m][s] = ok1 ? *(gp128)(na + 16) : z;
            }
#pragma unroll
        for (int m = 0; m < M; m++)
#pragma unroll
            for (int s = 0; s < S; s++) {
                const u32 c = c0 + G * s + j;
                const u32 q = sd[m] >> 2, sb = sd[m] & 3;
                // dwords q .. q+4 of the 8 new dwords (two select stages on named values: an array
                // here was turned into a dynamically indexed scratch copy)
                const u32x4 P0 = N0[m][s], P1 = N1[m][s];
                const bool s1 = q & 1, s2 = q & 2;
                const u32 b0 = s1 ? P0.y : P0.x, b1 = s1 ? P0.z : P0.y, b2 = s1 ? P0.w : P0.z;
                const u32 b3 = s1 ? P1.x : P0.w, b4 = s1 ? P1.y : P1.x, b5 = s1 ? P1.z : P1.y;
                const u32 b6 = s1 ? P1.w : P1.z;
                const u32 t2[5] = {s2 ? b2 : b0, s2 ? b3 : b1, s2 ? b4 : b2, s2 ? b5 : b3, s2 ? b6 : b4};
                const u32 o[4] = {O[m][s].x, O[m][s].y, O[m][s].z, O[m][s].w};
                // payload bytes of this chunk: t in [lo, hi)
                const int lo = c == 0 ? (int)sa[m] : 0;
                const int hi = (int)n[m] + (int)sa[m] - 16 * (int)c;
                u32 dd = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const u32 nw = __builtin_amdgcn_alignbyte(t2[k + 1], t2[k], sb);
                    const u32 lm = lo >= 4 * k + 4 ? 0u : lo <= 4 * k ? ~0u : ~0u << (8 * (lo - 4 * k));
                    const u32 hm = hi <= 4 * k ? 0u : hi >= 4 * k + 4 ? ~0u : (1u << (8 * (hi - 4 * k))) - 1;
                    dd |= (o[k] ^ nw) & lm & hm;
                }
                diff[m] |= c < nch[m] && dd != 0;
            }
    }
#pragma unroll
    for (int m = 0; m < M; m++) d[m] = ((__ballot(diff[m]) >> (G * grp)) & ((1ull << G) - 1)) != 0;
}

// Cooperative compare of M queued payloads by one G-lane group with byte-addressed 16-B loads (gfx950
// runs in unaligned mode): lane j of step s compares chunk c = G s + j of both payloads at the same
// payload offset min(16 c, n - 16) — the last chunk overlaps the one before it instead of running
// past the payload, so every byte read lies inside both payloads and nothing is masked or
// realigned.  Queued payloads are at least 16 B long (task_put); d[m] = "payload m differs", on
// every lane of the group; an absent payload has n = 0.
template <int M, int G, int S>
__device__ __forceinline__ void coop_differs_u(const u64 (&a)[M], const u64 (&b)[M], const u32 (&n)[M], bool (&d)[M]) {
    const u32 j = threadIdx.x & (G - 1), grp = (threadIdx.x & 63) / G;
    u32 nmax = 0;
    u32 diff[M];
#pragma unroll
    for (int m = 0; m < M; m++) {
        nmax = n[m] > nmax ? n[m] : nmax;
        diff[m] = 0;
    }
    for (u32 c0 = 0; 16 * c0 < nmax; c0 += G * S) {
        u32x4 A[M][S], B[M][S];
#pragma unroll
        for (int m = 0; m < M; m++)
#pragma unroll
            for (int s = 0; s < S; s++) {
                const u32 o = 16 * (c0 + G * s + j);
                const u32 off = min(o, n[m] - 16);
                const u32x4 z = {0, 0, 0, 0};
                A[m][s] = o < n[m] ? *(gp128b)(a[m] + off) : z;
                B[m][s] = o < n[m] ? *(gp128b)(b[m] + off) : z;
            }
#pragma unroll
        for (int m = 0; m < M; m++)
#pragma unroll
            for (int s = 0; s < S; s++) {
                const u32x4 x = A[m][s] ^ B[m][s];
                diff[m] |= x.x | x.y | x.z | x.w;
            }
    }
#pragma unroll
    for (int m = 0; m < M; m++) d[m] = ((__ballot(diff[m] != 0) >> (G * grp)) & ((1ull << G) - 1)) != 0;
}
#ifndef KD_FD_COOPU
#define KD_FD_COOPU 1  // the queued payloads by byte-addressed loads (0: aligned chunks + funnel shifts)
#endif
template <int M, int G, int S>
__device__ __forceinline__ void coop_cmp(const u64 (&a)[M], const u64 (&b)[M], const u32 (&n)[M], bool (&d)[M]) {
    if (KD_FD_COOPU) coop_differs_u<M, G, S>(a, b, n, d);
    else coop_differs<M, G, S>(a, b, n, d);
}

constexpr u32 FD_TAB_LDS_MAX = 16384;
// window shapes (updates per round, head chunks, tail chunks): small features / larger ones
#ifndef KD_FD_SHAPE_L
#ifndef KD_FD_TM_L
#define KD_FD_TM_L 3  // payloads per 16-lane group per pass (C3: 1 / 2 / 3 / 4 = 1.60 / 1.60 / 1.53-1.56 / 2.32 ms)
#endif
#ifndef KD_FD_TGS_L
#define KD_FD_TGS_L 16, 2  // lanes per payload, 16-B steps per lane per pass
#endif
#define KD_FD_SHAPE_L 64, 5, 4, KD_FD_TM_L, KD_FD_TGS_L  // C3 (update-order arenas, round 6): 56 / 60 / 64 updates per round = 1.371 / 1.337 / 1.299 ms
#endif
#ifndef KD_FD_SHAPE_S
#define KD_FD_SHAPE_S 32, 8, 3, 1, 16, 2  // C2 (10M points): tail 2 / 3 chunks = 40.5 / 37.4 us
#endif
template <int UPR, int NH, int NTL, int TM, int TG, int TS>
constexpr int fd_upr(const void*) { return UPR; }  // (the shape macros' first entry)
#ifndef KD_FD_SSHAPE
#define KD_FD_SSHAPE 32, 16384  // streamed kernel: updates per tile, LDS bytes per side
#endif
#ifndef KD_FD_SPF
#define KD_FD_SPF false  // streamed kernel: the next tile's spans prefetched into registers
#endif
#ifndef KD_FD_STREAM_DEFAULT
#define KD_FD_STREAM_DEFAULT 0
#endif
template <int T, int CAPB>
constexpr int fd_stream_t() { return T; }  // tables up to this size are copied into each block's LDS
typedef __attribute__((address_space(3))) void* fd_lds_vp;
typedef const __attribute__((address_space(1))) void* fd_glb_vp;

#ifdef KD_FD_WPE  // probe builds: a waves-per-SIMD floor (the register budget follows from it)
#define KD_FD_ATTR __attribute__((amdgpu_waves_per_eu(KD_FD_WPE)))
#else
#define KD_FD_ATTR
#endif
template <int UPR, int NH, int NTL, int TM, int TG, int TS, int MR>
__global__ __launch_bounds__(FD_NT) KD_FD_ATTR void k_fielddiff(const u8* __restrict__ od, const u64* __restrict__ ooff,
                                                     const u8* __restrict__ nd, const u64* __restrict__ noff,
                                                     const uint2* __restrict__ pairs, u64 n_upd_host,
                                                     const u64* __restrict__ n_upd_dev, FdTab tg, FdTabOff to,
                                                     const u8* __restrict__ tab_base,
                                                     u64* __restrict__ masks, u8* __restrict__ status) {
    constexpr int NC = NH + NTL;       // chunks per blob image
    constexpr int LS = 2 * NC;         // a lane's two images
    constexpr int NCH = (UPR * LS + 63) / 64 * 64;  // image chunks per round (whole instructions)
    constexpr u32 TCAP = UPR;          // queued payload compares per round (then a lane compares alone)
    static_assert(NTL >= 1, "window shape");
    __shared__ u32x4 s_img[NCH];
    __shared__ u64 s_task[2 * TCAP];
    __shared__ u64 s_res[UPR];         // mask bits (keys < 64) found by the cooperative compares
    __shared__ u32 s_ntask;
    extern __shared__ __attribute__((aligned(16))) u8 s_tab[];
    using BL = WBlob<NH, NTL>;
    const int lane = threadIdx.x;
    const bool owner = lane < UPR;
    const bool spec = n_upd_dev && n_upd_host;
    const u64 n_upd = n_upd_dev ? *n_upd_dev : n_upd_host;
    const u64 lim = spec ? n_upd_host : n_upd;
    const u64 end = min(lim, n_upd);
    // Rounds are assigned grid-stride.  (Handing them out by an atomic counter instead, so that a
    // block made resident late takes fewer rounds, measured ~20 % slower at C3.)
    const u64 step = (u64)gridDim.x * UPR;
    auto load_pair = [&](u64 uu) {
        uint2 p = make_uint2((u32)uu, (u32)uu);
        if (pairs && uu < lim && owner) p = pairs[uu];
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
    u64 u0 = (u64)blockIdx.x * UPR;
    if (u0 >= end) return;  // wave-uniform: no round for this block
    u64 u1 = u0 + step;
    u64 os, ns;
    u32 on, nn;
    // the first round's pair and offsets are in flight while the tables are copied to LDS
    load_off(load_pair(u0 + lane), owner && u0 + lane < n_upd, os, ns, on, nn);
    for (u32 i = 16 * lane; i < to.bytes; i += 16 * FD_NT) *(u32x4*)(s_tab + i) = *(gp128)(tab_base + i);
    mp_tab_to_lds();
    if (owner) s_res[lane] = 0;
    if (lane == 0) s_ntask = 0;
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
    const FdQueue queue{(lds_u64p)s_task, (lds_u32p)&s_ntask, TCAP};
    const u32 img0 = (u32)(size_t)(const __attribute__((address_space(3))) u32x4*)s_img;
    // window descriptors of one round, in the owner lanes' registers: head chunk and last chunk of
    // both blobs as 16-B chunk indices from the arenas' aligned bases (no chunk: last < head);
    // the staging lanes read them with lane shuffles (no LDS)
    const u64 obase = (u64)od & ~(u64)15, nbase = (u64)nd & ~(u64)15;
    u32 dha = 0, dla = 0, dhb = 0, dlb = 0;
    auto put_desc = [&](u64 os_, u32 an, u64 ns_, u32 bn, bool a) {
        const u64 xa = os_ + ((u64)od & 15), xb = ns_ + ((u64)nd & 15);  // offsets from the bases
        dha = (u32)(xa >> 4);
        dla = a && an ? (u32)((xa + an - 1) >> 4) : 0;
        dhb = (u32)(xb >> 4);
        dlb = a && bn ? (u32)((xb + bn - 1) >> 4) : 0;
        if (!(a && an)) dha = 1;  // no chunk: last < head
        if (!(a && bn)) dhb = 1;
    };
    // LDS-DMA of one round's windows: instruction k fills image chunks [64k, 64k + 64), lane l chunk
    // 64k + l (its blob and window position from the descriptors).  The old blobs' images come
    // first (owner o's at chunk NC o), then the new blobs' (at NC (UPR + o)): every instruction but
    // the one straddling the two halves stages one side only, so it shuffles two descriptor words,
    // not four (the fully unrolled stage keeps every shuffle result live until its one wait).
    constexpr u32 HALF = (u32)UPR * NC;
    // per staging instruction k, this lane's round-invariant part: the owner lane whose descriptors it
    // reads (src), the window chunk (head chunk i, or tail chunk j counted back from the blob's last)
    // and whether that owner is real — packed src | off << 8 | head << 12 | real << 13
    u32 spk[NCH / 64];
#pragma unroll
    for (int k = 0; k < NCH / 64; k++) {
        const u32 c = 64 * k + (lane & 63);
        const bool sb = c >= HALF;
        const u32 cs = sb ? c - HALF : c;
        const u32 ow = cs / NC, i = cs - ow * NC;
        const bool real = ow < (u32)UPR;
        const bool head = i < (u32)NH;
        const u32 off = head ? i : (u32)(NTL - 1) - (i - NH);
        spk[k] = (real ? ow : 0u) | off << 8 | (u32)head << 12 | (u32)real << 13;
    }
    auto stage = [&]() {
#pragma unroll
        for (int k = 0; k < NCH / 64; k++) {
            const u32 c = 64 * k + (lane & 63);
            const bool sb = c >= HALF;
            const int src = (int)(spk[k] & 63);
            const u32 off = (spk[k] >> 8) & 15;
            const bool head = (spk[k] >> 12) & 1, real = (spk[k] >> 13) & 1;
            u32 h, l;  // chunk indices
            if (64u * k + 63 < HALF) { h = __shfl(dha, src); l = __shfl(dla, src); }
            else if (64u * k >= HALF) { h = __shfl(dhb, src); l = __shfl(dlb, src); }
            else {
                const u32 ha = __shfl(dha, src), la = __shfl(dla, src), hb_ = __shfl(dhb, src), lb = __shfl(dlb, src);
                h = sb ? hb_ : ha;
                l = sb ? lb : la;
            }
            // head chunk h + off, or tail chunk l - off; it exists when the blob spans that many chunks
            // (no chunk at all: l < h)
            const u32 ci = head ? h + off : l - off;
            const bool valid = real && (int)(l - h) >= (int)off;
            const u64 addr = (sb ? nbase : obase) + 16ull * ci;
            // chunks holding no blob byte are not loaded (their LDS bytes are never decoded: every
            // read is bounded by the blob length)
            if (valid) __builtin_amdgcn_global_load_lds((fd_glb_vp)addr, (fd_lds_vp)(s_img + 64 * k), 16, 0, 0);
        }
    };
    // Software pipeline, one HBM round trip per round: round r's windows are parsed while nothing
    // is in flight but the next offsets; then round r+1's windows (LDS-DMA into the freed image)
    // and round r's queued payloads are loaded together.
    put_desc(os, on, ns, nn, owner && u0 + lane < n_upd);
    stage();
    uint2 pr_n = load_pair(u1 + lane);
    __syncthreads();  // vmcnt(0) + barrier: round 0's windows have landed
    for (;;) {
        const u64 u = u0 + lane;
        const bool act = owner && u < n_upd;
        const bool more = u1 < end;  // wave-uniform
        u64 os_n = 0, ns_n = 0, u2 = end;
        u32 on_n = 0, nn_n = 0;
        if (more) {
            load_off(pr_n, owner && u1 + lane < n_upd, os_n, ns_n, on_n, nn_n);
            u2 = u1 + step;
        }
        // ---- parse ----
        u64 mk[4] = {0, 0, 0, 0};  // mask words kept in registers for <= 256 keys
        u8 st = 0;
        u64* m = masks + u * tb.words;
        if (act) {
            for (int w = MR; w < tb.words; w++) m[w] = 0;
            const u64 a0 = (u64)od + os, b0 = (u64)nd + ns;
            BL A, B;
            A.start = a0; A.len = on; A.s0 = (u32)(a0 & 15);
            A.t0 = (int)(((a0 + (on ? on - 1 : 0)) & ~(u64)15) - (a0 & ~(u64)15)) - 16 * (NTL - 1);
            A.img = img0 + 16u * (u32)(lane * NC);
            B.start = b0; B.len = nn; B.s0 = (u32)(b0 & 15);
            B.t0 = (int)(((b0 + (nn ? nn - 1 : 0)) & ~(u64)15) - (b0 & ~(u64)15)) - 16 * (NTL - 1);
            B.img = img0 + 16u * (u32)(UPR * NC + lane * NC);
#if KD_FD_PROBE_NOPARSE  // timing probe only (results invalid): no parse, no queued payloads
            (void)queue;
#else
            st = KD_FD_HEADF ? diff_one_f<MR>(A, B, tb, mk, m, queue) : diff_one_w<MR>(A, B, tb, mk, m, queue);
#endif
        }
        __syncthreads();  // parse done: the image is free, the queue complete
        if (more) {
            put_desc(os_n, on_n, ns_n, nn_n, owner && u1 + lane < n_upd);
            stage();
            pr_n = load_pair(u2 + lane);
        }
        // ---- the queued payloads, 16 lanes per payload ----
#if KD_FD_PROBE_NOCMP  // timing probe only (results invalid): queued payloads dropped
        const u32 nt = 0;
#else
        const u32 nt = min(s_ntask, TCAP);
#endif
        // (M payloads per 16-lane group per pass: their loads share one memory round trip)
        constexpr int M = TM, G = TG, NG = 64 / TG;
        for (u32 t = (u32)lane / G; t < nt; t += NG * M) {
            u64 ta[M], tbb[M], tx[M];
            u32 tn[M];
#pragma unroll
            for (int m = 0; m < M; m++) {
                const u32 tm = t + NG * m;
                const bool h = tm < nt;
                const u64 w0 = h ? s_task[2 * tm] : 0, w1 = h ? s_task[2 * tm + 1] : 0;
                ta[m] = w0 & 0xFFFFFFFFFFFFull;
                tbb[m] = w1 & 0xFFFFFFFFFFFFull;
                tx[m] = w0 >> 48;  // lane | key << 6
                tn[m] = (u32)(w1 >> 48);
            }
            bool d[M];
            coop_cmp<M, G, TS>(ta, tbb, tn, d);
#pragma unroll
            for (int m = 0; m < M; m++)
                if (d[m] && (lane & (G - 1)) == 0) {
                    const u32 ow = (u32)tx[m] & 63, key = (u32)(tx[m] >> 6) & 63;
                    atomicOr((unsigned long long*)&s_res[ow], 1ull << key);
                }
        }
        __syncthreads();  // the compares are in s_res; vmcnt(0): the next windows have landed
        if (act) {
            mk[0] |= s_res[lane];
            if (st) { mk[0] = mk[1] = mk[2] = mk[3] = 0; }
            store_masks<MR>(m, tb.words, mk, st);
            status[u] = st;
        }
        if (owner) s_res[lane] = 0;
        if (lane == 0) s_ntask = 0;
        if (!more) break;
        __builtin_amdgcn_wave_barrier();  // (one wave: its LDS operations stay in program order)
        u0 = u1;
        u1 = u2;
        os = os_n; ns = ns_n; on = on_n; nn = nn_n;
    }
}

// ================================================================================================
// streamed variant (k_fielddiff_s): the updates' blobs lie back to back in update order (no pairs),
// so a tile of T consecutive updates owns one contiguous byte span per side.  Each workgroup (one
// wave) copies both spans whole into LDS by LDS-DMA — 16 B per lane, 1 KiB per instruction, the
// bytes of the arena read exactly once — and every lane then parses its update straight from LDS:
// headers, values and the payload compares, with no per-blob window descriptors, no offsets ->
// window round trip and no payload re-read from HBM.  A tile whose span exceeds the buffer keeps
// its first CAP bytes in LDS; the blobs past them are read from global memory.
// ================================================================================================
// one blob inside the tile image (or, past the buffer, in global memory only)
// LDS: every byte of the blob lies in the loaded part of the image (the decoder is compiled without
// global-memory paths, so no wait on other loads in flight lands in the parse); else HBM only
template <bool LDS>
struct SBlobT {
    static constexpr bool lds_only = LDS;
    u64 start;
    u32 len;
    u32 s0;    // start & 15: blob position p is at offset x = p + s0 from its aligned chunk
    u32 img;   // LDS byte address of that chunk
    __device__ __forceinline__ u32 win(u32 x, u32) const { return LDS ? x : ~0u; }
};

// one tile: its first update, both spans (aligned base, chunk counts) and this lane's blob offsets
struct FdTile {
    u64 u, co, cn, os, oe, ns, ne;
    u32 nco, ncn;
    bool act;
};

template <int T, u32 CAPC>
__device__ __forceinline__ void fd_load_tile(FdTile& f, u64 tile, u64 n_upd, const u8* od, const u64* ooff, const u8* nd,
                                             const u64* noff) {
    const int lane = threadIdx.x;
    const u64 u0 = tile * T, ue = min(u0 + T, n_upd);
    f.u = u0 + lane;
    f.act = lane < T && f.u < ue;
    const u64 so0 = ooff[u0], so1 = ooff[ue], sn0 = noff[u0], sn1 = noff[ue];
    f.os = f.oe = f.ns = f.ne = 0;
    if (f.act) {
        f.os = ooff[f.u]; f.oe = ooff[f.u + 1];
        f.ns = noff[f.u]; f.ne = noff[f.u + 1];
    }
    f.co = ((u64)od + so0) & ~(u64)15;
    f.cn = ((u64)nd + sn0) & ~(u64)15;
    f.nco = (u32)min<u64>((((u64)od + so1) - f.co + 15) >> 4, CAPC);
    f.ncn = (u32)min<u64>((((u64)nd + sn1) - f.cn + 15) >> 4, CAPC);
}

// PF: the spans of the next tile are loaded into registers (PL chunks per lane: the old span's
// chunks, then the new span's) while the current tile is parsed from LDS, and written to LDS after
// it — plain loads, so no wait on them precedes the parse's LDS reads (an LDS-DMA in flight makes
// the compiler drain every load before any LDS read).  Without PF: LDS-DMA, then the parse.
template <int T, int CAPB, bool PF>
__global__ __launch_bounds__(FD_NT) void k_fielddiff_s(const u8* __restrict__ od, const u64* __restrict__ ooff,
                                                       const u8* __restrict__ nd, const u64* __restrict__ noff,
                                                       u64 n_upd_host, const u64* __restrict__ n_upd_dev,
                                                       FdTab tg, FdTabOff to, const u8* __restrict__ tab_base,
                                                       u64* __restrict__ masks, u8* __restrict__ status) {
    static_assert(T <= FD_NT && CAPB % 512 == 0, "stream shape");
    constexpr u32 CAPC = CAPB / 16;             // chunks loaded per side at most
    constexpr int PL = (int)(2 * CAPC / FD_NT);  // PF: chunks per lane
    static_assert(!PF || PL * FD_NT == 2 * CAPC, "stream shape");
    __shared__ u32x4 s_img[2 * CAPC + 8];        // old span, new span (+ slack: reads past a blob's end)
    __shared__ u32 s_dummy;
    extern __shared__ __attribute__((aligned(16))) u8 s_tab[];
    const int lane = threadIdx.x;
    const u64 n_upd = n_upd_dev ? min(*n_upd_dev, n_upd_host ? n_upd_host : ~0ull) : n_upd_host;
    const u64 ntiles = (n_upd + T - 1) / T;
    if ((u64)blockIdx.x >= ntiles) return;  // wave-uniform
    for (u32 i = 16 * lane; i < to.bytes; i += 16 * FD_NT) *(u32x4*)(s_tab + i) = *(gp128)(tab_base + i);
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
    const FdQueue none{(lds_u64p) nullptr, (lds_u32p)&s_dummy, 0};  // payloads compare in place
    const u32 img_o = (u32)(size_t)(const __attribute__((address_space(3))) u32x4*)s_img;
    const u32 img_n = img_o + 16 * CAPC;
    typedef __attribute__((address_space(3))) u32x4* l128;
    u64 tile = blockIdx.x;
    FdTile cur, nxt;
    fd_load_tile<T, CAPC>(cur, tile, n_upd, od, ooff, nd, noff);
    u32x4 buf[PF ? PL : 1];
    if (PF) {  // the first tile's spans through registers too
#pragma unroll
        for (int p = 0; p < PL; p++) {
            const u32 i = 64 * p + lane;
            const bool o = i < cur.nco, n = !o && i < cur.nco + cur.ncn;
            const u64 src = o ? cur.co + 16ull * i : cur.cn + 16ull * (i - cur.nco);
            if (o || n) buf[p] = *(gp128)src;
        }
#pragma unroll
        for (int p = 0; p < PL; p++) {
            const u32 i = 64 * p + lane;
            const bool o = i < cur.nco, n = !o && i < cur.nco + cur.ncn;
            if (o || n) *(l128)(size_t)(o ? img_o + 16 * i : img_n + 16 * (i - cur.nco)) = buf[p];
        }
    }
    u64 nt = tile + gridDim.x;
    if (PF && nt < ntiles) fd_load_tile<T, CAPC>(nxt, nt, n_upd, od, ooff, nd, noff);
    for (;;) {
        const bool more = PF && nt < ntiles;  // wave-uniform
        if (PF) {
            // the next tile's spans into registers (its offsets were loaded during the last tile)
            if (more) {
#pragma unroll
                for (int p = 0; p < PL; p++) {
                    const u32 i = 64 * p + lane;
                    const bool o = i < nxt.nco, n = !o && i < nxt.nco + nxt.ncn;
                    const u64 src = o ? nxt.co + 16ull * i : nxt.cn + 16ull * (i - nxt.nco);
                    if (o || n) buf[p] = *(gp128)src;
                }
            }
        } else {
            for (u32 k = 0; k < cur.nco; k += FD_NT)
                if (k + lane < cur.nco)
                    __builtin_amdgcn_global_load_lds((fd_glb_vp)(cur.co + 16ull * (k + lane)), (fd_lds_vp)(s_img + k), 16, 0, 0);
            for (u32 k = 0; k < cur.ncn; k += FD_NT)
                if (k + lane < cur.ncn)
                    __builtin_amdgcn_global_load_lds((fd_glb_vp)(cur.cn + 16ull * (k + lane)), (fd_lds_vp)(s_img + CAPC + k), 16, 0, 0);
            __syncthreads();  // vmcnt(0) + barrier: the spans have landed
        }
        if (cur.act) {
            SBlobT<true> A, B;
            A.start = (u64)od + cur.os; A.len = (u32)(cur.oe - cur.os); A.s0 = (u32)(A.start & 15);
            A.img = img_o + (u32)((A.start & ~(u64)15) - cur.co);
            B.start = (u64)nd + cur.ns; B.len = (u32)(cur.ne - cur.ns); B.s0 = (u32)(B.start & 15);
            B.img = img_n + (u32)((B.start & ~(u64)15) - cur.cn);
            const bool res = A.start + A.len <= cur.co + 16ull * cur.nco && B.start + B.len <= cur.cn + 16ull * cur.ncn;
            u64* m = masks + cur.u * tb.words;
            for (int w = 4; w < tb.words; w++) m[w] = 0;
            u64 mk[4] = {0, 0, 0, 0};
#if KD_FD_PROBE_NOPARSE  // timing probe only (results invalid)
            u8 st = 0;
            (void)none;
            (void)res;
#else
            u8 st;
            if (res) {
                st = diff_one_w(A, B, tb, mk, m, none);
            } else {  // a tile whose span outgrew the buffer: this update from HBM
                SBlobT<false> GA, GB;
                GA.start = A.start; GA.len = A.len; GA.s0 = A.s0; GA.img = 0;
                GB.start = B.start; GB.len = B.len; GB.s0 = B.s0; GB.img = 0;
                st = diff_one_w(GA, GB, tb, mk, m, none);
            }
#endif
            if (st) { mk[0] = mk[1] = mk[2] = mk[3] = 0; }
            store_masks(m, tb.words, mk, st);
            status[cur.u] = st;
        }
        if (!PF) {
            __syncthreads();  // the image is free for the next tile
            tile += gridDim.x;
            if (tile >= ntiles) break;
            fd_load_tile<T, CAPC>(cur, tile, n_upd, od, ooff, nd, noff);
            continue;
        }
        if (!more) break;
        // the parse is done with the image (one wave: its LDS operations stay in order): the next
        // tile's spans go in, and the tile after it has its offsets loaded
        const u64 nn = nt + gridDim.x;
        FdTile aft;
        if (nn < ntiles) fd_load_tile<T, CAPC>(aft, nn, n_upd, od, ooff, nd, noff);
#pragma unroll
        for (int p = 0; p < PL; p++) {
            const u32 i = 64 * p + lane;
            const bool o = i < nxt.nco, n = !o && i < nxt.nco + nxt.ncn;
            if (o || n) *(l128)(size_t)(o ? img_o + 16 * i : img_n + 16 * (i - nxt.nco)) = buf[p];
        }
        cur = nxt;
        nt = nn;
        if (nn < ntiles) nxt = aft;
    }
}

// ================================================================================================
// walked variant (k_fdwalk, the default for larger features): no LDS images and no staging.  One
// wave per workgroup, 64 updates per round, one lane per update; each lane walks its two blobs value
// by value straight from global memory (HBlobT: one 16-B load per decode window, the header, legend
// and array header in one batch of three), compares scalars and payloads up to FD_LOCAL bytes in
// registers, and queues longer payloads (geometries of equal length) for the wave's cooperative
// compare.  A value the comparison does not need is never read: the middle of a geometry whose
// length changed costs no bytes.  With no LDS image the kernel keeps few registers and many waves
// per SIMD in flight, and the latency of the walk's dependent loads (mostly L2 hits after the
// blob's first line) hides behind the other waves.
// ================================================================================================
#ifndef KD_FDW_SHAPE
#define KD_FDW_SHAPE 1, 16, 2  // cooperative compare: payloads per 16-lane group per pass, lanes per payload, steps
#endif
#ifndef KD_FDW_CAP
#define KD_FDW_CAP 32  // resident workgroups per CU at most
#endif
template <int TM, int TG, int TS>
#ifndef KD_FDW_WPE
#define KD_FDW_WPE 4  // waves per SIMD the register budget is sized for
#endif
__global__ __launch_bounds__(FD_NT) __attribute__((amdgpu_waves_per_eu(KD_FDW_WPE))) void k_fdwalk(const u8* __restrict__ od, const u64* __restrict__ ooff,
                                                  const u8* __restrict__ nd, const u64* __restrict__ noff,
                                                  const uint2* __restrict__ pairs, u64 n_upd_host,
                                                  const u64* __restrict__ n_upd_dev, u64 n_ent_o, u64 n_ent_n,
                                                  FdTab tg, FdTabOff to, const u8* __restrict__ tab_base,
                                                  u64* __restrict__ masks, u8* __restrict__ status) {
    constexpr u32 TCAP = FD_NT;  // queued payload compares per round (then a lane compares alone)
    __shared__ u64 s_task[2 * TCAP];
    __shared__ u64 s_res[FD_NT];  // mask bits (keys < 64) found by the cooperative compares
    __shared__ u32 s_ntask;
    extern __shared__ __attribute__((aligned(16))) u8 s_tab[];
    const int lane = threadIdx.x;
    const bool spec = n_upd_dev && n_upd_host;
    const u64 n_upd = n_upd_dev ? *n_upd_dev : n_upd_host;
    const u64 lim = spec ? n_upd_host : n_upd;
    const u64 end = min(lim, n_upd);
    const u64 step = (u64)gridDim.x * FD_NT;
    u64 u0 = (u64)blockIdx.x * FD_NT;
    if (u0 >= end) return;  // wave-uniform
    // the arenas' ends: no load crosses them
    const u64 olim = (u64)od + ooff[n_ent_o], nlim = (u64)nd + noff[n_ent_n];
    auto load_pair = [&](u64 uu) {
        uint2 p = make_uint2((u32)uu, (u32)uu);
        if (pairs && uu < end) p = pairs[uu];
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
    u64 u1 = u0 + step;
    u64 os, ns;
    u32 on, nn;
    load_off(load_pair(u0 + lane), u0 + lane < end, os, ns, on, nn);
    for (u32 i = 16 * lane; i < to.bytes; i += 16 * FD_NT) *(u32x4*)(s_tab + i) = *(gp128)(tab_base + i);
    mp_tab_to_lds();
    s_res[lane] = 0;
    if (lane == 0) s_ntask = 0;
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
    const FdQueue queue{(lds_u64p)s_task, (lds_u32p)&s_ntask, TCAP};
    uint2 pr_n = load_pair(u1 + lane);
    __syncthreads();  // the tables are in LDS
    for (;;) {
        const u64 u = u0 + lane;
        const bool act = u < end;
        const bool more = u1 < end;  // wave-uniform
        u64 os_n = 0, ns_n = 0, u2 = end;
        u32 on_n = 0, nn_n = 0;
        if (more) {  // the next round's offsets are in flight during this round's walk
            load_off(pr_n, u1 + lane < end, os_n, ns_n, on_n, nn_n);
            u2 = u1 + step;
        }
        u64 mk[4] = {0, 0, 0, 0};
        u8 st = 0;
        u64* m = masks + u * tb.words;
        if (act) {
            for (int w = 1; w < tb.words; w++) m[w] = 0;
            const u64 a0 = (u64)od + os, b0 = (u64)nd + ns;
            // a blob within 16 B of its arena's end: every load bounded by it
            const HBlobT<true> A{a0, on, a0 + on + 16 > olim, olim}, B{b0, nn, b0 + nn + 16 > nlim, nlim};
            st = diff_one_f<1>(A, B, tb, mk, m, queue);
        }
        __syncthreads();  // the walk is done: the queue is complete
        if (more) pr_n = load_pair(u2 + lane);
        // ---- the queued payloads, TG lanes per payload, TM per group per pass ----
        const u32 nt = min(s_ntask, TCAP);
        constexpr int M = TM, G = TG, NG = 64 / TG;
        for (u32 t = (u32)lane / G; t < nt; t += NG * M) {
            u64 ta[M], tbb[M], tx[M];
            u32 tn[M];
#pragma unroll
            for (int k = 0; k < M; k++) {
                const u32 tm = t + NG * k;
                const bool h = tm < nt;
                const u64 w0 = h ? s_task[2 * tm] : 0, w1 = h ? s_task[2 * tm + 1] : 0;
                ta[k] = w0 & 0xFFFFFFFFFFFFull;
                tbb[k] = w1 & 0xFFFFFFFFFFFFull;
                tx[k] = w0 >> 48;  // lane | key << 6
                tn[k] = (u32)(w1 >> 48);
            }
            bool d[M];
            coop_cmp<M, G, TS>(ta, tbb, tn, d);
#pragma unroll
            for (int k = 0; k < M; k++)
                if (d[k] && (lane & (G - 1)) == 0) {
                    const u32 ow = (u32)tx[k] & 63, key = (u32)(tx[k] >> 6) & 63;
                    atomicOr((unsigned long long*)&s_res[ow], 1ull << key);
                }
        }
        __syncthreads();  // the compares are in s_res
        if (act) {
            mk[0] |= s_res[lane];
            if (st) { mk[0] = mk[1] = mk[2] = mk[3] = 0; }
            store_masks<1>(m, tb.words, mk, st);
            status[u] = st;
        }
        s_res[lane] = 0;
        if (lane == 0) s_ntask = 0;
        if (!more) break;
        __builtin_amdgcn_wave_barrier();
        u0 = u1;
        u1 = u2;
        os = os_n; ns = ns_n; on = on_n; nn = nn_n;
    }
}

// Fallback for tables too large for LDS: one lane per update, blobs parsed straight from global
// memory.
__global__ __launch_bounds__(FD_NT) void k_fielddiff_g(const u8* __restrict__ od, const u64* __restrict__ ooff,
                                                       const u8* __restrict__ nd, const u64* __restrict__ noff,
                                                       const uint2* __restrict__ pairs, u64 n_upd_host,
                                                       const u64* __restrict__ n_upd_dev, FdTab tb,
                                                       u64* __restrict__ masks, u8* __restrict__ status) {
    const int lane = threadIdx.x;
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
        for (int w = 4; w < tb.words; w++) m[w] = 0;
        u64 mk[4] = {0, 0, 0, 0};
        const u8 st = diff_one((gp8)(od + os), on, (gp8)(nd + ns), nn, tb, mk, m);
        if (st) { mk[0] = mk[1] = mk[2] = mk[3] = 0; }
        store_masks(m, tb.words, mk, st);
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
    // window shape from the typical blob: small features (points, ~90-150 B) fit a long head window
    // whole; larger ones (polygons) get head + tail windows around their geometry
    const bool small = typ <= 144;
    // the streamed kernel: contiguous update arenas (no pairs) of larger blobs; the fd_stream option
    // 0 / 1 forces it off / on
    const int stream_env = ctx->opt.fd_stream;
    const bool stream = lds_tab && d_pu == nullptr && (stream_env >= 0 ? stream_env > 0 : !small && KD_FD_STREAM_DEFAULT);
    // the walked kernel (no LDS images; slower: DESIGN §3.2): the fd_walk option 1 forces it
    const int walk_env = ctx->opt.fd_walk;
    const bool walk = lds_tab && !stream && walk_env > 0;
    // The kernel loops over rounds (grid stride), so its grid is the resident set (occupancy
    // calculator for this launch's LDS), capped at the measured optimum.
    const void* kern = walk ? (const void*)k_fdwalk<KD_FDW_SHAPE>
                       : stream ? (const void*)k_fielddiff_s<KD_FD_SSHAPE, KD_FD_SPF>
                       : !lds_tab ? (const void*)k_fielddiff_g
                       : small ? (W == 1 ? (const void*)k_fielddiff<KD_FD_SHAPE_S, 1> : (const void*)k_fielddiff<KD_FD_SHAPE_S, 4>)
                       : (W == 1 ? (const void*)k_fielddiff<KD_FD_SHAPE_L, 1> : (const void*)k_fielddiff<KD_FD_SHAPE_L, 4>);
    int per_cu = 0;
    KD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, FD_NT, lds_tab ? o_end : 0));
    // (the calculator can count one block per CU more than becomes resident: DESIGN.md §3.2)
#ifndef KD_FD_CAP
#define KD_FD_CAP 12  // C2 points: 10 / 12 blocks per CU = 36.8 / 35.1 us (C3 is LDS-bound at 8)
#endif
    per_cu = std::max(1, std::min(per_cu, walk ? KD_FDW_CAP : stream ? 16 : KD_FD_CAP));
    const u64 upr = walk ? (u64)FD_NT : stream ? (u64)fd_stream_t<KD_FD_SSHAPE>() : !lds_tab ? FD_NT : small ? fd_upr<KD_FD_SHAPE_S>(nullptr) : fd_upr<KD_FD_SHAPE_L>(nullptr);
    unsigned blocks = (unsigned)std::min<u64>((work + upr - 1) / upr, (u64)ctx->n_cu * (u64)per_cu);
    if (blocks == 0) blocks = 1;
    rc = launch(ctx, "k_fielddiff", [&] {
        auto args = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(FD_NT), o_end, ctx->stream, (const u8*)d_od, (const u64*)d_ooff,
                               (const u8*)d_nd, (const u64*)d_noff, (const uint2*)d_pu, n_upd, d_n_upd,
                               tb, to, (const u8*)dt, d_masks, d_status);
        };
        if (walk)
            hipLaunchKernelGGL((k_fdwalk<KD_FDW_SHAPE>), dim3(blocks), dim3(FD_NT), o_end, ctx->stream, (const u8*)d_od,
                               (const u64*)d_ooff, (const u8*)d_nd, (const u64*)d_noff, (const uint2*)d_pu, n_upd, d_n_upd,
                               (u64)ob->n, (u64)nb->n, tb, to, (const u8*)dt, d_masks, d_status);
        else if (stream)
            hipLaunchKernelGGL((k_fielddiff_s<KD_FD_SSHAPE, KD_FD_SPF>), dim3(blocks), dim3(FD_NT), o_end, ctx->stream, (const u8*)d_od,
                               (const u64*)d_ooff, (const u8*)d_nd, (const u64*)d_noff, n_upd, d_n_upd, tb, to,
                               (const u8*)dt, d_masks, d_status);
        else if (!lds_tab)
            hipLaunchKernelGGL(k_fielddiff_g, dim3(blocks), dim3(FD_NT), 0, ctx->stream, (const u8*)d_od, (const u64*)d_ooff,
                               (const u8*)d_nd, (const u64*)d_noff, (const uint2*)d_pu, n_upd, d_n_upd, tb, d_masks,
                               d_status);
        // (mask words kept in registers: one for up to 64 union keys, else four)
        else if (small) W == 1 ? args(k_fielddiff<KD_FD_SHAPE_S, 1>) : args(k_fielddiff<KD_FD_SHAPE_S, 4>);
        else W == 1 ? args(k_fielddiff<KD_FD_SHAPE_L, 1>) : args(k_fielddiff<KD_FD_SHAPE_L, 4>);
    });
    if (rc) return rc;
    if (out_mem == KD_MEM_HOST) {
        if ((rc = stage_d2h(ctx, masks, d_masks, n_upd * W * 8)) || (rc = stage_d2h(ctx, status, d_status, n_upd))) return rc;
        prof_flush(ctx);
    }
    return KD_OK;
}
