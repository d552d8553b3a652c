// kd_geom.h — GPKG geometry-header decoding, bbox test and the spatial-filter index envelope
// (EnvelopeEncoder), shared by k_envelopes (kd_spatial.hip) and the filtered diff (kd_geomfilter.hip).
// FP64 throughout; the translation units are built with -ffp-contract=off.
// Reference: kart/geometry.py:638-700 (geom_envelope), kart/spatial_filter/__init__.py:534-590,
// 709-734 (matches, bbox_intersects_fast), kart/spatial_filter/index.py:485-579,639-707,783-813.
#pragma once
#include "kd_internal.h"

namespace kd {
__device__ __forceinline__ double ld_f64(const u8* p, bool le) {
    u64 b = 0;
    if (le) {
#pragma unroll
        for (int i = 7; i >= 0; i--) b = (b << 8) | p[i];
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) b = (b << 8) | p[i];
    }
    return __longlong_as_double((i64)b);
}

__device__ __forceinline__ u32 ld_u32(const u8* p, bool le) {
    return le ? (u32)p[0] | (u32)p[1] << 8 | (u32)p[2] << 16 | (u32)p[3] << 24
              : (u32)p[3] | (u32)p[2] << 8 | (u32)p[1] << 16 | (u32)p[0] << 24;
}

__device__ __forceinline__ int env_size(int et) { return et == 0 ? 0 : et == 1 ? 32 : et <= 3 ? 48 : 64; }

// 1 stored env, 0 None (empty / NaN), 2 no stored env, -1 malformed/unsupported
__device__ __forceinline__ int gpkg_env(const u8* g, u64 n, double e[4]) {
    if (n < 8 || g[0] != 'G' || g[1] != 'P' || g[2] != 0) return -1;
    const u8 f = g[3];
    if (f & 0x20) return -1;
    if (f & 0x10) return 0;
    const int et = (f >> 1) & 7;
    if (et > 4) return -1;
    if (et == 0) return 2;
    if (n < (u64)(8 + env_size(et))) return -1;
    const bool le = f & 1;
    bool nan = false;
#pragma unroll
    for (int i = 0; i < 4; i++) { e[i] = ld_f64(g + 8 + 8 * i, le); nan |= e[i] != e[i]; }
    return nan ? 0 : 1;
}

// point WKB after the header: 1 ok (x,x,y,y), 0 empty point (NaN coords), -1 not a point
__device__ __forceinline__ int point_env(const u8* g, u64 n, double e[4]) {
    const int et = (g[3] >> 1) & 7;
    if (et > 4) return -1;
    const u64 off = 8 + env_size(et);
    if (n < off + 5) return -1;
    const bool le = g[off] == 1;
    u32 typ = ld_u32(g + off + 1, le) & 0x0fffffffu;
    if (typ >= 1000) typ %= 1000;
    if (typ != 1 || n < off + 21) return -1;
    const double x = ld_f64(g + off + 5, le), y = ld_f64(g + off + 13, le);
    if (x != x && y != y) { e[0] = e[1] = e[2] = e[3] = 0.0; return 0; }
    e[0] = x; e[1] = x; e[2] = y; e[3] = y;
    return 1;
}

// _range_overlaps: 1 / 0, -1 inverted range (reference raises)
__device__ __forceinline__ int range_ov(double a1, double a2, double b1, double b2) {
    if (a1 > a2 || b1 > b2) return -1;
    if (b1 < a1) return b2 > a1;
    if (a1 < b1) return a2 > b1;
    return (b2 != b1) && (a2 != a1);
}

// EnvelopeEncoder::decode of one big-endian record of 4 x bits (spatial_filter.cpp:106-128), then
// cyclic_range_overlaps(w, e, qw, qe) && range_overlaps(s, n, qs, qn) (:170-208, :249):
// 1 overlaps, 0 not, -1 an inverted range (the reference aborts)
__device__ __forceinline__ int enc_overlap(const u8* p, int bits, double qw, double qs, double qe, double qn) {
    const int nb = bits / 2;
    const double vmax = (double)((1ull << bits) - 1);
    const u64 mask = (1ull << bits) - 1;
    unsigned __int128 acc = 0;
    for (int k = 0; k < nb; k++) acc = (acc << 8) | p[k];
    double v[4];
    const double mins[4] = {-180, -90, -180, -90}, maxs[4] = {180, 90, 180, 90};
    for (int k = 3; k >= 0; k--) {
        const u64 q = (u64)(acc & mask);
        acc >>= bits;
        v[k] = ((double)q / vmax) * (maxs[k] - mins[k]) + mins[k];
    }
    double a1 = v[0], a2 = v[2], b1 = qw, b2 = qe;
    if (a1 > a2) a2 += 360;
    if (b1 > b2) b2 += 360;
    int r = range_ov(a1, a2, b1, b2);
    if (r == 0) {
        if (a1 < b1) { a1 += 360; a2 += 360; } else { b1 += 360; b2 += 360; }
        r = range_ov(a1, a2, b1, b2);
    }
    if (r > 0) r = range_ov(v[1], v[3], qs, qn);
    return r;
}

__device__ __attribute__((noinline)) double py_mod360_slow(double a) {
    double m = fmod(a, 360.0);
    if (m != 0.0) {
        if (m < 0) m += 360.0;  // b > 0: result takes the sign of b
    } else {
        m = 0.0;  // copysign(0, 360)
    }
    return m;
}

// Python float a % 360.  On (-360, 720) fmod is exact and needs at most one +-360 (Sterbenz: a - 360
// is exact for a in [360, 720)), so the common cases are plain selects; the rest call fmod.
__device__ __forceinline__ double py_mod360(double a) {
    double m;
    if (a >= 0.0 && a < 360.0) m = a;
    else if (a >= 360.0 && a < 720.0) m = a - 360.0;
    else if (a < 0.0 && a > -360.0) m = a + 360.0;
    else return py_mod360_slow(a);
    return m == 0.0 ? 0.0 : m;
}

__device__ __forceinline__ double wrap_lon(double x) { return py_mod360(x + 180.0) - 180.0; }

// encode one value (EnvelopeEncoder._encode_value); false if out of range (reference asserts)
__device__ __forceinline__ bool enc_val(double v, double lo, double hi, double vmax, bool up, u64* out) {
    if (!(lo <= v && v <= hi)) return false;
    double norm = (v - lo) / (hi - lo);
    double sc = norm * vmax;
    double r = up ? ceil(sc) : floor(sc);
    if (!(r >= 0 && r <= vmax)) return false;
    *out = (u64)r;
    return true;
}

// Fast header decode from registers.  The lane loads the 48 bytes from its blob start rounded down
// to 4 B (three dword-aligned 16-B loads instead of ~60 byte loads), realigns them with v_alignbyte
// (>= 45 valid bytes from the blob start), and decodes the GPKG header, a 32-B envelope (type 1) or
// a point WKB right after the header (type 0) at fixed byte positions — exactly gpkg_env /
// point_env.  Returns false (byte-wise slow path) where a field may lie past the window: envelope
// types 2-4, and a NaN type-1 envelope (whose point WKB would follow it).
__device__ __forceinline__ u64 f64_bits(u32 lo, u32 hi, bool le) {
    const u64 x = (u64)hi << 32 | lo;
    return le ? x : __builtin_bswap64(x);
}
__device__ __forceinline__ bool env_fast(const u32 r[11], u64 len, int& rc, double e[4], int& pc, double pe[4]) {
    const u32 h = r[0];
    const u32 f = h >> 24;
    pc = -1;
    if ((h & 0xFFFFFFu) != 0x005047u || (f & 0x20)) { rc = -1; return true; }  // 'G' 'P' version 0
    if (f & 0x10) { rc = 0; return true; }  // empty: no envelope or point read
    const int et = (f >> 1) & 7;
    if (et > 1) return false;
    const bool le = f & 1;
    if (et == 1) {
        if (len < 40) { rc = -1; return true; }
        bool nan = false;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            e[i] = __longlong_as_double((i64)f64_bits(r[2 + 2 * i], r[3 + 2 * i], le));
            nan |= e[i] != e[i];
        }
        rc = 1;
        return !nan;
    }
    rc = 2;  // no stored envelope: point WKB at byte 8, its fields 1 byte past dword boundaries
    if (len >= 13) {
        const bool wle = (r[2] & 0xFF) == 1;
        u32 typ = __builtin_amdgcn_alignbyte(r[3], r[2], 1);
        if (!wle) typ = __builtin_bswap32(typ);
        typ &= 0x0fffffffu;
        if (typ >= 1000) typ %= 1000;
        if (typ == 1 && len >= 29) {
            const double x = __longlong_as_double((i64)f64_bits(__builtin_amdgcn_alignbyte(r[4], r[3], 1),
                                                                __builtin_amdgcn_alignbyte(r[5], r[4], 1), wle));
            const double y = __longlong_as_double((i64)f64_bits(__builtin_amdgcn_alignbyte(r[6], r[5], 1),
                                                                __builtin_amdgcn_alignbyte(r[7], r[6], 1), wle));
            if (x != x && y != y) { pe[0] = pe[1] = pe[2] = pe[3] = 0.0; pc = 0; }
            else { pe[0] = x; pe[1] = x; pe[2] = y; pe[3] = y; pc = 1; }
        }
    }
    return true;
}

// EnvelopeEncoder bytes of the identity-CRS spatial-index envelope of one decoded geometry
// (get_envelope_for_indexing + transform_minmax_envelope + _buffer_minmax_envelope + encode):
// out(k, byte) receives bits/2 big-endian bytes; false when the indexer stores no row (empty,
// no envelope, too wide, out of range).  r/pc/e/pe as gpkg_env/point_env (or env_fast) left them.
template <class F>
__device__ __forceinline__ bool index_env(int r, int pc, const double e[4], const double pe[4], bool is_empty, int bits,
                                          double vmax, F&& out) {
    if (is_empty || r < 0) return false;
    double sv[4];
    if (r == 1) { sv[0] = e[0]; sv[1] = e[1]; sv[2] = e[2]; sv[3] = e[3]; }
    else if (r == 2 && pc == 1) { sv[0] = pe[0]; sv[1] = pe[1]; sv[2] = pe[2]; sv[3] = pe[3]; }
    else return false;
    // transpose -> (minx, miny, maxx, maxy)
    const double e0 = sv[0], e1 = sv[2], e2 = sv[1], e3 = sv[3];
    double wv, so, ea, no;
    if (e0 == e2 && e1 == e3) {
        wv = wrap_lon(e0); so = e1; ea = wv; no = e1;
    } else {
        const double width = e2 - e0, height = e3 - e1;
        if (width >= 180) return false;
        double big = width;
        if (height > big) big = height;
        const double buf = big < 1.0 ? 0.1 * big : 0.1;
        double t1 = e1 - buf; if (-90.0 > t1) t1 = -90.0;
        double t3 = e3 + buf; if (90.0 < t3) t3 = 90.0;
        wv = wrap_lon(e0 - buf); so = t1; ea = wrap_lon(e2 + buf); no = t3;
    }
    u64 q0, q1, q2, q3;
    if (!(enc_val(wv, -180, 180, vmax, false, &q0) && enc_val(so, -90, 90, vmax, false, &q1) &&
          enc_val(ea, -180, 180, vmax, true, &q2) && enc_val(no, -90, 90, vmax, true, &q3)))
        return false;
    // 4*bits big-endian bits -> bits/2 bytes
    unsigned __int128 acc = ((unsigned __int128)q0 << (3 * bits)) | ((unsigned __int128)q1 << (2 * bits)) |
                            ((unsigned __int128)q2 << bits) | (unsigned __int128)q3;
    for (int k = bits / 2 - 1; k >= 0; k--) { out(k, (u8)(acc & 0xFF)); acc >>= 8; }
    return true;
}

}  // namespace kd
