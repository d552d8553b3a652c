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

enum : u8 { V_NIL = 0, V_INT = 1, V_FLOAT = 2, V_STR = 3, V_BYTES = 4, V_EXT = 5 };

struct DVal {
    u8 cls;
    u8 big;     // V_INT: value in [2^63, 2^64) held in bits as uint64
    i8 ext;
    u64 bits;   // V_INT: int64 (or uint64 if big); V_FLOAT: double bits
    const u8* p;
    u32 len;
};

__device__ __forceinline__ u64 ld_be(const u8* p, int w) {
    u64 v = 0;
    for (int i = 0; i < w; i++) v = (v << 8) | p[i];
    return v;
}

// decode one value; returns bytes consumed, 0 on malformed / unsupported
__device__ u32 dv_decode(const u8* __restrict__ p, const u8* end, DVal& v) {
    if (p >= end) return 0;
    const u64 avail = (u64)(end - p);
    const u8 t = p[0];
    v.big = 0;
    if (t <= 0x7f) { v.cls = V_INT; v.bits = t; return 1; }
    if (t >= 0xe0) { v.cls = V_INT; v.bits = (u64)(i64)(int8_t)t; return 1; }
    if (t >= 0xa0 && t <= 0xbf) {
        u32 n = t & 31;
        if (1 + (u64)n > avail) return 0;
        v.cls = V_STR; v.p = p + 1; v.len = n; return 1 + n;
    }
    switch (t) {
    case 0xc0: v.cls = V_NIL; return 1;
    case 0xc2: v.cls = V_INT; v.bits = 0; return 1;
    case 0xc3: v.cls = V_INT; v.bits = 1; return 1;
    case 0xcc: case 0xcd: case 0xce: case 0xcf: {
        int w = 1 << (t - 0xcc);
        if ((u64)(1 + w) > avail) return 0;
        v.cls = V_INT; v.bits = ld_be(p + 1, w); v.big = (w == 8 && (v.bits >> 63)) ? 1 : 0;
        return 1 + w;
    }
    case 0xd0: case 0xd1: case 0xd2: case 0xd3: {
        int w = 1 << (t - 0xd0);
        if ((u64)(1 + w) > avail) return 0;
        int sh = 64 - 8 * w;
        v.cls = V_INT; v.bits = (u64)(((i64)(ld_be(p + 1, w) << sh)) >> sh);
        return 1 + w;
    }
    case 0xca: {
        if (5 > avail) return 0;
        u32 b = (u32)ld_be(p + 1, 4);
        v.cls = V_FLOAT; v.bits = (u64)__double_as_longlong((double)__uint_as_float(b));
        return 5;
    }
    case 0xcb: {
        if (9 > avail) return 0;
        v.cls = V_FLOAT; v.bits = ld_be(p + 1, 8);
        return 9;
    }
    case 0xd9: case 0xda: case 0xdb: case 0xc4: case 0xc5: case 0xc6: {
        int w = (t == 0xd9 || t == 0xc4) ? 1 : (t == 0xda || t == 0xc5) ? 2 : 4;
        if ((u64)(1 + w) > avail) return 0;
        u32 n = (u32)ld_be(p + 1, w);
        if ((u64)1 + w + n > avail) return 0;
        v.cls = t >= 0xd9 ? V_STR : V_BYTES; v.p = p + 1 + w; v.len = n;
        return 1 + w + n;
    }
    case 0xd4: case 0xd5: case 0xd6: case 0xd7: case 0xd8: case 0xc7: case 0xc8: case 0xc9: {
        u32 n, hdr;
        if (t <= 0xd8 && t >= 0xd4) { n = 1u << (t - 0xd4); hdr = 2; }
        else {
            int w = 1 << (t - 0xc7);
            if ((u64)(2 + w) > avail) return 0;
            n = (u32)ld_be(p + 1, w); hdr = 2 + w;
        }
        if ((u64)hdr + n > avail) return 0;
        v.ext = (i8)p[hdr - 1]; v.p = p + hdr; v.len = n;
        if (v.ext == 'G') {
            if (n == 0) { v.cls = V_NIL; return hdr; }           // Geometry.of(b"") -> None
            if (n < 2 || v.p[0] != 'G' || v.p[1] != 'P') return 0; // Geometry() raises
            v.cls = V_BYTES;
        } else {
            v.cls = V_EXT;
        }
        return hdr + n;
    }
    default: return 0;  // arrays / maps / 0xc1: not field values Kart writes
    }
}

__device__ __forceinline__ bool int_eq_float(const DVal& i, double d) {
    if (!(d == d)) return false;
    if (floor(d) != d) return false;
    if (i.big) {
        // value in [2^63, 2^64)
        if (!(d >= 9223372036854775808.0 && d < 18446744073709551616.0)) return false;
        return (u64)d == i.bits;
    }
    if (!(d >= -9223372036854775808.0 && d < 9223372036854775808.0)) return false;
    return (i64)d == (i64)i.bits;
}

__device__ bool bytes_eq(const u8* a, const u8* b, u32 n) {
    for (u32 k = 0; k < n; k++)
        if (a[k] != b[k]) return false;
    return true;
}

__device__ bool py_eq(const DVal& a, const DVal& b) {
    if (a.cls == V_NIL || b.cls == V_NIL) return a.cls == b.cls;
    if (a.cls == V_INT && b.cls == V_INT) return a.big == b.big && a.bits == b.bits;
    if (a.cls == V_FLOAT && b.cls == V_FLOAT) return __longlong_as_double((i64)a.bits) == __longlong_as_double((i64)b.bits);
    if (a.cls == V_INT && b.cls == V_FLOAT) return int_eq_float(a, __longlong_as_double((i64)b.bits));
    if (a.cls == V_FLOAT && b.cls == V_INT) return int_eq_float(b, __longlong_as_double((i64)a.bits));
    if (a.cls != b.cls) return false;
    if (a.cls == V_EXT && a.ext != b.ext) return false;
    return a.len == b.len && bytes_eq(a.p, b.p, a.len);
}

// header: 0x92, str(40) legend hex, array header -> returns 0 ok
__device__ int parse_header(const u8* b, u32 n, const u8** leg, u32* nvals, u32* off) {
    if (n < 3 || b[0] != 0x92) return 1;
    DVal lv;
    u32 c = dv_decode(b + 1, b + n, lv);
    if (!c || lv.cls != V_STR || lv.len != 40) return 1;
    *leg = lv.p;
    u32 o = 1 + c;
    if (o >= n) return 1;
    u8 t = b[o];
    if (t >= 0x90 && t <= 0x9f) { *nvals = t & 15; o += 1; }
    else if (t == 0xdc) { if (o + 3 > n) return 1; *nvals = (u32)ld_be(b + o + 1, 2); o += 3; }
    else if (t == 0xdd) { if (o + 5 > n) return 1; *nvals = (u32)ld_be(b + o + 1, 4); o += 5; }
    else return 1;
    *off = o;
    return 0;
}

// device-side tables (built by the host per call)
struct FdTab {
    int n_keys, words, n_lo, n_ln, maxv;
    const u8* leg_o;        // [n_lo*40]
    const u8* leg_n;        // [n_ln*40]
    const i16* map_o;       // [n_lo*n_keys]
    const i16* map_n;       // [n_ln*n_keys]
    const u64* cmp;         // [words]
    const u8* aligned;      // [n_lo*n_ln]: maps identical on every compared key
    const i16* key_of_val;  // [n_lo*maxv]: union key of value v of legend lo (-1 none / not compared)
    const u32* nv_o;        // [n_lo] value count of each old legend (number of non-pk columns)
};

__device__ __forceinline__ int find_legend(const u8* tab, int n, const u8* hex) {
    for (int l = 0; l < n; l++) {
        const u8* t = tab + 40 * l;
        bool eq = true;
        for (int k = 0; k < 40 && eq; k++) eq = t[k] == hex[k];
        if (eq) return l;
    }
    return -1;
}

constexpr int FD_MAXV = 128;
constexpr int FD_NT = 64;  // one wave per block: each lane owns one update and two LDS slots

// Stage [p, p+len) into an LDS slot with 16-B loads from the 16-B aligned-down address, all issued
// before any use (one HBM latency instead of one per byte).  Returns the LDS pointer of byte p, or
// nullptr when the blob does not fit (the lane then parses straight from global memory).
template <int SLOT>
__device__ __forceinline__ const u8* stage_blob(const u8* __restrict__ data, u64 start, u32 len, u64 arena_end,
                                                u32x4* slot) {
    (void)arena_end;
    // 16-byte chunks of the aligned-down *absolute* address: an aligned chunk that holds a valid
    // byte lies in one mapped page, so reading the whole chunk cannot fault.
    const u64 a0 = (u64)data + start;
    const u64 base = a0 & ~(u64)15;
    const u32 delta = (u32)(a0 - base);
    const u32 nch = (delta + len + 15) >> 4;
    if (nch * 16 > (u32)SLOT) return nullptr;
    typedef const __attribute__((address_space(1))) u32x4* gp;
    constexpr int B = 8;  // chunks in flight per batch (branch-free issue, then LDS stores)
#pragma unroll
    for (int c0 = 0; c0 < SLOT / 16; c0 += B) {
        if (c0 >= (int)nch) break;
        u32x4 v[B];
#pragma unroll
        for (int k = 0; k < B; k++) {
            const int c = c0 + k < (int)nch ? c0 + k : c0;
            v[k] = *(gp)(base + 16ull * c);
        }
#pragma unroll
        for (int k = 0; k < B; k++)
            if (c0 + k < (int)nch) slot[c0 + k] = v[k];
    }
    return (const u8*)slot + delta;
}

template <int SLOT>
__global__ __launch_bounds__(FD_NT) void k_fielddiff(const u8* __restrict__ od, const u64* __restrict__ ooff, u64 on_blobs,
                                                     const u8* __restrict__ nd, const u64* __restrict__ noff, u64 nn_blobs,
                                                     const uint2* __restrict__ pairs, u64 n_upd_host,
                                                     const u64* __restrict__ n_upd_dev, FdTab tb,
                                                     u64* __restrict__ masks, u8* __restrict__ status) {
    __shared__ u32x4 s_slots[SLOT > 0 ? FD_NT * 2 * (SLOT / 16) : 1];
    const u64 n_upd = n_upd_dev ? *n_upd_dev : n_upd_host;
    const u64 o_end = ooff[on_blobs], n_end = noff[nn_blobs];
    const int lane = threadIdx.x;
    for (u64 u0 = (u64)blockIdx.x * FD_NT; u0 < n_upd; u0 += (u64)gridDim.x * FD_NT) {
        const u64 u = u0 + lane;
        if (u >= n_upd) break;
        u64 oi = pairs ? pairs[u].x : u, ni = pairs ? pairs[u].y : u;
        const u64 os = ooff[oi], ns = noff[ni];
        const u32 on = (u32)(ooff[oi + 1] - os);
        const u32 nn = (u32)(noff[ni + 1] - ns);
        const u8* ob = nullptr;
        const u8* nb = nullptr;
        if constexpr (SLOT > 0) {
            u32x4* my = s_slots + (size_t)lane * 2 * (SLOT / 16);
            ob = stage_blob<SLOT>(od, os, on, o_end, my);
            nb = stage_blob<SLOT>(nd, ns, nn, n_end, my + SLOT / 16);
        }
        if (!ob) ob = od + os;
        if (!nb) nb = nd + ns;
        u64* m = masks + u * tb.words;
        u64 mk[4] = {0, 0, 0, 0};  // mask words kept in registers for <= 256 keys
        u8 st = 0;
        const u8 *lo, *ln;
        u32 cvo, cvn, po, pn;
        int li_o = -1, li_n = -1;
        if (parse_header(ob, on, &lo, &cvo, &po) || parse_header(nb, nn, &ln, &cvn, &pn)) st = 1;
        else {
            li_o = find_legend(tb.leg_o, tb.n_lo, lo);
            li_n = find_legend(tb.leg_n, tb.n_ln, ln);
            if (li_o < 0 || li_n < 0) st = 2;
        }
        if (!st && tb.aligned[li_o * tb.n_ln + li_n] && cvo == cvn) {
            // ---- lockstep: value v of both blobs belongs to the same union key ----
            const i16* kov = tb.key_of_val + (u64)li_o * tb.maxv;
            u32 pa = po, pb = pn;
            for (u32 v = 0; v < cvo; v++) {
                DVal a, b;
                u32 ca = dv_decode(ob + pa, ob + on, a), cb = dv_decode(nb + pb, nb + nn, b);
                if (!ca || !cb) { st = 4; break; }
                pa += ca; pb += cb;
                int k = v < (u32)tb.maxv ? kov[v] : -1;
                if (k >= 0 && !py_eq(a, b)) {
                    if (k < 256) mk[k >> 6] |= 1ull << (k & 63);
                    else m[k >> 6] |= 1ull << (k & 63);
                }
            }
            if (!st && (pa != on || pb != nn)) st = 4;  // trailing bytes: unpackb raises ExtraData
        } else if (!st) {
            // ---- general: resolve each union key through both maps ----
            if (cvo > FD_MAXV || cvn > FD_MAXV) st = 3;
            u32 vo[FD_MAXV], vn[FD_MAXV];
            u32 p = po;
            for (u32 v = 0; v < cvo && !st; v++) { DVal x; u32 c = dv_decode(ob + p, ob + on, x); if (!c) st = 4; vo[v] = p; p += c; }
            if (!st && p != on) st = 4;
            p = pn;
            for (u32 v = 0; v < cvn && !st; v++) { DVal x; u32 c = dv_decode(nb + p, nb + nn, x); if (!c) st = 4; vn[v] = p; p += c; }
            if (!st && p != nn) st = 4;
            const i16* mo = tb.map_o + (u64)(li_o < 0 ? 0 : li_o) * tb.n_keys;
            const i16* mn = tb.map_n + (u64)(li_n < 0 ? 0 : li_n) * tb.n_keys;
            for (int k = 0; k < tb.n_keys && !st; k++) {
                if (!((tb.cmp[k >> 6] >> (k & 63)) & 1)) continue;
                const int so = mo[k], sn = mn[k];
                bool changed;
                if (so == -1 || sn == -1) changed = !(so == -1 && sn == -1);
                else if (so == -3 || sn == -3) {
                    if (so == -3 && sn == -3) changed = false;
                    else { st = 4; break; }
                } else {
                    DVal a, b;
                    if (so == -2) a.cls = V_NIL;
                    else if ((u32)so >= cvo) { st = 1; break; }
                    else dv_decode(ob + vo[so], ob + on, a);
                    if (sn == -2) b.cls = V_NIL;
                    else if ((u32)sn >= cvn) { st = 1; break; }
                    else dv_decode(nb + vn[sn], nb + nn, b);
                    changed = !py_eq(a, b);
                }
                if (changed) {
                    if (k < 256) mk[k >> 6] |= 1ull << (k & 63);
                    else m[k >> 6] |= 1ull << (k & 63);
                }
            }
        }
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
    tb.leg_o = base + o_lo; tb.leg_n = base + o_ln;
    tb.map_o = (const i16*)(base + o_mo); tb.map_n = (const i16*)(base + o_mn);
    tb.cmp = (const u64*)(base + o_cmp); tb.aligned = base + o_al;
    tb.key_of_val = (const i16*)(base + o_kov); tb.nv_o = (const u32*)(base + o_nv);

    // ---- inputs ----
    const void *d_od, *d_ooff, *d_nd, *d_noff, *d_pu = nullptr;
    u64 ob_bytes = 0, nb_bytes = 0;
    if (ob->mem == KD_MEM_HOST) ob_bytes = ob->off[ob->n];
    if (nb->mem == KD_MEM_HOST) nb_bytes = nb->off[nb->n];
    if ((rc = stage_in(ctx, "fd.ooff", ob->off, (ob->n + 1) * 8, ob->mem, &d_ooff))) return rc;
    if ((rc = stage_in(ctx, "fd.od", ob->data, ob_bytes ? ob_bytes : 1, ob->mem, &d_od))) return rc;
    if ((rc = stage_in(ctx, "fd.noff", nb->off, (nb->n + 1) * 8, nb->mem, &d_noff))) return rc;
    if ((rc = stage_in(ctx, "fd.nd", nb->data, nb_bytes ? nb_bytes : 1, nb->mem, &d_nd))) return rc;
    if (pu && n_upd) {
        if ((rc = stage_in(ctx, "fd.pu", pu, n_upd * 8, pairs_mem, &d_pu))) return rc;
    } else if (pu) {
        d_pu = pu;  // device pairs with a device count
    }
    u64 *d_masks = masks;
    u8* d_status = status;
    if (out_mem == KD_MEM_HOST && n_upd) {
        void *a, *b;
        if ((rc = ensure(ctx, "fd.masks", n_upd * W * 8, &a))) return rc;
        if ((rc = ensure(ctx, "fd.status", n_upd, &b))) return rc;
        d_masks = (u64*)a;
        d_status = (u8*)b;
    }
    if (n_upd == 0 && d_n_upd == nullptr) return KD_OK;
    u64 work = d_n_upd ? (u64)1 << 22 : n_upd;  // device count: size the grid for the capacity
    unsigned blocks = (unsigned)std::min<u64>((work + FD_NT - 1) / FD_NT, 256ull * 32);
    if (blocks == 0) blocks = 1;
    // LDS slot per blob, from the largest typical blob (kd_blobs.size_hint; host arenas: measured).
    // Blobs that do not fit a slot are parsed from global memory by their lane.
    auto max_len = [](const kd_blobs* b) -> u64 {
        if (b->size_hint) return b->size_hint;
        u64 m = 0;
        if (b->mem == KD_MEM_HOST)
            for (u64 i = 0; i < b->n; i++) m = std::max<u64>(m, b->off[i + 1] - b->off[i]);
        return m ? m : 256;
    };
    const u64 need = std::max(max_len(ob), max_len(nb)) + 15;
    const int slot = need <= 160 ? 160 : need <= 256 ? 256 : need <= 512 ? 512 : 0;
    rc = launch(ctx, "k_fielddiff", [&] {
        auto args = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(FD_NT), 0, ctx->stream, (const u8*)d_od, (const u64*)d_ooff,
                               ob->n, (const u8*)d_nd, (const u64*)d_noff, nb->n, (const uint2*)d_pu, n_upd, d_n_upd,
                               tb, d_masks, d_status);
        };
        if (slot == 160) args(k_fielddiff<160>);
        else if (slot == 256) args(k_fielddiff<256>);
        else if (slot == 512) args(k_fielddiff<512>);
        else args(k_fielddiff<0>);
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
