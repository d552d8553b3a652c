// kd_geomheads.cpp — the geometry heads of feature blobs (host C++, multithreaded).
//
// The spatially filtered diff needs, per feature blob, only its geometry value's GPKG header and
// stored envelope (or point).  A blob reader that holds the blob bytes anyway (kd_odb_read_batch)
// extracts them here: one msgpack walk per blob, as msgpack.unpackb does it (nested values skipped,
// trailing bytes refused), the legend looked up, the geometry column's value located
// (kart/dataset3.py:185-223 get_feature, kart/schema.py:66-79 legend positions), and its first 40
// bytes kept with its length and offset.  kd_geom_filter_heads then reads 48 contiguous bytes per
// delta side instead of two or three scattered lines of every blob.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include "kartdiff.h"

namespace {

typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

u64 be(const u8* p, int w) {
    u64 v = 0;
    for (int i = 0; i < w; i++) v = (v << 8) | p[i];
    return v;
}

// one msgpack object at p (containers nested, a count of values still pending instead of
// recursion): bytes consumed, 0 when malformed or truncated
u64 skip_one(const u8* p, const u8* e) {
    const u8* q = p;
    u64 pending = 1;
    while (pending) {
        if (q >= e || pending > (u64)(e - q)) return 0;  // every value takes at least one byte
        const u8 c = *q++;
        pending--;
        u64 n = 0;
        if (c <= 0x7f || c >= 0xe0 || c == 0xc0 || c == 0xc2 || c == 0xc3) continue;
        if ((c & 0xe0) == 0xa0) n = c & 31;
        else if ((c & 0xf0) == 0x90) { pending += c & 15; continue; }
        else if ((c & 0xf0) == 0x80) { pending += 2 * (c & 15); continue; }
        else {
            auto len = [&](int w, u64 extra) -> bool {
                if ((u64)(e - q) < (u64)w) return false;
                n = be(q, w) + extra;
                q += w;
                return true;
            };
            switch (c) {
                case 0xcc: case 0xd0: n = 1; break;
                case 0xcd: case 0xd1: n = 2; break;
                case 0xce: case 0xd2: case 0xca: n = 4; break;
                case 0xcf: case 0xd3: case 0xcb: n = 8; break;
                case 0xd9: case 0xc4: if (!len(1, 0)) return 0; break;
                case 0xda: case 0xc5: if (!len(2, 0)) return 0; break;
                case 0xdb: case 0xc6: if (!len(4, 0)) return 0; break;
                case 0xd4: n = 2; break;
                case 0xd5: n = 3; break;
                case 0xd6: n = 5; break;
                case 0xd7: n = 9; break;
                case 0xd8: n = 17; break;
                case 0xc7: if (!len(1, 1)) return 0; break;
                case 0xc8: if (!len(2, 1)) return 0; break;
                case 0xc9: if (!len(4, 1)) return 0; break;
                case 0xdc: if ((u64)(e - q) < 2) return 0; pending += be(q, 2); q += 2; continue;
                case 0xdd: if ((u64)(e - q) < 4) return 0; pending += be(q, 4); q += 4; continue;
                case 0xde: if ((u64)(e - q) < 2) return 0; pending += 2 * be(q, 2); q += 2; continue;
                case 0xdf: if ((u64)(e - q) < 4) return 0; pending += 2 * be(q, 4); q += 4; continue;
                default: return 0;  // 0xc1
            }
        }
        if ((u64)(e - q) < n) return 0;
        q += n;
    }
    return (u64)(q - p);
}

// the head of one feature blob
void head_of(const u8* b, u64 n, int n_leg, const u8* leg_hex, const int16_t* gidx, kd_geom_head* h) {
    std::memset(h, 0, sizeof *h);
    h->goff_status = KD_GH_FALLBACK << 24;
    const u8* e = b + n;
    if (n == 0 || skip_one(b, e) != n) return;  // msgpack.unpackb raises (ExtraData included)
    u64 o, cnt;
    if (b[0] >= 0x90 && b[0] <= 0x9f) { cnt = b[0] & 15; o = 1; }
    else if (b[0] == 0xdc) { cnt = be(b + 1, 2); o = 3; }
    else if (b[0] == 0xdd) { cnt = be(b + 1, 4); o = 5; }
    else return;
    if (cnt != 2) return;  // legend, values = ...
    // the legend: a str of 40 bytes (str8 / str16 / str32 header)
    u64 sl, sh;
    const u8 t = b[o];
    if (t == 0xd9) { sl = be(b + o + 1, 1); sh = 2; }
    else if (t == 0xda) { sl = be(b + o + 1, 2); sh = 3; }
    else if (t == 0xdb) { sl = be(b + o + 1, 4); sh = 5; }
    else return;
    if (sl != 40) return;
    int li = -1;
    for (int l = 0; l < n_leg && li < 0; l++)
        if (!std::memcmp(leg_hex + 40 * l, b + o + sh, 40)) li = l;
    if (li < 0) return;
    const int gi = gidx[li];
    if (gi < 0) { h->goff_status = KD_GH_NULL << 24; return; }  // no geometry column: the value is None
    o += sh + 40;
    const u8 a = b[o];
    u64 nv;
    if (a >= 0x90 && a <= 0x9f) { nv = a & 15; o += 1; }
    else if (a == 0xdc) { nv = be(b + o + 1, 2); o += 3; }
    else if (a == 0xdd) { nv = be(b + o + 1, 4); o += 5; }
    else return;  // values not an array
    if ((u64)gi >= nv) return;
    for (int i = 0; i < gi; i++) o += skip_one(b + o, e);  // validated above: never 0
    const u8 v = b[o];
    if (v == 0xc0) { h->goff_status = KD_GH_NULL << 24; return; }
    u64 pl, ph;
    if (v >= 0xd4 && v <= 0xd8) { pl = 1ull << (v - 0xd4); ph = 2; }
    else if (v >= 0xc7 && v <= 0xc9) { const int w = 1 << (v - 0xc7); pl = be(b + o + 1, w); ph = 2 + w; }
    else return;  // not an ext value
    if (b[o + ph - 1] != 'G') return;
    const u64 goff = o + ph;
    if (goff >= (1ull << 24) || pl > 0xFFFFFFFFull) return;  // (the reference would not care: the host decides)
    h->glen = (u32)pl;
    std::memcpy(h->gpkg, b + goff, std::min<u64>(pl, sizeof h->gpkg));
    h->goff_status = (u32)goff | (KD_GH_GEOM << 24);
}

}  // namespace

extern "C" int kd_geom_heads(const uint8_t* data, const uint64_t* off, uint64_t n, int n_leg, const uint8_t* leg_hex,
                             const int16_t* gidx, int threads, kd_geom_head* out) {
    if ((n && (!data || !off || !out)) || n_leg < 0 || (n_leg && (!leg_hex || !gidx))) return KD_EINVAL;
    const unsigned hc = std::thread::hardware_concurrency();
    const int nt = threads > 0 ? std::min(threads, 256) : (int)std::max(1u, std::min(hc ? hc : 1u, 16u));
    constexpr u64 CH = 4096;
    const u64 nch = (n + CH - 1) / CH;
    std::atomic<u64> next{0};
    auto work = [&]() {
        for (;;) {
            const u64 c = next.fetch_add(1);
            if (c >= nch) break;
            for (u64 i = c * CH; i < std::min(n, (c + 1) * CH); i++)
                head_of(data + off[i], off[i + 1] - off[i], n_leg, leg_hex, gidx, out + i);
        }
    };
    const int use = (int)std::max<u64>(1, std::min<u64>((u64)nt, nch));
    std::vector<std::thread> th;
    for (int t = 1; t < use; t++) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    return KD_OK;
}
