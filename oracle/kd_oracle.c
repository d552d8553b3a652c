/*
 * kd_oracle.c — CPU restatement of the reference's bulk feature-diff path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker: it is linked/loaded only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product (kart_amd/, libkartdiff)
 * never includes, links or calls it.  Written independently of the HIP kernels (plain,
 * sequential C99 + __int128) so a bug is not shared between the checker and the checked.
 *
 * Parity pin: every function here is checked against the golden vectors under tests/golden/,
 * which were produced by running the reference's own Python (tests/golden/gen_golden.py).
 *
 * Reference semantics restated (file:line in /root/reference):
 *   classify2  — libgit2 tree-to-tree diff as consumed by RichBaseDataset.diff_feature
 *                (kart/rich_base_dataset.py:205-300): path only in old -> delete, only in new ->
 *                insert, both with different blob OID -> update.
 *   classify3  — libgit2 git_merge_trees OID rule (kart/merge.py:99-100).
 *   fielddiff  — Dataset3.get_feature (kart/dataset3.py:185-223) + Legend/Schema projection
 *                (kart/schema.py:66-79,288-293) + the text writer's field compare with Python ==
 *                (kart/text_diff_writer.py:135-145).
 *   envelopes  — geom_envelope (kart/geometry.py:638-700), SpatialFilter.matches bbox prefilter
 *                (kart/spatial_filter/__init__.py:534-590,709-734), identity-CRS
 *                get_envelope_for_indexing (kart/spatial_filter/index.py:551-579,639-707,783-813),
 *                EnvelopeEncoder (index.py:485-548 == vendor/spatial-filter/spatial_filter.cpp:30-152),
 *                cyclic_range_overlaps (spatial_filter.cpp:170-208).
 *
 * Must be compiled with -ffp-contract=off (see oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KDO_NONE 0xFFFFFFFFu

typedef __int128 i128;

/* ------------------------------------------------------------------------------------------ */
/* keys                                                                                       */
/* ------------------------------------------------------------------------------------------ */

/* Python floor division / modulo on 128-bit ints (dataset3_paths.py:292-299 uses // and %). */
static i128 pyfloordiv(i128 a, i128 b) {
    i128 q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1;
    return q;
}

/* int-PK join key: bucket24 (= IntPathEncoder tree number) | wrap(34, biased) | pk mod 64.
 * Bijective for pk in [-2^63, 2^63); returns -1 outside. */
int kdo_int_pk_key(int64_t pk_hi_sign, uint64_t pk_mag, uint64_t* key_out) {
    i128 pk = pk_hi_sign ? -(i128)pk_mag : (i128)pk_mag;
    i128 q = pyfloordiv(pk, 64);
    i128 r = pk - q * 64;
    i128 bucket = q - pyfloordiv(q, (i128)1 << 24) * ((i128)1 << 24);
    i128 k = pyfloordiv(pk, (i128)1 << 30) + ((i128)1 << 33);
    if (k < 0 || k >= ((i128)1 << 34)) return -1;
    *key_out = ((uint64_t)bucket << 40) | ((uint64_t)k << 6) | (uint64_t)r;
    return 0;
}

static const char B64URL[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

/* urlsafe base64 of msgpack([pk]) (serialise_util.py:34-41,64-66 + dataset3_paths.py:164-165): the
 * IntPathEncoder filename.  Returns its length. */
static int int_pk_filename(int64_t pk, char* out) {
    uint8_t m[10];
    int L = 0, w = 0;
    m[L++] = 0x91;
    if (pk >= -32 && pk <= 127) m[L++] = (uint8_t)pk;
    else if (pk > 0) {
        if (pk <= 0xff) { m[L++] = 0xcc; w = 1; }
        else if (pk <= 0xffff) { m[L++] = 0xcd; w = 2; }
        else if (pk <= 0xffffffffll) { m[L++] = 0xce; w = 4; }
        else { m[L++] = 0xcf; w = 8; }
    } else {
        if (pk >= -128) { m[L++] = 0xd0; w = 1; }
        else if (pk >= -32768) { m[L++] = 0xd1; w = 2; }
        else if (pk >= INT32_MIN) { m[L++] = 0xd2; w = 4; }
        else { m[L++] = 0xd3; w = 8; }
    }
    for (int k = w - 1; k >= 0; k--) m[L++] = (uint8_t)((uint64_t)pk >> (8 * k));
    int o = 0;
    for (int i = 0; i < L; i += 3) {
        uint32_t v = (uint32_t)m[i] << 16;
        if (i + 1 < L) v |= (uint32_t)m[i + 1] << 8;
        if (i + 2 < L) v |= m[i + 2];
        out[o++] = B64URL[(v >> 18) & 63];
        out[o++] = B64URL[(v >> 12) & 63];
        out[o++] = i + 1 < L ? B64URL[(v >> 6) & 63] : '=';
        out[o++] = i + 2 < L ? B64URL[v & 63] : '=';
    }
    return o;
}

static int ascii_rank(char c) {
    int r = 0;
    for (int i = 0; i < 64; i++) r += (unsigned char)B64URL[i] < (unsigned char)c;
    return r;
}

static int name_cmp(const char* a, int na, const char* b, int nb) {
    int n = na < nb ? na : nb;
    int c = memcmp(a, b, (size_t)n);
    return c ? c : (na > nb) - (na < nb);
}

/* The int-PK join key in git tree order, restated from its definition (DESIGN.md "join key"): the
 * four tree characters of the IntPathEncoder path (dataset3_paths.py:292-299) as ASCII ranks, the
 * pk's 2^30 wrap, and the filename's rank among the 64 filenames of its block [pk - pk%64, +64) —
 * found by encoding and comparing all 64 names, as git's bytewise tree order would. */
int kdo_int_walk_key(int64_t pk, uint64_t* key_out) {
    i128 q = pyfloordiv((i128)pk, 64);
    int64_t s = (int64_t)(q * 64);
    i128 bucket = q - pyfloordiv(q, (i128)1 << 24) * ((i128)1 << 24);
    uint64_t rb = 0;
    for (int k = 3; k >= 0; k--) rb = (rb << 6) | (uint64_t)ascii_rank(B64URL[(int)(bucket >> (6 * k)) & 63]);
    i128 wrap = pyfloordiv((i128)pk, (i128)1 << 30) + ((i128)1 << 33);
    char me[16], other[16];
    int nme = int_pk_filename(pk, me), rank = 0;
    for (int j = 0; j < 64; j++) {
        int no = int_pk_filename(s + j, other);
        rank += name_cmp(other, no, me, nme) < 0;
    }
    *key_out = rb << 40 | (uint64_t)wrap << 6 | (uint64_t)rank;
    return 0;
}

static int b64val(unsigned char c) {
    const char* p = (c == 0) ? NULL : strchr(B64URL, c);
    return p ? (int)(p - B64URL) : -1;
}

/* urlsafe base64 decode (serialise_util.py:69-71); returns length or -1 */
static int b64url_decode(const uint8_t* s, int n, uint8_t* out, int cap) {
    int o = 0, acc = 0, bits = 0;
    for (int i = 0; i < n; i++) {
        if (s[i] == '=') break;
        int v = b64val(s[i]);
        if (v < 0) return -1;
        acc = (acc << 6) | v;
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            if (o >= cap) return -1;
            out[o++] = (uint8_t)((acc >> bits) & 0xFF);
        }
    }
    return o;
}

/* filename -> int pk (Dataset3.decode_path_to_1pk, dataset3.py:250-259). 0 ok, -1 not an int pk */
int kdo_decode_int_filename(const uint8_t* name, int n, int64_t* neg, uint64_t* mag) {
    uint8_t buf[32];
    int m = b64url_decode(name, n, buf, sizeof buf);
    if (m < 2 || buf[0] != 0x91) return -1;
    const uint8_t* p = buf + 1;
    int rem = m - 1;
    uint8_t t = p[0];
    uint64_t u = 0;
    int64_t s = 0;
    int is_signed = 0, need = 0;
    if (t <= 0x7f) { u = t; need = 1; }
    else if (t >= 0xe0) { s = (int8_t)t; is_signed = 1; need = 1; }
    else if (t == 0xcc || t == 0xcd || t == 0xce || t == 0xcf) {
        int w = 1 << (t - 0xcc); need = 1 + w;
        if (rem < need) return -1;
        for (int i = 0; i < w; i++) u = (u << 8) | p[1 + i];
    } else if (t == 0xd0 || t == 0xd1 || t == 0xd2 || t == 0xd3) {
        int w = 1 << (t - 0xd0); need = 1 + w;
        if (rem < need) return -1;
        uint64_t v = 0;
        for (int i = 0; i < w; i++) v = (v << 8) | p[1 + i];
        int sh = 64 - 8 * w;
        s = (int64_t)(v << sh) >> sh;
        is_signed = 1;
    } else return -1;
    if (rem != need) return -1;
    if (is_signed) { *neg = s < 0; *mag = s < 0 ? (uint64_t)(-(i128)s) : (uint64_t)s; }
    else { *neg = 0; *mag = u; }
    return 0;
}

/* FNV-1a 64 of the filename bytes: within-bucket order key for hashed-path datasets. */
static uint64_t fnv1a64(const uint8_t* p, int n) {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; }
    return h;
}

/* Hashed-path join key (MsgpackHashPathEncoder, dataset3_paths.py:202-215): the tree levels
 * as a bucket number in git's tree order (each base64 character's ASCII rank, or the hex digit),
 * then 40/48 bits of FNV-1a of the filename.  path = "c1/c2/c3/c4/<filename>" relative to feature/.  levels*bits_per_level
 * bucket bits.  Returns -1 on malformed paths. */
int kdo_hash_path_key(const uint8_t* path, int n, int levels, int hex, uint64_t* key_out) {
    uint64_t bucket = 0;
    int pos = 0, bits = 0;
    for (int l = 0; l < levels; l++) {
        int seg_len = hex ? 2 : 1;
        for (int c = 0; c < seg_len; c++) {
            if (pos >= n) return -1;
            int v;
            uint8_t ch = path[pos++];
            if (hex) {
                if (ch >= '0' && ch <= '9') v = ch - '0';
                else if (ch >= 'a' && ch <= 'f') v = ch - 'a' + 10;
                else return -1;
                bucket = (bucket << 4) | (uint64_t)v; bits += 4;
            } else {
                v = b64val(ch);
                if (v < 0) return -1;
                /* git orders tree names bytewise: the digit's place in ASCII order */
                bucket = (bucket << 6) | (uint64_t)ascii_rank((char)ch); bits += 6;
            }
        }
        if (pos >= n || path[pos] != '/') return -1;
        pos++;
    }
    int low = 64 - bits;
    uint64_t h = fnv1a64(path + pos, n - pos);
    *key_out = (bucket << low) | (h >> (64 - low));
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* classify2 / classify3                                                                      */
/* ------------------------------------------------------------------------------------------ */

/* Sequential merge-join of two strictly ascending key arrays.  Writes deltas in key order as
 * (base index | KDO_NONE, target index | KDO_NONE).  counts[0..2] = inserts, updates, deletes.
 * Returns number of deltas, or -1 if a side is not strictly ascending. */
int64_t kdo_classify2(uint64_t nA, const uint64_t* kA, const uint8_t* oA,
                      uint64_t nB, const uint64_t* kB, const uint8_t* oB,
                      uint32_t* out_a, uint32_t* out_b, uint64_t* counts) {
    for (uint64_t i = 1; i < nA; i++) if (kA[i - 1] >= kA[i]) return -1;
    for (uint64_t j = 1; j < nB; j++) if (kB[j - 1] >= kB[j]) return -1;
    uint64_t i = 0, j = 0, d = 0;
    counts[0] = counts[1] = counts[2] = 0;
    while (i < nA || j < nB) {
        if (j >= nB || (i < nA && kA[i] < kB[j])) {
            out_a[d] = (uint32_t)i; out_b[d] = KDO_NONE; d++; counts[2]++; i++;
        } else if (i >= nA || kB[j] < kA[i]) {
            out_a[d] = KDO_NONE; out_b[d] = (uint32_t)j; d++; counts[0]++; j++;
        } else {
            if (memcmp(oA + 20 * i, oB + 20 * j, 20) != 0) {
                out_a[d] = (uint32_t)i; out_b[d] = (uint32_t)j; d++; counts[1]++;
            }
            i++; j++;
        }
    }
    return (int64_t)d;
}

static int oid_eq(const uint8_t* a, const uint8_t* b) { return memcmp(a, b, 20) == 0; }

/* Three-way merge classification (libgit2 OID rule), per key with (a,o,t):
 *   o==t -> o ; a==o -> t ; a==t -> o ; else conflict.   (x==y includes both-absent)
 * Outputs, in key order:
 *   conflicts (a,o,t indices | NONE)
 *   merge deltas (o,t) where result != ours: the entry to take from theirs (t) replacing
 *   ours' (o); t == NONE means delete ours' entry.
 * counts[0] = merged entries present (clean), counts[1] = conflicts, counts[2] = merge deltas.
 * Returns 0, or -1 if a side is not strictly ascending. */
int64_t kdo_classify3(uint64_t nA, const uint64_t* kA, const uint8_t* oA,
                      uint64_t nO, const uint64_t* kO, const uint8_t* oO,
                      uint64_t nT, const uint64_t* kT, const uint8_t* oT,
                      uint32_t* c_a, uint32_t* c_o, uint32_t* c_t,
                      uint32_t* m_o, uint32_t* m_t, uint64_t* counts) {
    for (uint64_t x = 1; x < nA; x++) if (kA[x - 1] >= kA[x]) return -1;
    for (uint64_t x = 1; x < nO; x++) if (kO[x - 1] >= kO[x]) return -1;
    for (uint64_t x = 1; x < nT; x++) if (kT[x - 1] >= kT[x]) return -1;
    uint64_t i = 0, j = 0, k = 0, nc = 0, nm = 0, clean = 0;
    while (i < nA || j < nO || k < nT) {
        uint64_t key = UINT64_MAX;
        if (i < nA && kA[i] < key) key = kA[i];
        if (j < nO && kO[j] < key) key = kO[j];
        if (k < nT && kT[k] < key) key = kT[k];
        int ha = i < nA && kA[i] == key, ho = j < nO && kO[j] == key, ht = k < nT && kT[k] == key;
        const uint8_t* a = ha ? oA + 20 * i : NULL;
        const uint8_t* o = ho ? oO + 20 * j : NULL;
        const uint8_t* t = ht ? oT + 20 * k : NULL;
#define EQ(x, y) ((!(x) && !(y)) || ((x) && (y) && oid_eq((x), (y))))
        int res; /* 0 = ours, 1 = theirs, 2 = conflict */
        if (EQ(o, t)) res = 0;
        else if (EQ(a, o)) res = 1;
        else if (EQ(a, t)) res = 0;
        else res = 2;
#undef EQ
        uint32_t ia = ha ? (uint32_t)i : KDO_NONE, io = ho ? (uint32_t)j : KDO_NONE, it = ht ? (uint32_t)k : KDO_NONE;
        if (res == 2) {
            c_a[nc] = ia; c_o[nc] = io; c_t[nc] = it; nc++;
        } else if (res == 0) {
            if (ho) clean++;
        } else {
            if (ht) clean++;
            m_o[nm] = io; m_t[nm] = it; nm++;
        }
        if (ha) i++;
        if (ho) j++;
        if (ht) k++;
    }
    counts[0] = clean; counts[1] = nc; counts[2] = nm;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* msgpack values + Python == (fielddiff)                                                     */
/* ------------------------------------------------------------------------------------------ */

enum { V_NIL = 0, V_INT = 1, V_FLOAT = 2, V_STR = 3, V_BYTES = 4, V_EXT = 5, V_BAD = 15 };

typedef struct {
    int cls;
    i128 ival;       /* V_INT (bool folded in: True == 1) */
    double fval;     /* V_FLOAT */
    const uint8_t* p; /* STR / BYTES / EXT payload */
    uint32_t len;
    int ext;         /* ext type code */
} kval;

static uint64_t be(const uint8_t* p, int w) {
    uint64_t v = 0;
    for (int i = 0; i < w; i++) v = (v << 8) | p[i];
    return v;
}

/* Decode one msgpack value at p (bounded by end).  Returns bytes consumed, 0 on error.
 * Mirrors msgpack.unpackb(raw=False, ext_hook=serialise_util._msg_unpack_ext_hook):
 * ext 'G' (71) -> Geometry (bytes; empty -> None); other ext -> ExtType; containers -> V_BAD. */
static uint32_t decode_value(const uint8_t* p, const uint8_t* end, kval* v) {
    if (p >= end) return 0;
    uint8_t t = p[0];
    uint64_t avail = (uint64_t)(end - p);
#define NEED(n) do { if ((uint64_t)(n) > avail) return 0; } while (0)
    v->cls = V_BAD;
    if (t <= 0x7f) { v->cls = V_INT; v->ival = t; return 1; }
    if (t >= 0xe0) { v->cls = V_INT; v->ival = (int8_t)t; return 1; }
    if (t >= 0xa0 && t <= 0xbf) { uint32_t n = t & 31; NEED(1 + n); v->cls = V_STR; v->p = p + 1; v->len = n; return 1 + n; }
    switch (t) {
    case 0xc0: v->cls = V_NIL; return 1;
    case 0xc2: v->cls = V_INT; v->ival = 0; return 1;
    case 0xc3: v->cls = V_INT; v->ival = 1; return 1;
    case 0xcc: case 0xcd: case 0xce: case 0xcf: {
        int w = 1 << (t - 0xcc); NEED(1 + w);
        v->cls = V_INT; v->ival = (i128)be(p + 1, w); return 1 + w; }
    case 0xd0: case 0xd1: case 0xd2: case 0xd3: {
        int w = 1 << (t - 0xd0); NEED(1 + w);
        int sh = 64 - 8 * w;
        v->cls = V_INT; v->ival = (i128)((int64_t)(be(p + 1, w) << sh) >> sh); return 1 + w; }
    case 0xca: { NEED(5); uint32_t b = (uint32_t)be(p + 1, 4); float f; memcpy(&f, &b, 4); v->cls = V_FLOAT; v->fval = (double)f; return 5; }
    case 0xcb: { NEED(9); uint64_t b = be(p + 1, 8); double d; memcpy(&d, &b, 8); v->cls = V_FLOAT; v->fval = d; return 9; }
    case 0xd9: case 0xda: case 0xdb: case 0xc4: case 0xc5: case 0xc6: {
        int w = (t == 0xd9 || t == 0xc4) ? 1 : (t == 0xda || t == 0xc5) ? 2 : 4;
        NEED(1 + w); uint32_t n = (uint32_t)be(p + 1, w); NEED((uint64_t)1 + w + n);
        v->cls = (t >= 0xd9) ? V_STR : V_BYTES; v->p = p + 1 + w; v->len = n; return 1 + w + n; }
    case 0xd4: case 0xd5: case 0xd6: case 0xd7: case 0xd8: {
        uint32_t n = 1u << (t - 0xd4); NEED(2 + n);
        v->ext = (int8_t)p[1]; v->p = p + 2; v->len = n; break; }
    case 0xc7: case 0xc8: case 0xc9: {
        int w = 1 << (t - 0xc7); NEED(2 + w); uint32_t n = (uint32_t)be(p + 1, w); NEED((uint64_t)2 + w + n);
        v->ext = (int8_t)p[1 + w]; v->p = p + 2 + w; v->len = n;
        if (v->ext == 'G') goto geom;
        v->cls = V_EXT; return 2 + w + n;
    geom:
        if (n == 0) { v->cls = V_NIL; return 2 + w + n; }     /* Geometry.of(b"") -> None */
        if (n < 2 || v->p[0] != 'G' || v->p[1] != 'P') { v->cls = V_BAD; return 0; }
        v->cls = V_BYTES; return 2 + w + n; }
    default:
        return 0; /* containers, 0xc1: unsupported as field values */
    }
    /* fixext */
    {
        uint32_t n = 1u << (t - 0xd4);
        if (v->ext == 'G') {
            if (n < 2 || v->p[0] != 'G' || v->p[1] != 'P') { v->cls = V_BAD; return 0; }
            v->cls = V_BYTES; return 2 + n;
        }
        v->cls = V_EXT; return 2 + n;
    }
#undef NEED
}

/* exact int == float (Python int/float comparison is exact) */
static int int_eq_float(i128 i, double d) {
    if (!(d == d)) return 0;
    if (d != floor(d)) return 0;
    if (d < -1.8446744073709552e19 * 2 || d > 1.8446744073709552e19 * 2) return 0;
    /* |d| < 2^65 here, exactly representable in i128 */
    return (i128)d == i;
}

static int py_eq(const kval* a, const kval* b) {
    if (a->cls == V_NIL || b->cls == V_NIL) return a->cls == b->cls;
    if (a->cls == V_INT && b->cls == V_INT) return a->ival == b->ival;
    if (a->cls == V_FLOAT && b->cls == V_FLOAT) return a->fval == b->fval;
    if (a->cls == V_INT && b->cls == V_FLOAT) return int_eq_float(a->ival, b->fval);
    if (a->cls == V_FLOAT && b->cls == V_INT) return int_eq_float(b->ival, a->fval);
    if (a->cls != b->cls) return 0;
    if (a->cls == V_EXT && a->ext != b->ext) return 0;
    return a->len == b->len && memcmp(a->p, b->p, a->len) == 0;
}

/* Legend-map codes (host precomputed per side, per legend, per union key) */
#define KD_SRC_NULL (-1)  /* key not in this side's schema: old.get(k, _NULL) -> _NULL */
#define KD_SRC_NONE (-2)  /* key in schema, column id absent from this legend -> None */
#define KD_SRC_PK   (-3)  /* primary-key column: value comes from the path */

/* Parse blob header: 0x92, str(40) legend hex, array header.  Returns value-array offset or -1. */
static int parse_header(const uint8_t* b, uint32_t n, const uint8_t** legend_hex, uint32_t* nvals, uint32_t* off) {
    if (n < 3 || b[0] != 0x92) return -1;
    kval lv;
    uint32_t c = decode_value(b + 1, b + n, &lv);
    if (!c || lv.cls != V_STR || lv.len != 40) return -1;
    *legend_hex = lv.p;
    uint32_t o = 1 + c;
    if (o >= n) return -1;
    uint8_t t = b[o];
    if (t >= 0x90 && t <= 0x9f) { *nvals = t & 15; o += 1; }
    else if (t == 0xdc) { if (o + 3 > n) return -1; *nvals = (uint32_t)be(b + o + 1, 2); o += 3; }
    else if (t == 0xdd) { if (o + 5 > n) return -1; *nvals = (uint32_t)be(b + o + 1, 4); o += 5; }
    else return -1;
    *off = o;
    return 0;
}

/* fielddiff: for each update u, mask bit k set iff union key k changed (Python !=).
 *   old blob of update u = old_data[old_off[oi]:old_off[oi+1]], oi = old_idx ? old_idx[u] : u
 *   legends: n_leg 40-byte hex strings per side; maps: [n_leg][n_keys] int16 source codes
 *   cmp_mask: [words] keys to compare (keys starting "__" are excluded by the host)
 *   status[u]: 0 ok, 1 malformed blob, 2 unknown legend, 3 too many values, 4 unsupported value
 * Returns 0. */
int kdo_fielddiff(uint64_t n_upd,
                  const uint8_t* old_data, const uint64_t* old_off, const uint32_t* old_idx,
                  const uint8_t* new_data, const uint64_t* new_off, const uint32_t* new_idx,
                  int n_keys, int words,
                  int n_leg_old, const uint8_t* leg_old_hex, const int16_t* map_old,
                  int n_leg_new, const uint8_t* leg_new_hex, const int16_t* map_new,
                  const uint64_t* cmp_mask,
                  uint64_t* masks, uint8_t* status) {
    enum { MAXV = 4096 };
    static __thread uint32_t voff_o[MAXV], voff_n[MAXV];  /* per thread: the bench runs shards in parallel */
    for (uint64_t u = 0; u < n_upd; u++) {
        uint64_t oi = old_idx ? old_idx[u] : u, ni = new_idx ? new_idx[u] : u;
        const uint8_t* ob = old_data + old_off[oi];
        uint32_t on = (uint32_t)(old_off[oi + 1] - old_off[oi]);
        const uint8_t* nb = new_data + new_off[ni];
        uint32_t nn = (uint32_t)(new_off[ni + 1] - new_off[ni]);
        uint64_t* m = masks + u * words;
        for (int w = 0; w < words; w++) m[w] = 0;
        status[u] = 0;
        const uint8_t *lo, *ln;
        uint32_t cvo, cvn, po, pn;
        if (parse_header(ob, on, &lo, &cvo, &po) || parse_header(nb, nn, &ln, &cvn, &pn)) { status[u] = 1; continue; }
        int li_o = -1, li_n = -1;
        for (int l = 0; l < n_leg_old; l++) if (!memcmp(leg_old_hex + 40 * l, lo, 40)) { li_o = l; break; }
        for (int l = 0; l < n_leg_new; l++) if (!memcmp(leg_new_hex + 40 * l, ln, 40)) { li_n = l; break; }
        if (li_o < 0 || li_n < 0) { status[u] = 2; continue; }
        if (cvo > MAXV || cvn > MAXV) { status[u] = 3; continue; }
        int bad = 0;
        uint32_t p = po;
        for (uint32_t i = 0; i < cvo && !bad; i++) { kval v; uint32_t c = decode_value(ob + p, ob + on, &v); if (!c) bad = 1; voff_o[i] = p; p += c; }
        if (!bad && p != on) bad = 1;   /* trailing bytes: msgpack.unpackb raises ExtraData */
        p = pn;
        for (uint32_t i = 0; i < cvn && !bad; i++) { kval v; uint32_t c = decode_value(nb + p, nb + nn, &v); if (!c) bad = 1; voff_n[i] = p; p += c; }
        if (!bad && p != nn) bad = 1;
        if (bad) { status[u] = 4; continue; }
        const int16_t* mo = map_old + (size_t)li_o * n_keys;
        const int16_t* mn = map_new + (size_t)li_n * n_keys;
        for (int k = 0; k < n_keys; k++) {
            if (!((cmp_mask[k >> 6] >> (k & 63)) & 1)) continue;
            int so = mo[k], sn = mn[k];
            int changed;
            if (so == KD_SRC_NULL || sn == KD_SRC_NULL) changed = !(so == KD_SRC_NULL && sn == KD_SRC_NULL);
            else if (so == KD_SRC_PK || sn == KD_SRC_PK) {
                if (so == KD_SRC_PK && sn == KD_SRC_PK) changed = 0;   /* same path -> same pk */
                else { status[u] = 4; break; }
            } else {
                kval a, b;
                if (so == KD_SRC_NONE) a.cls = V_NIL;
                else { if ((uint32_t)so >= cvo) { status[u] = 1; break; } decode_value(ob + voff_o[so], ob + on, &a); }
                if (sn == KD_SRC_NONE) b.cls = V_NIL;
                else { if ((uint32_t)sn >= cvn) { status[u] = 1; break; } decode_value(nb + voff_n[sn], nb + nn, &b); }
                changed = !py_eq(&a, &b);
            }
            if (changed) m[k >> 6] |= 1ull << (k & 63);
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* envelopes                                                                                  */
/* ------------------------------------------------------------------------------------------ */

static double rd_f64(const uint8_t* p, int le) {
    uint64_t b = 0;
    if (le) for (int i = 7; i >= 0; i--) b = (b << 8) | p[i];
    else for (int i = 0; i < 8; i++) b = (b << 8) | p[i];
    double d; memcpy(&d, &b, 8); return d;
}

static uint32_t rd_u32(const uint8_t* p, int le) {
    return le ? (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24
              : (uint32_t)p[3] | (uint32_t)p[2] << 8 | (uint32_t)p[1] << 16 | (uint32_t)p[0] << 24;
}

/* geom_envelope(g, only_2d=True) (geometry.py:638-700).
 * Returns 1 + env (minx,maxx,miny,maxy) when stored; 0 = None (empty, NaN);
 * 2 = no stored envelope (caller computes, e.g. point WKB); -1 malformed / unsupported. */
int kdo_gpkg_envelope(const uint8_t* g, uint64_t n, double env[4]) {
    if (n < 8 || g[0] != 'G' || g[1] != 'P') return -1;
    if (g[2] != 0) return -1;
    uint8_t flags = g[3];
    if (flags & 0x20) return -1;
    if (flags & 0x10) return 0;
    int et = (flags >> 1) & 7;
    static const int sizes[5] = {0, 32, 48, 48, 64};
    if (et > 4) return -1;
    if (et == 0) return 2;
    if (n < (uint64_t)(8 + sizes[et])) return -1;
    int le = flags & 1;
    for (int i = 0; i < 4; i++) env[i] = rd_f64(g + 8 + 8 * i, le);
    for (int i = 0; i < 4; i++) if (env[i] != env[i]) return 0;
    return 1;
}

/* Point envelope from WKB after the header (OGR GetEnvelope of a point = (x, x, y, y)).
 * Returns 1 ok, 0 empty point (NaN coords: OGR reports an empty point, envelope (0,0,0,0)),
 * -1 not a point / malformed. */
int kdo_point_envelope(const uint8_t* g, uint64_t n, double env[4]) {
    uint8_t flags = g[3];
    static const int sizes[5] = {0, 32, 48, 48, 64};
    int et = (flags >> 1) & 7;
    if (et > 4) return -1;
    uint64_t off = 8 + sizes[et];
    if (n < off + 5) return -1;
    int le = g[off] == 1;
    uint32_t typ = rd_u32(g + off + 1, le);
    uint32_t flat = typ & 0x0fffffff;
    if (flat >= 1000) flat %= 1000;
    if (flat != 1) return -1;
    if (n < off + 5 + 16) return -1;
    double x = rd_f64(g + off + 5, le), y = rd_f64(g + off + 13, le);
    if (x != x && y != y) { env[0] = env[1] = env[2] = env[3] = 0.0; return 0; }
    env[0] = x; env[1] = x; env[2] = y; env[3] = y;
    return 1;
}

/* _range_overlaps (spatial_filter/__init__.py:709-725). -1 = inverted range (reference raises). */
static int range_overlaps(double a1, double a2, double b1, double b2) {
    if (a1 > a2 || b1 > b2) return -1;
    if (b1 < a1) return b2 > a1;
    if (a1 < b1) return a2 > b1;
    return (b2 != b1) && (a2 != a1);
}

/* bbox_intersects_fast(a, b), a/b = (minx, maxx, miny, maxy).  1/0, -1 on inverted range. */
int kdo_bbox_intersects(const double a[4], const double b[4]) {
    int x = range_overlaps(a[0], a[1], b[0], b[1]);
    if (x <= 0) return x;
    return range_overlaps(a[2], a[3], b[2], b[3]);
}

/* Python float % (Objects/floatobject.c float_rem semantics) */
static double py_fmod(double a, double b) {
    double m = fmod(a, b);
    if (m != 0.0) {
        if ((b < 0) != (m < 0)) m += b;
    } else {
        m = copysign(0.0, b);
    }
    return m;
}

double kdo_wrap_lon(double x) { return py_fmod(x + 180.0, 360.0) - 180.0; }

/* identity-CRS get_envelope_for_indexing (index.py:551-579 with transform_minmax_envelope
 * :639-707 for an identity transform; the union of one envelope is itself).
 * in: 2D envelope (minx,maxx,miny,maxy).  out wsen.  Returns 1, or 0 = None (width >= 180). */
int kdo_index_envelope(const double gpkg[4], double out[4]) {
    double e0 = gpkg[0], e1 = gpkg[2], e2 = gpkg[1], e3 = gpkg[3]; /* transpose -> minx,miny,maxx,maxy */
    if (e0 == e2 && e1 == e3) {
        double x = kdo_wrap_lon(e0);
        out[0] = x; out[1] = e1; out[2] = x; out[3] = e1;
        return 1;
    }
    double width = e2 - e0, height = e3 - e1;
    if (width >= 180) return 0;
    double big = width;                       /* Python max(width, height) */
    if (height > big) big = height;
    double buf = (big < 1.0) ? 0.1 * big : 0.1;
    double t0 = e0 - buf;
    double t1 = e1 - buf; if (-90.0 > t1) t1 = -90.0;   /* max(e1 - b, -90) */
    double t2 = e2 + buf;
    double t3 = e3 + buf; if (90.0 < t3) t3 = 90.0;     /* min(e3 + b, 90) */
    out[0] = kdo_wrap_lon(t0); out[1] = t1; out[2] = kdo_wrap_lon(t2); out[3] = t3;
    return 1;
}

/* EnvelopeEncoder.encode (index.py:507-530; spatial_filter.cpp:74-107).  bits even, <= 32.
 * out: bits/2 bytes big-endian.  Returns 0, -1 if a value is out of range (reference asserts). */
int kdo_envelope_encode(const double wsen[4], int bits, uint8_t* out) {
    const double mins[4] = {-180, -90, -180, -90}, maxs[4] = {180, 90, 180, 90};
    double vmax = (double)(((uint64_t)1 << bits) - 1);
    unsigned __int128 acc = 0;
    for (int i = 0; i < 4; i++) {
        double v = wsen[i];
        if (!(mins[i] <= v && v <= maxs[i])) return -1;
        double norm = (v - mins[i]) / (maxs[i] - mins[i]);
        double sc = norm * vmax;
        double r = (i < 2) ? floor(sc) : ceil(sc);
        if (r < 0 || r > vmax) return -1;
        acc = (acc << bits) | (uint64_t)r;
    }
    int nbytes = bits / 2;
    for (int i = nbytes - 1; i >= 0; i--) { out[i] = (uint8_t)(acc & 0xFF); acc >>= 8; }
    return 0;
}

/* EnvelopeEncoder.decode (index.py:532-548; spatial_filter.cpp:109-130) */
void kdo_envelope_decode(const uint8_t* in, int bits, double wsen[4]) {
    const double mins[4] = {-180, -90, -180, -90}, maxs[4] = {180, 90, 180, 90};
    double vmax = (double)(((uint64_t)1 << bits) - 1);
    unsigned __int128 acc = 0;
    for (int i = 0; i < bits / 2; i++) acc = (acc << 8) | in[i];
    uint64_t m = ((uint64_t)1 << bits) - 1;
    for (int i = 3; i >= 0; i--) {
        uint64_t q = (uint64_t)(acc & m);
        acc >>= bits;
        double norm = (double)q / vmax;
        wsen[i] = norm * (maxs[i] - mins[i]) + mins[i];
    }
}

/* cyclic_range_overlaps (spatial_filter.cpp:187-208) */
static int cyclic_overlaps(double a1, double a2, double b1, double b2) {
    if (a1 > a2) a2 += 360;
    if (b1 > b2) b2 += 360;
    int r = range_overlaps(a1, a2, b1, b2);
    if (r) return r;
    if (a1 < b1) { a1 += 360; a2 += 360; } else { b1 += 360; b2 += 360; }
    return range_overlaps(a1, a2, b1, b2);
}

/* sf_filter_blob decision for an indexed blob (spatial_filter.cpp:212-260): decode and test
 * cyclic(w,e,qw,qe) && range(s,n,qs,qn).  Returns 1 match / 0 no / -1 inverted range (abort). */
int kdo_envelope_overlap(const uint8_t* enc, int bits, const double q[4]) {
    double e[4];
    kdo_envelope_decode(enc, bits, e);
    int c = cyclic_overlaps(e[0], e[2], q[0], q[2]);
    if (c <= 0) return c;
    return range_overlaps(e[1], e[3], q[1], q[3]);
}

/* Envelope used by SpatialFilter.matches (spatial_filter/__init__.py:556-568): the stored GPKG
 * envelope, else OGR GetEnvelope of the geometry (empty -> (0,0,0,0); point -> (x,x,y,y)).
 * Returns 1 with env set, -1 when a full geometry walk would be needed (CPU fallback). */
static int matches_envelope(const uint8_t* g, uint64_t n, double env[4]) {
    int r = kdo_gpkg_envelope(g, n, env);
    if (r == 1) return 1;
    if (r < 0) return -1;
    if (n >= 4 && (g[3] & 0x10)) { env[0] = env[1] = env[2] = env[3] = 0.0; return 1; }
    int p = kdo_point_envelope(g, n, env);
    return p >= 0 ? 1 : -1;
}

/* Envelope used for indexing: geom.envelope(only_2d=True, calculate_if_missing=True)
 * (geometry.py:638-700): stored env; NaN in stored -> None; EMPTY -> None (and the indexer
 * skips empties, index.py:346); no stored env -> OGR (empty point -> None, point -> x,x,y,y).
 * Returns 1 env set, 0 None, -1 fallback. */
static int index_source_envelope(const uint8_t* g, uint64_t n, double env[4]) {
    int r = kdo_gpkg_envelope(g, n, env);
    if (r == 1 || r == 0 || r < 0) return r;
    int p = kdo_point_envelope(g, n, env);
    return p == 1 ? 1 : (p == 0 ? 0 : -1);
}

/* Batch spatial work over n geometry blobs (GPKG bytes; length 0 = null geometry).
 *   match[i]: 0 NON_MATCHING, 1 CANDIDATE (bbox passed; GEOS refine is out of scope),
 *             2 MATCHING (null geometry), 3 FALLBACK (needs the CPU path)
 *   enc[i*bits/2 ..]: EnvelopeEncoder bytes of the identity-CRS index envelope, enc_ok[i] = 1
 *   when the indexer would store a row for this blob.
 * Returns the number of CANDIDATE results. */
int64_t kdo_envelope_batch(uint64_t n, const uint8_t* data, const uint64_t* off,
                           const double filt[4], int bits, uint8_t* match, uint8_t* enc, uint8_t* enc_ok) {
    int nb = bits / 2;
    int64_t npass = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t* g = data + off[i];
        uint64_t len = off[i + 1] - off[i];
        double env[4], src[4], wsen[4];
        memset(enc + i * nb, 0, nb);
        enc_ok[i] = 0;
        if (len == 0) { match[i] = 2; continue; }
        if (matches_envelope(g, len, env) < 0) { match[i] = 3; }
        else {
            int hit = kdo_bbox_intersects(filt, env);
            if (hit < 0) match[i] = 3;
            else { match[i] = (uint8_t)hit; npass += hit; }
        }
        if (len >= 4 && (g[3] & 0x10)) continue;          /* geom.is_empty(): not indexed */
        int r = index_source_envelope(g, len, src);
        if (r != 1) continue;
        if (kdo_index_envelope(src, wsen) != 1) continue;
        if (kdo_envelope_encode(wsen, bits, enc + i * nb) != 0) { memset(enc + i * nb, 0, nb); continue; }
        enc_ok[i] = 1;
    }
    return npass;
}

/* sf_filter_blob (vendor/spatial-filter/spatial_filter.cpp:212-260) over a batch of m objects.
 * The index (feature_envelopes) is given sorted by blob id (memcmp order, as sqlite's primary key
 * orders BLOBs): idx_oid [n_idx*20], idx_env [n_idx*bits/2].  is_feature [m] may be NULL (all
 * feature blobs).  out[i]: 0 MR_MATCH (not a feature path :219-223, not in the index :236-238, or
 * overlapping :249-255), 1 MR_NOT_MATCHED, 2 MR_ERROR (inverted range: the reference aborts). */
void kdo_sf_filter_batch(uint64_t n_idx, const uint8_t* idx_oid, const uint8_t* idx_env, int bits, uint64_t m,
                         const uint8_t* oid, const uint8_t* is_feature, const double q[4], uint8_t* out) {
    int nb = bits / 2;
    for (uint64_t i = 0; i < m; i++) {
        out[i] = 0;
        if (is_feature && !is_feature[i]) continue;
        uint64_t lo = 0, hi = n_idx;
        while (lo < hi) {
            uint64_t mid = lo + (hi - lo) / 2;
            if (memcmp(idx_oid + 20 * mid, oid + 20 * i, 20) < 0) lo = mid + 1; else hi = mid;
        }
        if (lo == n_idx || memcmp(idx_oid + 20 * lo, oid + 20 * i, 20) != 0) continue;
        int r = kdo_envelope_overlap(idx_env + (uint64_t)nb * lo, bits, q);
        out[i] = r < 0 ? 2 : (r ? 0 : 1);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* spatially filtered diff (kart/base_diff_writer.py:279-329 + SpatialFilter.matches,          */
/* kart/spatial_filter/__init__.py:534-605), envelope part: the C form of oracle.geom_filter     */
/* ------------------------------------------------------------------------------------------ */
enum { GF_NON = 0, GF_CAND = 1, GF_MATCH = 2, GF_FALLBACK = 3, GF_NONE = 4 };

/* one msgpack object of any kind (containers nested), as msgpack.unpackb walks it: bytes consumed,
 * 0 when malformed.  *top_ext_g / *is_nil describe a scalar (an ext 'G' payload, nil) */
static uint32_t skip_any(const uint8_t* p, const uint8_t* end, int depth) {
    if (p >= end || depth > 512) return 0;
    const uint8_t t = p[0];
    uint64_t avail = (uint64_t)(end - p), cnt = 0;
    uint32_t hdr = 0;
    int map = 0;
    if (t >= 0x90 && t <= 0x9f) { cnt = t & 15; hdr = 1; }
    else if (t >= 0x80 && t <= 0x8f) { cnt = t & 15; hdr = 1; map = 1; }
    else if (t == 0xdc || t == 0xde) { if (avail < 3) return 0; cnt = be(p + 1, 2); hdr = 3; map = t == 0xde; }
    else if (t == 0xdd || t == 0xdf) { if (avail < 5) return 0; cnt = be(p + 1, 4); hdr = 5; map = t == 0xdf; }
    else {
        kval v;
        uint32_t c = decode_value(p, end, &v);
        if (c) return c;
        /* decode_value refuses an ext 'G' payload not starting "GP"; unpackb with the oracle's hook
         * (oracle.py _gf_hook) accepts any payload: skip it by its length */
        if ((t >= 0xd4 && t <= 0xd8) || (t >= 0xc7 && t <= 0xc9)) {
            uint32_t n, h;
            if (t <= 0xd8 && t >= 0xd4) { n = 1u << (t - 0xd4); h = 2; }
            else { int w = 1 << (t - 0xc7); if (avail < (uint64_t)(2 + w)) return 0; n = (uint32_t)be(p + 1, w); h = 2 + w; }
            if ((uint64_t)h + n > avail) return 0;
            return h + n;
        }
        return 0;
    }
    uint64_t o = hdr;
    for (uint64_t i = 0; i < cnt * (map ? 2 : 1); i++) {
        uint32_t c = skip_any(p + o, end, depth + 1);
        if (!c) return 0;
        o += c;
    }
    return (uint32_t)o;
}

/* feature_geometry (oracle.py): status 0 with *g / *gn = the geometry payload (g NULL: None),
 * or GF_FALLBACK (malformed, unknown legend, value index out of range, not an ext 'G') */
static int feature_geometry_c(const uint8_t* b, uint32_t n, int n_leg, const uint8_t* leg_hex, const int16_t* gidx,
                              const uint8_t** g, uint32_t* gn) {
    *g = NULL;
    *gn = 0;
    const uint8_t* end = b + n;
    if (skip_any(b, end, 0) != n) return GF_FALLBACK;  /* unpackb raises (incl. ExtraData) */
    if (n < 1 || !((b[0] >= 0x90 && b[0] <= 0x9f) || b[0] == 0xdc || b[0] == 0xdd)) return GF_FALLBACK;
    uint32_t o = b[0] <= 0x9f ? 1 : b[0] == 0xdc ? 3 : 5;
    uint64_t cnt = b[0] <= 0x9f ? (uint64_t)(b[0] & 15) : be(b + 1, b[0] == 0xdc ? 2 : 4);
    if (cnt != 2) return GF_FALLBACK;                   /* legend, values = ... */
    kval lv;
    uint32_t c = decode_value(b + o, end, &lv);
    if (!c || lv.cls != V_STR || lv.len != 40) return GF_FALLBACK;
    int li = -1;
    for (int l = 0; l < n_leg; l++) if (!memcmp(leg_hex + 40 * l, lv.p, 40)) { li = l; break; }
    if (li < 0) return GF_FALLBACK;
    const int gi = gidx[li];
    if (gi < 0) return 0;
    o += c;
    const uint8_t t = b[o];
    uint64_t nv;
    uint32_t h;
    if (t >= 0x90 && t <= 0x9f) { nv = t & 15; h = 1; }
    else if (t == 0xdc) { nv = be(b + o + 1, 2); h = 3; }
    else if (t == 0xdd) { nv = be(b + o + 1, 4); h = 5; }
    else return GF_FALLBACK;  /* values not an array */
    if ((uint64_t)gi >= nv) return GF_FALLBACK;
    o += h;
    for (int i = 0; i < gi; i++) o += skip_any(b + o, end, 1);
    const uint8_t vt = b[o];
    if (vt == 0xc0) return 0;                          /* None */
    uint32_t pl, ph;
    if (vt >= 0xd4 && vt <= 0xd8) { pl = 1u << (vt - 0xd4); ph = 2; }
    else if (vt >= 0xc7 && vt <= 0xc9) { int w = 1 << (vt - 0xc7); pl = (uint32_t)be(b + o + 1, w); ph = 2 + w; }
    else return GF_FALLBACK;
    if ((int8_t)b[o + ph - 1] != 'G') return GF_FALLBACK;
    *g = b + o + ph;
    *gn = pl;
    return 0;
}

/* sf_envelope_code (oracle.py): SpatialFilter.matches without the exact Intersects */
static int sf_envelope_code_c(const uint8_t* g, uint32_t gn, const double filt[4], int rect) {
    static const uint8_t zero[1] = {0};
    if (!g) return GF_MATCH;                           /* geometry None: MATCHING (:549-551) */
    const uint8_t* gb = gn ? g : zero;
    double env[4];
    int r = kdo_gpkg_envelope(gb, gn, env);
    if (r < 0) return GF_FALLBACK;
    if (r == 0 && (gb[3] & 0x10)) return GF_NON;     /* empty: Intersects(empty) is False */
    if (r != 1) {
        int pc = kdo_point_envelope(gb, gn, env);
        if (pc == 0) return GF_NON;
        if (pc < 0) return GF_FALLBACK;
    }
    int x = kdo_bbox_intersects(filt, env);
    if (x < 0) return GF_FALLBACK;
    if (x == 0) return GF_NON;
    if (rect && filt[0] <= env[0] && env[1] <= filt[1] && filt[2] <= env[2] && env[3] <= filt[3]) return GF_MATCH;
    return GF_CAND;
}

/* the per-geometry body of kdo_envelope_batch */
static void envelope_one(const uint8_t* g, uint64_t len, const double filt[4], int bits, uint8_t* match, uint8_t* enc,
                         uint8_t* enc_ok) {
    int nb = bits / 2;
    double env[4], src[4], wsen[4];
    memset(enc, 0, nb);
    *enc_ok = 0;
    if (len == 0) { *match = 2; return; }
    if (matches_envelope(g, len, env) < 0) *match = 3;
    else {
        int hit = kdo_bbox_intersects(filt, env);
        *match = hit < 0 ? 3 : (uint8_t)hit;
    }
    if (len >= 4 && (g[3] & 0x10)) return;
    if (index_source_envelope(g, len, src) != 1) return;
    if (kdo_index_envelope(src, wsen) != 1) return;
    if (kdo_envelope_encode(wsen, bits, enc) != 0) { memset(enc, 0, nb); return; }
    *enc_ok = 1;
}

/* geom_filter (oracle.py): per delta d and side s, codes[2d+s] (GF_*), and the new side's index
 * envelope (enc [n*bits/2], enc_ok [n]) of the geometry when that side is neither NONE nor
 * FALLBACK.  pairs [2n] = (old blob | KD_NONE, new blob | KD_NONE).  Returns the kept count
 * (deltas with a side in CANDIDATE..FALLBACK). */
int64_t kdo_geom_filter(uint64_t n, const uint8_t* od, const uint64_t* ooff, const uint8_t* nd, const uint64_t* noff,
                        const uint32_t* pairs, int n_leg_o, const uint8_t* leg_o, const int16_t* gidx_o, int n_leg_n,
                        const uint8_t* leg_n, const int16_t* gidx_n, const double filt[4], int rect, int bits,
                        uint8_t* codes, uint8_t* enc, uint8_t* enc_ok) {
    int64_t kept = 0;
    const int nb = bits / 2;
    for (uint64_t d = 0; d < n; d++) {
        const uint8_t* gnew = NULL;
        uint32_t gnew_n = 0;
        int use_new = 0;
        for (int s = 0; s < 2; s++) {
            const uint32_t bi = pairs[2 * d + s];
            uint8_t code;
            const uint8_t* g = NULL;
            uint32_t gn = 0;
            if (bi == 0xFFFFFFFFu) code = GF_NONE;
            else {
                const uint8_t* data = s ? nd : od;
                const uint64_t* off = s ? noff : ooff;
                const int st = feature_geometry_c(data + off[bi], (uint32_t)(off[bi + 1] - off[bi]), s ? n_leg_n : n_leg_o,
                                                  s ? leg_n : leg_o, s ? gidx_n : gidx_o, &g, &gn);
                code = st ? (uint8_t)st : (uint8_t)sf_envelope_code_c(g, gn, filt, rect);
            }
            codes[2 * d + s] = code;
            if (s == 1 && code != GF_NONE && code != GF_FALLBACK) { gnew = g; gnew_n = gn; use_new = 1; }
        }
        uint8_t m;
        if (use_new && gnew) envelope_one(gnew, gnew_n, filt, bits, &m, enc + d * nb, enc_ok + d);
        else { memset(enc + d * nb, 0, nb); enc_ok[d] = 0; }
        const uint8_t a = codes[2 * d], b = codes[2 * d + 1];
        kept += (a >= 1 && a <= 3) || (b >= 1 && b <= 3);
    }
    return kept;
}

/* ------------------------------------------------------------------------------------------ */
/* writer formatting: gpkg_geom_to_hex_wkb over a geometry arena                               */
/* ------------------------------------------------------------------------------------------ */

/* kart/geometry.py:346-375 (gpkg_geom_to_hex_wkb) + :227-252 (header, envelope sizes): the WKB
 * after the GPKG header and envelope, as uppercase hex.  For blob i, status[i] = 0 with its hex at
 * hex[2 * (off[i] + start)] (start = 8 + envelope size, the layout kd_hex_encode writes), 1 for a
 * null (empty) value, 3 where the reference goes through OGR (big-endian WKB) or raises (invalid
 * GPKG, extended bit, unknown envelope, empty WKB). */
void kdo_hex_wkb_batch(uint64_t n, const uint8_t* data, const uint64_t* off, uint8_t* hex, uint8_t* status) {
    static const int env_size[8] = {0, 32, 48, 48, 64, -1, -1, -1};
    static const char digits[] = "0123456789ABCDEF";
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t* g = data + off[i];
        const uint64_t len = off[i + 1] - off[i];
        if (len == 0) { status[i] = 1; continue; }
        if (len < 8 || g[0] != 'G' || g[1] != 'P' || g[2] != 0 || (g[3] & 0x20)) { status[i] = 3; continue; }
        const int es = env_size[(g[3] >> 1) & 7];
        if (es < 0 || len <= (uint64_t)(8 + es) || g[8 + es] == 0) { status[i] = 3; continue; }
        for (uint64_t p = off[i] + 8 + es; p < off[i + 1]; p++) {
            hex[2 * p] = (uint8_t)digits[data[p] >> 4];
            hex[2 * p + 1] = (uint8_t)digits[data[p] & 15];
        }
        status[i] = 0;
    }
}
