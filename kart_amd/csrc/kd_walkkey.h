// kd_walkkey.h — the join keys, defined so that a side's leaves in git tree order (the order the
// tree walk lists them, kart/dataset3.py:225-231; libgit2's tree diff merges entries in that same
// name order, kart/rich_base_dataset.py:212-232) are already strictly ascending.
//
// KD_KEY_INT (IntPathEncoder, kart/dataset3_paths.py:283-299): a leaf's path is
//   <c1>/<c2>/<c3>/<c4>/<b64(msgpack([pk]))>,  c1..c4 = the base-64 digits of (pk // 64) % 2^24.
// git orders names bytewise, so the tree levels order by the ASCII rank of each digit's character
// ('-' < '0'..'9' < 'A'..'Z' < '_' < 'a'..'z'), not by digit value, and the filenames inside one leaf
// tree by their base-64 text.  The key
//   key = rank24(bucket) << 40 | (pk // 2^30 + 2^33) << 6 | frank(pk)
// is a bijection with pk in [-2^63, 2^63):
//   rank24  each 6-bit digit of the bucket replaced by its character's ASCII rank;
//   frank   the rank of pk's filename among the 64 filenames of its block
//           [pk - pk % 64, pk - pk % 64 + 64) — the pks sharing the bucket and the wrap.
// Every pk of one block has the same msgpack width (the width limits 128, 256, 2^16, 2^32 and
// -128, -2^15, -2^31 are multiples of 64; the one exception, [-64, -1] with fixint / int8, is a
// block of its own below), so the filenames differ only in the base-64 characters that carry the
// last msgpack byte's low 6 bits, and frank is one of 8 fixed permutations of pk % 64.  Leaves of
// one tree with one wrap value — every layer with pks in [-2^30, 2^30) whose buckets are not shared
// by a negative and a non-negative pk — are therefore in key order exactly as git lists them.  A leaf
// tree holding two wraps (|pk| >= 2^30) may list them in another order; the join's strict-order check
// reports that, and the caller sorts the side (kd_sort_side_into) — any consistent total order joins.
//
// KD_KEY_HASH (MsgpackHashPathEncoder, :202-215): key = rank-mapped bucket digits << low | FNV-1a
// bits of the filename.  The walk order is ascending in the bucket bits; inside a leaf tree it is
// filename order, which the FNV bits do not follow: kd_sort_segmented_into reorders each bucket's few
// entries (the hex legacy layout needs no rank map: '0'..'9' < 'a'..'f' in ASCII).
#pragma once
#include <cstdint>

namespace kd {
namespace wk {

typedef uint64_t wu64;
typedef int64_t wi64;

constexpr char B64[65] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

// b64(msgpack([pk])) (kart/serialise_util.py:34-41,64-66: msgpack canonical ints, urlsafe
// base64 with padding) into out; returns the length
constexpr int filename(wi64 pk, char* out) {
    unsigned char m[10] = {};
    int L = 0;
    m[L++] = 0x91;
    const wu64 u = (wu64)pk;
    int w = 0;  // payload bytes after the type byte
    if (pk >= 0 && pk <= 127) {
        m[L++] = (unsigned char)pk;
    } else if (pk < 0 && pk >= -32) {
        m[L++] = (unsigned char)(u & 0xff);
    } else if (pk > 0) {
        if (pk <= 255) { m[L++] = 0xcc; w = 1; }
        else if (pk <= 65535) { m[L++] = 0xcd; w = 2; }
        else if (pk <= 4294967295ll) { m[L++] = 0xce; w = 4; }
        else { m[L++] = 0xcf; w = 8; }
    } else {
        if (pk >= -128) { m[L++] = 0xd0; w = 1; }
        else if (pk >= -32768) { m[L++] = 0xd1; w = 2; }
        else if (pk >= -2147483648ll) { m[L++] = 0xd2; w = 4; }
        else { m[L++] = 0xd3; w = 8; }
    }
    for (int k = w - 1; k >= 0; k--) m[L++] = (unsigned char)((u >> (8 * k)) & 0xff);
    int o = 0;
    for (int i = 0; i < L; i += 3) {
        const unsigned v = (unsigned)m[i] << 16 | (i + 1 < L ? (unsigned)m[i + 1] << 8 : 0u) | (i + 2 < L ? m[i + 2] : 0u);
        out[o++] = B64[(v >> 18) & 63];
        out[o++] = B64[(v >> 12) & 63];
        out[o++] = i + 1 < L ? B64[(v >> 6) & 63] : '=';
        out[o++] = i + 2 < L ? B64[v & 63] : '=';
    }
    return o;
}

constexpr bool name_less(const char* a, int na, const char* b, int nb) {
    for (int i = 0; i < na && i < nb; i++)
        if (a[i] != b[i]) return (unsigned char)a[i] < (unsigned char)b[i];
    return na < nb;
}

// representative block starts of the 8 filename-order classes (block_class)
constexpr wi64 CLASS_BLOCK[8] = {128, 0, 64, 256, 320, 384, 448, -64};

struct Tables {
    unsigned char rank[64], irank[64];  // ASCII rank of a base-64 digit's character, and inverse
    unsigned char fr[8][64], ifr[8][64];  // frank per class: pk % 64 -> filename rank, and inverse
};

constexpr Tables make_tables() {
    Tables t{};
    for (int v = 0; v < 64; v++) {
        int r = 0;
        for (int x = 0; x < 64; x++) r += (unsigned char)B64[x] < (unsigned char)B64[v];
        t.rank[v] = (unsigned char)r;
        t.irank[r] = (unsigned char)v;
    }
    for (int c = 0; c < 8; c++) {
        char names[64][16] = {};
        int lens[64] = {};
        for (int j = 0; j < 64; j++) lens[j] = filename(CLASS_BLOCK[c] + j, names[j]);
        for (int j = 0; j < 64; j++) {
            int r = 0;
            for (int x = 0; x < 64; x++) r += name_less(names[x], lens[x], names[j], lens[j]);
            t.fr[c][j] = (unsigned char)r;
            t.ifr[c][r] = (unsigned char)j;
        }
    }
    return t;
}

// (device code reads these through the constant address space: constexpr namespace-scope data is
// implicitly __constant__ in HIP)
constexpr Tables T = make_tables();

// filename-order class of the block starting at s (s % 64 == 0): which msgpack width the block's
// pks take and which base-64 characters carry their low 6 bits
//   0  uint8 / int8 / uint32 / int32: the last character is the 6 bits themselves
//   1, 2  positive fixint blocks [0, 63], [64, 127]
//   3..6  uint16 / int16 / uint64 / int64, by bits 7..6 of the last byte
//   7  the block [-64, -1] (int8 and negative fixint names mixed)
__host__ __device__ inline int block_class(wi64 s) {
    if (s == -64) return 7;
    if (s >= 0 && s < 128) return 1 + (int)(s >> 6);
    const bool c0 = (s >= 128 && s < 256) || s == -128 || (s >= 65536 && s < 4294967296ll) ||
                    (s >= -2147483648ll && s < -32768);
    return c0 ? 0 : 3 + (int)((s & 0xff) >> 6);
}

__host__ __device__ inline wu64 rank_digits(wu64 x, int digits) {
    wu64 r = 0;
    for (int k = 0; k < digits; k++) r |= (wu64)T.rank[(x >> (6 * k)) & 63] << (6 * k);
    return r;
}

__host__ __device__ inline wu64 irank_digits(wu64 x, int digits) {
    wu64 r = 0;
    for (int k = 0; k < digits; k++) r |= (wu64)T.irank[(x >> (6 * k)) & 63] << (6 * k);
    return r;
}

// KD_KEY_INT key of pk (every int64 pk has one)
__host__ __device__ inline wu64 int_key(wi64 pk) {
    const wi64 q = pk >> 6;  // pk // 64 (arithmetic shift == floor division)
    const wi64 s = q * 64;   // block start
    const int r = (int)(pk - s);
    const wu64 bucket = (wu64)q & ((1ull << 24) - 1);
    const wu64 wrap = (wu64)((pk >> 30) + ((wi64)1 << 33));  // in [0, 2^34)
    return rank_digits(bucket, 4) << 40 | wrap << 6 | (wu64)T.fr[block_class(s)][r];
}

// inverse of int_key
__host__ __device__ inline wi64 int_key_pk(wu64 key) {
    const wu64 bucket = irank_digits(key >> 40, 4);
    const wu64 wrap = (key >> 6) & ((1ull << 34) - 1);
    // block start ((wrap - 2^33) * 2^24 + bucket) * 64, in wrapping unsigned arithmetic
    const wi64 s = (wi64)((((wrap - (1ull << 33)) << 24) + bucket) << 6);
    return s + (wi64)T.ifr[block_class(s)][key & 63];
}

}  // namespace wk
}  // namespace kd
