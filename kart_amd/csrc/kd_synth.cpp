// libkdsynth.so — host-only helpers of the seeded bench generators (kart_amd/synth.py).  Not part
// of the product ABI (include/kartdiff.h): bench.py and the tests use them to build the C4 table
//  at 50M rows in seconds instead of minutes of per-row Python.
//
//   kds_text_pks        the text pks: 12-24 characters, a fraction with multibyte UTF-8
//   kds_text_pk_paths   MsgpackHashPathEncoder paths of UTF-8 pks (kart/dataset3_paths.py:202-215)
//   kds_walk_order      git tree order of such paths
//   kds_gather_paths    a side's name arena from padded paths
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

// ---- SHA-256 (FIPS 180-4), enough for short messages ----
const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

void sha256_block(uint32_t h[8], const uint8_t* p) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
        uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = k + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

// the first word of sha256(msg) (len < 2^29)
uint32_t sha256_word0(const uint8_t* msg, size_t len) {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t full = len / 64;
    for (size_t i = 0; i < full; ++i) sha256_block(h, msg + 64 * i);
    uint8_t tail[128] = {0};
    size_t r = len - 64 * full;
    memcpy(tail, msg + 64 * full, r);
    tail[r] = 0x80;
    size_t tl = r + 9 <= 64 ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_block(h, tail);
    if (tl == 128) sha256_block(h, tail + 64);
    return h[0];
}

const char B64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

template <class F>
void parallel(uint64_t n, int threads, F f) {
    if (threads <= 1 || n < 4096) {
        f(0, n);
        return;
    }
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) {
        uint64_t a = n * t / threads, b = n * (t + 1) / threads;
        ts.emplace_back([=] { f(a, b); });
    }
    for (auto& t : ts) t.join();
}

const char PK_ASCII[] = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz-_.:";
const char* const PK_MB[] = {"\xc3\xa9", "\xc3\xbc", "\xc3\x9f", "\xc3\xb1", "\xc3\xb8", "\xc4\x81",
                             "\xce\xa9", "\xd0\xb6", "\xe4\xb8\xad", "\xe6\x97\xa5", "\xe8\xaa\x9e",
                             "\xed\x95\x9c", "\xe2\x82\xac", "\xe2\x9c\x93", "\xf0\x9f\x98\x80",
                             "\xf0\x9d\x94\x98"};

}  // namespace

extern "C" {

// Text pks of rows ``ids``: L = lmin + h % (lmax - lmin + 1) characters (h = a seeded mix of the
// id); characters 0-4 a bijective base-62 scramble of the id (pks are distinct for ids < 62^5), the
// rest seeded ASCII filler; with probability p_mb (per row) 1-3 filler characters replaced by
// 2-, 3- or 4-byte UTF-8 characters.  out: [n, w] zero-padded bytes; nb: byte lengths.
int kds_text_pks(const int64_t* ids, uint64_t n, uint64_t seed, int lmin, int lmax, double p_mb, uint8_t* out,
                 int w, int64_t* nb, int threads) {
    if (lmin < 6 || lmax < lmin || lmax > 32 || lmax + 9 > w) return -1;  // 3 multibyte chars add <= 9 B
    const int nasc = (int)sizeof(PK_ASCII) - 1, nmb = (int)(sizeof(PK_MB) / sizeof(PK_MB[0]));
    const uint64_t thr = (uint64_t)(p_mb * 9007199254740992.0);  // 2^53
    parallel(n, threads, [&](uint64_t a, uint64_t b) {
        for (uint64_t i = a; i < b; ++i) {
            uint8_t* o = out + i * (uint64_t)w;
            memset(o, 0, w);
            uint64_t id = (uint64_t)ids[i];
            uint64_t h = splitmix64(id ^ (seed * 0x9E3779B97F4A7C15ull));
            int L = lmin + (int)(h % (uint64_t)(lmax - lmin + 1));
            int code[32];
            uint64_t s = (id * 387420489ull + 0x1D3Full) % 916132832ull;  // 62^5; 3^18 coprime with it
            for (int k = 4; k >= 0; --k) {
                code[k] = (int)(s % 62);
                s /= 62;
            }
            uint64_t r = h;
            for (int j = 5; j < L; ++j) {
                r = splitmix64(r ^ (uint64_t)j);
                code[j] = (int)(r % (uint64_t)nasc);
            }
            uint64_t hm = splitmix64(h ^ 0xC4C4ull);
            if ((hm >> 11) < thr) {
                int k = 1 + (int)(splitmix64(hm) % 3);
                for (int t = 0; t < k; ++t) {
                    hm = splitmix64(hm ^ (uint64_t)(t + 1));
                    int pos = 5 + (int)(hm % (uint64_t)(L - 5));
                    code[pos] = nasc + (int)((hm >> 32) % (uint64_t)nmb);
                }
            }
            int p = 0;
            for (int j = 0; j < L; ++j) {
                if (code[j] < nasc) {
                    o[p++] = (uint8_t)PK_ASCII[code[j]];
                } else {
                    const char* m = PK_MB[code[j] - nasc];
                    size_t l = strlen(m);
                    memcpy(o + p, m, l);
                    p += (int)l;
                }
            }
            nb[i] = p;
        }
    });
    return 0;
}

// MsgpackHashPathEncoder paths of UTF-8 pks (kart/dataset3_paths.py:202-215): packed =
// msgpack([pk]) (fixstr up to 31 B, str8 up to 255 B; serialise_util.py:34-41); tree = the first 24
// bits of sha256(packed) as 4 base64 characters, one per level (b64hash, :82-85); filename =
// urlsafe base64 of packed with '=' padding (:64-66).  paths: [n, path_w] zero-padded; plen: lengths.
// Returns -1 if a path does not fit path_w.
int kds_text_pk_paths(const uint8_t* pkb, const int64_t* nb, uint64_t n, int pk_w, uint8_t* paths, int path_w,
                      int64_t* plen, int threads) {
    int bad = 0;
    parallel(n, threads, [&](uint64_t a, uint64_t b) {
        uint8_t packed[300];
        for (uint64_t i = a; i < b; ++i) {
            int64_t l = nb[i];
            uint8_t* o = paths + i * (uint64_t)path_w;
            memset(o, 0, path_w);
            if (l < 0 || l > 255 || l > pk_w) { bad = 1; continue; }
            int hl;
            packed[0] = 0x91;
            if (l <= 31) { packed[1] = (uint8_t)(0xA0 | l); hl = 2; }
            else { packed[1] = 0xD9; packed[2] = (uint8_t)l; hl = 3; }
            memcpy(packed + hl, pkb + i * (uint64_t)pk_w, (size_t)l);
            int pl = hl + (int)l;
            int fl = 4 * ((pl + 2) / 3);
            if (8 + fl > path_w) { bad = 1; continue; }
            uint32_t h = sha256_word0(packed, (size_t)pl) >> 8;  // first 24 bits
            for (int k = 0; k < 4; ++k) {
                o[2 * k] = (uint8_t)B64[(h >> (18 - 6 * k)) & 63];
                o[2 * k + 1] = '/';
            }
            uint8_t* f = o + 8;
            int q = 0;
            for (int g = 0; g < pl; g += 3) {
                uint32_t v = (uint32_t)packed[g] << 16 | (uint32_t)(g + 1 < pl ? packed[g + 1] : 0) << 8 |
                             (uint32_t)(g + 2 < pl ? packed[g + 2] : 0);
                f[q++] = (uint8_t)B64[(v >> 18) & 63];
                f[q++] = (uint8_t)B64[(v >> 12) & 63];
                f[q++] = g + 1 < pl ? (uint8_t)B64[(v >> 6) & 63] : '=';
                f[q++] = g + 2 < pl ? (uint8_t)B64[v & 63] : '=';
            }
            plen[i] = 8 + fl;
        }
    });
    return bad ? -1 : 0;
}

// Git tree order of zero-padded paths 'c/c/c/c/<filename>' (four one-character trees): by the
// tree characters, then the filename bytes (a shorter name that is a prefix of another first — the
// zero padding gives exactly that).  A counting sort on the 4 tree bytes, then each leaf tree's
// few entries sorted by memcmp.  order: [n] row indices.  Returns 1 if two paths are equal.
int kds_walk_order(const uint8_t* paths, uint64_t n, int path_w, int64_t* order, int threads) {
    // tree id = the 4 tree characters' ranks in ASCII order (24 bits)
    static int8_t rank[256];
    {
        int r = 0;
        for (int c = 0; c < 256; ++c) rank[c] = -1;
        for (int c = 0; c < 256; ++c)
            if (strchr(B64, c) && c) rank[c] = (int8_t)r++;  // ascending byte order
    }
    std::vector<uint32_t> tid(n);
    parallel(n, threads, [&](uint64_t a, uint64_t b) {
        for (uint64_t i = a; i < b; ++i) {
            const uint8_t* p = paths + i * (uint64_t)path_w;
            tid[i] = (uint32_t)rank[p[0]] << 18 | (uint32_t)rank[p[2]] << 12 | (uint32_t)rank[p[4]] << 6 | rank[p[6]];
        }
    });
    std::vector<uint64_t> start((1u << 24) + 1, 0);
    for (uint64_t i = 0; i < n; ++i) start[tid[i] + 1]++;
    for (uint32_t t = 0; t < (1u << 24); ++t) start[t + 1] += start[t];
    {
        std::vector<uint64_t> pos(start.begin(), start.end() - 1);
        for (uint64_t i = 0; i < n; ++i) order[pos[tid[i]]++] = (int64_t)i;
    }
    int dup = 0;
    parallel(1u << 24, threads, [&](uint64_t a, uint64_t b) {
        for (uint64_t t = a; t < b; ++t) {
            int64_t* s = order + start[t];
            int64_t* e = order + start[t + 1];
            if (e - s < 2) continue;
            auto less = [&](int64_t x, int64_t y) {
                return memcmp(paths + (uint64_t)x * path_w + 8, paths + (uint64_t)y * path_w + 8, path_w - 8) < 0;
            };
            std::sort(s, e, less);
            for (int64_t* q = s + 1; q < e; ++q)
                if (!less(q[-1], q[0])) dup = 1;
        }
    });
    return dup;
}

// A side's name arena: the rows' paths back to back (plen[rows[k]] bytes each); off[m+1] given
// (exclusive prefix of the lengths).
void kds_gather_paths(const uint8_t* paths, int path_w, const int64_t* plen, const int64_t* rows, uint64_t m,
                      const uint64_t* off, uint8_t* arena, int threads) {
    parallel(m, threads, [&](uint64_t a, uint64_t b) {
        for (uint64_t k = a; k < b; ++k)
            memcpy(arena + off[k], paths + (uint64_t)rows[k] * path_w, (size_t)plen[rows[k]]);
    });
}

}  // extern "C"
