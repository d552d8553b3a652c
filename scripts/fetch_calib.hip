// FETCH_SIZE calibration on gfx950 for k_fielddiff's access mix (MI355X_MICROARCH.md §HBM: only
// wide coalesced streaming reads are calibrated, at 1/2).  Each pattern reads its own 512-MiB
// region of a buffer (after a 1-GiB flush read, so nothing it touches is Infinity-Cache resident);
// the addresses are a function of the thread index (no address array is read), and the host
// enumerates the same function to print what the pattern touched: requested bytes and distinct
// 32 / 64 / 128-B blocks.  Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` and divide each
// dispatch's FETCH_SIZE by those figures (scripts/fetch_calib.py).
//   0 stream16   16 B per lane, consecutive (the calibrated case: FETCH = 1/2 of the bytes)
//   1 scat16_64  one 16-B load per random 64-B line
//   2 scat16_128 one 16-B load per random 128-B block
//   3 scat4_64   one 4-B load per random 64-B line (k_fielddiff's blob-offset loads)
//   4 seg256     16 lanes x 16 B = one 256-B segment per random 256-B-aligned position
//   5 windows    k_fielddiff's LDS windows: blobs of 245-582 B, one in eight read (the updates);
//                per read blob a 5-chunk head window from the 16-B-aligned start and the chunks of a
//                4-chunk tail window ending at the last byte that the head does not cover
//   6 payloads   k_fielddiff's cooperative compare: per read blob the 16-B chunks over its
//                geometry payload (blob bytes 50 .. len-30), 16 lanes per payload
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <unordered_set>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

constexpr u64 REGION = 512ull << 20;
constexpr u64 NL = 1ull << 20;             // loads of the scatter patterns
constexpr u64 NSTREAM = (256ull << 20) / 16;
constexpr u64 SLOT = 8 * 416;              // one read blob per 8 average-size blobs
constexpr u64 NBLOB = REGION / SLOT - 1;

__host__ __device__ inline u64 mix(u64 x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
// a bijection of [0, 2^bits): odd multiplier, masked
__host__ __device__ inline u64 perm(u64 i, int bits) { return (i * 0x9E3779B97F4A7C15ull + 0x1234567ull) & ((1ull << bits) - 1); }

__host__ __device__ inline void blob(u64 k, u64* s, u64* len) {
    const u64 h = mix(k + 77);
    *len = 245 + h % 338;
    *s = k * SLOT + (h >> 20) % (SLOT - 600);
}

// windows: 9 chunk slots per blob; returns false for a tail chunk the head covers
__host__ __device__ inline bool window_chunk(u64 t, u64* a) {
    u64 s, len;
    blob(t / 9, &s, &len);
    const int c = (int)(t % 9);
    const u64 a0 = s & ~15ull;
    if (c < 5) { *a = a0 + 16 * c; return true; }
    const u64 t0 = ((s + len - 1) & ~15ull) - 16 * 3 + 16 * (c - 5);
    *a = t0;
    return t0 >= a0 + 80;
}

__global__ void k_flush(const u32x4* p, u64 n, unsigned* sink) {
    unsigned acc = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) acc ^= p[i].x;
    if (acc == 0x12345678u) *sink = acc;
}

template <int P>
__global__ void k_pat(const unsigned char* base, unsigned* sink) {
    unsigned acc = 0;
    const u64 gid = (u64)blockIdx.x * blockDim.x + threadIdx.x, gs = (u64)gridDim.x * blockDim.x;
    auto ld16 = [&](u64 a) { const u32x4 v = *(const u32x4*)(base + a); acc ^= v.x ^ v.y ^ v.z ^ v.w; };
    if (P == 0) {
        for (u64 i = gid; i < NSTREAM; i += gs) ld16(16 * i);
    } else if (P == 1) {
        for (u64 i = gid; i < NL; i += gs) ld16(64 * perm(i, 23) + 16 * (i & 3));
    } else if (P == 2) {
        for (u64 i = gid; i < NL; i += gs) ld16(128 * perm(i, 22) + 16 * (i & 7));
    } else if (P == 3) {
        for (u64 i = gid; i < NL; i += gs) acc ^= *(const unsigned*)(base + 64 * perm(i, 23) + 4 * (i & 15));
    } else if (P == 4) {
        for (u64 i = gid; i < NL; i += gs) ld16(256 * perm(i / 16, 21) + 16 * (i & 15));
    } else if (P == 5) {
        for (u64 t = gid; t < 9 * NBLOB; t += gs) {
            u64 a;
            if (window_chunk(t, &a)) ld16(a);
        }
    } else {
        for (u64 t = gid; t < 16 * NBLOB; t += gs) {
            u64 s, len;
            blob(t / 16, &s, &len);
            const u64 a = (s + 50) & ~15ull, e = s + len - 30;
            for (u64 q = a + 16 * (t & 15); q < e; q += 256) ld16(q);
        }
    }
    if (acc == 0x12345678u) *sink = acc;
}

static const char* NAMES[7] = {"stream16", "scat16_64", "scat16_128", "scat4_64", "seg256", "windows", "payloads"};

static void report(int p) {
    std::unordered_set<u64> b32, b64, b128;
    u64 loads = 0, bytes = 0;
    auto add = [&](u64 a, int w) {
        loads++;
        bytes += w;
        for (u64 q = a; q < a + w; q += 4) { b32.insert(q / 32); b64.insert(q / 64); b128.insert(q / 128); }
    };
    if (p == 0) {
        loads = NSTREAM; bytes = 16 * NSTREAM;
        printf("{\"pattern\": \"%s\", \"kernel\": \"k_pat<%d>\", \"loads\": %llu, \"bytes\": %llu, \"b32\": %llu, \"b64\": %llu, "
               "\"b128\": %llu}\n", NAMES[p], p, (unsigned long long)loads, (unsigned long long)bytes,
               (unsigned long long)bytes, (unsigned long long)bytes, (unsigned long long)bytes);
        return;
    }
    if (p == 1) for (u64 i = 0; i < NL; i++) add(64 * perm(i, 23) + 16 * (i & 3), 16);
    if (p == 2) for (u64 i = 0; i < NL; i++) add(128 * perm(i, 22) + 16 * (i & 7), 16);
    if (p == 3) for (u64 i = 0; i < NL; i++) add(64 * perm(i, 23) + 4 * (i & 15), 4);
    if (p == 4) for (u64 i = 0; i < NL; i++) add(256 * perm(i / 16, 21) + 16 * (i & 15), 16);
    if (p == 5) for (u64 t = 0; t < 9 * NBLOB; t++) { u64 a; if (window_chunk(t, &a)) add(a, 16); }
    if (p == 6)
        for (u64 k = 0; k < NBLOB; k++) {
            u64 s, len;
            blob(k, &s, &len);
            for (u64 q = (s + 50) & ~15ull; q < s + len - 30; q += 16) add(q, 16);
        }
    printf("{\"pattern\": \"%s\", \"kernel\": \"k_pat<%d>\", \"loads\": %llu, \"bytes\": %llu, \"b32\": %llu, \"b64\": %llu, "
           "\"b128\": %llu}\n", NAMES[p], p, (unsigned long long)loads, (unsigned long long)bytes,
           (unsigned long long)(32 * b32.size()), (unsigned long long)(64 * b64.size()), (unsigned long long)(128 * b128.size()));
}

int main() {
    const u64 GB = 1ull << 30;
    unsigned char *buf, *flush;
    unsigned* sink;
    CK(hipMalloc(&buf, 8 * REGION));
    CK(hipMalloc(&flush, GB));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(buf, 1, 8 * REGION));
    CK(hipMemset(flush, 2, GB));
    CK(hipDeviceSynchronize());
#define RUN(P)                                                                                          \
    do {                                                                                                \
        report(P);                                                                                      \
        fflush(stdout);                                                                                 \
        hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, (const u32x4*)flush, GB / 16, sink);   \
        hipLaunchKernelGGL(k_pat<P>, dim3(2048), dim3(256), 0, 0, buf + REGION * (P + 1), sink);          \
        CK(hipDeviceSynchronize());                                                                     \
    } while (0)
    RUN(0); RUN(1); RUN(2); RUN(3); RUN(4); RUN(5); RUN(6);
    return 0;
}
