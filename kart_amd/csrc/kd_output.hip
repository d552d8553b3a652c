// kd_output.hip — writer formatting on gfx950: hex encoding of geometry WKB and bytes values.
//
// Reference (file:line under /root/reference):
//   gpkg_geom_to_wkb ............. kart/geometry.py:346-364  (WKB = blob[8 + envelope size:]; a
//                                   big-endian WKB (first byte 0) goes through OGR -> CPU path)
//   gpkg_geom_to_hex_wkb ......... kart/geometry.py:367-375  (binascii.hexlify(...).upper())
//   _validate_gpkg_geom .......... kart/geometry.py:227-244, gpkg_envelope_size :247-252
//   feature_as_json .............. kart/feature_output.py:34-56 (Geometry -> to_hex_wkb(),
//                                   bytes -> bytes.hex(v), lowercase)
//
// Layout: the hex of arena byte p is written at hex[2p .. 2p+2), so every blob's string is the
// contiguous range hex[2*(off[i] + start[i]) .. 2*off[i+1]) — no length scan, no per-blob output
// offsets.  k_hex is a pure streaming transform (16 B read -> 32 B written per lane, both fully
// coalesced); the GPKG header bytes are hex-encoded too and skipped by the reader (8 B of a 29-B
// point blob), which costs less than a per-blob gather would.  k_wkb_start reads 4 header bytes
// per blob.  Both are HBM-bound.
#include "kd_internal.h"

namespace kd {

// 4 nibbles (one per byte of v, each < 16) -> 4 ASCII hex digits; no carries cross bytes.
__device__ __forceinline__ u32 hex4(u32 v, u32 alpha) {
    const u32 ge10 = ((v + 0x06060606u) >> 4) & 0x01010101u;
    return v + 0x30303030u + ge10 * alpha;
}

// two input bytes (low 16 bits of x) -> 4 chars: hi(b0) lo(b0) hi(b1) lo(b1) in memory order
__device__ __forceinline__ u32 hex2b(u32 x, u32 alpha) {
    const u32 v = ((x >> 4) & 0xFu) | ((x & 0xFu) << 8) | (((x >> 12) & 0xFu) << 16) | (((x >> 8) & 0xFu) << 24);
    return hex4(v, alpha);
}

// Streaming hex encode of bytes [0, nbytes) of `src` into `dst` (2 chars per byte).  Aligned form:
// src 16-B and dst 32-B aligned.  Each lane issues U independent 16-B loads (units t, t+G, ..,
// t+(U-1)G for G lanes in the grid: every load instruction stays fully coalesced) before its 2U
// 16-B stores; NT selects nontemporal loads/stores (streamed once, no reuse).  Ragged tail
// byte-wise by block 0.
// Default: plain loads/stores, U = 4 (C6 measured: NT x1 3.48 ms, plain x1 3.48, NT x4 4.42,
// plain x4 3.37 per 5.96-GB arena).
#ifndef KD_HEX_VARIANT
#define KD_HEX_VARIANT 3
#endif
template <bool NT, int U>
__global__ __launch_bounds__(256) void k_hex(const u8* __restrict__ src, u64 nbytes, u8* __restrict__ dst, u32 alpha) {
    const u64 n16 = nbytes >> 4;
    const u64 G = (u64)gridDim.x * 256;
    const u32x4* s4 = (const u32x4*)src;
    u32x4* d4 = (u32x4*)dst;
    for (u64 t = (u64)blockIdx.x * 256 + threadIdx.x; t < n16; t += U * G) {
        u32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const u64 q = t + k * G;
            if (q < n16) v[k] = NT ? __builtin_nontemporal_load(s4 + q) : s4[q];
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const u64 q = t + k * G;
            if (q < n16) {
                u32x4 o0, o1;
                o0.x = hex2b(v[k].x, alpha); o0.y = hex2b(v[k].x >> 16, alpha);
                o0.z = hex2b(v[k].y, alpha); o0.w = hex2b(v[k].y >> 16, alpha);
                o1.x = hex2b(v[k].z, alpha); o1.y = hex2b(v[k].z >> 16, alpha);
                o1.z = hex2b(v[k].w, alpha); o1.w = hex2b(v[k].w >> 16, alpha);
                if (NT) {
                    __builtin_nontemporal_store(o0, d4 + 2 * q);
                    __builtin_nontemporal_store(o1, d4 + 2 * q + 1);
                } else {
                    d4[2 * q] = o0;
                    d4[2 * q + 1] = o1;
                }
            }
        }
    }
    if (blockIdx.x == 0) {
        for (u64 p = 16 * n16 + threadIdx.x; p < nbytes; p += 256) {
            const u32 h = hex2b(src[p], alpha);
            dst[2 * p] = (u8)h;
            dst[2 * p + 1] = (u8)(h >> 8);
        }
    }
}
#if KD_HEX_VARIANT == 1
#define K_HEX k_hex<false, 1>
#elif KD_HEX_VARIANT == 2
#define K_HEX k_hex<true, 4>
#elif KD_HEX_VARIANT == 3
#define K_HEX k_hex<false, 4>
#elif KD_HEX_VARIANT == 4
#define K_HEX k_hex<false, 8>
#elif KD_HEX_VARIANT == 5
#define K_HEX k_hex<false, 2>
#else
#define K_HEX k_hex<true, 1>
#endif

// Unaligned form (caller-provided device pointers off the 16/32-B grid): one byte per lane.
__global__ __launch_bounds__(256) void k_hex_bytes(const u8* __restrict__ src, u64 nbytes, u8* __restrict__ dst, u32 alpha) {
    const u64 stride = (u64)gridDim.x * 256;
    for (u64 p = (u64)blockIdx.x * 256 + threadIdx.x; p < nbytes; p += stride) {
        const u32 h = hex2b(src[p], alpha);
        dst[2 * p] = (u8)h;
        dst[2 * p + 1] = (u8)(h >> 8);
    }
}

// Per GPKG blob: start[i] = 8 + envelope size (the WKB offset), status[i]:
//   0 ok, 1 null geometry (length 0 -> None), 3 needs the CPU path (not GPKG v0 / extended /
//   bad envelope indicator / truncated / empty WKB — the reference raises — or big-endian WKB,
//   which the reference re-encodes through OGR).
// All candidate WKB first bytes (offsets 8, 40, 56, 72 for envelope types 0, 1, 2-3, 4) are loaded
// together with the header, so no load depends on the flags byte (one memory round trip per blob).
__global__ __launch_bounds__(256) void k_wkb_start(const u8* __restrict__ data, const u64* __restrict__ off, u64 n,
                                                   u32* __restrict__ start, u8* __restrict__ status) {
    const u64 stride = (u64)gridDim.x * 256;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const u64 o = off[i], len = off[i + 1] - o;
        u32 s = 0;
        u8 st = 3;
        if (len == 0) {
            st = 1;
        } else if (len >= 8) {
            const u8* g = data + o;
            const u8 g0 = g[0], g1 = g[1], g2 = g[2], f = g[3];
            const u8 w8 = len > 8 ? g[8] : 0, w40 = len > 40 ? g[40] : 0, w56 = len > 56 ? g[56] : 0,
                     w72 = len > 72 ? g[72] : 0;
            const int et = (f >> 1) & 7;
            if (g0 == 'G' && g1 == 'P' && g2 == 0 && !(f & 0x20) && et <= 4) {
                s = 8 + (et == 0 ? 0 : et == 1 ? 32 : et <= 3 ? 48 : 64);
                const u8 w = et == 0 ? w8 : et == 1 ? w40 : et <= 3 ? w56 : w72;
                if (len > s && w != 0) st = 0;
            }
        }
        start[i] = s;
        status[i] = st;
    }
}

static unsigned grid_for(u64 units) { return (unsigned)std::max<u64>(1, std::min<u64>((units + 255) / 256, 256ull * 16)); }

}  // namespace kd

using namespace kd;

extern "C" {

int kd_hex_encode(kd_ctx* ctx, const kd_blobs* blobs, uint32_t mode, uint8_t* hex, uint32_t* start, uint8_t* status,
                  uint32_t out_mem) {
    KD_CHECK(ctx && blobs && hex, "kd_hex_encode: NULL argument");
    KD_CHECK(mode == KD_HEX_BYTES || mode == KD_HEX_GPKG_WKB, "kd_hex_encode: unknown mode");
    KD_CHECK(mode != KD_HEX_GPKG_WKB || (start && status), "kd_hex_encode: GPKG mode needs start and status");
    KD_HIP(hipSetDevice(ctx->device));
    const u64 n = blobs->n;
    int rc;
    const void *d_data, *d_off;
    // host form: the arena size is known on the host; device form: read off[n] (one 8-B copy)
    u64 bytes = 0;
    if (blobs->mem == KD_MEM_HOST) bytes = blobs->off[n];
    if ((rc = stage_in(ctx, "hx.off", blobs->off, (n + 1) * 8, blobs->mem, &d_off))) return rc;
    if (blobs->mem != KD_MEM_HOST) {
        KD_HIP(hipMemcpyAsync(&bytes, (const u64*)d_off + n, 8, hipMemcpyDeviceToHost, ctx->stream));
        KD_HIP(hipStreamSynchronize(ctx->stream));
    }
    if ((rc = stage_in(ctx, "hx.data", blobs->data, bytes ? bytes : 1, blobs->mem, &d_data))) return rc;
    u8* d_hex = hex;
    u32* d_start = start;
    u8* d_status = status;
    if (out_mem == KD_MEM_HOST) {
        void *a, *b = nullptr, *c = nullptr;
        if ((rc = ensure(ctx, "hx.hex", 2 * bytes + 1, &a))) return rc;
        if (mode == KD_HEX_GPKG_WKB && ((rc = ensure(ctx, "hx.start", 4 * n + 4, &b)) || (rc = ensure(ctx, "hx.st", n + 1, &c))))
            return rc;
        d_hex = (u8*)a; d_start = (u32*)b; d_status = (u8*)c;
    }
    const u32 alpha = mode == KD_HEX_GPKG_WKB ? 7u : 39u;  // 'A'-'0'-10 (upper) / 'a'-'0'-10 (lower)
    if (mode == KD_HEX_GPKG_WKB && n) {
        rc = launch(ctx, "k_wkb_start", [&] {
            hipLaunchKernelGGL(k_wkb_start, dim3(grid_for(n)), dim3(256), 0, ctx->stream, (const u8*)d_data,
                               (const u64*)d_off, n, d_start, d_status);
        });
        if (rc) return rc;
    }
    if (bytes) {
        const bool aligned = ((u64)d_data & 15) == 0 && ((u64)d_hex & 31) == 0;
        rc = launch(ctx, "k_hex", [&] {
            if (aligned)
                hipLaunchKernelGGL(K_HEX, dim3(grid_for(bytes >> 4)), dim3(256), 0, ctx->stream, (const u8*)d_data, bytes,
                                   d_hex, alpha);
            else
                hipLaunchKernelGGL(k_hex_bytes, dim3(grid_for(bytes)), dim3(256), 0, ctx->stream, (const u8*)d_data, bytes,
                                   d_hex, alpha);
        });
        if (rc) return rc;
    }
    if (out_mem == KD_MEM_HOST) {
        if (bytes) KD_HIP(hipMemcpyAsync(hex, d_hex, 2 * bytes, hipMemcpyDeviceToHost, ctx->stream));
        if (mode == KD_HEX_GPKG_WKB && n) {
            KD_HIP(hipMemcpyAsync(start, d_start, 4 * n, hipMemcpyDeviceToHost, ctx->stream));
            KD_HIP(hipMemcpyAsync(status, d_status, n, hipMemcpyDeviceToHost, ctx->stream));
        }
        KD_HIP(hipStreamSynchronize(ctx->stream));
        prof_flush(ctx);
    }
    return KD_OK;
}

}  // extern "C"
