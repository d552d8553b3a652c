// kd_spatial.hip — GPKG envelope extraction, bbox prefilter, identity-CRS index envelope,
// EnvelopeEncoder quantisation and encoded-envelope overlap, all in FP64 on gfx950.
//
// Reference (file:line under /root/reference):
//   geom_envelope ................ kart/geometry.py:638-700   (GPKG flags / envelope indicator)
//   SpatialFilter.matches ........ kart/spatial_filter/__init__.py:534-590 (stored env, else OGR
//                                   GetEnvelope: point -> (x,x,y,y), empty -> (0,0,0,0))
//   bbox_intersects_fast ......... kart/spatial_filter/__init__.py:709-734
//   get_envelope_for_indexing .... kart/spatial_filter/index.py:551-579 + transform_minmax_envelope
//                                   :639-707 (identity CRS), _buffer_minmax_envelope :783-793,
//                                   _wrap_lon :811-813 (Python float %)
//   EnvelopeEncoder .............. index.py:485-548 == vendor/spatial-filter/spatial_filter.cpp:30-152
//   cyclic_range_overlaps ........ spatial_filter.cpp:170-208
// Built with -ffp-contract=off: `a - 0.1*b`, `n*(max-min)+min` must not fuse into FMAs.
// One lane per geometry; each lane reads the 8-byte header + 32-byte envelope (or the 21-byte
// point WKB) of its blob; HBM-bound.
#include "kd_geom.h"

namespace kd {

struct EnvArgs {
    const u8* data;
    const u64* off;
    u64 n;
    double f0, f1, f2, f3;  // filter env (minx, maxx, miny, maxy)
    int bits;
    u8* match;
    u8* enc;
    u8* enc_ok;
    unsigned long long* n_cand;
};

// One lane per geometry, 256 consecutive geometries per workgroup iteration; the outputs (match
// byte, encoded envelope, ok byte) are assembled in LDS and written as contiguous dwords.
__global__ __launch_bounds__(256) void k_envelopes(EnvArgs a) {
    typedef const __attribute__((address_space(1))) u32x4* gx4;
    __shared__ u8 s_enc[256 * 16];
    __shared__ u8 s_m[256], s_ok[256];
    const int nb = a.bits / 2;
    const double vmax = (double)((1ull << a.bits) - 1);
    const int tid = threadIdx.x;
    const u64 arena_end = (u64)a.data + a.off[a.n];
    u32 cand = 0;
    for (u64 i0 = (u64)blockIdx.x * 256; i0 < a.n; i0 += (u64)gridDim.x * 256) {
        const u64 i = i0 + tid;
        u8 m = 0, ok = 0;
        for (int k = 0; k < nb; k++) s_enc[tid * nb + k] = 0;
        if (i < a.n) {
            const u64 o = a.off[i], len = a.off[i + 1] - o;
            const u8* g = a.data + o;
            double e[4] = {0, 0, 0, 0}, pe[4] = {0, 0, 0, 0};
            int r = -1, pc = -1;
            u32 hflags = 0;
            bool fast = false;
            const u64 a0 = (u64)g, a4 = a0 & ~(u64)3;
            if (len >= 8 && a4 + 48 <= arena_end) {
                u32 w[12];
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const u32x4 v = *(gx4)(a4 + 16 * k);
                    w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
                }
                const u32 sh = (u32)(a0 - a4);
                u32 rr[11];
#pragma unroll
                for (int j = 0; j < 11; j++) rr[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
                fast = env_fast(rr, len, r, e, pc, pe);
                hflags = rr[0] >> 24;
            }
            if (!fast && len > 0) {  // byte-wise reference decode (short or unusual blobs)
                r = gpkg_env(g, len, e);
                pc = -1;
                if (r == 0 || r == 2) pc = point_env(g, len, pe);
                if (r >= 0) hflags = g[3];
            }
            if (len == 0) {
                m = 2;
            } else {
                // the GPKG empty bit (r == 0 may also mean a NaN envelope); r >= 0 implies len >= 8
                const bool is_empty = r >= 0 && (hflags & 0x10);
                bool have = false;
                if (r == 1) have = true;
                else if (r >= 0) {
                    if (is_empty) { e[0] = e[1] = e[2] = e[3] = 0.0; have = true; }
                    else if (pc >= 0) { e[0] = pe[0]; e[1] = pe[1]; e[2] = pe[2]; e[3] = pe[3]; have = true; }
                }
                if (!have) m = 3;
                else {
                    int x = range_ov(a.f0, a.f1, e[0], e[1]);
                    if (x > 0) x = range_ov(a.f2, a.f3, e[2], e[3]);
                    m = x < 0 ? 3 : (u8)x;
                    cand += x > 0;
                }
                // ---- index envelope (skip empties: index.py:346) ----
                ok = index_env(r, pc, e, pe, is_empty, a.bits, vmax, [&](int k, u8 b) { s_enc[tid * nb + k] = b; });
            }
        }
        // ---- outputs through LDS: contiguous dword stores ----
        s_m[tid] = m;
        s_ok[tid] = ok;
        __syncthreads();
        const u32 cnt = (u32)(a.n - i0 < 256 ? a.n - i0 : 256);
        auto copy = [&](u8* dst, const u8* src, u32 bytes) {
            if ((((u64)dst) & 3) == 0) {
                const u32 nw = bytes >> 2;
                for (u32 k = tid; k < nw; k += 256) ((u32*)dst)[k] = ((const u32*)src)[k];
                for (u32 k = 4 * nw + tid; k < bytes; k += 256) dst[k] = src[k];
            } else {
                for (u32 k = tid; k < bytes; k += 256) dst[k] = src[k];
            }
        };
        copy(a.match + i0, s_m, cnt);
        copy(a.enc_ok + i0, s_ok, cnt);
        copy(a.enc + i0 * nb, s_enc, cnt * nb);
        __syncthreads();
    }
    // candidate count: wave reduce then one atomic per wave
    u64 c = cand;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(a.n_cand, (unsigned long long)c);
}

// 1024 consecutive encoded envelopes per workgroup iteration are moved HBM <-> LDS as contiguous
// 16-B (or 4-B) chunks — 10 KB in flight per workgroup; the per-lane byte loads of nb-byte records
// were the bound — and each lane decodes four of them.  BITS > 0: compile-time bit width (the shifts
// of the 4*bits-bit record fold to constants).
template <int BITS>
__global__ __launch_bounds__(256) void k_env_overlap(const u8* __restrict__ enc, u64 n, int bits_rt, double qw, double qs,
                                                     double qe, double qn, u8* __restrict__ out) {
    constexpr int CH = 1024;
    __shared__ __attribute__((aligned(16))) u8 s_in[CH * 16];
    __shared__ __attribute__((aligned(16))) u8 s_out[CH];
    const int bits = BITS > 0 ? BITS : bits_rt;
    const int nb = bits / 2, tid = threadIdx.x;
    const double vmax = (double)((1ull << bits) - 1);
    const u64 mask = (1ull << bits) - 1;
    auto copy = [&](u8* dst, const u8* src, u32 bytes) {
        const u64 al = ((u64)dst) | ((u64)src);
        if ((al & 15) == 0) {
            const u32 nq = bytes >> 4;
            for (u32 k = tid; k < nq; k += 256) ((u32x4*)dst)[k] = ((const u32x4*)src)[k];
            for (u32 k = 16 * nq + tid; k < bytes; k += 256) dst[k] = src[k];
        } else if ((al & 3) == 0) {
            const u32 nw = bytes >> 2;
            for (u32 k = tid; k < nw; k += 256) ((u32*)dst)[k] = ((const u32*)src)[k];
            for (u32 k = 4 * nw + tid; k < bytes; k += 256) dst[k] = src[k];
        } else {
            for (u32 k = tid; k < bytes; k += 256) dst[k] = src[k];
        }
    };
    for (u64 i0 = (u64)blockIdx.x * CH; i0 < n; i0 += (u64)gridDim.x * CH) {
        const u32 cnt = (u32)(n - i0 < CH ? n - i0 : CH);
        copy(s_in, enc + i0 * nb, cnt * nb);
        __syncthreads();
        for (u32 e = tid; e < cnt; e += 256) {
            const u8* p = s_in + e * nb;
            unsigned __int128 acc = 0;
            for (int k = 0; k < nb; k++) acc = (acc << 8) | p[k];
            double v[4];
            const double mins[4] = {-180, -90, -180, -90}, maxs[4] = {180, 90, 180, 90};
            for (int k = 3; k >= 0; k--) {
                u64 q = (u64)(acc & mask);
                acc >>= bits;
                double norm = (double)q / vmax;
                v[k] = norm * (maxs[k] - mins[k]) + mins[k];
            }
            // cyclic_range_overlaps(w, e, qw, qe) && range_overlaps(s, n, qs, qn)
            double a1 = v[0], a2 = v[2], b1 = qw, b2 = qe;
            if (a1 > a2) a2 += 360;
            if (b1 > b2) b2 += 360;
            int r = range_ov(a1, a2, b1, b2);
            if (r == 0) {
                if (a1 < b1) { a1 += 360; a2 += 360; } else { b1 += 360; b2 += 360; }
                r = range_ov(a1, a2, b1, b2);
            }
            if (r > 0) r = range_ov(v[1], v[3], qs, qn);
            s_out[e] = r < 0 ? 2 : (u8)r;
        }
        __syncthreads();
        copy(out + i0, s_out, cnt);
        __syncthreads();
    }
}

}  // namespace kd

using namespace kd;

extern "C" {

int kd_envelopes(kd_ctx* ctx, const kd_blobs* geoms, const double filt_env[4], int bits, uint8_t* match, uint8_t* enc,
                 uint8_t* enc_ok, uint32_t out_mem, uint64_t* n_candidates) {
    KD_CHECK(ctx && geoms && filt_env && match && enc && enc_ok, "kd_envelopes: NULL argument");
    KD_CHECK(bits >= 2 && bits <= 32 && bits % 2 == 0, "kd_envelopes: bits must be even and <= 32");
    KD_CHECK(filt_env[0] <= filt_env[1] && filt_env[2] <= filt_env[3], "kd_envelopes: inverted filter envelope");
    KD_HIP(hipSetDevice(ctx->device));
    const u64 n = geoms->n;
    const int nb = bits / 2;
    int rc;
    const void *d_data, *d_off;
    u64 bytes = geoms->mem == KD_MEM_HOST ? geoms->off[n] : 0;
    if ((rc = stage_in(ctx, "sp.off", geoms->off, (n + 1) * 8, geoms->mem, &d_off))) return rc;
    if ((rc = stage_in(ctx, "sp.data", geoms->data, bytes ? bytes : 1, geoms->mem, &d_data))) return rc;
    u8 *dm = match, *de = enc, *dk = enc_ok;
    if (out_mem == KD_MEM_HOST) {
        void *a, *b, *c;
        if ((rc = ensure(ctx, "sp.match", n + 1, &a)) || (rc = ensure(ctx, "sp.enc", n * nb + 1, &b)) ||
            (rc = ensure(ctx, "sp.ok", n + 1, &c)))
            return rc;
        dm = (u8*)a; de = (u8*)b; dk = (u8*)c;
    }
    void* dc;
    if ((rc = ensure(ctx, "sp.cnt", 8, &dc))) return rc;
    KD_HIP(hipMemsetAsync(dc, 0, 8, ctx->stream));
    if (n) {
        EnvArgs a;
        a.data = (const u8*)d_data; a.off = (const u64*)d_off; a.n = n;
        a.f0 = filt_env[0]; a.f1 = filt_env[1]; a.f2 = filt_env[2]; a.f3 = filt_env[3];
        a.bits = bits; a.match = dm; a.enc = de; a.enc_ok = dk; a.n_cand = (unsigned long long*)dc;
        unsigned blocks = (unsigned)std::min<u64>((n + 255) / 256, 256ull * 32);
        rc = launch(ctx, "k_envelopes", [&] {
            hipLaunchKernelGGL(k_envelopes, dim3(blocks), dim3(256), 0, ctx->stream, a);
        });
        if (rc) return rc;
    }
    if (out_mem == KD_MEM_HOST || n_candidates) {
        u64 hc = 0;
        KD_HIP(hipMemcpyAsync(&hc, dc, 8, hipMemcpyDeviceToHost, ctx->stream));
        if (out_mem == KD_MEM_HOST && n) {
            KD_HIP(hipMemcpyAsync(match, dm, n, hipMemcpyDeviceToHost, ctx->stream));
            KD_HIP(hipMemcpyAsync(enc, de, n * nb, hipMemcpyDeviceToHost, ctx->stream));
            KD_HIP(hipMemcpyAsync(enc_ok, dk, n, hipMemcpyDeviceToHost, ctx->stream));
        }
        KD_HIP(hipStreamSynchronize(ctx->stream));
        if (n_candidates) *n_candidates = hc;
        prof_flush(ctx);
    }
    return KD_OK;
}

int kd_env_overlap(kd_ctx* ctx, const uint8_t* enc, uint64_t n, int bits, const double q[4], uint8_t* out, uint32_t mem) {
    KD_CHECK(ctx && enc && q && out, "kd_env_overlap: NULL argument");
    KD_CHECK(bits >= 2 && bits <= 32 && bits % 2 == 0, "kd_env_overlap: bad bits");
    KD_HIP(hipSetDevice(ctx->device));
    const int nb = bits / 2;
    int rc;
    const void* d_enc;
    if ((rc = stage_in(ctx, "ov.enc", enc, n * nb + 1, mem, &d_enc))) return rc;
    u8* d_out = out;
    if (mem == KD_MEM_HOST) {
        void* p;
        if ((rc = ensure(ctx, "ov.out", n + 1, &p))) return rc;
        d_out = (u8*)p;
    }
    if (n) {
        unsigned blocks = (unsigned)std::min<u64>((n + 1023) / 1024, 256ull * 32);
        rc = launch(ctx, "k_env_overlap", [&] {
            if (bits == 20) hipLaunchKernelGGL(k_env_overlap<20>, dim3(blocks), dim3(256), 0, ctx->stream, (const u8*)d_enc, n, bits, q[0],
                               q[1], q[2], q[3], d_out);
            else hipLaunchKernelGGL(k_env_overlap<0>, dim3(blocks), dim3(256), 0, ctx->stream, (const u8*)d_enc, n, bits, q[0],
                               q[1], q[2], q[3], d_out);
        });
        if (rc) return rc;
    }
    if (mem == KD_MEM_HOST) {
        if (n) KD_HIP(hipMemcpyAsync(out, d_out, n, hipMemcpyDeviceToHost, ctx->stream));
        KD_HIP(hipStreamSynchronize(ctx->stream));
        prof_flush(ctx);
    }
    return KD_OK;
}

}  // extern "C"
