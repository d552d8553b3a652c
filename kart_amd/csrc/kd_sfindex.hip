// kd_sfindex.hip — the clone-time spatial filter over a batch of objects (gfx950).
//
// Reference: sf_filter_blob (vendor/spatial-filter/spatial_filter.cpp:212-260), called by git once
// per object of a partial clone / fetch with `--filter=extension:spatial=w,s,e,n`:
//   * a path outside "/.sno-dataset/feature/" and "/.table-dataset/feature/" matches;
//   * a blob whose id is not in feature_envelopes matches (SQLITE_DONE);
//   * otherwise its stored envelope is decoded (EnvelopeEncoder, bits = 8 * bytes / 4) and the blob
//     matches iff cyclic_range_overlaps(w, e, qw, qe) && range_overlaps(s, n, qs, qn).
// The reference does one sqlite primary-key lookup per object.  Here the index is loaded once into
// HBM (kd_sf_index_build) and a whole batch of object ids is answered by one kernel:
//   key[i]  = the index OID's first 8 bytes, big-endian, sorted on the GPU (kd_sort_side_into);
//   order[i] = the index row of sorted key i (OIDs and envelopes stay in row order: late reads);
//   bucket[b] = first sorted position whose key's top `bb` bits are >= b (a direct-address table
//   sized for ~16 keys per bucket), so a query costs one table read plus a ~4-step binary search
//   inside its bucket, then the 20-byte compare of the (rare) equal 64-bit prefixes.
#include <algorithm>

#include "kd_internal.h"
#include "kd_geom.h"

struct kd_sf_index {
    kd_ctx* ctx = nullptr;
    uint64_t n = 0;
    int bits = 20, nb = 10, bb = 1;
    uint64_t* key = nullptr;     // [n] sorted 64-bit OID prefixes
    uint32_t* order = nullptr;   // [n] row of sorted key i
    uint8_t* oid = nullptr;      // [n*20] row order
    uint8_t* env = nullptr;      // [n*nb] row order
    uint32_t* bucket = nullptr;  // [(1 << bb) + 1]
};

namespace kd {

__device__ __forceinline__ u64 oid_prefix(u32 w0, u32 w1) {
    return ((u64)__builtin_bswap32(w0) << 32) | (u64)__builtin_bswap32(w1);
}

__global__ __launch_bounds__(256) void k_sf_keys(const u8* __restrict__ oid, u64 n, u64* __restrict__ key) {
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) {
        const u32* w = (const u32*)(oid + 20 * i);
        key[i] = oid_prefix(w[0], w[1]);
    }
}

// bucket[b] = lower bound of b << (64 - bb) in the sorted keys: thread i fills the buckets whose
// lower edge falls in (key[i-1], key[i]]; the last thread also closes the table with n
__global__ __launch_bounds__(256) void k_sf_buckets(const u64* __restrict__ key, u64 n, int bb, u32* __restrict__ bucket) {
    const int sh = 64 - bb;
    const u64 nbk = 1ull << bb;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) {
        const u64 p = key[i] >> sh;
        const u64 q = i ? (key[i - 1] >> sh) + 1 : 0;
        for (u64 b = q; b <= p; b++) bucket[b] = (u32)i;
        if (i == n - 1)
            for (u64 b = p + 1; b <= nbk; b++) bucket[b] = (u32)n;
    }
}

struct SfArgs {
    const u64* key;
    const u32* order;
    const u8* ioid;
    const u8* env;
    const u32* bucket;
    u64 n_idx;
    int bits, nb, bb;
    const u8* qoid;
    const u8* is_feature;  // may be null: every object is a feature blob
    u64 n;
    double qw, qs, qe, qn;
    u8* out;
};

// one lane per object; MR_MATCH 0 / MR_NOT_MATCHED 1 / MR_ERROR 2 as the reference's enum
__global__ __launch_bounds__(256) void k_sf_filter(SfArgs a) {
    const int sh = 64 - a.bb;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (u64)gridDim.x * 256) {
        u8 res = 0;
        if (!a.is_feature || a.is_feature[i]) {
            const u32* q = (const u32*)(a.qoid + 20 * i);
            const u32 w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
            const u64 k = oid_prefix(w0, w1);
            const u64 b = k >> sh;
            u64 lo = a.bucket[b], hi = a.bucket[b + 1];
            while (lo < hi) {
                const u64 mid = (lo + hi) >> 1;
                if (a.key[mid] < k) lo = mid + 1; else hi = mid;
            }
            for (u64 p = lo; p < a.n_idx && a.key[p] == k; p++) {
                const u64 r = a.order[p];
                const u32* o = (const u32*)(a.ioid + 20 * r);
                if (o[0] == w0 && o[1] == w1 && o[2] == w2 && o[3] == w3 && o[4] == w4) {
                    const int ov = enc_overlap(a.env + r * a.nb, a.bits, a.qw, a.qs, a.qe, a.qn);
                    res = ov < 0 ? 2 : ov ? 0 : 1;
                    break;
                }
            }
        }
        a.out[i] = res;
    }
}

static unsigned grid_for(kd_ctx* ctx, u64 n) {
    return (unsigned)std::max<u64>(1, std::min<u64>((n + 255) / 256, (u64)ctx->n_cu * 16));
}

}  // namespace kd

using namespace kd;

extern "C" {

int kd_sf_index_free(kd_sf_index* ix) {
    if (!ix) return KD_OK;
    hipError_t e = ix->ctx ? hipSetDevice(ix->ctx->device) : hipSuccess;
    for (void* p : {(void*)ix->key, (void*)ix->order, (void*)ix->oid, (void*)ix->env, (void*)ix->bucket}) {
        const hipError_t f = hipFree(p);
        if (e == hipSuccess) e = f;
    }
    delete ix;
    if (e != hipSuccess) {
        set_error("kd_sf_index_free: %s", hipGetErrorString(e));
        return KD_EHIP;
    }
    return KD_OK;
}

int kd_sf_index_build(kd_ctx* ctx, const uint8_t* oid, const uint8_t* env, uint64_t n, int bits, uint32_t mem,
                      kd_sf_index** out) {
    KD_CHECK(ctx && out && (n == 0 || (oid && env)), "kd_sf_index_build: NULL argument");
    KD_CHECK(bits >= 2 && bits <= 32 && bits % 2 == 0, "kd_sf_index_build: bits must be even and <= 32");
    KD_CHECK(n < 0xFFFFFFFFull, "kd_sf_index_build: index too large for uint32 positions");
    KD_HIP(hipSetDevice(ctx->device));
    *out = nullptr;
    kd_sf_index* ix = new kd_sf_index();
    ix->ctx = ctx;
    ix->n = n;
    ix->bits = bits;
    ix->nb = bits / 2;
    u64 want = std::max<u64>(n / 16, 2);
    while (ix->bb < 24 && (1ull << ix->bb) < want) ix->bb++;
    const u64 m = std::max<u64>(n, 1);
    hipError_t e = hipMalloc((void**)&ix->key, m * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&ix->order, m * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&ix->oid, m * 20);
    if (e == hipSuccess) e = hipMalloc((void**)&ix->env, m * ix->nb);
    if (e == hipSuccess) e = hipMalloc((void**)&ix->bucket, ((1ull << ix->bb) + 1) * 4);
    if (e != hipSuccess) {
        kd_sf_index_free(ix);
        set_error("kd_sf_index_build: hipMalloc: %s", hipGetErrorString(e));
        return KD_EHIP;
    }
    int rc = KD_OK;
    auto fail = [&](int r) { kd_sf_index_free(ix); return r; };
    const hipMemcpyKind kind = mem == KD_MEM_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    if (n) {
        if (hipMemcpyAsync(ix->oid, oid, n * 20, kind, ctx->stream) != hipSuccess ||
            hipMemcpyAsync(ix->env, env, n * ix->nb, kind, ctx->stream) != hipSuccess) {
            set_error("kd_sf_index_build: copy-in failed");
            return fail(KD_EHIP);
        }
        void* kin;
        if ((rc = ensure(ctx, "sf.kin", n * 8, &kin))) return fail(rc);
        rc = launch(ctx, "k_sf_keys", [&] {
            hipLaunchKernelGGL(k_sf_keys, dim3(grid_for(ctx, n)), dim3(256), 0, ctx->stream, (const u8*)ix->oid, n, (u64*)kin);
        });
        if (rc) return fail(rc);
        // equal 64-bit prefixes of different OIDs are legal here (the lookup compares all 20 bytes)
        if ((rc = kd_sort_side_into(ctx, (const u64*)kin, nullptr, ix->key, nullptr, ix->order, n, nullptr, nullptr)))
            return fail(rc);
        rc = launch(ctx, "k_sf_buckets", [&] {
            hipLaunchKernelGGL(k_sf_buckets, dim3(grid_for(ctx, n)), dim3(256), 0, ctx->stream, (const u64*)ix->key, n,
                               ix->bb, ix->bucket);
        });
        if (rc) return fail(rc);
    } else if (hipMemsetAsync(ix->bucket, 0, ((1ull << ix->bb) + 1) * 4, ctx->stream) != hipSuccess) {
        set_error("kd_sf_index_build: memset failed");
        return fail(KD_EHIP);
    }
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) {
        set_error("kd_sf_index_build: %s", hipGetErrorString(hipGetLastError()));
        return fail(KD_EHIP);
    }
    prof_flush(ctx);
    *out = ix;
    return KD_OK;
}

int kd_sf_filter(kd_ctx* ctx, const kd_sf_index* ix, const uint8_t* oid, const uint8_t* is_feature, uint64_t n,
                 const double q[4], uint8_t* result, uint32_t mem) {
    KD_CHECK(ctx && ix && q && result && (n == 0 || oid), "kd_sf_filter: NULL argument");
    KD_CHECK(ix->ctx == ctx, "kd_sf_filter: index built on another context");
    // sf_init takes the rectangle as given (an inverted latitude range included): range_overlaps
    // rejects it per object, only for objects whose longitudes overlap (result 2, MR_ERROR)
    KD_HIP(hipSetDevice(ctx->device));
    if (n == 0) return KD_OK;
    int rc;
    const void *d_oid, *d_feat = nullptr;
    if ((rc = stage_in(ctx, "sf.qoid", oid, n * 20, mem, &d_oid))) return rc;
    if (is_feature && (rc = stage_in(ctx, "sf.qfeat", is_feature, n, mem, &d_feat))) return rc;
    u8* d_out = result;
    if (mem == KD_MEM_HOST) {
        void* p;
        if ((rc = ensure(ctx, "sf.out", n, &p))) return rc;
        d_out = (u8*)p;
    }
    SfArgs a;
    a.key = ix->key; a.order = ix->order; a.ioid = ix->oid; a.env = ix->env; a.bucket = ix->bucket;
    a.n_idx = ix->n; a.bits = ix->bits; a.nb = ix->nb; a.bb = ix->bb;
    a.qoid = (const u8*)d_oid; a.is_feature = (const u8*)d_feat; a.n = n;
    a.qw = q[0]; a.qs = q[1]; a.qe = q[2]; a.qn = q[3];
    a.out = d_out;
    rc = launch(ctx, "k_sf_filter", [&] {
        hipLaunchKernelGGL(k_sf_filter, dim3(grid_for(ctx, n)), dim3(256), 0, ctx->stream, a);
    });
    if (rc) return rc;
    if (mem == KD_MEM_HOST) {
        KD_HIP(hipMemcpyAsync(result, d_out, n, hipMemcpyDeviceToHost, ctx->stream));
        KD_HIP(hipStreamSynchronize(ctx->stream));
        prof_flush(ctx);
    }
    return KD_OK;
}

}  // extern "C"
