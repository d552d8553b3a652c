// kd_comm.hip — device memory for framework-free callers, and the multi-GPU path: bucket-range
// shards of one diff with the per-shard counts and compacted delta records all-gathered over RCCL
// (xGMI), the only exchange the path has.
//
// RCCL is loaded on first use (dlopen by soname, so a process that already loaded it — e.g.
// through a framework — shares that copy); a single-GPU caller never touches it.
#include <dlfcn.h>

#include <algorithm>

#include <rccl/rccl.h>

#include "kd_internal.h"

namespace kd {

// ---- RCCL entry points, resolved at run time ----
struct Rccl {
    void* h = nullptr;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommInitAll) commInitAll = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
    decltype(&ncclCommCount) commCount = nullptr;
    decltype(&ncclCommUserRank) commUserRank = nullptr;
    decltype(&ncclCommCuDevice) commDevice = nullptr;
};
static Rccl g_rccl;
static std::mutex g_rccl_m;

static int rccl(Rccl** out) {
    std::lock_guard<std::mutex> g(g_rccl_m);
    if (!g_rccl.h) {
        const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        for (const char* n : names)
            if ((g_rccl.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
        if (!g_rccl.h) { set_error("RCCL not loadable: %s", dlerror()); return KD_EHIP; }
#define KD_SYM(f, s) g_rccl.f = (decltype(g_rccl.f))dlsym(g_rccl.h, s)
        KD_SYM(getUniqueId, "ncclGetUniqueId");
        KD_SYM(commInitRank, "ncclCommInitRank");
        KD_SYM(commInitAll, "ncclCommInitAll");
        KD_SYM(commDestroy, "ncclCommDestroy");
        KD_SYM(allGather, "ncclAllGather");
        KD_SYM(groupStart, "ncclGroupStart");
        KD_SYM(groupEnd, "ncclGroupEnd");
        KD_SYM(errorString, "ncclGetErrorString");
        KD_SYM(commCount, "ncclCommCount");
        KD_SYM(commUserRank, "ncclCommUserRank");
        KD_SYM(commDevice, "ncclCommCuDevice");
#undef KD_SYM
        if (!g_rccl.getUniqueId || !g_rccl.commInitRank || !g_rccl.commInitAll || !g_rccl.commDestroy ||
            !g_rccl.allGather || !g_rccl.groupStart || !g_rccl.groupEnd || !g_rccl.errorString || !g_rccl.commCount ||
            !g_rccl.commUserRank || !g_rccl.commDevice) {
            set_error("RCCL: missing symbols");
            dlclose(g_rccl.h);
            g_rccl.h = nullptr;
            return KD_EHIP;
        }
    }
    *out = &g_rccl;
    return KD_OK;
}

#define KD_NCCL(R, call)                                                             \
    do {                                                                             \
        ncclResult_t r_ = (call);                                                    \
        if (r_ != ncclSuccess) {                                                     \
            ::kd::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, (R)->errorString(r_)); \
            return KD_EHIP;                                                          \
        }                                                                            \
    } while (0)

// shard-local record indices -> global sorted indices (KD_NONE stays KD_NONE); the count is read
// on the device (no host round trip between the join and the gather)
__global__ __launch_bounds__(256) void k_rebase(uint2* __restrict__ rec, const u64* __restrict__ n_dev, u64 cap,
                                                u32 off_a, u32 off_b) {
    const u64 n = std::min<u64>(*n_dev, cap);
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) {
        uint2 x = rec[i];
        x.x = x.x == KD_NONE ? KD_NONE : x.x + off_a;
        x.y = x.y == KD_NONE ? KD_NONE : x.y + off_b;
        rec[i] = x;
    }
}

static int rebase(kd_ctx* ctx, u32* d_rec, const u64* d_n, u64 cap, u64 off_a, u64 off_b) {
    if (off_a == 0 && off_b == 0) return KD_OK;
    const unsigned blocks = (unsigned)std::max<u64>(1, std::min<u64>((cap + 255) / 256, (u64)ctx->n_cu * 4));
    return launch(ctx, "k_rebase", [&] {
        hipLaunchKernelGGL(k_rebase, dim3(blocks), dim3(256), 0, ctx->stream, (uint2*)d_rec, d_n, cap, (u32)off_a,
                           (u32)off_b);
    });
}

// first index of a sorted key array at or after bucket b (keys carry the bucket in their top bits)
static u64 bucket_lower(const u64* key, u64 n, u64 b, int bits) {
    if (b >= (1ull << bits)) return n;
    const u64 edge = b << (64 - bits);
    return (u64)(std::lower_bound(key, key + n, edge) - key);
}

void comm_release(kd_ctx* ctx) {
    if (!g_rccl.h) return;
    if (ctx->comm) g_rccl.commDestroy((ncclComm_t)ctx->comm);
    for (void* c : ctx->group_comms)
        if (c) g_rccl.commDestroy((ncclComm_t)c);
    ctx->comm = nullptr;
    ctx->group_comms.clear();
    ctx->group_devs.clear();
}

void gather_release(kd_ctx* ctx) {
    if (ctx->ev_counts) (void)hipEventDestroy(ctx->ev_counts);
    if (ctx->ev_gathered) (void)hipEventDestroy(ctx->ev_gathered);
    if (ctx->comm_stream) (void)hipStreamDestroy(ctx->comm_stream);
    if (ctx->h_counts_pin) (void)hipHostFree(ctx->h_counts_pin);
    ctx->ev_counts = ctx->ev_gathered = nullptr;
    ctx->comm_stream = nullptr;
    ctx->h_counts_pin = nullptr;
    ctx->h_counts_ranks = 0;
}

}  // namespace kd

using namespace kd;

extern "C" {

// ------------------------------------------------------------------------------------------
// device memory
int kd_malloc(kd_ctx* ctx, uint64_t bytes, void** dptr) {
    KD_CHECK(ctx && dptr, "kd_malloc: NULL");
    KD_HIP(hipSetDevice(ctx->device));
    KD_HIP(hipMalloc(dptr, bytes ? bytes : 16));
    return KD_OK;
}

int kd_mfree(kd_ctx* ctx, void* dptr) {
    KD_CHECK(ctx, "kd_mfree: NULL ctx");
    if (!dptr) return KD_OK;
    KD_HIP(hipSetDevice(ctx->device));
    KD_HIP(hipFree(dptr));
    return KD_OK;
}

int kd_host_alloc(uint64_t bytes, void** hptr) {
    KD_CHECK(hptr, "kd_host_alloc: NULL");
    KD_HIP(hipHostMalloc(hptr, bytes ? bytes : 16, hipHostMallocDefault));
    return KD_OK;
}

int kd_host_free(void* hptr) {
    if (!hptr) return KD_OK;
    KD_HIP(hipHostFree(hptr));
    return KD_OK;
}

int kd_memcpy(kd_ctx* ctx, void* dst, const void* src, uint64_t bytes, uint32_t kind) {
    KD_CHECK(ctx && (bytes == 0 || (dst && src)), "kd_memcpy: NULL");
    KD_CHECK(kind == KD_COPY_H2D || kind == KD_COPY_D2H || kind == KD_COPY_D2D, "kd_memcpy: bad kind %u", kind);
    if (!bytes) return KD_OK;
    const hipMemcpyKind k = kind == KD_COPY_H2D ? hipMemcpyHostToDevice
                            : kind == KD_COPY_D2H ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    KD_HIP(hipSetDevice(ctx->device));
    KD_HIP(hipMemcpyAsync(dst, src, bytes, k, ctx->stream));
    return KD_OK;
}

int kd_memset(kd_ctx* ctx, void* dst, int value, uint64_t bytes) {
    KD_CHECK(ctx && (bytes == 0 || dst), "kd_memset: NULL");
    if (!bytes) return KD_OK;
    KD_HIP(hipSetDevice(ctx->device));
    KD_HIP(hipMemsetAsync(dst, value, bytes, ctx->stream));
    return KD_OK;
}

int kd_device_sync(kd_ctx* ctx) {
    KD_CHECK(ctx, "kd_device_sync: NULL");
    KD_HIP(hipSetDevice(ctx->device));
    KD_HIP(hipDeviceSynchronize());
    return prof_flush(ctx);
}

// ------------------------------------------------------------------------------------------
// multi-process: one rank per GPU, one communicator per context
int kd_comm_unique_id(uint8_t id[KD_COMM_ID_BYTES]) {
    KD_CHECK(id, "kd_comm_unique_id: NULL");
    static_assert(sizeof(ncclUniqueId) == KD_COMM_ID_BYTES, "ncclUniqueId size");
    Rccl* R;
    int rc;
    if ((rc = rccl(&R))) return rc;
    ncclUniqueId u;
    KD_NCCL(R, R->getUniqueId(&u));
    std::memcpy(id, &u, sizeof u);
    return KD_OK;
}

int kd_comm_init(kd_ctx* ctx, int nranks, int rank, const uint8_t id[KD_COMM_ID_BYTES]) {
    KD_CHECK(ctx && id && nranks >= 1 && rank >= 0 && rank < nranks, "kd_comm_init: bad args");
    KD_CHECK(ctx->comm == nullptr, "kd_comm_init: context already has a communicator");
    Rccl* R;
    int rc;
    if ((rc = rccl(&R))) return rc;
    KD_HIP(hipSetDevice(ctx->device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclComm_t c;
    KD_NCCL(R, R->commInitRank(&c, nranks, u, rank));
    ctx->comm = c;
    ctx->nranks = nranks;
    ctx->rank = rank;
    return KD_OK;
}

int kd_comm_info(kd_ctx* ctx, int32_t out[3]) {
    KD_CHECK(ctx && out, "kd_comm_info: NULL");
    KD_CHECK(ctx->comm, "kd_comm_info: no communicator (kd_comm_init)");
    Rccl* R;
    int rc;
    if ((rc = rccl(&R))) return rc;
    int count = 0, rank = -1, dev = -1;
    KD_NCCL(R, R->commCount((ncclComm_t)ctx->comm, &count));
    KD_NCCL(R, R->commUserRank((ncclComm_t)ctx->comm, &rank));
    KD_NCCL(R, R->commDevice((ncclComm_t)ctx->comm, &dev));
    out[0] = count;
    out[1] = rank;
    out[2] = dev;
    return KD_OK;
}

int kd_comm_fini(kd_ctx* ctx) {
    KD_CHECK(ctx, "kd_comm_fini: NULL");
    if (!ctx->comm) return KD_OK;
    Rccl* R;
    int rc;
    if ((rc = rccl(&R))) return rc;
    KD_HIP(hipSetDevice(ctx->device));
    KD_HIP(hipStreamSynchronize(ctx->stream));
    KD_NCCL(R, R->commDestroy((ncclComm_t)ctx->comm));
    ctx->comm = nullptr;
    return KD_OK;
}

int kd_allgather_u64(kd_ctx* ctx, const uint64_t* d_send, uint64_t* d_recv, uint64_t n) {
    KD_CHECK(ctx && ctx->comm, "kd_allgather_u64: no communicator (kd_comm_init)");
    Rccl* R;
    int rc;
    if ((rc = rccl(&R))) return rc;
    KD_HIP(hipSetDevice(ctx->device));
    KD_NCCL(R, R->allGather(d_send, d_recv, n, ncclUint64, (ncclComm_t)ctx->comm, ctx->stream));
    return KD_OK;
}

int kd_diff2_gather_begin(kd_ctx* ctx, const kd_side* base, const kd_side* target, uint64_t base_off,
                          uint64_t target_off, uint32_t flags, uint32_t* d_delta, uint32_t* d_upd, uint64_t* d_counts,
                          uint32_t* d_err, uint64_t* d_all_counts) {
    KD_CHECK(ctx && ctx->comm, "kd_diff2_gather: no communicator (kd_comm_init)");
    KD_CHECK(base && target && base->mem == KD_MEM_DEVICE && target->mem == KD_MEM_DEVICE,
             "kd_diff2_gather: sides must be device-resident");
    KD_CHECK(d_delta && d_counts && d_err && d_all_counts, "kd_diff2_gather: NULL");
    KD_CHECK(base_off + base->n < 0xFFFFFFFFull && target_off + target->n < 0xFFFFFFFFull,
             "kd_diff2_gather: global indices exceed uint32");
    Rccl* R;
    int rc;
    if ((rc = rccl(&R))) return rc;
    KD_HIP(hipSetDevice(ctx->device));
    if (!ctx->ev_counts) {
        KD_HIP(hipEventCreateWithFlags(&ctx->ev_counts, hipEventDisableTiming));
        KD_HIP(hipEventCreateWithFlags(&ctx->ev_gathered, hipEventDisableTiming));
        KD_HIP(hipStreamCreateWithFlags(&ctx->comm_stream, hipStreamNonBlocking));
    }
    if (ctx->h_counts_ranks < ctx->nranks) {
        if (ctx->h_counts_pin) KD_HIP(hipHostFree(ctx->h_counts_pin));
        ctx->h_counts_pin = nullptr;
        KD_HIP(hipHostMalloc((void**)&ctx->h_counts_pin, (size_t)ctx->nranks * 64, hipHostMallocDefault));
        ctx->h_counts_ranks = ctx->nranks;
    }
    // 1. this rank's shard (the device form; counts stay on the device)
    if ((rc = diff2_device(ctx, base, target, flags, d_delta, d_upd, d_counts, d_err))) return rc;
    ctx->gather_send_cap = base->n + target->n + 1;  // records d_delta holds (the documented capacity)
    // 2. records -> global sorted indices
    if ((rc = rebase(ctx, d_delta, d_counts + 3, base->n + target->n, base_off, target_off))) return rc;
    // 3. all-gather the counts (+ the error word): [nranks][8] u64, then to pinned host memory
    //    (asynchronous: the caller's next work is queued before anything waits for them)
    void* pack;
    if ((rc = ensure(ctx, "gather.pack", 64, &pack))) return rc;
    KD_HIP(hipMemcpyAsync(pack, d_counts, 32, hipMemcpyDeviceToDevice, ctx->stream));
    KD_HIP(hipMemsetAsync((u8*)pack + 32, 0, 32, ctx->stream));
    KD_HIP(hipMemcpyAsync((u8*)pack + 32, d_err, 4, hipMemcpyDeviceToDevice, ctx->stream));
    KD_NCCL(R, R->allGather(pack, d_all_counts, 8, ncclUint64, (ncclComm_t)ctx->comm, ctx->stream));
    KD_HIP(hipMemcpyAsync(ctx->h_counts_pin, d_all_counts, (size_t)ctx->nranks * 64, hipMemcpyDeviceToHost,
                          ctx->stream));
    KD_HIP(hipEventRecord(ctx->ev_counts, ctx->stream));
    return KD_OK;
}

int kd_diff2_gather_end(kd_ctx* ctx, const uint32_t* d_delta, uint32_t* d_all_delta, uint64_t all_cap,
                        uint64_t* h_all_counts) {
    KD_CHECK(ctx && ctx->comm && ctx->ev_counts, "kd_diff2_gather_end: no kd_diff2_gather_begin");
    KD_CHECK(d_delta && d_all_delta && h_all_counts, "kd_diff2_gather_end: NULL");
    Rccl* R;
    int rc;
    if ((rc = rccl(&R))) return rc;
    KD_HIP(hipSetDevice(ctx->device));
    // 4. the counts (the one host wait: the record stride), then the delta records, each rank's
    //    padded to the largest count (no all-gatherv), on the communication stream
    KD_HIP(hipEventSynchronize(ctx->ev_counts));
    std::memcpy(h_all_counts, ctx->h_counts_pin, (size_t)ctx->nranks * 64);
    // Every decision before the collective uses only the gathered counts, which every rank holds
    // identically: no rank may return early while the others enter the all-gather.
    u64 mx = 0;
    for (int r = 0; r < ctx->nranks; r++) mx = std::max<u64>(mx, h_all_counts[8 * r + 3]);
    const bool fits = mx * (u64)ctx->nranks <= all_cap;
    if (mx) {
        const u64 mine = h_all_counts[8 * ctx->rank + 3];
        const void* send = d_delta;
        void* recv = d_all_delta;
        KD_HIP(hipStreamWaitEvent(ctx->comm_stream, ctx->ev_counts, 0));  // the records are final by then
        if (mx > ctx->gather_send_cap) {  // this shard's d_delta is shorter than the padded stride
            void* sb;
            if ((rc = ensure(ctx, "gather.send", mx * 8, &sb))) return rc;
            if (mine) KD_HIP(hipMemcpyAsync(sb, d_delta, mine * 8, hipMemcpyDeviceToDevice, ctx->comm_stream));
            send = sb;
        }
        if (!fits) {  // still take part (into scratch), then report the short buffer
            if ((rc = ensure(ctx, "gather.recv", mx * (u64)ctx->nranks * 8, &recv))) return rc;
        }
        KD_NCCL(R, R->allGather(send, recv, 2 * mx, ncclUint32, (ncclComm_t)ctx->comm, ctx->comm_stream));
        KD_HIP(hipEventRecord(ctx->ev_gathered, ctx->comm_stream));
        KD_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_gathered, 0));  // later work on the stream sees the records
    }
    KD_CHECK(fits, "kd_diff2_gather: d_all_delta holds %llu records, %llu needed (this rank took part in the "
                   "all-gather; records not delivered)",
             (unsigned long long)all_cap, (unsigned long long)(mx * ctx->nranks));
    return KD_OK;
}

int kd_diff2_gather(kd_ctx* ctx, const kd_side* base, const kd_side* target, uint64_t base_off, uint64_t target_off,
                    uint32_t flags, uint32_t* d_delta, uint32_t* d_upd, uint64_t* d_counts, uint32_t* d_err,
                    uint32_t* d_all_delta, uint64_t all_cap, uint64_t* d_all_counts, uint64_t* h_all_counts) {
    int rc;
    if ((rc = kd_diff2_gather_begin(ctx, base, target, base_off, target_off, flags, d_delta, d_upd, d_counts, d_err,
                                    d_all_counts)))
        return rc;
    return kd_diff2_gather_end(ctx, d_delta, d_all_delta, all_cap, h_all_counts);
}

// ------------------------------------------------------------------------------------------
// bucket-range cuts (host only): shard s holds buckets [cut[s], cut[s+1]) — cut[s] the smallest
// bucket at or after cut[s-1] with at least total*s/g entries of both sides before it — and the
// sorted entries [a_lo[s], a_lo[s+1]) / [b_lo[s], b_lo[s+1]) of each side
int kd_shard_cuts(const uint64_t* key_a, uint64_t n_a, const uint64_t* key_b, uint64_t n_b, int g, int bucket_bits,
                  uint64_t* cut, uint64_t* a_lo, uint64_t* b_lo) {
    KD_CHECK(g >= 1 && cut && a_lo && b_lo && (n_a == 0 || key_a) && (n_b == 0 || key_b), "kd_shard_cuts: bad args");
    KD_CHECK(bucket_bits >= 1 && bucket_bits <= 32, "kd_shard_cuts: bucket_bits %d", bucket_bits);
    const u64 total = n_a + n_b;
    cut[0] = 0;
    cut[g] = 1ull << bucket_bits;
    for (int s = 1; s < g; s++) {
        const u64 want = total * (u64)s / (u64)g;
        u64 lo = cut[s - 1], hi = cut[g];
        while (lo < hi) {  // smallest bucket whose lower edge has >= want entries before it
            const u64 mid = lo + (hi - lo) / 2;
            const u64 c = bucket_lower(key_a, n_a, mid, bucket_bits) + bucket_lower(key_b, n_b, mid, bucket_bits);
            if (c >= want) hi = mid; else lo = mid + 1;
        }
        cut[s] = lo;
    }
    for (int s = 0; s <= g; s++) {
        a_lo[s] = bucket_lower(key_a, n_a, cut[s], bucket_bits);
        b_lo[s] = bucket_lower(key_b, n_b, cut[s], bucket_bits);
    }
    return KD_OK;
}

// ------------------------------------------------------------------------------------------
// single process, g GPUs: the library cuts the sides, runs every shard and owns the communicator
int kd_diff2_sharded(kd_ctx** ctxs, int g, const kd_side* base, const kd_side* target, int bucket_bits,
                     uint32_t flags, kd_diff_result** out) {
    KD_CHECK(ctxs && g >= 1 && base && target && out, "kd_diff2_sharded: bad args");
    KD_CHECK(base->mem == KD_MEM_HOST && target->mem == KD_MEM_HOST, "kd_diff2_sharded: host sides");
    KD_CHECK(base->key_mode == target->key_mode, "kd_diff2_sharded: key modes differ");
    KD_CHECK(bucket_bits >= 1 && bucket_bits <= 32, "kd_diff2_sharded: bucket_bits %d", bucket_bits);
    KD_CHECK(!(flags & KD_DIFF_UNORDERED), "kd_diff2_sharded: ordered results only");
    for (int i = 0; i < g; i++) KD_CHECK(ctxs[i], "kd_diff2_sharded: ctx %d NULL", i);
    int rc;
    Rccl* R;
    if ((rc = rccl(&R))) return rc;
    // ---- bucket cuts: shard s holds buckets [cut[s], cut[s+1]), about total/g entries ----
    std::vector<u64> cut(g + 1, 0), a_lo(g + 1), b_lo(g + 1);
    if ((rc = kd_shard_cuts(base->key, base->n, target->key, target->n, g, bucket_bits, cut.data(), a_lo.data(),
                            b_lo.data())))
        return rc;
    // ---- communicator over these devices (kept on ctxs[0] for the same device set) ----
    std::vector<int> devs(g);
    for (int i = 0; i < g; i++) devs[i] = ctxs[i]->device;
    if (ctxs[0]->group_devs != devs) {
        for (void* c : ctxs[0]->group_comms)
            if (c) R->commDestroy((ncclComm_t)c);
        ctxs[0]->group_comms.assign(g, nullptr);
        KD_NCCL(R, R->commInitAll((ncclComm_t*)ctxs[0]->group_comms.data(), g, devs.data()));
        ctxs[0]->group_devs = devs;
    }
    // ---- every shard on its GPU: stage, join, rebase, counts ----
    std::vector<u32*> dd(g), dall(g);
    std::vector<u64*> dc(g), dcall(g);
    for (int i = 0; i < g; i++) {
        kd_ctx* c = ctxs[i];
        KD_HIP(hipSetDevice(c->device));
        kd_side A = *base, B = *target, dA, dB;
        A.n = a_lo[i + 1] - a_lo[i];
        A.key = base->key + a_lo[i];
        A.oid = base->oid + 20 * a_lo[i];
        B.n = b_lo[i + 1] - b_lo[i];
        B.key = target->key + b_lo[i];
        B.oid = target->oid + 20 * b_lo[i];
        if (base->key_mode == KD_KEY_HASH) {  // name offsets stay absolute: the arena is shared
            A.name_off = base->name_off + a_lo[i];
            B.name_off = target->name_off + b_lo[i];
        }
        if ((rc = stage_side(c, &A, "sh.a", &dA)) || (rc = stage_side(c, &B, "sh.b", &dB))) return rc;
        void *d, *cnt;
        if ((rc = ensure(c, "sh.delta", (A.n + B.n + 1) * 8, &d))) return rc;
        if ((rc = ensure(c, "sh.counts", 64, &cnt))) return rc;
        dd[i] = (u32*)d;
        dc[i] = (u64*)cnt;
        u32* derr = (u32*)(dc[i] + 4);
        if ((rc = diff2_device(c, &dA, &dB, flags, dd[i], nullptr, dc[i], derr))) return rc;
        if ((rc = rebase(c, dd[i], dc[i] + 3, A.n + B.n, a_lo[i], b_lo[i]))) return rc;
        KD_HIP(hipMemsetAsync((u8*)cnt + 40, 0, 24, c->stream));
        void* ca;
        if ((rc = ensure(c, "sh.counts_all", (size_t)g * 64, &ca))) return rc;
        dcall[i] = (u64*)ca;
    }
    // ---- all-gather counts, then records padded to the largest shard ----
    KD_NCCL(R, R->groupStart());
    for (int i = 0; i < g; i++)
        KD_NCCL(R, R->allGather(dc[i], dcall[i], 8, ncclUint64, (ncclComm_t)ctxs[0]->group_comms[i], ctxs[i]->stream));
    KD_NCCL(R, R->groupEnd());
    std::vector<u64> hc((size_t)g * 8);
    KD_HIP(hipSetDevice(ctxs[0]->device));
    KD_HIP(hipMemcpyAsync(hc.data(), dcall[0], (size_t)g * 64, hipMemcpyDeviceToHost, ctxs[0]->stream));
    KD_HIP(hipStreamSynchronize(ctxs[0]->stream));
    u64 mx = 0, nd = 0, ni = 0, nu = 0, nx = 0;
    u32 err = 0;
    for (int s = 0; s < g; s++) {
        ni += hc[8 * s]; nu += hc[8 * s + 1]; nx += hc[8 * s + 2]; nd += hc[8 * s + 3];
        mx = std::max<u64>(mx, hc[8 * s + 3]);
        err |= (u32)(hc[8 * s + 4] & 0xFFFFFFFFu);
    }
    if (err) {
        set_error("kd_diff2_sharded: %s", (err & 1) ? "side keys not strictly ascending" : "hash key collision between different filenames");
        return KD_EUNSUPPORTED;
    }
    if (mx) {
        std::vector<const u32*> send(g);
        for (int i = 0; i < g; i++) {
            void* a;
            KD_HIP(hipSetDevice(ctxs[i]->device));
            if ((rc = ensure(ctxs[i], "sh.all", (size_t)g * mx * 8, &a))) return rc;
            dall[i] = (u32*)a;
            send[i] = dd[i];
            const u64 cap = a_lo[i + 1] - a_lo[i] + b_lo[i + 1] - b_lo[i] + 1;  // records sh.delta holds
            if (mx > cap) {  // a shard shorter than the padded stride sends from a copy of stride size
                void* sb;
                if ((rc = ensure(ctxs[i], "sh.send", mx * 8, &sb))) return rc;
                if (hc[8 * i + 3])
                    KD_HIP(hipMemcpyAsync(sb, dd[i], hc[8 * i + 3] * 8, hipMemcpyDeviceToDevice, ctxs[i]->stream));
                send[i] = (const u32*)sb;
            }
        }
        KD_NCCL(R, R->groupStart());
        for (int i = 0; i < g; i++)
            KD_NCCL(R, R->allGather(send[i], dall[i], 2 * mx, ncclUint32, (ncclComm_t)ctxs[0]->group_comms[i], ctxs[i]->stream));
        KD_NCCL(R, R->groupEnd());
    }
    // ---- result from GPU 0: the shards in bucket order = key order ----
    kd_diff_result* r = (kd_diff_result*)std::malloc(sizeof(kd_diff_result) + (nd + nu) * 8 + 16);
    KD_CHECK(r, "kd_diff2_sharded: out of host memory");
    r->n_insert = ni; r->n_update = nu; r->n_delete = nx; r->n_delta = nd;
    r->delta = (u32*)(r + 1);
    r->upd = r->delta + 2 * nd;
    u64 pos = 0;
    hipError_t e = hipSuccess;
    for (int s = 0; s < g && e == hipSuccess; s++) {
        const u64 n = hc[8 * s + 3];
        if (n) e = hipMemcpyAsync(r->delta + 2 * pos, dall[0] + 2 * s * mx, n * 8, hipMemcpyDeviceToHost, ctxs[0]->stream);
        pos += n;
    }
    if (e == hipSuccess) e = hipStreamSynchronize(ctxs[0]->stream);
    for (int i = 1; i < g && e == hipSuccess; i++) e = hipStreamSynchronize(ctxs[i]->stream);
    if (e != hipSuccess) { std::free(r); set_error("kd_diff2_sharded: %s", hipGetErrorString(e)); return KD_EHIP; }
    u64 k = 0;
    for (u64 i = 0; i < nd; i++)
        if (r->delta[2 * i] != KD_NONE && r->delta[2 * i + 1] != KD_NONE) {
            r->upd[2 * k] = r->delta[2 * i];
            r->upd[2 * k + 1] = r->delta[2 * i + 1];
            k++;
        }
    for (int i = 0; i < g; i++) prof_flush(ctxs[i]);
    *out = r;
    return KD_OK;
}

}  // extern "C"
