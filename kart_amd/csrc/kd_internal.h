// kd_internal.h — shared internals of libkartdiff (gfx950 / MI355X).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <utility>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "kartdiff.h"

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t i64;
typedef int16_t i16;
typedef int8_t i8;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // native 16-B vector (SROA-friendly)
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

namespace kd {

void set_error(const char* fmt, ...);

#define KD_HIP(call)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess) {                                                             \
            ::kd::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
            return KD_EHIP;                                                                 \
        }                                                                                   \
    } while (0)

#define KD_CHECK(cond, ...)            \
    do {                               \
        if (!(cond)) {                 \
            ::kd::set_error(__VA_ARGS__); \
            return KD_EINVAL;          \
        }                              \
    } while (0)

// grow-only device buffer
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool slab = false;  // carved from the context's slab (never freed on its own)
};

struct ProfStat {
    u64 launches = 0;
    double ms = 0;
};

struct PendingEv {
    std::string name;
    hipEvent_t a, b;
};

}  // namespace kd

// Tuning options of a context (kd_set_option; kd_init seeds them once from the KD_* environment
// variables of the same names, documented in kartdiff.h).  Defaults are the measured optima.
struct kd_opts {
    int merge3_join = 1;             // KD_MERGE3_JOIN: 0 = round 3's two-step merge (classify2 + k_resolve3)
    int merge3_split = 0;            // KD_MERGE3_SPLIT: 1 = k_join3 stages candidates, k_resolve3 applies the rule
    int j3_ol = 0;                   // KD_J3_OL: 1 = k_join3 stages ours'/theirs' OIDs in LDS (sorted-form sides)
    int j3_v = 1;                    // KD_J3_V: 1 = k_join3b (one DMA batch per tile), 0 = k_join3
    uint64_t j2_oidlds_min = 1ull << 26;  // KD_J2_OIDLDS_MIN: k_join2 stages OIDs in LDS from this many entries
    int j2r = 0;                     // KD_J2R: 1 = the persistent register-prefetched k_join2r
    int fd_stream = -1;              // KD_FD_STREAM: -1 auto, 0 windowed k_fielddiff, 1 streamed k_fielddiff_s
    int fd_walk = -1;                // KD_FD_WALK: -1 / 0 off, 1 the walked k_fdwalk (A/B)
    uint64_t pkm_max_blocks = 1ull << 26;  // KD_PKM_MAX_BLOCKS: largest pk range (64-pk blocks) of the bitmap pk order
    int trace_host = 0;              // KD_TRACE_HOST: 1 = stream-synced wall-clock marks to stderr
};

struct kd_ctx {
    int device = 0;
    kd_opts opt;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::map<std::string, kd::DevBuf> bufs;
    // profiling
    bool prof = false;
    std::string prof_only;  // ",name,name," selection (empty = every kernel)
    std::vector<hipEvent_t> ev_pool;
    std::vector<kd::PendingEv> pending;
    std::map<std::string, kd::ProfStat> stats;
    // last uploaded kd_fielddiff table (host copy kept alive for the async upload, and reused
    // when the next call's tables are identical)
    std::vector<uint8_t> fd_tab;
    int n_cu = 256;  // compute units (grid sizing of grid-stride kernels)
    // multi-GPU (kd_comm.hip): this rank's communicator, and kd_diff2_sharded's per-device set
    void* comm = nullptr;
    int nranks = 1, rank = 0;
    std::vector<int> group_devs;
    std::vector<void*> group_comms;
    // kd_diff2_gather_begin / _end: the counts' pinned landing area, the event after it, and the
    // stream the record all-gather runs on (overlapping whatever the caller queued in between)
    hipStream_t comm_stream = nullptr;
    hipEvent_t ev_counts = nullptr, ev_gathered = nullptr;
    uint64_t* h_counts_pin = nullptr;
    int h_counts_ranks = 0;
    uint64_t gather_send_cap = 0;  // records the last _begin's d_delta holds (base.n + target.n + 1)
    int occ_resolve3 = 0;  // resident k_resolve3 workgroups per CU
    // resident workgroups per CU by (kernel, block size, dynamic LDS): asked once per context (kd::occupancy)
    std::map<std::tuple<const void*, int, size_t>, int> occ;
    uint32_t rs_epoch = 0;  // kd_sort: epoch of the last pass's look-back words (kd_sort.hip)
    // kd_delta_pk_order's two mask buffers: a call marks one and its scan zeroes the other for the
    // next call; zeroed = (buffer address, blocks known zero) — a reallocated buffer is zeroed again
    int pkm_cur = 0;
    void* pkm_zero_ptr[2] = {nullptr, nullptr};
    uint64_t pkm_zero_nb[2] = {0, 0};
    // small workspaces come from one slab (one hipMalloc instead of one per slot on a process's
    // first calls); grown slots take a fresh piece, the slab is freed with the context
    char* slab = nullptr;
    size_t slab_used = 0;
    // host inputs / results cross PCIe through two pinned chunks (stage_h2d / stage_d2h): a
    // pageable hipMemcpy pins the caller's pages on first use, which a one-shot process pays for
    // every buffer it hands over
    char* pin[2] = {nullptr, nullptr};
    void* pin_dev[2] = {nullptr, nullptr};  // the chunks' device-side addresses (k_to_host writes them)
    hipEvent_t pin_ev[2] = {nullptr, nullptr};
    int pin_next = 0;
};

namespace kd {

// device scratch slot, grown as needed (never shrinks).  Not called inside timed regions once
// kd_reserve() has sized it.
void gather_release(kd_ctx* ctx);  // kd_comm.hip: kd_diff2_gather_begin/_end resources
int ensure(kd_ctx* ctx, const char* slot, size_t bytes, void** out);
// host -> device on ctx->stream through the pinned chunks (returns when src may be reused);
// device -> host, blocking (the stream is synchronised)
int stage_h2d(kd_ctx* ctx, void* dst, const void* src, size_t bytes);
// KD_TRACE_HOST=1: stream sync + wall time since the previous mark to stderr (diagnosis only;
// name nullptr starts a sequence)
void host_mark(kd_ctx* ctx, const char* name);
int stage_d2h(kd_ctx* ctx, void* dst, const void* src, size_t bytes);

// 256 zero bytes of device memory: what empty inputs point at, and the target of loads issued by
// masked-off lanes in branch-free load batches (never a host address)
int device_zeros(kd_ctx* ctx, void** out);

// resident workgroups per CU of `kernel` at `block` threads and `lds` dynamic LDS bytes on the
// context's device (>= 1), from the occupancy calculator once per context
int occupancy(kd_ctx* ctx, const void* kernel, int block, size_t lds);

// profiling wrappers around a launch on ctx->stream
void prof_begin(kd_ctx* ctx, const char* name, hipEvent_t* a);
void prof_end(kd_ctx* ctx, const char* name, hipEvent_t a);
int prof_flush(kd_ctx* ctx);

inline bool prof_on(const kd_ctx* ctx, const char* name) {
    return ctx->prof && (ctx->prof_only.empty() || ctx->prof_only.find("," + std::string(name) + ",") != std::string::npos);
}

template <typename F>
inline int launch(kd_ctx* ctx, const char* name, F&& f) {
    hipEvent_t a = nullptr;
    const bool prof = prof_on(ctx, name);
    if (prof) prof_begin(ctx, name, &a);
    f();
    hipError_t e = hipGetLastError();
    if (prof) prof_end(ctx, name, a);
    if (e != hipSuccess) {
        set_error("launch %s: %s", name, hipGetErrorString(e));
        return KD_EHIP;
    }
    return KD_OK;
}

// copy a host/device side array to device (returns device pointer; device input is passed through)
int stage_in(kd_ctx* ctx, const char* slot, const void* p, size_t bytes, u32 mem, const void** dev);
// a side's arrays staged to device scratch slots "<tag>.*" (device sides pass through); checks
int stage_side(kd_ctx* ctx, const kd_side* s, const char* tag, kd_side* dev);
int check_side(const kd_side* s, const char* which);
// destroy the context's communicators (kd_fini)
void comm_release(kd_ctx* ctx);

// ---- classify2 (device form), kd_classify.hip ----
// ordA / ordB (both or neither): the sides' OIDs and filename offsets are in another order, row
// ord[i] belongs to sorted entry i (kd_diff2_device_perm)
// d_dkey / d_ukey (optional): the join key of every delta / update record, beside the lists
// three-way merge in one pass (k_join3): conflicts (a, o, t) and merge deltas (o, t) in path order,
// counts = clean, conflicts, merge deltas, 0; ord*: late materialisation (walk rows of sorted entries)
// k_resolve3 over k_join3's candidates (a, o, t) with the ancestor entries already found
int resolve3_have_a(kd_ctx* ctx, const kd_side& K, const kd_side& O, const kd_side& T, const u32* cand3, const u64* c2,
                    u32* d_conf, uint2* d_md, u64* d_counts, u32* d_err, const u32* ordK, const u32* ordO,
                    const u32* ordT);
int merge3_join_device(kd_ctx* ctx, const kd_side& K, const kd_side& O, const kd_side& T, u32* d_conf, uint2* d_md,
                       u64* d_counts, u32* d_err, const u32* ordK = nullptr, const u32* ordO = nullptr,
                       const u32* ordT = nullptr);
int diff2_device(kd_ctx* ctx, const kd_side* A, const kd_side* B, u32 flags, u32* d_delta,
                 u32* d_upd, u64* d_counts, u32* d_err, const u32* ordA = nullptr, const u32* ordB = nullptr,
                 u64* d_dkey = nullptr, u64* d_ukey = nullptr);
#ifndef KD_C2_NT
#define KD_C2_NT 256
#endif
constexpr int C2_NT = KD_C2_NT;
#ifndef KD_C2_IPT
#define KD_C2_IPT 4
#endif
constexpr int C2_IPT = KD_C2_IPT;
constexpr int C2_TILE = C2_NT * C2_IPT;

}  // namespace kd
