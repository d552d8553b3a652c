// kd_classify.hip — classify3 (three-way merge) on gfx950 + the host-form C API of both joins.
// (classify2's kernels live in kd_classify2.hip.)
//
// classify2 replaces libgit2's tree-to-tree diff as consumed by RichBaseDataset.diff_feature
// (/root/reference/kart/rich_base_dataset.py:205-300): both commits' feature leaves arrive as
// strictly ascending join keys + 20-byte blob OIDs; a pair present on one side only is an
// insert/delete, a pair present on both with different OIDs is an update.
//
// (kernels: kd_classify2.hip)
//
// classify3 replaces libgit2 git_merge_trees (kart/merge.py:99-100): key-range tiles cut on the
// ancestor∪ours merge path, theirs split by lower_bound; per item LDS binary searches find the
// (ancestor, ours, theirs) triple and the libgit2 OID rule classifies it.
#include <cstdlib>

#include "kd_join.h"

namespace kd {

// ============================================================================================
// classify3 = classify2(ours, theirs) + k_resolve3 over the ours/theirs deltas
// ============================================================================================
// libgit2's per-path rule (o == t -> o; a == o -> t; a == t -> o; else conflict) only needs the
// ancestor where ours and theirs differ: every path with o == t is clean and takes ours.  So the
// three-way merge is (1) the two-way join of ours against theirs (k_partition2/k_join2/k_place2,
// which also verify hash-mode filenames of every matched pair), giving the key-ordered list of
// paths where they differ (~2 x the edit rate of the entries), then (2) k_resolve3: per differing
// path, look the key up in the ancestor, compare the OIDs, apply the rule and compact conflicts and
// merge deltas in key order with a decoupled look-back.  The ancestor's keys are read only along
// the lookups' paths and its OIDs only where a path differs; k_sorted3 checks it is strictly
// ascending (one streaming pass over its keys).
#ifndef KD_RS3_PROBE_NOSEARCH
#define KD_RS3_PROBE_NOSEARCH 0
#endif
#ifndef KD_RS3_PROBE_NOOID
#define KD_RS3_PROBE_NOOID 0
#endif
#ifndef KD_RS3_PROBE_NONAMES
#define KD_RS3_PROBE_NONAMES 0
#endif
constexpr int C3_NT = 256;
constexpr int C3_CH = 1024;  // differing paths per resolve chunk (4 per thread, contiguous)
#ifndef KD_C3_SAMPLE_BITS
#define KD_C3_SAMPLE_BITS 11  // 2048 samples: C4 k_resolve3 0.745 -> 0.721 ms (8 / 9 bits: no better)
#endif
constexpr int C3_SAMPLE_BITS = KD_C3_SAMPLE_BITS;
constexpr int C3_SAMPLES = 1 << C3_SAMPLE_BITS;  // ancestor keys sampled per chunk bracket (LDS)

struct Resolve3Args {
    const u64 *A, *O, *T;
    const u32 *oA, *oO, *oT;
    u64 nA, nO;
    const u8 *nmA, *nmO, *nmT;
    const u64 *noA, *noO, *noT;
    int hash_mode;
    const uint2* cand;      // classify2(ours, theirs) delta list: (ours | NONE, theirs | NONE)
    const u32* cand3;       // HAVE_A: k_join3's differing paths with their ancestor entry (a, o, t)
    const u64* c2;          // its counts: inserts, updates, deletes, deltas
    const u32 *pA, *pO, *pT;  // PERM: row of sorted entry i in the side's OID / filename arrays
    u64* desc;              // look-back descriptors [2][nchunk]
    u64 nchunk;
    u32* aux;               // [0] chunk ticket, [1] ancestor-order error (k_sorted3)
    u32* out_conf;          // (a, o, t) per conflict
    uint2* out_md;          // (o, t) per merge delta
    u64* counts;            // clean, conflicts, mdeltas, 0
    u32* err;
};

// ancestor strictly ascending (-> aux[1]), and the resolve's counters zeroed
__global__ __launch_bounds__(256) void k_sorted3(const u64* __restrict__ A, u64 nA, u64* __restrict__ desc, u64 ndesc,
                                                 u32* __restrict__ aux, u64* __restrict__ counts) {
    const u64 tid = (u64)blockIdx.x * blockDim.x + threadIdx.x, stride = (u64)gridDim.x * blockDim.x;
    if (tid == 0) {
        aux[0] = 0;  // (aux[1] is cleared by the k_resolve3 that consumes it)
        counts[0] = counts[1] = counts[2] = counts[3] = 0;
    }
    for (u64 k = tid; k < ndesc; k += stride) desc[k] = 0;
    u32 bad = 0;
    // pairs (2i, 2i+1), and (2i+1, 2i+2) with the next pair's first key
    const u64 np = nA / 2;
    for (u64 p = tid; p < np; p += stride) {
        const u64 x = A[2 * p], y = A[2 * p + 1];  // (the side may start at any 8-B offset)
        bad |= x >= y;
        if (2 * p + 2 < nA) bad |= y >= A[2 * p + 2];
    }
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(aux + 1, 1u);
}

// smallest index in [0, n) with X[index] >= key (n if none), for one key per 32-lane half-wave:
// 32 probes per round, ~6 rounds for 50M keys
__device__ __forceinline__ u64 half_lower_bound(const u64* __restrict__ X, u64 n, u64 key) {
    const int lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31;
    u64 lo = 0, hi = n;  // answer in [lo, hi]
    while (__ballot(lo < hi)) {
        const u64 span = hi - lo, step = (span + 31) / 32;
        const u64 p = lo + (u64)l * step;
        const bool probe = lo < hi && p < hi;
        const bool below = probe && X[p] < key;
        const u32 c = __popc((u32)(__ballot(below) >> (32 * h)));
        if (lo < hi) {
            if (c == 0) hi = lo;
            else {
                const u64 nlo = lo + (u64)(c - 1) * step + 1, nhi = lo + (u64)c * step;
                lo = nlo;
                hi = nhi < hi ? nhi : hi;
            }
        }
    }
    return lo;
}

// HAVE_A: the candidates come from k_join3 (split form) with the ancestor entry found in its LDS:
// no bracket, sample or search; c2 = the join's counts (clean paths where ours == theirs, candidates)
template <int NT, bool PERM, bool HAVE_A>
__global__ __launch_bounds__(NT) void k_resolve3(Resolve3Args g) {
    constexpr int PT = C3_CH / NT;
    constexpr int NS = C3_SAMPLES;
    __shared__ u32 s_wave[NT / 64];
    __shared__ u64 s_b[4];  // ticket, bracket lo, bracket hi, -
    __shared__ u64 s_ex[2];
    __shared__ u64 s_smp[HAVE_A ? 1 : NS];  // ancestor keys at NS evenly spaced bracket positions
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const u64 n = HAVE_A ? g.c2[1] : g.c2[3];
    while (true) {
        if (tid == 0) s_b[0] = atomicAdd(g.aux, 1u);
        __syncthreads();
        const u64 t = s_b[0];
        if (t == 0 && tid == 0) {  // paths where ours == theirs: clean, and the ancestor-order check
            atomicAdd((unsigned long long*)g.counts, (unsigned long long)(HAVE_A ? g.c2[0] : g.nO - g.c2[1] - g.c2[2]));
            if (g.aux[1]) { atomicOr(g.err, 1u); g.aux[1] = 0; }  // consumed: k_sorted3 only sets it
        }
        const u64 base = t * C3_CH;
        if (base >= n) break;
        const u32 cnt = (u32)(n - base < (u64)C3_CH ? n - base : (u64)C3_CH);
        auto key_of = [&](uint2 r) { return *(r.x != KD_NONE ? g.O + r.x : g.T + r.y); };  // one load
        // the chunk's ancestor bracket: [lower_bound(first key), lower_bound(last key) + 1)
        if (!HAVE_A && wid == 0) {
            const u64 k = key_of(g.cand[base + (lane < 32 ? 0 : cnt - 1)]);
            const u64 p = half_lower_bound(g.A, g.nA, k);
            if (lane == 0) s_b[1] = p;
            if (lane == 32) s_b[2] = p < g.nA ? p + 1 : g.nA;
        }
        uint2 rec[PT];
        u64 key[PT];
        u32 ia3[PT];
#pragma unroll
        for (int j = 0; j < PT; j++) {
            const u32 r = tid * PT + j;
            if (HAVE_A) {
                const u32* c3 = g.cand3 + 3 * (base + r);
                ia3[j] = r < cnt ? c3[0] : KD_NONE;
                rec[j] = r < cnt ? make_uint2(c3[1], c3[2]) : make_uint2(KD_NONE, KD_NONE);
            } else {
                rec[j] = r < cnt ? g.cand[base + r] : make_uint2(KD_NONE, KD_NONE);
            }
        }
#pragma unroll
        for (int j = 0; j < PT; j++) key[j] = (!HAVE_A && tid * PT + j < cnt) ? key_of(rec[j]) : 0;
        __syncthreads();
        u32 lo[PT], hi[PT];
        bool found[PT];
        if (HAVE_A) {
#pragma unroll
            for (int j = 0; j < PT; j++) { found[j] = ia3[j] != KD_NONE; lo[j] = hi[j] = ia3[j]; }
        } else {
        const u32 blo = (u32)s_b[1], bhi = (u32)s_b[2];
        const u32 span = bhi - blo;
        // sample level: NS keys at positions blo + s*span/NS in LDS (one gather), each key's
        // sub-bracket from an LDS search, then the global search inside it (~log2(span/NS) rounds)
        for (int x = tid; x < NS; x += NT) {
            const u32 pos = blo + (u32)(((u64)x * span) / NS);
#if KD_RS3_PROBE_NOSEARCH  // timing probe only (results invalid)
            s_smp[x] = (u64)pos;
#else
            s_smp[x] = pos < bhi ? g.A[pos] : ~0ull;
#endif
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PT; j++) {
            // c = number of samples < key: lower_bound lies in (pos(c-1), pos(c)]
            int l = 0, h = NS;
#pragma unroll
            for (int r = 0; r < C3_SAMPLE_BITS + 1; r++) {
                const int m = (l + h) >> 1;
                const bool act = l < h;
                const bool lt = s_smp[m < NS ? m : NS - 1] < key[j];
                l = act && lt ? m + 1 : l;
                h = act && !lt ? m : h;
            }
            lo[j] = l == 0 ? blo : blo + (u32)(((u64)(l - 1) * span) / NS) + 1;
            hi[j] = l == NS ? bhi : blo + (u32)(((u64)l * span) / NS);
            found[j] = l < NS && s_smp[l] == key[j];
            if (found[j]) lo[j] = hi[j];  // the sample itself is the match
        }
        u32 sub = 0;
#pragma unroll
        for (int j = 0; j < PT; j++) sub = max(sub, hi[j] - lo[j]);
#if KD_RS3_PROBE_NOSEARCH
        const int rounds = 0;
#else
        const int rounds = sub ? 32 - __clz(sub) : 0;
#endif
        for (int it = 0; it < rounds; it++) {
            u64 v[PT];
            u32 m[PT];
#pragma unroll
            for (int j = 0; j < PT; j++) {
                m[j] = (lo[j] + hi[j]) >> 1;
                v[j] = g.A[m[j] < g.nA ? m[j] : 0];
            }
#pragma unroll
            for (int j = 0; j < PT; j++) {
                const bool act = lo[j] < hi[j];
                const bool lt = v[j] < key[j];
                found[j] |= act && v[j] == key[j];
                lo[j] = act && lt ? m[j] + 1 : lo[j];
                hi[j] = act && !lt ? m[j] : hi[j];
            }
        }
        }  // (!HAVE_A)
        // every OID of the chunk's paths loaded before any compare
        u32 ia[PT], io[PT], itt[PT];
        u32 ra[PT], ro[PT], rt[PT];  // their rows in the OID / filename arrays
        u32 xa[PT][5], xo[PT][5], xt[PT][5];
#pragma unroll
        for (int j = 0; j < PT; j++) {
            ia[j] = found[j] ? lo[j] : KD_NONE;
            io[j] = rec[j].x;
            itt[j] = rec[j].y;
            ra[j] = ia[j]; ro[j] = io[j]; rt[j] = itt[j];
        }
        if (PERM) {  // late materialisation: the sides' OIDs and names stay in walk order
#pragma unroll
            for (int j = 0; j < PT; j++) {
                ra[j] = ia[j] != KD_NONE ? g.pA[ia[j]] : KD_NONE;
                ro[j] = io[j] != KD_NONE ? g.pO[io[j]] : KD_NONE;
                rt[j] = itt[j] != KD_NONE ? g.pT[itt[j]] : KD_NONE;
            }
        }
#pragma unroll
        for (int j = 0; j < PT; j++) {
            const u32* qa = g.oA + (u64)(ra[j] != KD_NONE ? ra[j] : 0) * 5;
            const u32* qo = g.oO + (u64)(ro[j] != KD_NONE ? ro[j] : 0) * 5;
            const u32* qt = g.oT + (u64)(rt[j] != KD_NONE ? rt[j] : 0) * 5;
#if KD_RS3_PROBE_NOOID  // timing probe only (results invalid)
#pragma unroll
            for (int w = 0; w < 5; w++) { xa[j][w] = (u32)(size_t)qa; xo[j][w] = (u32)(size_t)qo; xt[j][w] = (u32)(size_t)qt; }
#else
#pragma unroll
            for (int w = 0; w < 5; w++) { xa[j][w] = qa[w]; xo[j][w] = qo[w]; xt[j][w] = qt[w]; }
#endif
        }
        if (g.hash_mode && !KD_RS3_PROBE_NONAMES) {  // a matched ancestor path must carry the same filename
            u32 act_o = 0, act_t = 0;
#pragma unroll
            for (int j = 0; j < PT; j++) {
                act_o |= (u32)(ia[j] != KD_NONE && io[j] != KD_NONE) << j;
                // with ours present, theirs' name = ours' (classify2 checked the matched pair) = the
                // ancestor's (checked here): only ancestor-and-theirs-without-ours needs its own check
                act_t |= (u32)(ia[j] != KD_NONE && itt[j] != KD_NONE && io[j] == KD_NONE) << j;
            }
            if (names_ne_batch<PT, 8>(g.nmA, g.noA, ra, g.nmO, g.noO, ro, act_o) |
                names_ne_batch<PT, 8>(g.nmA, g.noA, ra, g.nmT, g.noT, rt, act_t))
                atomicOr(g.err, 2u);
        }
        u32 fc = 0, fm = 0, clean = 0;
        u32 cls[PT];
#pragma unroll
        for (int j = 0; j < PT; j++) {
            const bool valid = tid * PT + j < cnt;
            const bool pa = ia[j] != KD_NONE, po = io[j] != KD_NONE, pt = itt[j] != KD_NONE;
            auto same = [](const u32* x, const u32* y) {
                return ((x[0] ^ y[0]) | (x[1] ^ y[1]) | (x[2] ^ y[2]) | (x[3] ^ y[3]) | (x[4] ^ y[4])) == 0;
            };
            // ours != theirs here (classify2 emitted the path), so the rule reduces to two tests
            const bool a_eq_o = pa == po && (!pa || same(xa[j], xo[j]));
            const bool a_eq_t = pa == pt && (!pa || same(xa[j], xt[j]));
            u32 c = a_eq_o ? 1u : a_eq_t ? 0u : 2u;  // 0 ours (clean), 1 theirs (merge delta), 2 conflict
            if (!valid) c = 3;
            cls[j] = c;
            fc += c == 2;
            fm += c == 1;
            clean += (c == 0 && po) || (c == 1 && pt);
        }
        u32 tot;
        const u32 off = block_excl_scan<NT>(fc | (fm << 16), s_wave, &tot);
        const u32 tc = tot & 0xFFFF, tm = tot >> 16;
        const u32 tclean = block_sum<NT>(clean, s_wave);
        if (wid == 0) {
            const u64 ex = lookback(g.desc, g.nchunk, t, tc, tm);
            if (lane == 0) s_ex[0] = ex;
            if (lane == 32) s_ex[1] = ex;
        }
        __syncthreads();
        const u64 exc = s_ex[0], exm = s_ex[1];
        if (tid == 0) {
            if (tclean) atomicAdd((unsigned long long*)g.counts, (unsigned long long)tclean);
            if (base + cnt == n) {
                g.counts[1] = exc + tc;
                g.counts[2] = exm + tm;
            }
        }
        u64 pc = exc + (off & 0xFFFF), pm = exm + (off >> 16);
#pragma unroll
        for (int j = 0; j < PT; j++) {
            if (cls[j] == 2) {
                u32* o = g.out_conf + 3 * pc;
                o[0] = ia[j]; o[1] = io[j]; o[2] = itt[j];
                pc++;
            } else if (cls[j] == 1) {
                g.out_md[pm] = rec[j];
                pm++;
            }
        }
    }
}

}  // namespace kd

using namespace kd;

int kd::resolve3_have_a(kd_ctx* ctx, const kd_side& A, const kd_side& O, const kd_side& T, const u32* cand3,
                        const u64* c2, u32* d_conf, uint2* d_md, u64* counts, u32* derr, const u32* pA, const u32* pO,
                        const u32* pT) {
    const bool perm = pA || pO || pT;
    int rc;
    const u64 nA = A.n, nO = O.n, nT = T.n;
    const u64 nchunk = (nO + nT) / C3_CH + 2;
    void *desc, *aux, *dz;
    if ((rc = ensure(ctx, "c3.desc", 2 * nchunk * 8, &desc))) return rc;
    const bool fresh_aux = ctx->bufs["c3.aux"].p == nullptr;
    if ((rc = ensure(ctx, "c3.aux", 64, &aux))) return rc;
    if (fresh_aux) KD_HIP(hipMemsetAsync(aux, 0, 64, ctx->stream));
    if ((rc = device_zeros(ctx, &dz))) return rc;
    // the resolve's counters and look-back words cleared (no ancestor scan: k_join3 checked its order)
    rc = launch(ctx, "k_sorted3", [&] {
        const u64 blocks = std::min<u64>((2 * nchunk + 255) / 256, (u64)ctx->n_cu * 8);
        hipLaunchKernelGGL(k_sorted3, dim3((unsigned)std::max<u64>(blocks, 1)), dim3(256), 0, ctx->stream,
                           (const u64*)dz, (u64)0, (u64*)desc, 2 * nchunk, (u32*)aux, counts);
    });
    if (rc) return rc;
    const int occ_r3a = occupancy(ctx, perm ? (const void*)k_resolve3<C3_NT, true, true> : (const void*)k_resolve3<C3_NT, false, true>,
                                  C3_NT, 0);
    auto ptr = [&](const void* p, u64 n) { return n && p ? p : (const void*)dz; };
    Resolve3Args g{};
    g.A = (const u64*)dz; g.O = (const u64*)ptr(O.key, nO); g.T = (const u64*)ptr(T.key, nT);
    g.oA = (const u32*)ptr(A.oid, nA); g.oO = (const u32*)ptr(O.oid, nO); g.oT = (const u32*)ptr(T.oid, nT);
    g.nA = nA; g.nO = nO;
    g.nmA = (const u8*)ptr(A.name, nA); g.nmO = (const u8*)ptr(O.name, nO); g.nmT = (const u8*)ptr(T.name, nT);
    g.noA = (const u64*)ptr(A.name_off, nA); g.noO = (const u64*)ptr(O.name_off, nO); g.noT = (const u64*)ptr(T.name_off, nT);
    g.hash_mode = A.key_mode == KD_KEY_HASH;
    g.cand = nullptr; g.cand3 = cand3; g.c2 = c2;
    g.pA = (const u32*)ptr(pA, nA); g.pO = (const u32*)ptr(pO, nO); g.pT = (const u32*)ptr(pT, nT);
    g.desc = (u64*)desc; g.nchunk = nchunk; g.aux = (u32*)aux;
    g.out_conf = d_conf; g.out_md = d_md; g.counts = counts; g.err = derr;
    const u64 grid = std::min<u64>((nO + nT) / C3_CH + 1, (u64)ctx->n_cu * (u64)occ_r3a);
    return launch(ctx, "k_resolve3", [&] {
        if (perm) hipLaunchKernelGGL((k_resolve3<C3_NT, true, true>), dim3((unsigned)grid), dim3(C3_NT), 0, ctx->stream, g);
        else hipLaunchKernelGGL((k_resolve3<C3_NT, false, true>), dim3((unsigned)grid), dim3(C3_NT), 0, ctx->stream, g);
    });
}

// --------------------------------------------------------------------------------------------
// host-form helpers
int kd::stage_side(kd_ctx* ctx, const kd_side* s, const char* tag, kd_side* dev) {
    *dev = *s;
    dev->mem = KD_MEM_DEVICE;
    std::string p(tag);
    int rc;
    if ((rc = stage_in(ctx, (p + ".key").c_str(), s->key, s->n * 8, s->mem, (const void**)&dev->key))) return rc;
    if ((rc = stage_in(ctx, (p + ".oid").c_str(), s->oid, s->n * 20, s->mem, (const void**)&dev->oid))) return rc;
    if (s->key_mode == KD_KEY_HASH && s->n) {
        KD_CHECK(s->name_off && s->name, "KD_KEY_HASH side without filenames");
        u64 nbytes = s->mem == KD_MEM_HOST ? s->name_off[s->n] : 0;
        if (s->mem == KD_MEM_DEVICE) {
            KD_HIP(hipMemcpy(&nbytes, s->name_off + s->n, 8, hipMemcpyDeviceToHost));
        }
        if ((rc = stage_in(ctx, (p + ".noff").c_str(), s->name_off, (s->n + 1) * 8, s->mem, (const void**)&dev->name_off))) return rc;
        if ((rc = stage_in(ctx, (p + ".name").c_str(), s->name, nbytes ? nbytes : 1, s->mem, (const void**)&dev->name))) return rc;
    }
    return KD_OK;
}

int kd::check_side(const kd_side* s, const char* which) {
    KD_CHECK(s, "%s side is NULL", which);
    KD_CHECK(s->n == 0 || (s->key && s->oid), "%s side: key/oid NULL", which);
    KD_CHECK(s->mem == KD_MEM_HOST || s->mem == KD_MEM_DEVICE, "%s side: bad mem", which);
    KD_CHECK(s->key_mode == KD_KEY_INT || s->key_mode == KD_KEY_HASH, "%s side: bad key_mode", which);
    return KD_OK;
}

// classify3 on device-resident sides: conflicts (a, o, t index triples, path order) -> d_conf,
// merge deltas -> d_md, counts[4] <- clean, conflicts, mdeltas, 0; *derr <- error bits.  Nothing
// needs zeroing by the caller.
static int merge3_device(kd_ctx* ctx, const kd_side& A, const kd_side& O, const kd_side& T, u32* d_conf, uint2* d_md,
                         u64* counts, u32* derr, const u32* pA = nullptr, const u32* pO = nullptr,
                         const u32* pT = nullptr) {
    const bool perm = pA || pO || pT;
    int rc;
    const u64 nA = A.n, nO = O.n, nT = T.n;
    // the one-pass join (k_join3) unless the union is empty (then only the ancestor's order check
    // remains) or the merge3_join option selects the two-step path (classify2 + k_resolve3)
    if (nO + nT > 0 && ctx->opt.merge3_join)
        return merge3_join_device(ctx, A, O, T, d_conf, d_md, counts, derr, pA, pO, pT);
    const u64 nchunk = (nO + nT) / C3_CH + 2;
    void *cand, *c2, *desc, *aux, *dz;
    if ((rc = ensure(ctx, "c3.cand", (nO + nT + 1) * 8, &cand))) return rc;
    if ((rc = ensure(ctx, "c3.c2", 64, &c2))) return rc;
    if ((rc = ensure(ctx, "c3.desc", 2 * nchunk * 8, &desc))) return rc;
    const bool fresh_aux = ctx->bufs["c3.aux"].p == nullptr;
    if ((rc = ensure(ctx, "c3.aux", 64, &aux))) return rc;
    if (fresh_aux) KD_HIP(hipMemsetAsync(aux, 0, 64, ctx->stream));
    if ((rc = device_zeros(ctx, &dz))) return rc;
    const u64* kA = nA ? A.key : (const u64*)dz;
    rc = launch(ctx, "k_sorted3", [&] {
        const u64 work = std::max<u64>(nA / 2, 2 * nchunk);
        const u64 blocks = std::min<u64>((work + 255) / 256, (u64)ctx->n_cu * 8);
        hipLaunchKernelGGL(k_sorted3, dim3((unsigned)std::max<u64>(blocks, 1)), dim3(256), 0, ctx->stream, kA, nA,
                           (u64*)desc, 2 * nchunk, (u32*)aux, counts);
    });
    if (rc) return rc;
    // ours vs theirs: key-ordered differing paths (+ filename checks, order check, error bits)
    if ((rc = diff2_device(ctx, &O, &T, 0, (u32*)cand, nullptr, (u64*)c2, derr, perm ? pO : nullptr,
                           perm ? pT : nullptr)))
        return rc;
    ctx->occ_resolve3 = occupancy(ctx, perm ? (const void*)k_resolve3<C3_NT, true, false> : (const void*)k_resolve3<C3_NT, false, false>,
                                  C3_NT, 0);
    // an empty side (or an absent filename arena) points at device zeros: lanes without an entry
    // load from index 0 of every array instead of branching, so each array must be readable
    auto ptr = [&](const void* p, u64 n) { return n && p ? p : (const void*)dz; };
    Resolve3Args g;
    g.A = kA; g.O = (const u64*)ptr(O.key, nO); g.T = (const u64*)ptr(T.key, nT);
    g.oA = (const u32*)ptr(A.oid, nA); g.oO = (const u32*)ptr(O.oid, nO); g.oT = (const u32*)ptr(T.oid, nT);
    g.nA = nA; g.nO = nO;
    g.nmA = (const u8*)ptr(A.name, nA); g.nmO = (const u8*)ptr(O.name, nO); g.nmT = (const u8*)ptr(T.name, nT);
    g.noA = (const u64*)ptr(A.name_off, nA); g.noO = (const u64*)ptr(O.name_off, nO); g.noT = (const u64*)ptr(T.name_off, nT);
    g.hash_mode = A.key_mode == KD_KEY_HASH;
    g.cand = (const uint2*)cand; g.c2 = (const u64*)c2;
    g.pA = (const u32*)ptr(pA, nA); g.pO = (const u32*)ptr(pO, nO); g.pT = (const u32*)ptr(pT, nT);
    g.desc = (u64*)desc; g.nchunk = nchunk; g.aux = (u32*)aux;
    g.out_conf = d_conf; g.out_md = d_md; g.counts = counts; g.err = derr;
    // persistent: at most every resident workgroup, at most one per chunk (+1 so someone adds the
    // clean count when there are no differing paths)
    const u64 grid = std::min<u64>((nO + nT) / C3_CH + 1, (u64)ctx->n_cu * (u64)ctx->occ_resolve3);
    return launch(ctx, "k_resolve3", [&] {
        if (perm) hipLaunchKernelGGL((k_resolve3<C3_NT, true, false>), dim3((unsigned)grid), dim3(C3_NT), 0, ctx->stream, g);
        else hipLaunchKernelGGL((k_resolve3<C3_NT, false, false>), dim3((unsigned)grid), dim3(C3_NT), 0, ctx->stream, g);
    });
}

extern "C" {

int kd_reserve(kd_ctx* ctx, uint64_t max_entries_per_side, uint64_t max_updates) {
    KD_CHECK(ctx, "kd_reserve: ctx NULL");
    KD_HIP(hipSetDevice(ctx->device));
    u64 total = 2 * max_entries_per_side;
    u64 ntiles = (total + C2_TILE - 1) / C2_TILE + 1;
    void* p;
    int rc;
    if ((rc = ensure(ctx, "c2.part", (ntiles + 1) * 8, &p))) return rc;
    if ((rc = ensure(ctx, "c2.tcnt", ntiles * 16, &p))) return rc;
    if ((rc = ensure(ctx, "c2.gsum", 2 * (ntiles / 64 + 1) * 8, &p))) return rc;
    if ((rc = ensure(ctx, "c2.sdel", ntiles * (C2_TILE + 64) * 8, &p))) return rc;
    if ((rc = ensure(ctx, "c2.supd", ntiles * (C2_TILE + 64) * 8, &p))) return rc;
    (void)max_updates;
    return KD_OK;
}

int kd_diff2_device(kd_ctx* ctx, const kd_side* base, const kd_side* target, uint32_t flags, uint32_t* d_delta,
                    uint32_t* d_upd, uint64_t* d_counts, uint32_t* d_err) {
    KD_CHECK(ctx, "kd_diff2_device: ctx NULL");
    int rc;
    if ((rc = check_side(base, "base")) || (rc = check_side(target, "target"))) return rc;
    KD_CHECK(base->mem == KD_MEM_DEVICE && target->mem == KD_MEM_DEVICE, "kd_diff2_device: sides must be device memory");
    KD_CHECK(d_delta && d_counts && d_err, "kd_diff2_device: NULL output");
    KD_HIP(hipSetDevice(ctx->device));
    return diff2_device(ctx, base, target, flags, d_delta, d_upd, d_counts, d_err);
}

int kd_diff2_device_perm(kd_ctx* ctx, const kd_side* base, const kd_side* target, const uint32_t* base_order,
                         const uint32_t* target_order, uint32_t flags, uint32_t* d_delta, uint32_t* d_upd,
                         uint64_t* d_counts, uint32_t* d_err) {
    KD_CHECK(ctx, "kd_diff2_device_perm: ctx NULL");
    int rc;
    if ((rc = check_side(base, "base")) || (rc = check_side(target, "target"))) return rc;
    KD_CHECK(base->mem == KD_MEM_DEVICE && target->mem == KD_MEM_DEVICE, "kd_diff2_device_perm: sides must be device memory");
    KD_CHECK(d_delta && d_counts && d_err, "kd_diff2_device_perm: NULL output");
    KD_CHECK((base->n == 0 || base_order) && (target->n == 0 || target_order), "kd_diff2_device_perm: NULL order");
    KD_HIP(hipSetDevice(ctx->device));
    return diff2_device(ctx, base, target, flags, d_delta, d_upd, d_counts, d_err,
                        base_order ? base_order : (const u32*)nullptr, target_order);
}

int kd_diff2_device_ex(kd_ctx* ctx, const kd_side* base, const kd_side* target, const uint32_t* base_order,
                       const uint32_t* target_order, uint32_t flags, uint32_t* d_delta, uint32_t* d_upd,
                       uint64_t* d_delta_key, uint64_t* d_upd_key, uint64_t* d_counts, uint32_t* d_err) {
    KD_CHECK(ctx, "kd_diff2_device_ex: ctx NULL");
    int rc;
    if ((rc = check_side(base, "base")) || (rc = check_side(target, "target"))) return rc;
    KD_CHECK(base->mem == KD_MEM_DEVICE && target->mem == KD_MEM_DEVICE, "kd_diff2_device_ex: sides must be device memory");
    KD_CHECK(d_delta && d_counts && d_err, "kd_diff2_device_ex: NULL output");
    KD_CHECK(!base_order == !target_order, "kd_diff2_device_ex: both orders or neither");
    KD_CHECK(!d_upd_key || (d_upd && d_delta_key), "kd_diff2_device_ex: update keys need the update list and delta keys");
    KD_HIP(hipSetDevice(ctx->device));
    void* dz = nullptr;
    if (base_order && (rc = device_zeros(ctx, &dz))) return rc;
    const u32* oa = base_order ? (base->n ? base_order : (const u32*)dz) : nullptr;
    const u32* ob = target_order ? (target->n ? target_order : (const u32*)dz) : nullptr;
    return diff2_device(ctx, base, target, flags, d_delta, d_upd, d_counts, d_err, oa, ob, d_delta_key, d_upd_key);
}

int kd_diff2(kd_ctx* ctx, const kd_side* base, const kd_side* target, uint32_t flags, kd_diff_result** out) {
    KD_CHECK(ctx && out, "kd_diff2: NULL");
    int rc;
    if ((rc = check_side(base, "base")) || (rc = check_side(target, "target"))) return rc;
    KD_HIP(hipSetDevice(ctx->device));
    host_mark(ctx, nullptr);
    kd_side A, B;
    if ((rc = stage_side(ctx, base, "in.a", &A)) || (rc = stage_side(ctx, target, "in.b", &B))) return rc;
    host_mark(ctx, "kd_diff2 stage");
    u64 total = base->n + target->n;
    void *dd, *du, *dc;
    if ((rc = ensure(ctx, "out.delta", (total + 1) * 8, &dd))) return rc;
    if ((rc = ensure(ctx, "out.upd", (total + 1) * 8, &du))) return rc;
    if ((rc = ensure(ctx, "out.counts", 64, &dc))) return rc;
    host_mark(ctx, "kd_diff2 ensure");
    u64* counts = (u64*)dc;
    u32* derr = (u32*)(counts + 4);
    if ((rc = diff2_device(ctx, &A, &B, flags, (u32*)dd, (u32*)du, counts, derr))) return rc;
    host_mark(ctx, "kd_diff2 kernels");
    u64 hc[5];
    KD_HIP(hipMemcpyAsync(hc, dc, 40, hipMemcpyDeviceToHost, ctx->stream));
    KD_HIP(hipStreamSynchronize(ctx->stream));
    u32 err = (u32)(hc[4] & 0xFFFFFFFFu);
    if (err) {
        set_error("kd_diff2: %s", (err & 1) ? "side keys not strictly ascending" : "hash key collision between different filenames");
        return KD_EUNSUPPORTED;
    }
    u64 nd = hc[3], nu = hc[1];
    host_mark(ctx, "kd_diff2 counts");
    size_t bytes = sizeof(kd_diff_result) + (nd + nu) * 8 + 16;
    kd_diff_result* r = (kd_diff_result*)std::malloc(bytes);
    KD_CHECK(r, "kd_diff2: out of host memory");
    host_mark(ctx, "kd_diff2 malloc");
    r->n_insert = hc[0]; r->n_update = hc[1]; r->n_delete = hc[2]; r->n_delta = nd;
    r->delta = (u32*)(r + 1);
    r->upd = r->delta + 2 * nd;
    if (nd) {
        if ((rc = stage_d2h(ctx, r->delta, dd, nd * 8)) || (nu && (rc = stage_d2h(ctx, r->upd, du, nu * 8)))) {
            std::free(r);
            return rc;
        }
    }
    host_mark(ctx, "kd_diff2 results");
    prof_flush(ctx);
    *out = r;
    return KD_OK;
}

int kd_merge3(kd_ctx* ctx, const kd_side* anc, const kd_side* ours, const kd_side* theirs, uint32_t flags,
              kd_merge_result** out) {
    (void)flags;
    KD_CHECK(ctx && out, "kd_merge3: NULL");
    int rc;
    if ((rc = check_side(anc, "ancestor")) || (rc = check_side(ours, "ours")) || (rc = check_side(theirs, "theirs"))) return rc;
    KD_CHECK(anc->key_mode == ours->key_mode && ours->key_mode == theirs->key_mode, "kd_merge3: key modes differ");
    KD_CHECK(anc->n < 0xFFFFFFFFull && ours->n < 0xFFFFFFFFull && theirs->n < 0xFFFFFFFFull, "kd_merge3: side too large");
    KD_HIP(hipSetDevice(ctx->device));
    kd_side A, O, T;
    if ((rc = stage_side(ctx, anc, "in.a", &A)) || (rc = stage_side(ctx, ours, "in.b", &O)) ||
        (rc = stage_side(ctx, theirs, "in.c", &T)))
        return rc;
    const u64 nA = A.n, nO = O.n, nT = T.n;
    void *oc, *om, *dc;
    if ((rc = ensure(ctx, "c3.oc", (nA + nO + nT + 1) * 12, &oc))) return rc;
    if ((rc = ensure(ctx, "c3.om", (nO + nT + 1) * 8, &om))) return rc;
    if ((rc = ensure(ctx, "c3.counts", 64, &dc))) return rc;
    u64* counts = (u64*)dc;
    u32* derr = (u32*)(counts + 4);
    if ((rc = merge3_device(ctx, A, O, T, (u32*)oc, (uint2*)om, counts, derr))) return rc;
    u64 hc[5];
    KD_HIP(hipMemcpyAsync(hc, dc, 40, hipMemcpyDeviceToHost, ctx->stream));
    KD_HIP(hipStreamSynchronize(ctx->stream));
    u32 err = (u32)(hc[4] & 0xFFFFFFFFu);
    if (err) {
        set_error("kd_merge3: err=0x%x (%s)", err,
                  (err & 1) ? "keys not strictly ascending" : (err & 2) ? "hash key collision" : "tile overflow");
        return KD_EUNSUPPORTED;
    }
    u64 nc = hc[1], nm = hc[2];
    kd_merge_result* r = (kd_merge_result*)std::malloc(sizeof(kd_merge_result) + nc * 12 + nm * 8 + 16);
    KD_CHECK(r, "kd_merge3: out of host memory");
    r->n_clean = hc[0]; r->n_conflict = nc; r->n_mdelta = nm;
    r->conflict = (u32*)(r + 1);
    r->mdelta = r->conflict + 3 * nc;
    if ((nc && (rc = stage_d2h(ctx, r->conflict, oc, nc * 12))) || (nm && (rc = stage_d2h(ctx, r->mdelta, om, nm * 8)))) {
        std::free(r);
        return rc;
    }
    prof_flush(ctx);
    *out = r;
    return KD_OK;
}

int kd_merge3_device(kd_ctx* ctx, const kd_side* anc, const kd_side* ours, const kd_side* theirs, uint32_t flags,
                     uint32_t* d_conflict, uint32_t* d_mdelta, uint64_t* d_counts, uint32_t* d_err) {
    (void)flags;
    KD_CHECK(ctx && d_conflict && d_mdelta && d_counts && d_err, "kd_merge3_device: NULL");
    int rc;
    if ((rc = check_side(anc, "ancestor")) || (rc = check_side(ours, "ours")) || (rc = check_side(theirs, "theirs"))) return rc;
    KD_CHECK(anc->mem == KD_MEM_DEVICE && ours->mem == KD_MEM_DEVICE && theirs->mem == KD_MEM_DEVICE,
             "kd_merge3_device: sides must be device memory");
    KD_CHECK(anc->key_mode == ours->key_mode && ours->key_mode == theirs->key_mode, "kd_merge3_device: key modes differ");
    KD_CHECK(anc->n < 0xFFFFFFFFull && ours->n < 0xFFFFFFFFull && theirs->n < 0xFFFFFFFFull,
             "kd_merge3_device: side too large");
    KD_HIP(hipSetDevice(ctx->device));
    return merge3_device(ctx, *anc, *ours, *theirs, d_conflict, (uint2*)d_mdelta, d_counts, d_err);
}

int kd_merge3_device_perm(kd_ctx* ctx, const kd_side* anc, const kd_side* ours, const kd_side* theirs,
                          const uint32_t* anc_order, const uint32_t* ours_order, const uint32_t* theirs_order,
                          uint32_t flags, uint32_t* d_conflict, uint32_t* d_mdelta, uint64_t* d_counts, uint32_t* d_err) {
    (void)flags;
    KD_CHECK(ctx && d_conflict && d_mdelta && d_counts && d_err, "kd_merge3_device_perm: NULL");
    int rc;
    if ((rc = check_side(anc, "ancestor")) || (rc = check_side(ours, "ours")) || (rc = check_side(theirs, "theirs"))) return rc;
    KD_CHECK(anc->mem == KD_MEM_DEVICE && ours->mem == KD_MEM_DEVICE && theirs->mem == KD_MEM_DEVICE,
             "kd_merge3_device_perm: sides must be device memory");
    KD_CHECK(anc->key_mode == ours->key_mode && ours->key_mode == theirs->key_mode, "kd_merge3_device_perm: key modes differ");
    KD_CHECK(anc->n < 0xFFFFFFFFull && ours->n < 0xFFFFFFFFull && theirs->n < 0xFFFFFFFFull,
             "kd_merge3_device_perm: side too large");
    KD_CHECK((anc->n == 0 || anc_order) && (ours->n == 0 || ours_order) && (theirs->n == 0 || theirs_order),
             "kd_merge3_device_perm: NULL order");
    KD_HIP(hipSetDevice(ctx->device));
    void* dz;
    if ((rc = device_zeros(ctx, &dz))) return rc;
    auto ord = [&](const uint32_t* p) { return p ? p : (const u32*)dz; };
    return merge3_device(ctx, *anc, *ours, *theirs, d_conflict, (uint2*)d_mdelta, d_counts, d_err, ord(anc_order),
                         ord(ours_order), ord(theirs_order));
}

}  // extern "C"
