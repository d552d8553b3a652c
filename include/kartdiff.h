/*
 * kartdiff.h — C ABI of libkartdiff.so, the MI355X (gfx950) bulk feature-diff engine.
 *
 * Drop-in boundary.  Each entry point replaces one reference interface:
 *
 *   kd_diff2       <- libgit2 tree-to-tree diff as consumed by RichBaseDataset.diff_feature
 *                     (/root/reference/kart/rich_base_dataset.py:205-300; the FFI call is
 *                     Tree.diff_to_tree at :212-232).  Returns the insert/update/delete delta set.
 *   kd_fielddiff   <- Dataset3.get_feature (kart/dataset3.py:185-223) + Schema.feature_from_raw_dict
 *                     (kart/schema.py:288-293) + the per-field Python `==` compare of
 *                     TextDiffWriter.write_feature_delta (kart/text_diff_writer.py:135-145).
 *   kd_merge3      <- repo.merge_trees(ancestor, ours, theirs) (kart/merge.py:99-100; libgit2
 *                     git_merge_trees) feeding MergeIndex.from_pygit2_index (kart/merge_util.py:92-103).
 *   kd_envelopes   <- SpatialFilter.matches envelope quick-check (kart/spatial_filter/__init__.py:534-590,
 *                     709-734) + get_envelope_for_indexing/EnvelopeEncoder.encode for an identity
 *                     CRS (kart/spatial_filter/index.py:485-579,639-707).
 *   kd_env_overlap <- sf_filter_blob decode + cyclic_range_overlaps
 *                     (vendor/spatial-filter/spatial_filter.cpp:170-260).
 *   kd_sf_index_build / kd_sf_filter
 *                  <- sf_filter_blob (vendor/spatial-filter/spatial_filter.cpp:212-260): the clone-time
 *                     spatial filter over a batch of object ids against feature_envelopes.
 *   kd_geom_filter <- BaseDiffWriter.filtered_ds_feature_deltas (kart/base_diff_writer.py:279-329):
 *                     the geometry of each delta's old/new feature blob, envelope-tested, kept
 *                     deltas compacted on the GPU.  kd_geom_heads + kd_geom_filter_heads: the same
 *                     from 48-byte geometry heads the blob reader extracts on the host.
 *   kd_hex_encode  <- Geometry.to_hex_wkb / gpkg_geom_to_hex_wkb (kart/geometry.py:346-375) and
 *                     bytes.hex(v), as feature_as_json formats them (kart/feature_output.py:34-56).
 *   kd_diff2_sharded / kd_diff2_gather
 *                  <- the same diff split by dataset3 path-bucket range over several GPUs (the
 *                     reference's own sharding idea: kart/fast_import.py:289-337), counts and
 *                     compacted delta records all-gathered over RCCL (xGMI).
 *   kd_malloc / kd_memcpy / kd_host_alloc ...
 *                  device HBM and pinned host staging for callers without a GPU framework.
 *   kd_pack_*      <- Dataset3.decode_path_to_1pk / PathEncoder (kart/dataset3.py:250-259,
 *                     kart/dataset3_paths.py:202-215,292-299): host-side key packing.
 *   kd_odb_* / kd_walk
 *                  <- libgit2's ODB reads and tree iteration under Dataset3 (kart/dataset3.py:
 *                     26-35,225-231; kart/base_dataset.py:230-265), with diff_to_tree's subtree
 *                     pruning: the leaves the packer above consumes, read natively.
 *
 * Conventions: plain pointers and sizes only; return 0 on success, KD_EINVAL (-1) on bad
 * arguments, KD_EHIP (-2) on a HIP runtime error, KD_EUNSUPPORTED (-3) when the input needs
 * the CPU path (caller falls back); kd_last_error() gives a thread-local message.  One kd_ctx per
 * GPU; calls on one context are serialised by the caller.  Index arrays are uint32 (a side may
 * hold at most 2^32-2 entries per GPU); KD_NONE marks "absent".
 */
#ifndef KARTDIFF_H
#define KARTDIFF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KD_ABI_VERSION 1

#define KD_OK 0
#define KD_EINVAL (-1)
#define KD_EHIP (-2)
#define KD_EUNSUPPORTED (-3)

#define KD_NONE 0xFFFFFFFFu

/* where a buffer lives */
#define KD_MEM_HOST 0u
#define KD_MEM_DEVICE 1u

/* key modes (see DESIGN.md "join key") */
#define KD_KEY_INT 0u  /* IntPathEncoder: key = rank24(bucket) | wrap34 | frank(pk), bijective with
                          pk and ascending in git's tree order (DESIGN.md "join key")            */
#define KD_KEY_HASH 1u /* MsgpackHashPathEncoder: key = rank-mapped bucket bits | FNV-1a(filename)
                          bits; matched keys are verified against the filename bytes           */

typedef struct kd_ctx kd_ctx;

/* One commit's dataset feature tree, flattened: n leaf entries sorted by strictly ascending key.
 * KD_KEY_INT keys of a tree walk's leaves are ascending as listed (git tree order), unless a leaf
 * tree mixes pks of different 2^30 wraps; KD_KEY_HASH leaves need kd_sort_segmented_into. */
typedef struct kd_side {
    uint64_t n;
    const uint64_t* key;      /* [n] join keys, strictly ascending                                 */
    const uint8_t* oid;       /* [n*20] git blob OIDs (raw bytes)                                  */
    const uint8_t* name;      /* KD_KEY_HASH only: concatenated filenames (may be NULL for INT)    */
    const uint64_t* name_off; /* [n+1] offsets into name (KD_KEY_HASH only)                        */
    uint32_t mem;             /* KD_MEM_HOST or KD_MEM_DEVICE: where the arrays above live         */
    uint32_t key_mode;        /* KD_KEY_INT or KD_KEY_HASH                                         */
} kd_side;

/* A blob arena: blob b = data[off[b] .. off[b+1]).  Feature blobs are msgpack
 * [legend_hex40, [values...]] (kart/dataset3.py:185-215); geometry blobs are GPKG binary. */
typedef struct kd_blobs {
    uint64_t n;
    const uint8_t* data;
    const uint64_t* off; /* [n+1] */
    uint32_t mem;
    uint32_t size_hint; /* typical (mean) blob size in bytes (0 = unknown); sizes the LDS staging pool */
} kd_blobs;

/* Legend -> union-key maps for kd_fielddiff (host memory).  Union keys are the old schema's
 * column names in order, then the new schema's names not in the old one
 * (BaseDiffWriter._all_feature_keys, kart/base_diff_writer.py:181-187).
 * map[l*n_keys + k] = value index in legend l's non-pk array, or
 *   -1 key not in that side's schema (_NULL), -2 column absent from the legend (None),
 *   -3 the primary-key column (value from the path). */
typedef struct kd_legend_maps {
    int32_t n_keys;
    int32_t words;            /* ceil(n_keys / 64): uint64 mask words per update */
    int32_t n_leg_old;
    int32_t n_leg_new;
    const uint8_t* leg_old_hex; /* [n_leg_old*40] legend hexhash strings */
    const int16_t* map_old;     /* [n_leg_old*n_keys] */
    const uint8_t* leg_new_hex;
    const int16_t* map_new;
    const uint64_t* cmp_mask;   /* [words] keys to compare ("__"-prefixed keys are excluded) */
} kd_legend_maps;

typedef struct kd_diff_result {
    uint64_t n_insert, n_update, n_delete, n_delta;
    uint32_t* delta;  /* [2*n_delta] (base index | KD_NONE, target index | KD_NONE), key order */
    uint32_t* upd;    /* [2*n_update] (base index, target index) of the updates, key order     */
} kd_diff_result;

typedef struct kd_merge_result {
    uint64_t n_clean;     /* merged entries present without conflict                          */
    uint64_t n_conflict;
    uint64_t n_mdelta;    /* entries where the merge result differs from ours                 */
    uint32_t* conflict;   /* [3*n_conflict] (ancestor, ours, theirs) index | KD_NONE          */
    uint32_t* mdelta;     /* [2*n_mdelta] (ours | KD_NONE, theirs | KD_NONE): take theirs     */
} kd_merge_result;

/* -------- context -------- */
int kd_abi_version(void);
const char* kd_last_error(void);
/* Creates the context and warms the first-diff path (runtime copy kernels, DMA queues, the pinned
 * staging chunks, one 1 + 1-entry classify2), so a one-shot process's first diff runs warm. */
int kd_init(int device_ordinal, kd_ctx** out);
int kd_fini(kd_ctx* ctx);
/* Launch on an external HIP stream (e.g. torch's current stream); NULL = the context's own. */
int kd_set_stream(kd_ctx* ctx, void* hip_stream);
/* Tuning options of a context (A/B switches of the measured alternatives; defaults are the measured
 * optima).  kd_init seeds each from the environment variable in brackets, once; kd_set_option changes
 * it for later calls on the context.  Unknown names: KD_EINVAL.
 *   merge3_join    [KD_MERGE3_JOIN]    1: one-pass three-way join (k_join3); 0: classify2 + k_resolve3
 *   merge3_split   [KD_MERGE3_SPLIT]   1: k_join3 stages candidates, k_resolve3 applies the rule
 *   j3_ol          [KD_J3_OL]          1: k_join3 stages ours'/theirs' OIDs in LDS (sorted-form sides)
 *   j3_v           [KD_J3_V]           1: k_join3b (every tile range in one LDS-DMA batch); 0: k_join3
 *   j2_oidlds_min  [KD_J2_OIDLDS_MIN]  k_join2 stages OIDs in LDS from this many entries (2^26)
 *   j2r            [KD_J2R]            1: the persistent register-prefetched int-key join
 *   fd_stream      [KD_FD_STREAM]      -1 auto, 0 windowed, 1 streamed field diff (contiguous arenas)
 *   fd_walk        [KD_FD_WALK]        -1 / 0 off, 1 the walked field diff (A/B)
 *   pkm_max_blocks [KD_PKM_MAX_BLOCKS] largest pk range (64-pk blocks) kd_delta_pk_order places by bitmap
 *   trace_host     [KD_TRACE_HOST]     1: stream-synced wall-clock marks of host phases to stderr */
int kd_set_option(kd_ctx* ctx, const char* name, int64_t value);
int kd_get_option(kd_ctx* ctx, const char* name, int64_t* value);
int kd_sync(kd_ctx* ctx);
/* Pre-size device workspaces so the first timed call does not allocate. */
int kd_reserve(kd_ctx* ctx, uint64_t max_entries_per_side, uint64_t max_updates);
void kd_free(void* p); /* frees kd_diff_result / kd_merge_result and their arrays */

/* -------- two-way diff: classify2 (+ optional fused field diff) -------- */
/* Host-convenience form: sides may be host or device; results are host memory (kd_free). */
int kd_diff2(kd_ctx* ctx, const kd_side* base, const kd_side* target, uint32_t flags,
             kd_diff_result** out);
/* flags for kd_diff2 / kd_diff2_device */
#define KD_DIFF_UNORDERED 0x1u /* device form only: deltas/updates grouped per 1024-pair tile, tiles in
                                  completion order (each tile key-ordered) — skips the ordering
                                  scan + scatter; the delta SET is identical                      */

/* Device form: everything device-resident, asynchronous on the context stream.
 * d_delta / d_upd capacity must cover the worst case (base.n + target.n pairs).
 * d_counts[4] <- inserts, updates, deletes, deltas.  d_err <- nonzero if a side is not strictly
 * ascending (1) or a KD_KEY_HASH key matched two different filenames (2). */
int kd_diff2_device(kd_ctx* ctx, const kd_side* base, const kd_side* target, uint32_t flags,
                    uint32_t* d_delta, uint32_t* d_upd, uint64_t* d_counts, uint32_t* d_err);

/* Late-materialised form, what follows kd_sort_side_into(..., d_oid_out = NULL, ...): each side's
 * keys are sorted but its OIDs (and KD_KEY_HASH filename offsets) are still in the order the tree
 * walk produced them; row order[i] belongs to sorted entry i.  The join reads OIDs through the order
 * (one extra coalesced 4-B load per matched entry), so no side's OIDs are ever permuted.  Results are
 * identical to kd_diff2_device on the permuted sides (indices are sorted-entry indices). */
int kd_diff2_device_perm(kd_ctx* ctx, const kd_side* base, const kd_side* target, const uint32_t* base_order,
                         const uint32_t* target_order, uint32_t flags, uint32_t* d_delta, uint32_t* d_upd,
                         uint64_t* d_counts, uint32_t* d_err);

/* kd_diff2_device / kd_diff2_device_perm with more outputs: base_order / target_order (both or
 * NULL) as kd_diff2_device_perm; d_delta_key [cap] / d_upd_key [cap] (optional, device) <- the join key
 * of every delta / update record, written beside the lists (what kd_delta_pk_order reads instead of
 * gathering them from the sides). */
int kd_diff2_device_ex(kd_ctx* ctx, const kd_side* base, const kd_side* target, const uint32_t* base_order,
                       const uint32_t* target_order, uint32_t flags, uint32_t* d_delta, uint32_t* d_upd,
                       uint64_t* d_delta_key, uint64_t* d_upd_key, uint64_t* d_counts, uint32_t* d_err);

/* -------- field diff -------- */
/* For each update u: old blob = old->data[old->off[pu[2u]] ..], new blob = neu->...[pu[2u+1]]
 * (pu = the (base, target) update pairs, or NULL: blob u on both sides).  masks[u*words + w]
 * bit k set iff union key k changed under Python `==`.  status[u]: 0 ok, 1 malformed blob,
 * 2 unknown legend, 3 too many values, 4 unsupported value (nested container, invalid ext 'G'):
 * nonzero -> the caller recomputes that update on the CPU path.
 * pairs_mem / out_mem say where pu and masks/status live.  Device form: with d_n_upd != NULL the
 * update count is read from that device counter (no host sync between classify and diff), pu
 * and the outputs must be device memory, and n_upd is the capacity — an upper bound of *d_n_upd
 * used to size the grid (0 = unknown). */
int kd_fielddiff(kd_ctx* ctx, const kd_blobs* old_blobs, const kd_blobs* new_blobs,
                 const uint32_t* pu, uint64_t n_upd, const uint64_t* d_n_upd, uint32_t pairs_mem,
                 const kd_legend_maps* maps, uint64_t* masks, uint8_t* status, uint32_t out_mem);

/* -------- three-way merge classification -------- */
int kd_merge3(kd_ctx* ctx, const kd_side* ancestor, const kd_side* ours, const kd_side* theirs,
              uint32_t flags, kd_merge_result** out);
/* Device form of kd_merge3 (no host sync): all three sides in device memory; d_conflict
 * [(a.n + o.n + t.n) * 3] <- conflict triples (ancestor, ours, theirs index, 0xFFFFFFFF = absent)
 * in path order, d_mdelta [(o.n + t.n) * 2] <- merge deltas, d_counts[4] <- clean entries,
 * conflicts, merge deltas, 0; d_err <- 1 unsorted side, 2 hash key collision, 8 tile overflow. */
int kd_merge3_device(kd_ctx* ctx, const kd_side* ancestor, const kd_side* ours, const kd_side* theirs,
                     uint32_t flags, uint32_t* d_conflict, uint32_t* d_mdelta, uint64_t* d_counts,
                     uint32_t* d_err);

/* Late-materialised form (after kd_sort_segmented_into / kd_sort_side_into without OIDs): keys
 * sorted, each side's OIDs and KD_KEY_HASH filename offsets still in walk order, row order[i]
 * belonging to sorted entry i.  Results identical to kd_merge3_device on the permuted sides. */
int kd_merge3_device_perm(kd_ctx* ctx, const kd_side* ancestor, const kd_side* ours, const kd_side* theirs,
                          const uint32_t* ancestor_order, const uint32_t* ours_order, const uint32_t* theirs_order,
                          uint32_t flags, uint32_t* d_conflict, uint32_t* d_mdelta, uint64_t* d_counts,
                          uint32_t* d_err);

/* -------- spatial -------- */
/* Per geometry blob (GPKG; length 0 = null geometry):
 *   match[i]: 0 NON_MATCHING, 1 CANDIDATE (bbox passed; exact GEOS test is the caller's),
 *             2 MATCHING (null geometry), 3 FALLBACK (needs the CPU path)
 *   enc[i*bits/2 ..] EnvelopeEncoder bytes of the identity-CRS index envelope; enc_ok[i]=1 when
 *   the spatial indexer would store a row.
 * filt_env = (min-x, max-x, min-y, max-y) of the filter (SpatialFilter.filter_env). */
int kd_envelopes(kd_ctx* ctx, const kd_blobs* geoms, const double filt_env[4], int bits,
                 uint8_t* match, uint8_t* enc, uint8_t* enc_ok, uint32_t out_mem,
                 uint64_t* n_candidates);
/* Decode n encoded envelopes (bits/2 bytes each) and test them against q = (w, s, e, n):
 * out[i] = cyclic(w,e) && range(s,n) overlap (spatial_filter.cpp:187-260). */
int kd_env_overlap(kd_ctx* ctx, const uint8_t* enc, uint64_t n, int bits, const double q[4],
                   uint8_t* out, uint32_t mem);

/* -------- clone-time spatial filter -------- */
/* sf_filter_blob (vendor/spatial-filter/spatial_filter.cpp:212-260) for a batch of objects.  The
 * feature_envelopes table (blob id -> EnvelopeEncoder bytes, bits/2 each: bits = 8 * bytes / 4 as
 * the reference derives it) is loaded once into HBM: oid [n*20] and env [n*bits/2] in any row order
 * (mem: where they live).  kd_sf_filter answers m objects: oid [m*20] (4-byte aligned), is_feature
 * [m] (may be NULL = all are feature blobs: 1 when the object's path contains
 * "/.table-dataset/feature/" or "/.sno-dataset/feature/"), q = (w, s, e, n) of the filter;
 * result[i] = 0 MATCH (not a feature, not in the index, or the envelope overlaps), 1 NOT_MATCHED,
 * 2 ERROR (an inverted range reached by range_overlaps, per object as the reference decides it: a
 * query with south > north errors only the objects whose longitude range overlaps). */
typedef struct kd_sf_index kd_sf_index;
int kd_sf_index_build(kd_ctx* ctx, const uint8_t* oid, const uint8_t* env, uint64_t n, int bits, uint32_t mem,
                      kd_sf_index** out);
int kd_sf_filter(kd_ctx* ctx, const kd_sf_index* index, const uint8_t* oid, const uint8_t* is_feature, uint64_t m,
                 const double q[4], uint8_t* result, uint32_t mem);
int kd_sf_index_free(kd_sf_index* index);

/* -------- spatially filtered diff -------- */
/* BaseDiffWriter.filtered_ds_feature_deltas (kart/base_diff_writer.py:279-329) with
 * SpatialFilter.matches (kart/spatial_filter/__init__.py:534-605): for every delta, the geometry
 * column is located in the old and new feature blobs (legend -> value position), its GPKG
 * envelope (or point) tested against the filter envelope in FP64.  Per side (match[2d], match[2d+1]):
 *   0 NON_MATCHING, 1 CANDIDATE (bbox passes: the exact Intersects is the caller's),
 *   2 MATCHING (null geometry / no geometry column / inside a KD_GF_RECT filter),
 *   3 FALLBACK (the caller decides on the CPU: unknown legend, nested value, envelope needs OGR),
 *   4 NONEXISTENT (KD_NONE side).  Empty geometries are NON_MATCHING (Intersects(empty) is false).
 * keep[0..*n_keep) <- the delta indices (in delta order) with either side 1, 2 or 3.
 * enc/enc_ok (optional, NULL): the new side's spatial-index envelope (EnvelopeEncoder, bits/2
 * bytes per delta), as kd_envelopes computes it.  pairs = (old blob | KD_NONE, new blob | KD_NONE)
 * per delta — classify2's delta list with the arenas indexed by sorted entry.  With d_n the count
 * is read on the device (pairs and outputs device memory, n = capacity).  match must be 2-B aligned. */
#define KD_GF_RECT 0x1u /* the filter geometry is its own envelope (an axis-aligned rectangle) */
/* kd_geom_filter_heads / kd_geom_filter_deltas: the heads are already in delta order — heads_old[d] /
 * heads_new[d] belong to delta d (an absent side's slot is never read), as the drop-in's blob reader
 * lays them out after classification; pairs then give each side's presence and its blob in the
 * arenas (the slow path).  n_old and n_new must each cover whole 64-delta chunks of the capacity
 * (>= ceil(n / 64) * 64; heads device memory in kd_geom_filter_deltas). */
#define KD_GF_DELTA_HEADS 0x2u
typedef struct kd_geom_cols {
    int32_t n_leg_old, n_leg_new;
    const uint8_t* leg_old_hex; /* [n_leg_old*40] legend hexhashes (host memory) */
    const int16_t* gidx_old;    /* [n_leg_old] value index of the geometry column, -1 none */
    const uint8_t* leg_new_hex;
    const int16_t* gidx_new;
} kd_geom_cols;
int kd_geom_filter(kd_ctx* ctx, const kd_blobs* old_blobs, const kd_blobs* new_blobs, const uint32_t* pairs,
                   uint64_t n, const uint64_t* d_n, uint32_t pairs_mem, const kd_geom_cols* cols,
                   const double filt_env[4], uint32_t flags, int bits, uint8_t* match, uint32_t* keep,
                   uint64_t* n_keep, uint8_t* enc, uint8_t* enc_ok, uint32_t out_mem);

/* Geometry heads (host, multithreaded): the filtered diff from 48 contiguous bytes per blob.  For
 * each feature blob (msgpack [legend_hex, [values]]) the geometry column's value is located as
 * msgpack.unpackb + Dataset3.get_feature would (kart/dataset3.py:185-223; the whole blob validated:
 * nested values skipped, trailing bytes refused) and its GPKG bytes summarised: */
#define KD_GH_GEOM 0u     /* a geometry: gpkg[] = its first min(glen, 40) bytes (header + XY envelope) */
#define KD_GH_NULL 2u     /* null geometry, or no geometry column in the blob's legend (MATCHING)    */
#define KD_GH_FALLBACK 3u /* malformed blob, unknown legend, value not an ext 'G': the caller decides */
typedef struct kd_geom_head {
    uint8_t gpkg[40];
    uint32_t glen;        /* GPKG value length                                                        */
    uint32_t goff_status; /* (status << 24) | offset of the GPKG value in its blob (< 2^24)           */
} kd_geom_head;
/* n_leg legends (40-byte hex each) with gidx[l] = the geometry value's index (-1: none); threads
 * 0 = up to 16.  Blob i = data[off[i] .. off[i+1]) (host memory). */
int kd_geom_heads(const uint8_t* data, const uint64_t* off, uint64_t n, int n_leg, const uint8_t* leg_hex,
                  const int16_t* gidx, int threads, kd_geom_head* out);
/* kd_geom_filter from the heads: same codes, keep list and index envelopes.  heads_old [n_old] /
 * heads_new [n_new] in heads_mem; pairs index them.  A geometry whose decode needs bytes past its
 * head (an XYZ/XYM/XYZM envelope, a NaN envelope) is read from old_blobs / new_blobs (the arenas
 * the heads came from, device or host); with NULL arenas such a side is 3 FALLBACK. */
int kd_geom_filter_heads(kd_ctx* ctx, const kd_geom_head* heads_old, uint64_t n_old, const kd_geom_head* heads_new,
                         uint64_t n_new, uint32_t heads_mem, const kd_blobs* old_blobs, const kd_blobs* new_blobs,
                         const uint32_t* pairs, uint64_t n, const uint64_t* d_n, uint32_t pairs_mem,
                         const double filt_env[4], uint32_t flags, int bits, uint8_t* match, uint32_t* keep,
                         uint64_t* n_keep, uint8_t* enc, uint8_t* enc_ok, uint32_t out_mem);

/* kd_geom_filter_heads over classify2's delta list on the device (all buffers device memory, the delta
 * count *d_n on the device, cap the list's capacity): filtered from heads in delta order (the layout
 * the drop-in's blob reader produces: it reads the deltas' blobs after classification); a geometry
 * whose head cannot decide it is read from old_blobs / new_blobs at the delta's own blob (the pairs).
 * With KD_GF_DELTA_HEADS in flags the heads are given in delta order; without it heads_old [n_old] /
 * heads_new [n_new] are indexed like the arenas (per entry) and first gathered into delta order.
 * Outputs as kd_geom_filter_heads (match [cap * 2], keep [cap], n_keep, enc, enc_ok: device). */
int kd_geom_filter_deltas(kd_ctx* ctx, const kd_geom_head* heads_old, uint64_t n_old, const kd_geom_head* heads_new,
                          uint64_t n_new, const kd_blobs* old_blobs, const kd_blobs* new_blobs, const uint32_t* pairs,
                          uint64_t cap, const uint64_t* d_n, const double filt_env[4], uint32_t flags, int bits,
                          uint8_t* match, uint32_t* keep, uint64_t* n_keep, uint8_t* enc, uint8_t* enc_ok);

/* -------- writer formatting -------- */
#define KD_HEX_BYTES 0u    /* bytes.hex(v): lowercase hex of every byte of every blob                */
#define KD_HEX_GPKG_WKB 1u /* gpkg_geom_to_hex_wkb: uppercase hex of the WKB after the GPKG header   */
/* hex[2*off[n]]: the hex of arena byte p lands at hex[2p], so blob i's string is
 * hex[2*(off[i] + start[i]) .. 2*off[i+1]) (start = 0 in KD_HEX_BYTES mode; start/status may then
 * be NULL).  KD_HEX_GPKG_WKB: start[i] = WKB offset in blob i (8 + envelope size), status[i] =
 * 0 ok, 1 null geometry (length 0: the reference returns None), 3 needs the CPU path (invalid
 * GPKG or empty WKB: the reference raises; big-endian WKB: the reference re-encodes via OGR).
 * blobs->mem says where the arena lives, out_mem where hex/start/status live. */
int kd_hex_encode(kd_ctx* ctx, const kd_blobs* blobs, uint32_t mode, uint8_t* hex, uint32_t* start,
                  uint8_t* status, uint32_t out_mem);

/* -------- packing on the GPU (the sort that follows the leaf-path decode) -------- */
/* Sort one side's n entries by join key on the device: an onesweep LSD radix sort over the keys'
 * varying bits (LDS-ranked, LDS-reordered tiles, decoupled look-back; stable).  d_key [n] is sorted in place; d_order [n] <- original index of
 * sorted entry k; d_oid [n*20] (may be NULL) is permuted in place.  *h_dup (may be NULL) <- 1 when
 * the sorted keys are not strictly ascending (two entries share a key: the caller's fallback).
 * Replaces the host sort of the packer (Dataset3 leaves arrive in git path order, not key order). */
int kd_sort_side(kd_ctx* ctx, uint64_t* d_key, uint8_t* d_oid, uint32_t* d_order, uint64_t n, uint32_t* h_dup);
/* What a sort needs to know about a side's keys (host scan, kd_keys_scan): the bits that vary
 * (OR of key[i] ^ key[0]) and key[0]; whether the keys are strictly ascending already (a walk-order
 * KD_KEY_INT side usually is: no sort); for KD_KEY_INT the smallest and largest pk; seg_max: the
 * longest run of consecutive keys sharing their top 24 bits (the leaf tree: a walk lists each leaf
 * tree's entries together), or -1 when those bits descend somewhere — a side with 0 < seg_max <= 512
 * that is not ascending sorts per leaf tree (kd_sort_segmented_into, seg_bits 24). */
typedef struct kd_keys_info {
    uint64_t vary;
    uint64_t key0;
    int64_t pk_min, pk_max; /* KD_KEY_INT only */
    int32_t ascending;
    int32_t seg_max;
} kd_keys_info;
int kd_keys_scan(const uint64_t* keys, uint64_t n, uint32_t key_mode, kd_keys_info* out);
/* Out-of-place form (what a device pipeline runs): d_key_in / d_oid_in hold the side in walk order
 * and are left unchanged; d_key_out [n] <- the keys ascending, d_oid_out [n*20] <- the OIDs in that
 * order (both oid pointers NULL to skip: kd_diff2_device_perm then reads them through the order),
 * d_order [n] <- input index of sorted entry k.  d_dup (device, may be NULL: a following
 * kd_diff2_device checks strict order anyway) <- 1 when two entries share a key.  Outputs must not
 * alias inputs.  info (host, from kd_keys_scan) sizes the passes; with NULL one 16-byte read-back
 * finds the varying bits.  Otherwise asynchronous on the context stream.  This is the fallback of a
 * side whose walk order is not key order (a leaf tree mixing pk wraps). */
int kd_sort_side_into(kd_ctx* ctx, const uint64_t* d_key_in, const uint8_t* d_oid_in, uint64_t* d_key_out,
                      uint8_t* d_oid_out, uint32_t* d_order, uint64_t n, uint32_t* d_dup, const kd_keys_info* info);
/* A side in walk order whose keys ascend in their top seg_bits bucket bits (KD_KEY_HASH: inside a leaf
 * tree the leaves are in filename order, not FNV order; KD_KEY_INT: a leaf tree mixing pk wraps):
 * each bucket's entries ordered by key.
 * d_key_out [n] <- keys ascending, d_order [n] <- walk index of sorted entry k (the OIDs and
 * filenames stay in walk order: kd_diff2_device_perm / kd_merge3_device_perm read through it).
 * *d_err |= 1 on a duplicate key or descending bucket bits, 4 on a bucket of more than 512 entries
 * (then sort with kd_sort_side_into).  max_seg: the longest bucket the caller knows of (kd_keys_scan's
 * seg_max; 0 = unknown): at most 128 stages a smaller halo per tile.  One kernel, no host sync. */
int kd_sort_segmented_into(kd_ctx* ctx, const uint64_t* d_key_in, uint64_t* d_key_out, uint32_t* d_order,
                           uint64_t n, int seg_bits, int max_seg, uint32_t* d_err);
/* The deltas in pk order (DeltaDiff.sorted_items, kart/diff_structs.py:442-458; classify2 emits them in
 * git walk order): for KD_KEY_INT device sides and a device record list d_delta [cap] of (base | KD_NONE,
 * target | KD_NONE) records (classify2's deltas or updates) with *d_n of them, d_pk [cap] <- their pks
 * ascending, d_perm [cap] <- the record index of pk rank k.  d_keys (optional, device): the records'
 * keys as kd_diff2_device_ex wrote them (else each is gathered from the sides).  pk_lo / pk_hi bound
 * every pk of both sides (kd_keys_scan's pk_min / pk_max): a range of at most 2^26 64-pk blocks is
 * placed through a bitmap (one mask per block: every pk occurs once), a wider one radix-sorted with
 * passes sized by the range — no read-back either way.  Stable, asynchronous. */
int kd_delta_pk_order(kd_ctx* ctx, const kd_side* base, const kd_side* target, const uint32_t* d_delta,
                      const uint64_t* d_keys, uint64_t cap, const uint64_t* d_n, int64_t pk_lo, int64_t pk_hi,
                      int64_t* d_pk, uint32_t* d_perm);

/* -------- device memory and copies (no GPU framework needed by the caller) -------- */
#define KD_COPY_H2D 1u
#define KD_COPY_D2H 2u
#define KD_COPY_D2D 3u
int kd_malloc(kd_ctx* ctx, uint64_t bytes, void** dptr);   /* HBM of the context's device      */
int kd_mfree(kd_ctx* ctx, void* dptr);
int kd_host_alloc(uint64_t bytes, void** hptr);            /* pinned (page-locked) host memory */
int kd_host_free(void* hptr);
/* asynchronous on the context stream (host buffers should be pinned for a true async copy) */
int kd_memcpy(kd_ctx* ctx, void* dst, const void* src, uint64_t bytes, uint32_t kind);
int kd_memset(kd_ctx* ctx, void* dst, int value, uint64_t bytes);
int kd_device_sync(kd_ctx* ctx);                           /* hipDeviceSynchronize + profiling */

/* -------- multi-GPU: bucket-range shards, RCCL all-gather -------- */
#define KD_COMM_ID_BYTES 128
/* One process per GPU: rank 0 makes the id, the caller broadcasts it (any channel), every rank
 * calls kd_comm_init with it.  The library owns the communicator (RCCL, loaded at first use). */
int kd_comm_unique_id(uint8_t id[KD_COMM_ID_BYTES]);
int kd_comm_init(kd_ctx* ctx, int nranks, int rank, const uint8_t id[KD_COMM_ID_BYTES]);
int kd_comm_fini(kd_ctx* ctx);
/* the communicator's own view, from RCCL: out[0] = ncclCommCount (ranks that joined), out[1] =
 * ncclCommUserRank, out[2] = ncclCommCuDevice (the HIP device it drives) */
int kd_comm_info(kd_ctx* ctx, int32_t out[3]);
/* d_recv[nranks * n] <- every rank's d_send[n] (device buffers, context stream) */
int kd_allgather_u64(kd_ctx* ctx, const uint64_t* d_send, uint64_t* d_recv, uint64_t n);
/* One rank's step of a sharded diff: kd_diff2_device on this rank's shard (device sides holding
 * the global sorted entries [base_off, base_off + base.n) / [target_off, ...) of one bucket range),
 * its delta records rebased to global indices, then all-gathered with the counts:
 *   d_all_counts / h_all_counts [nranks * 8]: rank r's inserts, updates, deletes, deltas, error word;
 *   d_all_delta [all_cap * 2]: rank r's records at 2 * r * stride, stride = max_r deltas(r).
 * Ranks hold consecutive bucket ranges, so the gathered records in rank order are key-ordered.
 * One host sync (the record stride).  d_upd may be NULL. */
int kd_diff2_gather(kd_ctx* ctx, const kd_side* base, const kd_side* target, uint64_t base_off,
                    uint64_t target_off, uint32_t flags, uint32_t* d_delta, uint32_t* d_upd,
                    uint64_t* d_counts, uint32_t* d_err, uint32_t* d_all_delta, uint64_t all_cap,
                    uint64_t* d_all_counts, uint64_t* h_all_counts);
/* kd_diff2_gather in two halves, so the caller can queue work between them (the shard's
 * kd_fielddiff): _begin queues the join, the rebase and the counts' all-gather (no host wait);
 * _end waits for the counts, queues the records' all-gather on the context's communication
 * stream (overlapping the work queued in between) and makes the context stream wait for it.
 * kd_diff2_gather = _begin + _end. */
int kd_diff2_gather_begin(kd_ctx* ctx, const kd_side* base, const kd_side* target, uint64_t base_off,
                          uint64_t target_off, uint32_t flags, uint32_t* d_delta, uint32_t* d_upd,
                          uint64_t* d_counts, uint32_t* d_err, uint64_t* d_all_counts);
int kd_diff2_gather_end(kd_ctx* ctx, const uint32_t* d_delta, uint32_t* d_all_delta, uint64_t all_cap,
                        uint64_t* h_all_counts);
/* One process driving g GPUs (one context each): host sides are cut into g bucket ranges of about
 * equal entry count (bucket = the key's top bucket_bits bits: 24 for KD_KEY_INT, 6 per tree level
 * for base64 hash paths, 8 per level for hex), each shard diffed on its GPU, and the records
 * all-gathered over a communicator the library keeps on ctxs[0].  Result as kd_diff2. */
int kd_diff2_sharded(kd_ctx** ctxs, int g, const kd_side* base, const kd_side* target, int bucket_bits,
                     uint32_t flags, kd_diff_result** out);
/* The cut kd_diff2_sharded uses (host only, no GPU): cut [g+1] bucket edges, shard s = buckets
 * [cut[s], cut[s+1]), each cut the smallest bucket with at least total*s/g entries of both sorted
 * key arrays before it; a_lo / b_lo [g+1] the matching entry ranges of each side. */
int kd_shard_cuts(const uint64_t* key_a, uint64_t n_a, const uint64_t* key_b, uint64_t n_b, int g, int bucket_bits,
                  uint64_t* cut, uint64_t* a_lo, uint64_t* b_lo);

/* -------- host-side key packing (CPU, multithreaded) -------- */
/* KD_KEY_INT: filenames b64(msgpack([pk])) -> keys (entries may be whole relative paths
 * "c/c/c/c/<filename>": the part after the last '/' is decoded).  status[i] = 0 ok / 1 not an int
 * pk / 2 pk outside [-2^63, 2^63).  Returns number of bad entries. */
int64_t kd_pack_int_keys(const uint8_t* names, const uint64_t* name_off, uint64_t n,
                         uint64_t* keys, uint8_t* status);
/* KD_KEY_HASH: "c1/../cL/<filename>" relative paths -> keys (levels, hex=0 base64 / 1 hex). */
int64_t kd_pack_hash_keys(const uint8_t* paths, const uint64_t* path_off, uint64_t n, int levels,
                          int hex, uint64_t* keys, uint8_t* status);
/* Inverse of the KD_KEY_INT key: pk = ((wrap - 2^33) * 2^24 + bucket) * 64 + low6, bucket and low6
 * through the inverse rank maps. */
int kd_int_keys_to_pks(const uint64_t* keys, uint64_t n, int64_t* pks);

/* -------- git object database + leaf walk (host, no GPU) -------- */
/* Replaces libgit2's ODB and tree iteration under Dataset3 (kart/dataset3.py:26-35,225-231,
 * kart/base_dataset.py:230-265) and the subtree pruning of Tree.diff_to_tree
 * (kart/rich_base_dataset.py:212-232).  Loose objects, pack v2 (idx v1/v2), zlib, OFS/REF delta
 * chains, objects/info/alternates.  The pack set is read at open: reopen to see new packs. */
#define KD_ENOTFOUND (-4) /* object not in the odb (missing, or promised by a partial clone) */
typedef struct kd_odb kd_odb;
int kd_odb_open(const char* gitdir, kd_odb** out);
/* Options of an object store (A/B switches; kd_odb_open seeds each from the environment variable in
 * brackets).  Unknown names: KD_EINVAL.
 *   zlib           [KD_ODB_ZLIB]       1: inflate with zlib even when libdeflate.so.0 is present */
int kd_odb_set_option(kd_odb* odb, const char* name, int64_t value);
int kd_odb_get_option(kd_odb* odb, const char* name, int64_t* value);
int kd_odb_close(kd_odb* odb);
/* One object (*type 1 commit, 2 tree, 3 blob, 4 tag); *data malloc'd (kd_free). */
int kd_odb_read(kd_odb* odb, const uint8_t oid[20], int* type, uint8_t** data, uint64_t* len);
/* n blobs into one arena *data (kd_free): blob i = (*data)[off[i] .. off[i+1]) (off [n+1]);
 * status[i] 0 ok, 1 missing (empty), 2 corrupt / not a blob (empty).  threads 0 = up to 16. */
int kd_odb_read_batch(kd_odb* odb, const uint8_t* oids, uint64_t n, int threads, uint8_t** data,
                      uint64_t* off, uint8_t* status);
/* A walk's leaves for one root, one block (kd_free): leaf i = path[path_off[i] .. path_off[i+1])
 * relative to the walked tree, '/'-separated, in git path order (what `git ls-tree -r` lists). */
typedef struct kd_leaves {
    uint64_t n;
    uint64_t* path_off; /* [n+1] */
    uint32_t* mode;     /* [n] git file modes (0100644, 0100755, 0120000, 0160000)  */
    uint8_t* oid;       /* [n*20] */
    uint8_t* path;
    int32_t present;    /* 0: the walked tree does not exist in this root */
} kd_leaves;
#define KD_WALK_ALL (-1)
/* Walk the tree at `subpath` ("" or NULL = the root) of k roots (commit, tag or tree OIDs, 20 raw
 * bytes each, k <= 3) into out[0..k).  cmp0/cmp1 (root indices) prune: an entry (subtree or leaf)
 * identical in roots cmp0 and cmp1 — same mode and OID, or absent from both — is skipped in every
 * root and a pruned subtree is never read.  KD_WALK_ALL (both) lists everything.  The first levels
 * are expanded breadth-first, then subtrees are walked depth-first by `threads` (0 = up to 16). */
int kd_walk(kd_odb* odb, const uint8_t* roots, int k, const char* subpath, int cmp0, int cmp1,
            int threads, kd_leaves** out);

/* -------- profiling (hipEvents around every launch on the context stream) -------- */
int kd_prof_enable(kd_ctx* ctx, int on);
/* Time only the named kernels ("k_join2,k_fielddiff"; NULL or "" = every kernel): each timed
 * launch adds two events to the stream, so a bench times just the kernels it reports. */
int kd_prof_select(kd_ctx* ctx, const char* names);
/* name = kernel name; returns launches and summed milliseconds since the last reset. */
int kd_prof_get(kd_ctx* ctx, const char* name, uint64_t* launches, double* total_ms);
int kd_prof_reset(kd_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* KARTDIFF_H */
