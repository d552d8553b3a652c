#!/usr/bin/env python3
"""Bench: device-resident bulk feature diff on MI355X (one JSON line on rank 0).

Default workload (BASELINE.json configs[2], "C3", the north-star config): ONE synthetic
100M-MULTIPOLYGON int-PK layer, 10 % edits (4 % geometry + 4 % attribute updates, 1 % deletes, 1 %
inserts; kart_amd.synth.polygons_layer: the reference's feature blob and path encodings, synthetic
OIDs), both sides as the tree walk lists them (git tree order, which is KD_KEY_INT key order: no side
sort).  One *step* = one full pass of the hot path over that layer: merge-path join + OID compare +
walk-ordered compaction of the delta set (k_partition2, k_join2, k_place2), the msgpack field decode +
Python-== column compare of every update (k_fielddiff), then the delta and update records radix-sorted
into pk order (kd_delta_pk_order: DeltaDiff.sorted_items) — all on the device, inputs resident in HBM
before the timed region.

--gpus N (one process per GPU, launched by torch.distributed.run): the SAME layer split into N
bucket ranges (whole leaf trees, contiguous runs of the walk: synth.shard_rank_range); each rank generates and diffs its
range, and every step all-gathers the per-rank counts and the compacted delta records (rebased to
global indices) over RCCL inside libkartdiff (kd_diff2_gather) — strong scaling.  The harness
(barrier, max-over-ranks time, the RCCL id broadcast) uses torch.distributed's gloo backend on the
CPU; no device memory, stream or collective of the measured path goes through torch, and at N=1
torch is not imported at all.

--workload c2 (configs[1]): a 10M-point layer per GPU, 1 % upd/del/ins (weak scaling at N>1);
c4 (configs[3]): 50M-row string-PK three-way merge classification; c5 (configs[4]): the spatially
filtered diff of a 100M-feature layer on SURVEY §8(d)'s mix (classify2 + the deltas' geometry heads
gathered into delta order + per-delta envelope filter + EnvelopeEncoder + the blob fallback); c5env: the envelope kernels alone over a raw geometry arena; c6:
hex WKB of every geometry.

Timing: W untimed warmup steps (their results checked), then — after a burst of untimed steps worth
BENCH_PREWARM_S = 0.1 s (the count from one timed step, the slowest rank's, so every rank runs the
same steps), so the clocks are up after the host's checks — a barrier + device sync, exactly K timed
steps, device sync + barrier; the max over ranks.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5|c5env|c6] [--n UNITS]
                       [--no-cpu-baseline] [--no-host-timing]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "feature deltas classified+field-diffed/sec (M/s) at 1/2/4/8 GPUs; % HBM peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# the reference's own hot path (kart's Python diff_feature + get_feature/== loop, git
# diff-tree for libgit2) measured on 1 core in the build container on a 1M-feature 1 % layer
REFERENCE_CPU_PATH = {"value": 0.54, "unit": "M feature-pairs/s", "cores": 1, "kind": "reference",
                      "sample": "BASELINE.md: reference kart diff hot path (Python + git diff-tree), synthetic 1M "
                                "points, 1 % U/I/D, build container (the reference cannot run on the GPU box)"}
# the same reference path measured on C3's own edit mix (8 % updates, 1 % deletes, 1 % inserts of a 3M
# polygon layer): profiles/r05/ref_path_3m.json (scripts/ref_path_bench.py, build container, 1 core)
REFERENCE_CPU_PATH_C3 = {"value": 0.097, "unit": "M feature-pairs/s", "cores": 1, "kind": "reference",
                         "mix": "C3's mix: 8 % updates / 1 % deletes / 1 % inserts, 3M-polygon layer",
                         "file": "profiles/r05/ref_path_3m.json",
                         "sample": "the reference's Dataset3.diff + get_feature of both sides of every update + the "
                                   "Python == field compare, 1 thread; libgit2's tree diff by git diff-tree (C)",
                         "differently_mixed": dict(REFERENCE_CPU_PATH, mix="BASELINE.md's points layer at 1 / 1 / 1 % edits")}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=["c2", "c3", "c3v", "c4", "c5", "c5env", "c6"])
    ap.add_argument("--same-len", type=float, default=0.6,
                    help="c3v: fraction of features whose geometry edits keep the blob length (vertex moves)")
    ap.add_argument("--n", type=int, default=0,
                    help="units (c3: polygons of the whole layer, 100M; c2: points per GPU, 10M; c4: rows, 50M; "
                         "c5: features of the filtered layer, 100M; c5env/c6: geometries, 20M)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-timing", action="store_true", help="skip the host pack / H2D timings")
    ap.add_argument("--unordered", action="store_true",
                    help="c2/c3: tile-grouped delta list (per-tile atomic appends, no k_place2); default: key order")
    ap.add_argument("--sort-gather", action="store_true",
                    help="fallback steps: permute the OIDs in the sort (k_gather_oid) instead of reading them "
                         "through the order in the join")
    ap.add_argument("--no-sort", action="store_true",
                    help="c2/c3: skip timing the fallback steps (sides in a non-key order: both GPU side sorts in "
                         "the step); c4: skip the presorted comparison")
    ap.add_argument("--no-radix", action="store_true", help="c2/c3: skip timing the radix-sort fallback beside the "
                                                             "per-leaf-tree one")
    ap.add_argument("--no-pk-order", action="store_true",
                    help="c2/c3: leave the deltas in walk (key) order (no kd_delta_pk_order in the step)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--arena", action="store_true",
                    help="c5: filter from the blob arenas (kd_geom_filter) instead of the geometry heads")
    ap.add_argument("--per-entry", action="store_true",
                    help="c5: the heads kernel straight on the per-entry heads (pair-indexed k_gf_heads)")
    ap.add_argument("--gh-gather", action="store_true",
                    help="c5: gather the per-entry heads into delta order on the device inside every step "
                         "(k_gh_gather) instead of the blob reader's delta-order heads")
    ap.add_argument("--c3-layer", action="store_true",
                    help="c5: the C3 polygon layer instead of SURVEY's C5 mix (points, straddles, wide, EMPTY, edge)")
    ap.add_argument("--no-arena-timing", action="store_true", help="c5: skip timing the arena path beside the heads")
    ap.add_argument("--pair-arenas", action="store_true",
                    help="c2/c3: field-diff from the per-entry arenas through the join's update pairs instead of "
                         "update-order arenas (the drop-in's form: the blob reader writes update i's blobs at index i)")
    ap.add_argument("--traffic-json", default=None, help="measured HBM bytes per launch (the newest profiles/<round>/traffic_<wl>.json)")
    ap.add_argument("--no-heads-path", action="store_true", help="c5env: skip the indexer's heads-path timing")
    ap.add_argument("--no-check", action="store_true", help="profiling variants only: skip the correctness check")
    ap.add_argument("--no-events", action="store_true", help="no per-kernel HIP events in the timed region")
    ap.add_argument("--time-all", action="store_true",
                    help="HIP events around every kernel of a step (default: only the dominant kernel, "
                         "so the events do not inflate the step time)")
    a = ap.parse_args()
    if not a.n:
        a.n = {"c2": 10_000_000, "c3": 100_000_000, "c3v": 100_000_000, "c4": 50_000_000, "c5": 100_000_000, "c5env": 20_000_000,
               "c6": 20_000_000}[a.workload]
    if a.traffic_json is None:
        for d in PROFILE_ROUNDS + ("",):  # the newest PMC passes of the workload
            a.traffic_json = os.path.join(ROOT, "profiles", d, f"traffic_{a.workload}.json")
            if os.path.exists(a.traffic_json):
                break
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cores():
    try:
        c = len(os.sched_getaffinity(0))
    except AttributeError:
        c = os.cpu_count() or 1
    return max(1, min(c, 16))  # the GPU box's CPU share is 16 cores (nproc shows the whole host)


class Harness:
    """rank / world from the launcher's env; barrier, max and object exchange over gloo (CPU) when
    world > 1.  Nothing of the measured path goes through it."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.comm = None  # set by engine_for
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return x
        out = [None] * self.world
        self.dist.all_gather_object(out, float(x))
        return max(out)

    def allgather(self, obj):
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def bcast(self, obj):
        if not self.dist:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def engine_for(H):
    from kart_amd.engine import Engine

    eng = Engine(H.local)
    if H.world > 1:  # the library's own RCCL communicator; the id travels over the harness
        uid = H.bcast(Engine.comm_unique_id() if H.rank == 0 else None)
        eng.comm_init(H.world, H.rank, uid)
        # the communicator's own count (ncclCommCount) and every rank's (rank, device) as RCCL sees
        # them: the JSON line shows that N ranks joined one communicator
        info = eng.comm_info()
        views = H.allgather((info["count"], info["rank"], info["device"]))
        H.comm = {"backend": "rccl", "ncclCommCount": info["count"],
                  "ranks": [v[1] for v in views], "devices": [v[2] for v in views],
                  "all_ranks_agree": all(v[0] == H.world for v in views)}
    else:
        H.comm = {"backend": None, "ncclCommCount": None, "ranks": [0]}
    return eng


# The warmup ends with untimed steps for at least this long directly before the timed bracket: the
# GPU clocks down while the host checks the warmup's results, and the first ~20 ms after an idle
# spell run slow (r4pw: C5-envelopes 1.51 -> 0.73 ms per step over 20 steps, C3 3.46 -> 3.41)
PREWARM_S = float(os.environ.get("BENCH_PREWARM_S", "0.1"))


def timed(H, eng, step, steps):
    """barrier + device sync, K steps, device sync + barrier; the max-over-ranks seconds"""
    if PREWARM_S > 0:
        # untimed steps right before the bracket for at least PREWARM_S seconds.  A step may hold
        # collectives (the gathered records at N > 1), so every rank runs the same count: one step
        # timed on each rank, the count from the slowest
        H.barrier()
        t0 = time.perf_counter()
        step()
        eng.sync()
        one = H.max(time.perf_counter() - t0)
        for _ in range(min(10_000, int(PREWARM_S / max(one, 1e-6)))):
            step()
        eng.sync()
    H.barrier()
    eng.device_sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    eng.device_sync()
    H.barrier()
    return H.max(time.perf_counter() - t0)


PROFILE_ROUNDS = ("r06", "r05", "r04")  # committed profiles, newest first


def rocprof_stats_path(workload):
    """the newest committed `rocprofv3 --kernel-trace --stats` summary of the workload"""
    for d in PROFILE_ROUNDS:
        path = os.path.join(ROOT, "profiles", d, f"{workload}_kernel_stats.csv")
        if os.path.exists(path):
            return path
    return None


# the HIP-event name a role is timed under -> the kernel symbols rocprof lists for it
# (kd_geom_filter_deltas times k_gf_dense, the dense-heads form, under "k_gf_heads")
# (kd_merge3_device times k_join3b, the one-batch join, under "k_join3")
KERNEL_SYMBOLS = {"k_gf_heads": ("k_gf_dense", "k_gf_heads"), "k_join3": ("k_join3b", "k_join3")}


def rocprof_avg_ms(workload, kernel):
    """the kernel's average duration in the committed `rocprofv3 --kernel-trace --stats` summary of
    this workload (the newest of PROFILE_ROUNDS), or None"""
    path = rocprof_stats_path(workload)
    if path is None:
        return None
    names = KERNEL_SYMBOLS.get(kernel, (kernel,))
    try:
        import csv

        with open(path) as f:
            rows = {r["Name"].split("(")[0].split("<")[0]: r for r in csv.DictReader(f)}
        for name in names:
            if name in rows:
                return float(rows[name]["AverageNs"]) / 1e6, os.path.relpath(path, ROOT)
    except (OSError, KeyError, ValueError):
        pass
    return None


def roofline(kern, dom, alg_bytes, traffic_json, n_units, workload=None):
    """roofline object of the dominant kernel: algorithmic bytes per launch / its average launch time
    (HIP events on the launch stream); next to it the same from the committed rocprofv3 summary of
    the workload (the rocprof duration is the conservative one: quote both)"""
    if dom not in kern:
        return None
    achieved = alg_bytes / (kern[dom][1] * 1e-3) / 1e9
    traffic = None
    try:
        with open(traffic_json) as f:
            tj = json.load(f)
        if tj.get("kernel") in KERNEL_SYMBOLS.get(dom, (dom,)) and int(tj.get("n_units", tj.get("n_points", -1))) == n_units:
            traffic = tj.get("hbm_bytes_per_launch")
    except (OSError, ValueError, TypeError):
        pass
    out = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "algorithmic_bytes_per_launch": int(alg_bytes),
           "avg_launch_ms": round(kern[dom][1], 5)}
    rp = rocprof_avg_ms(workload, dom) if workload else None
    if rp:
        ms, path = rp
        out["rocprof"] = {"avg_launch_ms": round(ms, 5), "frac": round(alg_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "stats": path}
    return out


def kernel_times(eng, names):
    kern = {}
    for name in names:
        launches, ms = eng.prof_get(name)
        if launches:
            kern[name] = (launches, ms / launches)
    return kern


def oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle as O

    return O


# ---------------------------------------------------------------------------------------------
# c2 / c3: two-way diff + field diff
def run_diff(args, H, polygons):
    from kart_amd import shard, synth
    from kart_amd.device import DiffPipeline
    from kart_amd.schema import FieldMaps

    n, world, rank = args.n, H.world, H.rank
    split = polygons and world > 1  # C3: one layer split by bucket range (strong scaling)
    t0 = time.time()
    if polygons:
        L = synth.polygons_layer(n, shard=(rank, world) if split else None,
                                 same_len=args.same_len if args.workload == "c3v" else 0.0)
    else:
        L = synth.points_layer(n, seed=synth.SEED + rank, pk0=shard.rank_pk_base(rank, n))
    gen_s = time.time() - t0
    log(f"[rank {rank}] generated {L.base.n}+{L.target.n} entries in {gen_s:.1f}s "
        f"(+{L.n_insert} ins, {L.n_update} upd, -{L.n_delete} del)")
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    eng = engine_for(H)
    gather = None
    if split:  # global walk index of this shard's first entry on each side
        sizes = H.allgather((L.base.n, L.target.n))
        gather = (sum(s[0] for s in sizes[:rank]), sum(s[1] for s in sizes[:rank]))
    t0 = time.perf_counter()
    pipe = DiffPipeline(eng, L.base, L.target, L.base_blobs, L.target_blobs, maps, ordered=not args.unordered,
                        gather=gather, pk_order=not args.no_pk_order)
    h2d_s = time.perf_counter() - t0
    h2d_bytes = 28 * (L.base.n + L.target.n) + int(L.base_blobs[0].size + L.target_blobs[0].size) + \
        8 * int(L.base_blobs[1].size + L.target_blobs[1].size)

    # ---- warmup + correctness of the resident pipeline against the generator's own counts ----
    for _ in range(max(1, args.warmup)):
        pipe.step()
    eng.sync()
    counts, delta, upd, masks, status = pipe.results()
    if not args.pair_arenas:  # the drop-in's arena form: update-order blobs, no pairs (same bytes)
        pipe.use_update_arenas(upd)
        pipe.step()
        eng.sync()
        counts, delta, upd2, masks, status = pipe.results()
        assert np.array_equal(upd2, upd)
    plan = (L.n_insert, L.n_update, L.n_delete)
    if not args.no_check:
        assert (counts["inserts"], counts["updates"], counts["deletes"]) == plan, (counts, plan)
        assert not status.any(), "fielddiff status flags set"
        if pipe.pk_order:  # the pk-ordered records: a stable argsort of the records' pks
            check_pk_order(pipe, L, delta, upd)
    if split:
        mx = max(x for x in H.allgather(counts["deltas"]))
        pipe.reserve_gather(mx)
        pipe.step()
        eng.sync()
        g_counts, g_delta = pipe.gathered()
        tot = [sum(x) for x in zip(*H.allgather(plan))]
        if not args.no_check:  # every rank holds the whole diff: counts of all ranks, global key order
            assert (g_counts["inserts"], g_counts["updates"], g_counts["deletes"]) == tuple(tot), (g_counts, tot)
            assert g_delta.shape[0] == g_counts["deltas"]
    n_pairs = L.base.n + L.n_insert

    eng.prof_reset()
    eng.prof_select(None if args.time_all else ["k_fielddiff" if polygons else "k_join2"])
    eng.prof_enable(not args.no_events)
    elapsed = timed(H, eng, pipe.step, args.steps)  # walk-order device-resident sides: the whole step
    eng.prof_enable(False)
    total_pairs = sum(H.allgather(n_pairs))
    total_deltas = sum(H.allgather(counts["deltas"]))
    kern = kernel_times(eng, ("k_partition2", "k_join2", "k_place2", "k_fielddiff", "k_rebase"))
    # every kernel of the step once more with events around each launch (untimed steps): the parts
    eng.prof_reset()
    eng.prof_select(None)
    eng.prof_enable(True)
    for _ in range(3):
        pipe.step()
    eng.sync()
    eng.prof_enable(False)
    parts = kernel_times(eng, STEP_KERNELS)
    pk_sort = pk_sort_summary(pipe, parts, counts) if pipe.pk_order else None
    sort = None
    if not args.no_sort and not split:  # the fallback: sides in a non-key order, both GPU side sorts in the step
        del pipe
        sort = fallback_sort(args, H, eng, L, maps, elapsed, total_pairs)
    # ---- roofline of the dominant kernel (algorithmic bytes per launch) ----
    nA, nB = L.base.n, L.target.n
    ob_off, nb_off = L.base_blobs[1], L.target_blobs[1]
    ok_u = (upd[:, 0] < nA) & (upd[:, 1] < nB)  # (profiling variants with --no-check may emit junk)
    u0, u1 = upd[ok_u, 0], upd[ok_u, 1]
    upd_bytes = int((ob_off[u0 + 1] - ob_off[u0]).sum() + (nb_off[u1 + 1] - nb_off[u1]).sum())
    alg = {
        "k_join2": 28 * (nA + nB) + 8 * counts["deltas"] + 8 * counts["updates"],
        "k_fielddiff": upd_bytes + counts["updates"] * (8 + 8 * maps.words + 1),
    }
    dom = max((k for k in kern if k in alg), key=lambda k: kern[k][1]) if kern else None
    # (the committed traffic files are 1-GPU profiles of the whole layer: not a shard's bytes)
    # (the committed traffic and rocprof files profile the default update-order arenas)
    roof = roofline(kern, dom, alg.get(dom, 0), "" if args.pair_arenas else args.traffic_json, n if world == 1 else -1,
                    args.workload if world == 1 and not args.pair_arenas else None) if dom else None
    cpu = host = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_diff(L, maps, args.cpu_seconds, "C3" if polygons else "C2")
    if rank == 0 and world == 1 and not args.no_host_timing:
        host = host_timing(eng, L, h2d_s, h2d_bytes)
    eng.close()
    wl = (f"C3: ONE {n}-polygon int-PK layer{f' split into {world} bucket-range shards' if split else ''}, 10% edits "
          "(4% geometry + 4% attribute updates, 1% del, 1% ins), two-commit diff + field diff" +
          (f"; geometry edits keep the blob length for {args.same_len:.0%} of features (vertex moves)"
           if args.workload == "c3v" else "")) if polygons else \
        f"C2: {n}-point int-PK layer per GPU, 1% upd/del/ins, two-commit diff + field diff"
    out = {
        "metric": METRIC,
        "value": round(total_pairs * args.steps / elapsed / 1e6, 2),
        "unit": "M feature-pairs/s",
        "n_gpus": world, "rccl_comm": H.comm,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if polygons else "weak",
        "vs_baseline": None,
        "dtype": "u8/u64 (integer + fp64 compare)",
        "data": ("synthetic (seeded MULTIPOLYGON layer: reference blob/path encodings, synthetic OIDs; "
                 "blobs materialised for updated features only)") if polygons else
                "synthetic (seeded points layer: reference blob/path encodings, synthetic OIDs)",
        "config": {"workload": wl, "features": n if polygons else n * world, "pairs_per_step": total_pairs,
                   "deltas_per_step": total_deltas, "updates_per_step": sum(H.allgather(counts["updates"])),
                   "delta_order": "tile-grouped (same delta set)" if args.unordered else
                   ("walk (= key) order, then pk order (kd_delta_pk_order)" if pk_sort else "walk (= key) order"),
                   "side_order": "git tree (walk) order as listed, no side sort",
                   "blob_arenas": ("per-entry arenas read through the join's update pairs" if args.pair_arenas else
                                   "update-order arenas (the drop-in's form: update i's blobs at index i; the field "
                                   "diff reads the join's device update count)"),
                   "parallelism": f"bucket-range shards x{world}" + (", RCCL all-gather of counts + delta records"
                                                                      if split else "")},
        "kernels_avg_ms": {k: round(v[1], 5) for k, v in kern.items()},
        "step_kernels_avg_ms": {k: round(v[1], 5) for k, v in parts.items()},
        "step_kernel_launches": {k: v[0] // 3 for k, v in parts.items()},
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    if pk_sort:
        out["pk_order"] = pk_sort
    if sort:
        out["fallback_sort"] = sort
    if host:
        out["host"] = host
    return out


SORT_KERNELS = ("k_rs_bits", "k_sort_hist", "k_sort_scan", "k_sort_pass", "k_gather_oid")
C4_KERNELS = ("k_seg_sort", "k_sorted3", "k_partition2", "k_apart3", "k_join2", "k_join3", "k_gscan2", "k_place2",
              "k_place3", "k_resolve3")
STEP_KERNELS = ("k_partition2", "k_join2", "k_gscan2", "k_place2", "k_fielddiff", "k_dpk_keys", "k_sort_scan",
                "k_sort_pass", "k_pkm_mark", "k_pkm_scan", "k_pkm_cscan", "k_pkm_place")
PKM_MAX_BLOCKS = 1 << 26  # kd_delta_pk_order's bitmap path: pk ranges of at most this many 64-pk blocks
RS_RB = 9  # digit bits per radix pass (kd_sort.hip RS_RB): passes = ceil(varying bits / 9)


def radix_passes(bits):
    return -(-int(bits) // RS_RB) if bits else 0


def check_pk_order(pipe, L, delta, upd):
    from kart_amd import walkkey

    d_pk, d_perm, u_pk, u_perm = pipe.pk_results()
    for rec, pk_out, perm_out in ((delta, d_pk, d_perm), (upd, u_pk, u_perm)):
        keys = np.where(rec[:, 0] != 0xFFFFFFFF, L.base.key[np.minimum(rec[:, 0], L.base.n - 1)],
                        L.target.key[np.minimum(rec[:, 1], L.target.n - 1)])
        pks = walkkey.int_keys_to_pks(keys)
        want = np.argsort(pks, kind="stable")
        assert np.array_equal(perm_out, want.astype(np.uint32)), "pk order differs from a stable argsort"
        assert np.array_equal(pk_out, pks[want]), "pk-ordered pks differ"


def pk_sort_summary(pipe, parts, counts):
    """the deltas' and updates' pk order (kd_delta_pk_order, two calls per step).  A bounded pk range
    takes the bitmap placement (one 64-bit mask per 64-pk block; every pk occurs once per list):
    algorithmic bytes per record = the record (8 B) + its key (8 B) read, the pk (8 B) + the record
    index (4 B) written; per block its mask written and read (16 B) and its in-chunk prefix (8 B).
    Otherwise the radix path: the library's own pass count (the pk range's varying bits, 9-bit digits)."""
    lo, hi = pipe.pk_range
    nb = (hi >> 6) - (lo >> 6) + 1
    recs = counts["deltas"] + counts["updates"]
    if nb <= PKM_MAX_BLOCKS:
        kk = ("k_pkm_mark", "k_pkm_scan", "k_pkm_cscan", "k_pkm_place")
        alg = 28 * recs + 2 * 24 * nb
        how = {"path": "bitmap", "blocks": nb}
    else:
        d = (lo ^ (1 << 63)) ^ (hi ^ (1 << 63)) if hi != lo else 0
        bits = d.bit_length()
        npass = max(1, radix_passes(bits))
        ck = 4 if bits <= 32 else 8
        per_rec = 8 + 8 + ck + sum((ck if p == 0 else ck + 4) + (12 if p == npass - 1 else ck + 4) for p in range(npass))
        kk = ("k_dpk_keys", "k_sort_scan", "k_sort_pass")
        alg = per_rec * recs
        how = {"path": "radix", "varying_bits": bits, "passes_per_sort": npass}
    ms = sum(parts[k][0] * parts[k][1] for k in kk if k in parts) / 3
    return {"what": "deltas and updates put in pk order on the device (kd_delta_pk_order x2), the order "
                    "DeltaDiff.sorted_items yields", "records_per_step": recs, **how,
            "ms_per_step_events": round(ms, 4),
            "roofline": {"bound": "hbm", "algorithmic_bytes_per_step": int(alg),
                         "achieved": round(alg / (ms * 1e-3) / 1e9, 1) if ms else None, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if ms else None}}


def sort_bytes(info, n, gather_oids):
    """algorithmic HBM bytes of kd_sort_side_into over one side, with the pass count the
    library derives from the same kd_keys_scan (9-bit digits): the all-pass histogram (8 B read per
    key), the digit passes (first: 8-B key read, compact key + 4-B index written; middle: compact key
    + index read and written; last: compact key + index read, 8-B key + 4-B order written), and the OID
    gather (4-B order + 20-B row read, 20 B written) unless the join reads the OIDs through the order
    (late materialisation).  No varying-bit pass: the host scan sized the sort.  Returns (bytes, passes)."""
    if n < 2:
        return 0, 0
    bits = bin(int(info.vary)).count("1")  # compact width (gaps absorbed only beyond 4 runs: not for int keys)
    npass = radix_passes(bits)
    ck = 4 if bits <= 32 else 8
    b = 8 * n  # histogram
    for p in range(npass):
        rd = 8 if p == 0 else ck + 4
        wr = 12 if p == npass - 1 else ck + 4
        b += (rd + wr) * n
    if gather_oids:
        b += 44 * n
    return b, npass


def fallback_sort(args, H, eng, L, maps, elapsed, total_pairs, radix=False):
    """The fallback the drop-in takes for a side whose walk order is not key order (leaf trees mixing
    2**30 pk wraps): the same step from sides whose rows are shuffled inside every leaf tree, both GPU
    side sorts inside it — per leaf tree (kd_sort_segmented_into: the walk lists each leaf tree's
    entries together, so only they are out of order; planned from the host's kd_keys_scan, no
    read-back) or, ``radix`` (a leaf tree longer than 512 entries), the onesweep radix sort of the
    compacted varying key bits — then the join reading OIDs through the sort orders."""
    from kart_amd.device import DiffPipeline

    def leaf_scramble(keys, seed):
        """rows shuffled inside each leaf tree (the entries sharing the key's top 24 bucket bits): what
        a walk of leaf trees mixing pk wraps looks like — key order broken inside leaf trees, kept
        between them"""
        r = np.random.default_rng(seed)
        b = keys >> np.uint64(40)
        return np.lexsort((r.random(keys.shape[0]), b))  # stable by bucket, random inside

    perms = (leaf_scramble(L.base.key, 1), leaf_scramble(L.target.key, 2))
    fp = DiffPipeline(eng, L.base, L.target, L.base_blobs, L.target_blobs, maps, unsorted=perms,
                      late=not args.sort_gather, pk_order=not args.no_pk_order, radix=radix)
    for _ in range(max(1, args.warmup)):
        fp.step()
    eng.sync()
    if not args.no_check:
        fp.results()  # (raises on a device error flag: the join's order checks, the per-leaf-tree sort's)
        for S, side, perm, order in zip((fp.A, fp.B), (L.base, L.target), perms, fp.orders()):
            assert np.array_equal(S.key.download(np.uint64, side.n), side.key), "sorted keys differ"
            assert np.array_equal(perm[order], np.arange(side.n)), "sort order differs"
    eng.prof_reset()
    eng.prof_select(None)
    eng.prof_enable(False)
    el = timed(H, eng, fp.step, args.steps)
    eng.prof_reset()
    eng.prof_enable(True)
    for _ in range(3):
        fp.sort_step()
    eng.sync()
    eng.prof_enable(False)
    sk = kernel_times(eng, SORT_KERNELS + ("k_seg_sort",))
    ms_sorts = sum(v[0] * v[1] for v in sk.values()) / 3
    if fp.segmented:  # per entry: the key read, the key + 4-B order written (the leaf tree's neighbours hit the cache)
        bb, bt = 20 * L.base.n, 20 * L.target.n
        pb = pt = 0
    else:
        (bb, pb), (bt, pt) = [sort_bytes(w[3], w[2], not fp.late) for w in fp.walk]
    eng.prof_reset()
    eng.prof_select(["k_join2"])
    eng.prof_enable(True)
    for _ in range(3):
        fp.step()
    eng.sync()
    eng.prof_enable(False)
    jp = kernel_times(eng, ("k_join2",))
    how = ("per leaf tree (kd_sort_segmented_into: one kernel per side, planned from the host kd_keys_scan's "
           "seg_max)" if fp.segmented else "by the onesweep LSD radix sort of the compacted varying key bits "
           "(kd_sort_side_into, passes sized by the host kd_keys_scan)")
    out = {"what": "the drop-in's fallback for sides whose walk order is not key order: each step sorts both "
                   "sides (rows shuffled inside every leaf tree, as a walk of leaf trees mixing pk wraps) on the GPU "
                   + how + ", then classify2 + field diff + pk order; " +
                   ("the join reads the OIDs through the sort orders (kd_diff2_device_perm)" if fp.late else
                    "the OIDs are gathered into key order by the sort"),
           "value": round(total_pairs * args.steps / el / 1e6, 2), "ms_per_step": round(el / args.steps * 1e3, 4),
           "sort_ms_per_step_wall": round((el - elapsed) / args.steps * 1e3, 4),
           "passes": [pb, pt], "kernels_avg_ms": {k: round(v[1], 5) for k, v in sk.items()},
           "kernel_launches_per_step": {k: v[0] // 3 for k, v in sk.items()},
           "sort_ms_per_step_events": round(ms_sorts, 4),
           "k_join2_perm_avg_ms": round(jp["k_join2"][1], 5) if "k_join2" in jp else None,
           "roofline": {"bound": "hbm", "algorithmic_bytes_per_step": int(bb + bt),
                        "achieved": round((bb + bt) / (ms_sorts * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round((bb + bt) / (ms_sorts * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}
    assert out["kernel_launches_per_step"].get("k_sort_pass", 0) == pb + pt, "pass accounting differs from launches"
    if fp.segmented:
        assert out["kernel_launches_per_step"].get("k_seg_sort", 0) == 2, "one per-leaf-tree sort per side"
    del fp
    if not radix and not args.no_radix:  # the radix path beside it (a leaf tree longer than 512 entries)
        out["radix"] = fallback_sort(args, H, eng, L, maps, elapsed, total_pairs, radix=True)
    return out


def _shard_bounds(L, parts):
    from kart_amd import shard

    bits = shard.bucket_bits(L.base.key_mode, L.base.encoding)
    cuts = shard.cut_points([L.base.key, L.target.key], parts, bits)
    return shard.slice_bounds(L.base.key, cuts, bits), shard.slice_bounds(L.target.key, cuts, bits)


def _oracle_shard(O, L, maps, ba, bb, s):
    """oracle classify2 + fielddiff of bucket-range shard s (the C restatement; ctypes drops the GIL)"""
    A, B = L.base, L.target
    a0, a1, b0, b1 = int(ba[s]), int(ba[s + 1]), int(bb[s]), int(bb[s + 1])
    delta, c = O.classify2(A.key[a0:a1], A.oid[a0:a1], B.key[b0:b1], B.oid[b0:b1])
    upd = delta[(delta[:, 0] != O.NONE) & (delta[:, 1] != O.NONE)].astype(np.int64)
    ob, oo = L.base_blobs
    nb, no = L.target_blobs
    O.fielddiff(ob, oo, nb, no, np.stack([upd[:, 0] + a0, upd[:, 1] + b0], 1).astype(np.uint32), maps)
    return (a1 - a0) + c["inserts"]


def cpu_baseline_diff(L, maps, seconds, tag):
    """The C oracle's classify2 + fielddiff (test infrastructure, kd_oracle.c) on the host cores:
    all cores over bucket-range shards of the whole layer, and one thread over one shard."""
    from concurrent.futures import ThreadPoolExecutor

    O = oracle()
    cores = host_cores()
    parts = 4 * cores
    ba, bb = _shard_bounds(L, parts)
    with ThreadPoolExecutor(cores) as ex:
        t0 = time.perf_counter()
        reps = 0
        while True:
            pairs = sum(ex.map(lambda s: _oracle_shard(O, L, maps, ba, bb, s), range(parts)))
            reps += 1
            if time.perf_counter() - t0 >= seconds:
                break
        dt = time.perf_counter() - t0
    allc = pairs * reps / dt / 1e6
    t0 = time.perf_counter()
    reps1 = 0
    while True:
        p1 = _oracle_shard(O, L, maps, ba, bb, 0)
        reps1 += 1
        if time.perf_counter() - t0 >= seconds / 2:
            break
    dt1 = time.perf_counter() - t0
    return {"value": round(allc, 2), "unit": "M feature-pairs/s", "cores": cores, "kind": "port",
            "sample": f"the full {tag} layer ({pairs} pairs) x {reps} reps in {dt:.1f}s: oracle/kd_oracle.c classify2 + "
                      f"fielddiff on {cores} threads over {parts} bucket-range shards",
            "one_thread": {"value": round(p1 * reps1 / dt1 / 1e6, 3), "unit": "M feature-pairs/s", "cores": 1,
                           "sample": f"one shard ({p1} pairs, 1/{parts} of the layer) x {reps1} reps in {dt1:.1f}s"},
            "reference_path": REFERENCE_CPU_PATH_C3 if tag == "C3" else REFERENCE_CPU_PATH}


def cpu_sharded(work, parts, seconds):
    """A CPU baseline on the host cores: ``work(s)`` processes shard s of ``parts`` (the oracle's C
    code, which releases the GIL) and returns its units.  All cores run every shard repeatedly for
    ``seconds``; then shard 0 alone on one thread for ``seconds / 2``.  Returns
    (cores, units per rep, reps, seconds, shard-0 units, its reps, its seconds)."""
    from concurrent.futures import ThreadPoolExecutor

    cores = host_cores()
    with ThreadPoolExecutor(cores) as ex:
        t0 = time.perf_counter()
        reps = 0
        while True:
            units = sum(ex.map(work, range(parts)))
            reps += 1
            if time.perf_counter() - t0 >= seconds:
                break
        dt = time.perf_counter() - t0
    t0 = time.perf_counter()
    reps1 = 0
    while True:
        u1 = work(0)
        reps1 += 1
        if time.perf_counter() - t0 >= seconds / 2:
            break
    return cores, units, reps, dt, u1, reps1, time.perf_counter() - t0


def cpu_line(res, unit, what, tag):
    """the cpu_baseline object of a cpu_sharded result"""
    cores, units, reps, dt, u1, reps1, dt1 = res
    return {"value": round(units * reps / dt / 1e6, 3), "unit": unit, "cores": cores, "kind": "port",
            "sample": f"the full {tag} ({units} units) x {reps} reps in {dt:.1f}s: {what} on {cores} threads",
            "one_thread": {"value": round(u1 * reps1 / dt1 / 1e6, 3), "unit": unit, "cores": 1,
                           "sample": f"one shard ({u1} units) x {reps1} reps in {dt1:.1f}s"}}


def host_timing(eng, L, h2d_s, h2d_bytes):
    """What the drop-in path spends outside the timed device step, for the same layer:
    * pack: the base side's relative leaf paths ('c/c/c/c/<b64(msgpack([pk]))>', in the order the tree
      walk yields them) -> join keys (native, multithreaded) -> kd_keys_scan (already ascending: no
      sort; the pk range for the pk-order passes) -> H2D of keys + OIDs from pinned staging;
    * h2d: uploading both sides + the update blob arenas from pageable numpy arrays (the pipeline
      setup above)."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor

    from kart_amd import _native as N
    from kart_amd import packing, synth
    from kart_amd.device import DevBuf

    n = L.base.n
    pks = packing.int_keys_to_pks(L.base.key)
    chunks = [(a, min(n, a + 4_000_000)) for a in range(0, n, 4_000_000)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(host_cores()) as ex:
        parts = list(ex.map(lambda c: synth.int_pk_paths(pks[c[0]:c[1]]), chunks))
    arena = np.concatenate([p[0] for p in parts])
    off = np.zeros(n + 1, np.uint64)
    pos = 0
    for (a, b), (_, o) in zip(chunks, parts):
        off[a + 1:b + 1] = o[1:] + np.uint64(pos)
        pos += int(o[-1])
    gen_paths_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    keys = packing.parse_keys(arena, off, packing.INT_PK_ENCODING)
    parse_s = time.perf_counter() - t0
    del arena, off
    assert np.array_equal(keys, L.base.key)
    t0 = time.perf_counter()
    info = packing.keys_scan(keys, N.KD_KEY_INT)
    scan_s = time.perf_counter() - t0
    assert info.ascending == 1, "the walk-order side is not key-ordered"
    # pinned staging -> HBM
    nbytes = 28 * n
    hp = ctypes.c_void_p()
    N.check(N.lib().kd_host_alloc(nbytes, ctypes.byref(hp)), "kd_host_alloc")
    try:
        pinned = np.ctypeslib.as_array(ctypes.cast(hp, ctypes.POINTER(ctypes.c_uint8)), (nbytes,))
        pinned[:8 * n] = keys.view(np.uint8)
        pinned[8 * n:] = L.base.oid.reshape(-1)
        dk, do = DevBuf(eng, 8 * n), DevBuf(eng, 20 * n)
        eng.sync()
        t0 = time.perf_counter()
        N.check(eng.L.kd_memcpy(eng.ctx, dk.ptr, hp.value, 8 * n, N.KD_COPY_H2D), "kd_memcpy")
        N.check(eng.L.kd_memcpy(eng.ctx, do.ptr, hp.value + 8 * n, 20 * n, N.KD_COPY_H2D), "kd_memcpy")
        eng.sync()
        pinned_s = time.perf_counter() - t0
    finally:
        N.lib().kd_host_free(hp)
    return {"pack_entries": n, "host_pack_s": round(parse_s, 3), "keys_scan_s": round(scan_s, 4), "gpu_sort_s": 0.0,
            "pack_h2d_pinned_s": round(pinned_s, 4), "pack_h2d_pinned_GBps": round(nbytes / pinned_s / 1e9, 1),
            "h2d_s": round(h2d_s, 3), "h2d_bytes": h2d_bytes, "h2d_GBps": round(h2d_bytes / h2d_s / 1e9, 1),
            "note": f"host_pack_s = native parse of {n} relative leaf paths ('c/c/c/c/<b64 msgpack pk>', in walk "
                    f"order, generated in {gen_paths_s:.1f}s, not counted) into join keys on {host_cores()} threads; "
                    "keys_scan_s = kd_keys_scan (strictly ascending as walked: no sort; vary bits + pk range); then H2D "
                    "of keys + OIDs from pinned memory leaves a device-resident side. h2d_s = the pipeline setup's "
                    "uploads of both sides + update blobs from pageable memory."}


# ---------------------------------------------------------------------------------------------
def run_c5(args, H):
    """C5 (configs[4]): the spatially filtered diff of a 100M-feature layer — the C3 polygon layer,
    one step = classify2 (k_partition2 / k_join2 / k_place2) + kd_geom_filter over its key-ordered
    delta list (each delta's old and new geometry located in its feature blob, GPKG envelope bbox-
    tested against the filter in FP64, matching deltas compacted, the new side's EnvelopeEncoder
    index envelope written), all on the device (BaseDiffWriter.filtered_ds_feature_deltas)."""
    import types

    from kart_amd import synth
    from kart_amd.device import FilterPipeline
    from kart_amd.spatial import GeomCols

    n, bits = args.n, 20
    t0 = time.time()
    shard = (H.rank, H.world) if H.world > 1 else None
    L = synth.polygons_layer(n, shard=shard, delta_blobs=True) if args.c3_layer else synth.c5_layer(n, shard=shard)
    log(f"[rank {H.rank}] generated {L.base.n}+{L.target.n} entries in {time.time() - t0:.1f}s")
    ver = types.SimpleNamespace(schema=L.schema, legends=L.legends)
    cols = GeomCols(ver, ver, "geom", "geom")
    eng = engine_for(H)
    heads = not args.arena
    pipe = FilterPipeline(eng, L.base, L.target, L.base_blobs, L.target_blobs, cols, synth.C5_FILTER, False, bits,
                          heads=heads, delta_order=heads and not args.per_entry, gather=args.gh_gather)
    for _ in range(max(1, args.warmup)):
        pipe.step()
    eng.sync()
    counts, delta, codes, keep, enc, enc_ok = pipe.results()
    plan = (L.n_insert, L.n_update, L.n_delete)
    if not args.no_check:
        assert (counts["inserts"], counts["updates"], counts["deletes"]) == plan, (counts, plan)
        # size-independent: kept = deltas with a side that may match, in delta order; codes in range
        may = ((codes >= 1) & (codes <= 3)).any(axis=1)
        assert np.array_equal(keep, np.nonzero(may)[0]), "kept deltas differ from the per-delta codes"
        assert codes.max() <= 4 and not (codes == 3).any(), "fallback codes left (the blob fallback runs in the step)"
        assert ((delta[:, 0] == 0xFFFFFFFF) == (codes[:, 0] == 4)).all() and \
            ((delta[:, 1] == 0xFFFFFFFF) == (codes[:, 1] == 4)).all()
    kname = "k_gf_heads" if heads else "k_gf_match"
    eng.prof_reset()
    eng.prof_select(None if args.time_all else [kname])
    eng.prof_enable(not args.no_events)
    elapsed = timed(H, eng, pipe.step, args.steps)
    eng.prof_enable(False)
    kern = kernel_times(eng, ("k_partition2", "k_join2", "k_place2", kname, "k_gf_scan", "k_gf_place"))
    eng.prof_reset()
    eng.prof_select(None)
    eng.prof_enable(True)
    for _ in range(3):
        pipe.step()
    eng.sync()
    eng.prof_enable(False)
    parts = kernel_times(eng, ("k_partition2", "k_join2", "k_gscan2", "k_place2", "k_gh_gather", kname, "k_gf_scan",
                               "k_gf_place"))
    n_pairs = L.base.n + L.n_insert
    total_pairs = sum(H.allgather(n_pairs))
    nd = counts["deltas"]
    ob_off, nb_off = L.base_blobs[1], L.target_blobs[1]
    pres = int((delta[:, 0] != 0xFFFFFFFF).sum() + (delta[:, 1] != 0xFFFFFFFF).sum())
    gather = None
    if heads:
        # algorithmic bytes per k_gf_heads launch: the delta pairs (8 B), one 48-B head per present
        # side, codes (2 B) + index envelope (bits/2 + 1 B) written per delta
        alg = 8 * nd + 48 * pres + nd * (2 + bits // 2 + 1)
        if pipe.gather and "k_gh_gather" in parts:  # the gather: pairs read, heads read + written, pairs written
            galg = 8 * nd + 96 * pres + 8 * nd
            gms = parts["k_gh_gather"][1]
            gather = {"what": "k_gh_gather: the deltas' 48-B heads copied into delta order (one per present side)",
                      "avg_launch_ms": round(gms, 5), "algorithmic_bytes_per_launch": galg,
                      "frac": round(galg / (gms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    # per k_gf_match launch (the arena path): the delta pairs (8 B); per present side its offsets (16 B)
    # and the blob head up to the end of the GPKG envelope (<= 96 B); codes + index envelope written
    head = 0
    for col, off in ((delta[:, 0], ob_off), (delta[:, 1], nb_off)):
        prs = col[col != 0xFFFFFFFF].astype(np.int64)
        head += int(np.minimum(off[prs + 1] - off[prs], 96).sum()) + 16 * prs.size
    alg_arena = 8 * nd + head + nd * (2 + bits // 2 + 1)
    if not heads:
        alg = alg_arena
    roof = roofline(kern, kname, alg, args.traffic_json, n, "c5" if heads and H.world == 1 else None)
    arena_path = None
    if heads and not args.no_arena_timing:  # the same step through kd_geom_filter (blob arenas, msgpack walk)
        pa = FilterPipeline(eng, L.base, L.target, L.base_blobs, L.target_blobs, cols, synth.C5_FILTER, False, bits)
        pa.step()
        eng.sync()
        eng.prof_reset()
        eng.prof_select(["k_gf_match"])
        eng.prof_enable(not args.no_events)
        el_a = timed(H, eng, pa.step, args.steps)
        eng.prof_enable(False)
        ka = kernel_times(eng, ("k_gf_match",))
        eng.prof_reset()
        eng.prof_select(None)
        eng.prof_enable(True)
        for _ in range(3):
            pa.step()
        eng.sync()
        eng.prof_enable(False)
        pa_parts = kernel_times(eng, ("k_partition2", "k_join2", "k_gscan2", "k_place2", "k_gf_match", "k_gf_scan",
                                      "k_gf_place"))
        # the arena path's own roofline: k_gf_match's algorithmic bytes over its HIP-event time, and the
        # measured HBM bytes of its rocprofv3 PMC passes (profiles/<round>/traffic_c5arena.json)
        ta = args.traffic_json.replace("traffic_c5.json", "traffic_c5arena.json") if args.traffic_json else ""
        arena_path = {"value": round(total_pairs * args.steps / el_a / 1e6, 2),
                      "ms_per_step": round(el_a / args.steps * 1e3, 4),
                      "kernels_avg_ms": {k: round(v[1], 5) for k, v in ka.items()},
                      "step_kernels_avg_ms": {k: round(v[1], 5) for k, v in pa_parts.items()},
                      "largest_step_kernel": max(pa_parts, key=lambda k: pa_parts[k][1]) if pa_parts else None,
                      "roofline": roofline(ka, "k_gf_match", alg_arena, ta if os.path.exists(ta) else "", n,
                                           "c5arena" if H.world == 1 else None)}
        del pa
    cpu = None
    if H.rank == 0 and H.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_filter(L, delta, codes, keep, enc, enc_ok, args, bits)
    eng.close()
    out = {
        "metric": METRIC, "value": round(total_pairs * args.steps / elapsed / 1e6, 2), "unit": "M feature-pairs/s",
        "n_gpus": H.world, "rccl_comm": H.comm, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong" if H.world > 1 else "weak", "vs_baseline": None,
        "dtype": "u8/u64 (integer join) + f64 (envelopes, EnvelopeEncoder)",
        "data": ("synthetic (the C3 MULTIPOLYGON layer" if args.c3_layer else
                 "synthetic (SURVEY §8d's C5 mix: 30% points incl. EMPTY, polygons with straddling / >=180-degree-wide / "
                 "filter-edge / XYZ envelopes, EPSG:4326") + "; blobs materialised for every delta's old/new version)",
        "config": {"workload": f"C5: spatially filtered diff of ONE {n}-feature polygon layer"
                               f"{f' split into {H.world} bucket-range shards' if H.world > 1 else ''}: classify2 + "
                               "per-delta geometry envelope filter + EnvelopeEncoder of the new side" +
                               ((" (from the 48-B geometry heads the blob reader extracts on the host, kd_geom_heads, "
                                 "in delta order as the reader leaves them after classification; blob fallback through "
                                 "the step's delta pairs)" if pipe.delta_order and not pipe.gather else
                                 " (from the 48-B per-entry geometry heads, gathered into delta order on the device in "
                                 "the step)" if pipe.gather else " (from the 48-B per-entry geometry heads)")
                                if heads else " (msgpack walk of the blob arenas on the GPU)"),
                   "features": n, "pairs_per_step": total_pairs, "deltas_per_step": sum(H.allgather(nd)),
                   "kept_per_step": sum(H.allgather(counts["kept"])), "bits": bits, "filter": list(synth.C5_FILTER),
                   "parallelism": f"bucket-range shards x{H.world} (counts per rank, no exchange)"},
        "kernels_avg_ms": {k: round(v[1], 5) for k, v in kern.items()},
        "step_kernels_avg_ms": {k: round(v[1], 5) for k, v in parts.items()},
        "roofline": roof, "cpu_baseline": cpu, "heads_gather": gather,
        "largest_step_kernel": max(parts, key=lambda k: parts[k][1]) if parts else None,
    }
    if heads:
        blobs = int(np.count_nonzero(np.diff(L.base_blobs[1])) + np.count_nonzero(np.diff(L.target_blobs[1])))
        out["host"] = {"geom_heads_s": round(pipe.heads_s, 4), "blobs": blobs,
                       "geom_heads_M_blobs_per_s": round(blobs / pipe.heads_s / 1e6, 2),
                       "delta_heads_s": round(pipe.delta_heads_s, 4) if pipe.delta_heads_s is not None else None,
                       # one diff's device step plus its host layout of the heads in delta order (the
                       # headline's step excludes that layout: ADVICE r5)
                       "step_plus_delta_heads_ms": (round(elapsed / args.steps * 1e3 + pipe.delta_heads_s * 1e3, 2)
                                                    if pipe.delta_heads_s is not None else None),
                       "note": "kd_geom_heads: the blob reader's host pass (msgpack walk of every materialised blob, "
                               f"{host_cores()} threads) that leaves 48 B per blob for the GPU; delta_heads_s: those "
                               "heads laid out in delta order (the reader reads the deltas' blobs after "
                               "classification); both outside the timed step, per pass over the layer"}
        out["arena_path"] = arena_path
    return out


def cpu_baseline_filter(L, delta, codes, keep, enc, enc_ok, args, bits):
    """The C oracle's classify2 + filtered-diff decision (kdo_classify2 + kdo_geom_filter: msgpack walk,
    envelope, bbox, EnvelopeEncoder) on the host cores over bucket-range shards of the whole layer,
    and one thread over one shard.  The first shard doubles as a bit-exact check of the device codes."""
    from concurrent.futures import ThreadPoolExecutor

    O = oracle()
    cols = {h: 0 for h in L.legends}
    (od, oo), (nd, no) = L.base_blobs, L.target_blobs
    cores = host_cores()
    parts = 4 * cores
    ba, bb = _shard_bounds(L, parts)
    filt = synth_filter()

    def shard(s):
        A, B = L.base, L.target
        a0, a1, b0, b1 = int(ba[s]), int(ba[s + 1]), int(bb[s]), int(bb[s + 1])
        d, c = O.classify2(A.key[a0:a1], A.oid[a0:a1], B.key[b0:b1], B.oid[b0:b1])
        g = d.astype(np.int64)
        g[:, 0] = np.where(d[:, 0] == O.NONE, O.NONE, g[:, 0] + a0)
        g[:, 1] = np.where(d[:, 1] == O.NONE, O.NONE, g[:, 1] + b0)
        res = O.geom_filter(od, oo, nd, no, g.astype(np.uint32), cols, cols, filt, False, bits)
        return (a1 - a0) + c["inserts"], g.astype(np.uint32), res

    if not args.no_check:  # shard 0 against the device's first deltas
        _, g0, (oc, okeep, oenc, ook) = shard(0)
        m = g0.shape[0]
        assert np.array_equal(delta[:m], g0), "classify2 differs from the oracle"
        assert np.array_equal(codes[:m], oc), "kd_geom_filter codes differ from the oracle"
        assert np.array_equal(keep[keep < m], okeep), "kept deltas differ from the oracle"
        assert np.array_equal(enc_ok[:m], ook) and np.array_equal(enc[:m][ook == 1], oenc[ook == 1])
    with ThreadPoolExecutor(cores) as ex:
        t0 = time.perf_counter()
        reps = 0
        while True:
            pairs = sum(r[0] for r in ex.map(shard, range(parts)))
            reps += 1
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        dt = time.perf_counter() - t0
    t0 = time.perf_counter()
    reps1 = 0
    while True:
        p1 = shard(0)[0]
        reps1 += 1
        if time.perf_counter() - t0 >= args.cpu_seconds / 2:
            break
    dt1 = time.perf_counter() - t0
    return {"value": round(pairs * reps / dt / 1e6, 2), "unit": "M feature-pairs/s", "cores": cores, "kind": "port",
            "sample": f"the full C5 layer ({pairs} pairs) x {reps} reps in {dt:.1f}s: oracle/kd_oracle.c classify2 + "
                      f"geom_filter on {cores} threads over {parts} bucket-range shards",
            "one_thread": {"value": round(p1 * reps1 / dt1 / 1e6, 3), "unit": "M feature-pairs/s", "cores": 1,
                           "sample": f"one shard ({p1} pairs, 1/{parts} of the layer) x {reps1} reps in {dt1:.1f}s"}}


def synth_filter():
    from kart_amd import synth

    return synth.C5_FILTER


# ---------------------------------------------------------------------------------------------
def run_c5env(args, H):
    """k_envelopes + k_env_overlap over a raw GPKG geometry arena (the spatial-index envelope
    kernels alone, no diff)"""
    import ctypes

    from kart_amd import _native as N
    from kart_amd import synth
    from kart_amd.device import DevBuf

    n, bits = args.n, 20
    nb = bits // 2
    t0 = time.time()
    data, off, is_pt = synth.geometry_layer(n, seed=synth.SEED + H.rank)
    log(f"[rank {H.rank}] generated {n} geometries ({data.size / 1e9:.2f} GB) in {time.time() - t0:.1f}s")
    eng = engine_for(H)
    d_data, d_off = DevBuf.from_numpy(eng, data), DevBuf.from_numpy(eng, off)
    g = N.KdBlobs()
    g.n, g.data, g.off, g.mem, g.size_hint = n, d_data.ptr, d_off.ptr, N.KD_MEM_DEVICE, 0
    match, enc, ok, ovl = DevBuf(eng, n), DevBuf(eng, n * nb), DevBuf(eng, n), DevBuf(eng, n)
    fe = (ctypes.c_double * 4)(*synth.C5_FILTER)
    q = (ctypes.c_double * 4)(synth.C5_FILTER[0], synth.C5_FILTER[2], synth.C5_FILTER[1], synth.C5_FILTER[3])
    L, ctx = eng.L, eng.ctx

    def step():
        N.check(L.kd_envelopes(ctx, ctypes.byref(g), fe, bits, match.ptr, enc.ptr, ok.ptr, N.KD_MEM_DEVICE, None),
                "kd_envelopes")
        N.check(L.kd_env_overlap(ctx, enc.ptr, n, bits, q, ovl.ptr, N.KD_MEM_DEVICE), "kd_env_overlap")

    for _ in range(max(1, args.warmup)):
        step()
    eng.sync()
    h_match, h_ok = match.download(np.uint8, n), ok.download(np.uint8, n)
    if not args.no_check:  # size-independent: an encoded envelope only where the indexer stores one
        assert not (h_ok.astype(bool) & (h_match == 2)).any(), "enc_ok on a null geometry"
    eng.prof_reset()
    eng.prof_select(None if args.time_all else ["k_envelopes"])
    eng.prof_enable(not args.no_events)
    elapsed = timed(H, eng, step, args.steps)
    eng.prof_enable(False)
    total = sum(H.allgather(n))
    kern = kernel_times(eng, ("k_envelopes", "k_env_overlap"))
    npt = int(is_pt.sum())
    # algorithmic bytes per k_envelopes launch: offsets (8 B) + GPKG header (8 B) + stored envelope
    # (32 B, polygons) or point WKB (21 B) read; match + enc_ok flags (2 B) + encoded envelope written
    alg = n * (8 + 8 + 2 + nb) + npt * 21 + (n - npt) * 32
    roof = roofline(kern, "k_envelopes", alg, args.traffic_json, n, "c5env")
    heads_path = None
    if not args.no_heads_path:
        heads_path = c5env_heads_path(args, H, eng, data, off, d_data, d_off, n, bits, nb, enc, ok)
    cpu = None
    if H.rank == 0 and H.world == 1 and not args.no_cpu_baseline:
        O = oracle()
        nsh = 4 * host_cores()
        cut = np.linspace(0, n, nsh + 1).astype(np.int64)
        h_enc = enc.download(np.uint8, n * nb).reshape(n, nb)
        got = [None] * nsh

        def work(s):
            a, b = int(cut[s]), int(cut[s + 1])
            o0 = int(off[a])
            got[s] = O.envelope_batch(data[o0:int(off[b])], off[a:b + 1] - np.uint64(o0), synth.C5_FILTER, bits)
            return b - a

        res = cpu_sharded(work, nsh, min(args.cpu_seconds, 10.0))
        if not args.no_check:  # the baseline's last run doubles as a bit-exact check of the whole layer
            assert np.array_equal(h_match, np.concatenate([g[0] for g in got])), "k_envelopes flags differ from the oracle"
            assert np.array_equal(h_ok, np.concatenate([g[2] for g in got])), "k_envelopes enc_ok differs from the oracle"
            assert np.array_equal(h_enc, np.concatenate([g[1] for g in got])), "EnvelopeEncoder bytes differ"
        del got, h_enc
        cpu = cpu_line(res, "M geometries/s", "oracle/kd_oracle.c envelope batch (bbox test + index envelope + "
                                              f"EnvelopeEncoder) over {nsh} geometry ranges", f"layer ({n} geometries)")
    eng.close()
    return {
        "metric": METRIC, "value": round(total * args.steps / elapsed / 1e6, 2), "unit": "M geometries/s",
        "n_gpus": H.world, "rccl_comm": H.comm, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64 (envelopes, EnvelopeEncoder) + u8",
        "data": "synthetic (seeded GPKG geometries: 30% points, 70% multipolygons, EPSG:4326)",
        "config": {"workload": f"C5-envelopes: {n} raw GPKG geometries per GPU: spatial-filter envelopes + "
                               "EnvelopeEncoder + encoded-envelope overlap (no diff)",
                   "geoms_per_gpu": n, "points": npt, "bits": bits, "filter": list(synth.C5_FILTER),
                   "parallelism": f"independent shards x{H.world}"},
        "kernels_avg_ms": {k: round(v[1], 5) for k, v in kern.items()},
        "roofline": roof, "cpu_baseline": cpu, "heads_path": heads_path,
    }


def c5env_heads_path(args, H, eng, data, off, d_data, d_off, n, bits, nb, enc, ok):
    """the spatial indexer's path over the same geometries (spatial_index._index_envelopes): one
    48-B head per geometry (what kd_geom_heads leaves for a blob whose geometry value this is; built
    here straight from the geometry arena, outside the timing) through kd_geom_filter_heads with the
    arena for the heads that cannot decide; its index envelopes must equal k_envelopes'"""
    import ctypes

    from kart_amd import _native as N
    from kart_amd.device import DevBuf
    from kart_amd.spatial import GEOM_HEAD

    heads = np.zeros(n, GEOM_HEAD)
    lens = np.diff(off).astype(np.int64)
    heads["glen"] = lens
    heads["goff_status"] = np.where(lens > 0, N.KD_GH_GEOM << 24, N.KD_GH_NULL << 24).astype(np.uint32)
    col = np.arange(40, dtype=np.int64)
    for a in range(0, n, 1 << 19):  # first 40 bytes of each geometry (zeros past its end)
        b = min(n, a + (1 << 19))
        idx = off[a:b, None].astype(np.int64) + col
        inside = col < lens[a:b, None]
        heads["gpkg"][a:b] = np.where(inside, data[np.minimum(idx, data.size - 1)], 0)
    dh = DevBuf.from_numpy(eng, heads.view(np.uint8).reshape(-1))
    pairs = np.full((n, 2), N.KD_NONE, np.uint32)
    pairs[:, 1] = np.arange(n, dtype=np.uint32)
    dp = DevBuf.from_numpy(eng, pairs.reshape(-1))
    m2, kp, nk = DevBuf(eng, 2 * n + 2), DevBuf(eng, 4 * n + 4), DevBuf(eng, 8)
    e2, ok2 = DevBuf(eng, n * nb + 4), DevBuf(eng, n + 4)
    empty_off = DevBuf.from_numpy(eng, np.zeros(1, np.uint64))
    blobs = []
    for d_, o_, cnt in ((d_data, empty_off, 0), (d_data, d_off, n)):
        b_ = N.KdBlobs()
        b_.n, b_.data, b_.off, b_.mem, b_.size_hint = cnt, d_.ptr, o_.ptr, N.KD_MEM_DEVICE, 0
        blobs.append(b_)
    fe = (ctypes.c_double * 4)(-180.0, 180.0, -90.0, 90.0)  # the indexer's world envelope

    def filt():
        N.check(eng.L.kd_geom_filter_heads(eng.ctx, dh.ptr, 0, dh.ptr, n, N.KD_MEM_DEVICE, ctypes.byref(blobs[0]),
                                           ctypes.byref(blobs[1]), dp.ptr, n, None, N.KD_MEM_DEVICE, fe, 0, bits,
                                           m2.ptr, kp.ptr, ctypes.cast(nk.ptr, N.c_u64p), e2.ptr, ok2.ptr,
                                           N.KD_MEM_DEVICE), "kd_geom_filter_heads")

    filt()
    eng.sync()
    if not args.no_check:
        g_ok, h_ok = ok2.download(np.uint8, n), ok.download(np.uint8, n)
        assert np.array_equal(g_ok, h_ok), "heads path enc_ok differs from k_envelopes"
        g_enc, h_enc = e2.download(np.uint8, n * nb).reshape(n, nb), enc.download(np.uint8, n * nb).reshape(n, nb)
        sel = h_ok == 1
        assert np.array_equal(g_enc[sel], h_enc[sel]), "heads path envelopes differ from k_envelopes"
    eng.prof_reset()
    eng.prof_select(["k_gf_heads"])
    eng.prof_enable(True)
    el = timed(H, eng, filt, args.steps)
    eng.prof_enable(False)
    kd = kernel_times(eng, ("k_gf_heads",))
    alg = 8 * n + 48 * n + n * (2 + nb + 1)
    for b_ in (dh, dp, m2, kp, nk, e2, ok2, empty_off):
        b_.free()
    return {"what": "the spatial indexer's path: 48-B geometry heads (built from the arena outside the timing) "
                    "through kd_geom_filter_heads, envelopes equal to k_envelopes'",
            "ms_per_call": round(el / args.steps * 1e3, 4),
            "roofline": roofline(kd, "k_gf_heads", alg, "", -1)}


# ---------------------------------------------------------------------------------------------
def run_c6(args, H):
    """Writer formatting: hex WKB of every geometry of the C5 layer (kd_hex_encode,
    KD_HEX_GPKG_WKB), the formatting `kart diff -o json` applies per geometry value."""
    import ctypes

    from kart_amd import _native as N
    from kart_amd import synth
    from kart_amd.device import DevBuf

    n = args.n
    t0 = time.time()
    data, off, is_pt = synth.geometry_layer(n, seed=synth.SEED + H.rank)
    nbytes = int(off[-1])
    log(f"[rank {H.rank}] generated {n} geometries ({nbytes / 1e9:.2f} GB) in {time.time() - t0:.1f}s")
    eng = engine_for(H)
    d_data, d_off = DevBuf.from_numpy(eng, data), DevBuf.from_numpy(eng, off)
    g = N.KdBlobs()
    g.n, g.data, g.off, g.mem, g.size_hint = n, d_data.ptr, d_off.ptr, N.KD_MEM_DEVICE, 0
    hexbuf, start, status = DevBuf(eng, 2 * nbytes), DevBuf(eng, 4 * n), DevBuf(eng, n)
    L, ctx = eng.L, eng.ctx

    def step():
        N.check(L.kd_hex_encode(ctx, ctypes.byref(g), N.KD_HEX_GPKG_WKB, hexbuf.ptr, start.ptr, status.ptr,
                                N.KD_MEM_DEVICE), "kd_hex_encode")

    for _ in range(max(1, args.warmup)):
        step()
    eng.sync()
    O = oracle()
    if not args.no_check:  # every geometry is valid LE GPKG; sampled strings equal the oracle's
        assert int(status.download(np.uint8, n).max()) == 0, "kd_hex_encode flagged a valid geometry"
        st = start.download(np.uint32, n)
        for i in list(range(0, n, max(1, n // 2000))) + [n - 1]:
            o, e = int(off[i]), int(off[i + 1])
            a = 2 * (o + int(st[i]))
            got = hexbuf.download(np.uint8, 2 * e - a, offset=a).tobytes().decode()
            assert got == O.hex_wkb(data[o:e].tobytes()), f"hex WKB of geometry {i} differs from the oracle"
    eng.prof_reset()
    eng.prof_select(None if args.time_all else ["k_hex"])
    eng.prof_enable(not args.no_events)
    elapsed = timed(H, eng, step, args.steps)
    eng.prof_enable(False)
    total = sum(H.allgather(n))
    kern = kernel_times(eng, ("k_hex", "k_wkb_start"))
    # algorithmic bytes per k_hex launch: the geometry arena read once, two hex chars written per byte
    roof = roofline(kern, "k_hex", 3 * nbytes, args.traffic_json, n, "c6")
    cpu = None
    if H.rank == 0 and H.world == 1 and not args.no_cpu_baseline:
        m = min(n, 200_000)
        blobs = [data[int(off[i]):int(off[i + 1])].tobytes() for i in range(m)]
        nsh = 4 * host_cores()
        cut = np.linspace(0, n, nsh + 1).astype(np.int64)
        first = {}

        def work(s):
            a, b = int(cut[s]), int(cut[s + 1])
            hx, st = O.hex_wkb_batch(data, off[a:b + 1])
            if s == 0:
                first["hex"], first["st"] = hx, st
            return b - a

        res = cpu_sharded(work, nsh, min(args.cpu_seconds, 10.0))
        if not args.no_check:  # shard 0 of the C restatement equals the kernel's hex bytes
            b0 = int(cut[1])
            st0 = start.download(np.uint32, b0)
            gh = hexbuf.download(np.uint8, 2 * int(off[b0]))
            assert not first["st"].any()
            for i in range(b0):
                a, e = 2 * (int(off[i]) + int(st0[i])), 2 * int(off[i + 1])
                if not np.array_equal(gh[a:e], first["hex"][a:e]):
                    raise AssertionError(f"hex of geometry {i} differs from the C restatement")
        cpu = cpu_line(res, "M geometries/s", "oracle/kd_oracle.c kdo_hex_wkb_batch (gpkg_geom_to_hex_wkb "
                                              f"restated: slice + uppercase hex) over {nsh} geometry ranges",
                       f"layer ({n} geometries)")
        # the drop-in as Kart would call it: host values in, Python strs out (arena join, H2D, kernel,
        # D2H, one decode + numpy-bounded slicing), against a per-value binascii.hexlify loop
        import binascii

        from kart_amd.output import hex_wkb_arena, hex_wkb_batch

        e2e = eng
        hx, fb = hex_wkb_batch(e2e, blobs[:1000])  # warm the staging slots
        t0 = time.perf_counter()
        hx, fb = hex_wkb_batch(e2e, blobs)
        t_batch = time.perf_counter() - t0
        t0 = time.perf_counter()
        hb, lo, hi, st = hex_wkb_arena(e2e, blobs)
        t_arena = time.perf_counter() - t0
        t0 = time.perf_counter()
        ref = [binascii.hexlify(b[8 + (32 if (b[3] >> 1) & 7 else 0):]).decode().upper() for b in blobs]
        t_loop = time.perf_counter() - t0
        if not args.no_check:
            assert not fb and hx == ref, "hex_wkb_batch differs from the per-value loop"
        cpu["end_to_end"] = {
            "hex_wkb_batch": {"value": round(m / t_batch / 1e6, 3), "unit": "M geometries/s",
                              "sample": f"{m} host geometries -> list of str via kart_amd.output.hex_wkb_batch "
                                        "(arena join + H2D + kd_hex_encode + D2H + slicing), 1 GPU"},
            "hex_wkb_arena": {"value": round(m / t_arena / 1e6, 3), "unit": "M geometries/s",
                              "sample": f"the same {m} geometries -> one hex buffer + bounds (no str per value)"},
            "per_value_hexlify": {"value": round(m / t_loop / 1e6, 3), "unit": "M geometries/s",
                                  "sample": f"the same {m} geometries, binascii.hexlify(wkb).upper() per value, 1 thread"}}
    eng.close()
    return {
        "metric": METRIC, "value": round(total * args.steps / elapsed / 1e6, 2), "unit": "M geometries/s",
        "n_gpus": H.world, "rccl_comm": H.comm, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded GPKG geometries: 30% points, 70% multipolygons, EPSG:4326)",
        "config": {"workload": f"C6 (SURVEY 8f #2, {n} geometries per GPU): hex WKB of every geometry "
                               "(Geometry.to_hex_wkb for kart diff -o json)",
                   "geoms_per_gpu": n, "points": int(is_pt.sum()), "arena_bytes": nbytes,
                   "parallelism": f"independent shards x{H.world}"},
        "kernels_avg_ms": {k: round(v[1], 5) for k, v in kern.items()},
        "roofline": roof, "cpu_baseline": cpu,
    }


# ---------------------------------------------------------------------------------------------
def run_c4(args, H):
    """C4 (configs[3]): three-way merge classification of a 50M-row string-PK table.  The sides come as
    the tree walk lists them (git tree order: buckets ascending, each leaf tree's few entries in
    filename order, not FNV-key order); one step = the three per-bucket sorts
    (kd_sort_segmented_into) + the one-pass three-way join (k_partition2, k_apart3, k_join3, k_place3),
    OIDs and filenames read through the orders (kd_merge3_device_perm).  The table is SURVEY §8(d)'s
    mix (synth.table3_layers).  Beside it (``presorted``) the same merge over key-sorted sides."""
    from kart_amd import synth
    from kart_amd.device import MergePipeline

    n = args.n
    t0 = time.time()
    M = synth.table3_layers(n, seed=synth.SEED + H.rank, walk=True)
    A, O_, T = M.ancestor, M.ours, M.theirs
    log(f"[rank {H.rank}] generated ancestor/ours/theirs {A.n}/{O_.n}/{T.n} string-pk rows (walk order) in "
        f"{time.time() - t0:.1f}s ({M.n_conflict} conflicts planned)")
    eng = engine_for(H)
    pipe = MergePipeline(eng, A, O_, T, segmented=True)
    for _ in range(max(1, args.warmup)):
        pipe.step()
    eng.sync()
    n_clean, conf, md = pipe.results()
    srt = []
    for S, order in zip((A, O_, T), pipe.orders()):
        if not args.no_check:  # the per-bucket sorts == a full sort of the keys
            ko = S.key[order]
            assert np.all(ko[1:] > ko[:-1]), "segmented sort: keys not ascending"
        srt.append((S.key[order], S.oid[order], order))
    if not args.no_check:  # the generator's own plan (libgit2 rule over planned edits)
        assert conf.shape[0] == M.n_conflict, (conf.shape[0], M.n_conflict)
    eng.prof_reset()
    eng.prof_select(None if args.time_all else ["k_join2", "k_join3"])
    eng.prof_enable(not args.no_events)
    elapsed = timed(H, eng, pipe.step, args.steps)
    eng.prof_enable(False)
    nall = A.n + O_.n + T.n
    total = sum(H.allgather(nall))
    kern = kernel_times(eng, C4_KERNELS)
    eng.prof_reset()
    eng.prof_select(None)
    eng.prof_enable(True)
    for _ in range(3):
        pipe.step()
    eng.sync()
    eng.prof_enable(False)
    parts = kernel_times(eng, C4_KERNELS)
    # classify3 in one pass (k_join3b): dominant kernel k_join3, algorithmic bytes per
    # launch — what the join must read with the sides in walk order (late materialisation):
    #   per ours / theirs entry: key 8 + OID 20 + walk row 4 B, and its filename;
    #   per matched pair: both name offsets (8 B each: a hash key is verified against the names);
    #   every ancestor key (8 B);
    #   per differing path with an ancestor entry: its walk row, OID, name offset and filename, and
    #   the path's own name offset when it is one-sided;
    #   per differing path the staged result (12 B).
    # (Round 4's formula — 28 B per ours / theirs entry + names + 8 B per ancestor key + 12 B per
    # differing path + 4 B per matched pair — left out the walk rows, the name offsets and the
    # ancestor's reads; it is reported beside, `algorithmic_bytes_r4_formula`.)
    (kA, _, ordA), (kO, oO, _), (kT, oT, _) = srt[0], srt[1], srt[2]
    _, io, it = np.intersect1d(kO, kT, assume_unique=True, return_indices=True)
    chg = (oO[io] != oT[it]).any(axis=1)
    n_cand = int(O_.n + T.n - 2 * io.size + np.count_nonzero(chg))
    one_o = np.ones(O_.n, bool)
    one_o[io] = False
    one_t = np.ones(T.n, bool)
    one_t[it] = False
    one_keys = np.concatenate([kO[one_o], kT[one_t]])
    dif_keys = np.concatenate([one_keys, kO[io][chg]])
    pa = np.searchsorted(kA, dif_keys)
    has_a = (pa < kA.size) & (kA[np.minimum(pa, kA.size - 1)] == dif_keys)
    rows = ordA[pa[has_a]]
    anc_name = int((A.name_off[rows + 1] - A.name_off[rows]).sum())
    n_anc = int(np.count_nonzero(has_a))
    n_one_anc = int(np.count_nonzero(has_a[:one_keys.size]))
    alg_r4 = 28 * (O_.n + T.n) + int(O_.name.size + T.name.size) + 8 * A.n + 12 * n_cand + 4 * io.size
    j3 = "k_join3" in kern
    if j3:
        alg = (32 * (O_.n + T.n) + int(O_.name.size + T.name.size) + 16 * io.size + 8 * A.n
               + 32 * n_anc + anc_name + 8 * n_one_anc + 12 * n_cand)
    else:  # (KD_MERGE3_JOIN=0: the two-step path, k_join2 + k_resolve3, k_join2 dominant)
        alg = 28 * (O_.n + T.n) + int(O_.name.size + T.name.size) + 8 * n_cand + 8 * io.size
    roof = roofline(kern, "k_join3" if j3 else "k_join2", alg, args.traffic_json, n, "c4" if H.world == 1 else None)
    if roof and j3:
        roof["algorithmic_bytes_r4_formula"] = int(alg_r4)
    seg_alg = 20 * nall  # per entry: the key read, key + 4-B order written (neighbours hit the cache)
    seg = {"what": "kd_sort_segmented_into x3: each bucket's entries (git filename order) ordered by key",
           "ms_per_step_events": round(parts["k_seg_sort"][0] * parts["k_seg_sort"][1] / 3, 4) if "k_seg_sort" in parts else None,
           "algorithmic_bytes_per_step": seg_alg}
    if seg["ms_per_step_events"]:
        seg["frac"] = round(seg_alg / (seg["ms_per_step_events"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    presorted = None
    if not args.no_sort:  # the same merge over key-sorted sides (what the walk would give if it were key order)
        from kart_amd import packing

        ks = []
        for S, (k, o, order) in zip((A, O_, T), srt):
            P = packing.PackedSide(np.ascontiguousarray(k), np.ascontiguousarray(o), S.key_mode, np.arange(S.n),
                                   encoding=S.encoding)
            P.name, P.name_off = packing._gather_names(S.name, S.name_off, order)
            ks.append(P)
        del pipe
        pp = MergePipeline(eng, *ks)
        pp.step()
        eng.sync()
        c2, conf2, md2 = pp.results()
        if not args.no_check:
            assert np.array_equal(conf2, conf) and np.array_equal(md2, md) and c2 == n_clean, "presorted merge differs"
        el2 = timed(H, eng, pp.step, args.steps)
        presorted = {"value": round(total * args.steps / el2 / 1e6, 2), "ms_per_step": round(el2 / args.steps * 1e3, 4)}
        del pp
    cpu = None
    if H.rank == 0 and H.world == 1 and not args.no_cpu_baseline:
        Orc = oracle()
        (kA, oA, _), (kO, oO, _), (kT, oT, _) = srt
        nsh = 4 * host_cores()
        # bucket-range shards (keys ascend in their bucket bits): cut at ancestor key quantiles
        ck = kA[np.linspace(0, A.n, nsh + 1).astype(np.int64)[1:-1]] if A.n else np.zeros(0, np.uint64)
        bnd = [np.concatenate([[0], np.searchsorted(k, ck), [k.shape[0]]]).astype(np.int64) for k in (kA, kO, kT)]
        got = [None] * nsh

        def work(s):
            sl = [slice(int(bd[s]), int(bd[s + 1])) for bd in bnd]
            got[s] = Orc.classify3(kA[sl[0]], oA[sl[0]], kO[sl[1]], oO[sl[1]], kT[sl[2]], oT[sl[2]])
            return sum(x.stop - x.start for x in sl)

        res = cpu_sharded(work, nsh, min(args.cpu_seconds, 10.0))
        if not args.no_check:  # the baseline's last run, re-based to whole-side indices, is a bit-exact check
            NONE = np.uint32(0xFFFFFFFF)

            def rebase(rows, s, cols):
                rows = rows.copy()
                for c, side in enumerate(cols):
                    m = rows[:, c] != NONE
                    rows[m, c] += np.uint32(bnd[side][s])
                return rows

            oc = np.concatenate([rebase(got[s][0], s, (0, 1, 2)) for s in range(nsh)])
            om = np.concatenate([rebase(got[s][1], s, (1, 2)) for s in range(nsh)])
            assert np.array_equal(conf, oc), "classify3 conflicts differ from the oracle"
            assert np.array_equal(md, om), "classify3 merge deltas differ from the oracle"
            assert n_clean == sum(got[s][2] for s in range(nsh))
        del got
        cpu = cpu_line(res, "M entries/s", f"oracle/kd_oracle.c classify3 over {nsh} bucket-range shards",
                       f"C4 layer ({nall} entries, key-sorted)")
    eng.close()
    return {
        "metric": METRIC, "value": round(total * args.steps / elapsed / 1e6, 2), "unit": "M entries/s",
        "n_gpus": H.world, "rccl_comm": H.comm, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8/u64 (integer)",
        "data": "synthetic (seeded text-PK table: MsgpackHashPathEncoder paths in git tree order, synthetic OIDs)",
        "config": {"workload": f"C4: {n}-row string-PK table per GPU (SURVEY 8(d) mix: 12-24-char text pks, 5% "
                               "multibyte UTF-8; per side 5% updates, 0.5% inserts, 0.5% deletes from independent "
                               "seeds; +0.5% rows edited differently on both sides, +0.5% identically; add/add), "
                               "three-way merge classification (ancestor/ours/theirs join + libgit2 conflict rule) "
                               "from walk-order sides",
                   "rows_per_gpu": n, "entries_per_step": total, "mix": M.plan, "conflicts": int(conf.shape[0]),
                   "merge_deltas": int(md.shape[0]), "differing_paths": n_cand,
                   "parallelism": f"independent shards x{H.world}"},
        "kernels_avg_ms": {k: round(v[1], 5) for k, v in kern.items()},
        "step_kernels_avg_ms": {k: round(v[1], 5) for k, v in parts.items()},
        "segmented_sort": seg, "presorted": presorted,
        "roofline": roof, "cpu_baseline": cpu,
    }


def main():
    args = parse()
    H = Harness()
    out = {"c2": lambda a, h: run_diff(a, h, polygons=False), "c3": lambda a, h: run_diff(a, h, polygons=True),
           "c3v": lambda a, h: run_diff(a, h, polygons=True),
           "c4": run_c4, "c5": run_c5, "c5env": run_c5env, "c6": run_c6}[args.workload](args, H)
    if H.rank == 0:
        print(json.dumps(out), flush=True)
    H.close()


if __name__ == "__main__":
    main()
