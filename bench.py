#!/usr/bin/env python3
"""Bench: device-resident bulk feature diff on MI355X (one JSON line on rank 0).

Default workload (BASELINE.json configs[1], "C2"): a synthetic 10M-point int-PK layer per GPU with
seeded 1% updates / 1% deletes / 1% inserts (kart_amd.synth.points_layer; the reference's feature
blob and path encodings, synthetic OIDs).  One *step* = one full pass of the hot path over that
layer: merge-path join + OID compare + key-ordered compaction of the delta set (k_partition2,
k_join2, k_place2), then the msgpack field decode + Python-== column compare of every update
(k_fielddiff) — all on the device, inputs resident in HBM before the timed region.

--workload c3 (BASELINE configs[2]): a 100M-polygon int-PK layer per GPU (--n), 10% edits: 4% geometry
updates, 4% attribute updates, 1% deletes, 1% inserts; same step as C2 (blobs materialised only for the
updated features: nothing else is read).

--workload c4 (BASELINE configs[3]): a 50M-row string-PK table per GPU (MsgpackHashPathEncoder paths)
three-way merge classification: classify2(ours, theirs) + k_resolve3 (ancestor lookup + the libgit2
conflict rule) over the paths where ours and theirs differ.

--workload c5 (BASELINE configs[4], scaled: --n geometries per GPU, default 20M): GPKG geometry
blobs of a spatially filtered layer (synth.geometry_layer); one step = k_envelopes (header /
stored envelope or point WKB -> SpatialFilter bbox test + identity-CRS index envelope +
EnvelopeEncoder bytes) + k_env_overlap (decode + cyclic overlap of the encoded envelopes).

--workload c6 (--n geometries per GPU, default 20M): the C5 geometry arena hex-encoded
as `kart diff -o json` formats geometries (kd_hex_encode: k_wkb_start WKB offsets + k_hex
streaming 16 B -> 32 B hex per lane).

Multi-GPU (torch.distributed, one process per GPU, RCCL): each rank owns a disjoint dataset3
path-bucket range (its own shard; weak scaling); the only collective is the all-gather of per-rank
counts each step.  value = units of all ranks / max-rank time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c5|c6] [--n UNITS]
                       [--no-cpu-baseline]
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c5", "c6"])
    ap.add_argument("--n", type=int, default=0, help="units per GPU (c2: points, default 10M; c3: polygons, 100M; c4: rows, 50M; c5: geometries, 20M)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--unordered", action="store_true",
                    help="c2: tile-grouped delta list (per-tile atomic appends, no k_place2); default: key order")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--traffic-json", default=None, help="measured HBM bytes per launch (profiles/traffic_<wl>.json)")
    ap.add_argument("--no-check", action="store_true", help="profiling variants only: skip the correctness check")
    ap.add_argument("--no-events", action="store_true", help="no per-kernel HIP events in the timed region")
    ap.add_argument("--time-all", action="store_true",
                    help="HIP events around every kernel of a step (default: only the dominant kernel, "
                         "so the events do not inflate the step time)")
    a = ap.parse_args()
    if not a.n:
        a.n = {"c2": 10_000_000, "c3": 100_000_000, "c4": 50_000_000, "c5": 20_000_000, "c6": 20_000_000}[a.workload]
    if a.traffic_json is None:
        a.traffic_json = os.path.join(ROOT, "profiles", f"traffic_{a.workload}.json")
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Dist:
    def __init__(self):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", rank=self.rank, world_size=self.world, device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(0)
        self.dev = torch.device("cuda", torch.cuda.current_device())

    def timed(self, step, steps, exchange=None):
        """barrier + sync, K steps, sync + barrier; returns the max-over-ranks seconds"""
        torch, dist = self.torch, self.dist
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
            if exchange is not None and self.world > 1:
                exchange()
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if self.world > 1:
            e = torch.tensor([el], device=self.dev, dtype=torch.float64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
        return el

    def total(self, *vals):
        if self.world == 1:
            return vals
        t = self.torch.tensor(list(vals), device=self.dev, dtype=self.torch.int64)
        self.dist.all_reduce(t)
        return tuple(int(x) for x in t.tolist())

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def roofline(kern, dom, alg_bytes, traffic_json, units_tag, n_units):
    """roofline object of the dominant kernel: algorithmic bytes per launch / its average launch time"""
    if dom not in kern:
        return None
    achieved = alg_bytes / (kern[dom][1] * 1e-3) / 1e9
    traffic = None
    try:
        with open(traffic_json) as f:
            tj = json.load(f)
        if tj.get("kernel") == dom and int(tj.get("n_units", tj.get("n_points", -1))) == n_units:
            traffic = tj.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "algorithmic_bytes_per_launch": int(alg_bytes),
            "avg_launch_ms": round(kern[dom][1], 5)}


def kernel_times(eng, names):
    kern = {}
    for name in names:
        launches, ms = eng.prof_get(name)
        if launches:
            kern[name] = (launches, ms / launches)
    return kern


# ---------------------------------------------------------------------------------------------
def run_c2(args, D, polygons=False):
    torch = D.torch
    from kart_amd import shard, synth
    from kart_amd.device import DiffPipeline
    from kart_amd.engine import Engine
    from kart_amd.schema import FieldMaps

    n = args.n
    t0 = time.time()
    if polygons:  # C3: 10 % edits (4 % geometry + 4 % attribute updates, 1 % del, 1 % ins)
        L = synth.polygons_layer(n, seed=synth.SEED + D.rank, pk0=shard.rank_pk_base(D.rank, n))
    else:
        L = synth.points_layer(n, seed=synth.SEED + D.rank, pk0=shard.rank_pk_base(D.rank, n))
    log(f"[rank {D.rank}] generated {n} {'polygons' if polygons else 'points'} in {time.time() - t0:.1f}s "
        f"(+{L.n_insert} ins, ~{L.n_update} upd, -{L.n_delete} del)")
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    eng = Engine(torch.cuda.current_device())
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    pipe = DiffPipeline(eng, L.base, L.target, L.base_blobs, L.target_blobs, maps, D.dev, ordered=not args.unordered)
    torch.cuda.synchronize()

    # ---- warmup + correctness of the resident pipeline against the generator's own counts ----
    for _ in range(max(1, args.warmup)):
        pipe.step()
    torch.cuda.synchronize()
    counts, delta, upd, masks, status = pipe.results()
    if not args.no_check:
        assert (counts["inserts"], counts["updates"], counts["deletes"]) == (L.n_insert, L.n_update, L.n_delete), counts
        assert not status.any(), "fielddiff status flags set"
    n_pairs = L.base.n + L.n_insert
    counts_t = torch.tensor([counts["inserts"], counts["updates"], counts["deletes"]], device=D.dev, dtype=torch.int64)
    gathered = [torch.empty_like(counts_t) for _ in range(D.world)]

    eng.prof_reset()
    eng.prof_select(None if args.time_all else ["k_join2"])
    eng.prof_enable(not args.no_events)
    elapsed = D.timed(pipe.step, args.steps, lambda: D.dist.all_gather(gathered, counts_t))
    eng.prof_enable(False)
    total_pairs, total_deltas = D.total(n_pairs, counts["deltas"])
    kern = kernel_times(eng, ("k_partition2", "k_join2", "k_place2", "k_fielddiff"))

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
    dom = max(kern, key=lambda k: kern[k][1]) if kern else None
    roof = roofline(kern, dom, alg.get(dom, 0), args.traffic_json, "n_points", n) if dom in alg else None
    cpu = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_c2(L, maps, args.cpu_seconds, "C3" if polygons else "C2")
    eng.close()
    return {
        "metric": METRIC,
        "value": round(total_pairs * args.steps / elapsed / 1e6, 2),
        "unit": "M feature-pairs/s",
        "n_gpus": D.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u64 (integer + fp64 compare)",
        "data": ("synthetic (seeded MULTIPOLYGON layer: reference blob/path encodings, synthetic OIDs; "
                 "blobs materialised for updated features only)") if polygons else
                "synthetic (seeded points layer: reference blob/path encodings, synthetic OIDs)",
        "config": {"workload": (f"C3: {n}-polygon int-PK layer per GPU, 10% edits (4% geometry + 4% attribute "
                                "updates, 1% del, 1% ins), two-commit diff + field diff") if polygons else
                               "C2: 10M-point int-PK layer per GPU, 1% upd/del/ins, two-commit diff + field diff",
                   "features_per_gpu": n, "pairs_per_step": total_pairs, "deltas_per_step": total_deltas,
                   "updates_per_step": counts["updates"],
                   "delta_order": "tile-grouped (same delta set)" if args.unordered else "key",
                   "parallelism": f"bucket-range shards x{D.world}"},
        "kernels_avg_ms": {k: round(v[1], 5) for k, v in kern.items()},
        "roofline": roof,
        "cpu_baseline": cpu,
    }


def cpu_baseline_c2(L, maps, seconds, tag="C2"):
    """oracle classify2 + fielddiff (sequential C, 1 core) on the same layer, repeated for ~N s"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle as O

    A, B = L.base, L.target
    t0 = time.perf_counter()
    reps = 0
    while True:
        delta, counts = O.classify2(A.key, A.oid, B.key, B.oid)
        upd = delta[(delta[:, 0] != O.NONE) & (delta[:, 1] != O.NONE)]
        O.fielddiff(*L.base_blobs, *L.target_blobs, upd, maps)
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    pairs = (A.n + L.n_insert) * reps
    return {"value": round(pairs / dt / 1e6, 3), "unit": "M feature-pairs/s", "cores": 1, "kind": "port",
            "sample": f"the full {tag} layer ({A.n + L.n_insert} pairs) x {reps} reps in {dt:.1f}s: oracle/kd_oracle.c "
                      f"classify2 + fielddiff, 1 thread"}


# ---------------------------------------------------------------------------------------------
def run_c5(args, D):
    import ctypes

    torch = D.torch
    from kart_amd import _native as N
    from kart_amd import synth
    from kart_amd.device import to_dev
    from kart_amd.engine import Engine

    n, bits = args.n, 20
    nb = bits // 2
    t0 = time.time()
    data, off, is_pt = synth.geometry_layer(n, seed=synth.SEED + D.rank)
    log(f"[rank {D.rank}] generated {n} geometries ({data.size / 1e9:.2f} GB) in {time.time() - t0:.1f}s")
    eng = Engine(torch.cuda.current_device())
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    d_data, d_off = to_dev(data, D.dev), to_dev(off, D.dev)
    g = N.KdBlobs()
    g.n, g.data, g.off, g.mem, g.size_hint = n, d_data.data_ptr(), d_off.data_ptr(), N.KD_MEM_DEVICE, 0
    match = torch.empty(n, dtype=torch.uint8, device=D.dev)
    enc = torch.empty(n * nb, dtype=torch.uint8, device=D.dev)
    ok = torch.empty(n, dtype=torch.uint8, device=D.dev)
    ovl = torch.empty(n, dtype=torch.uint8, device=D.dev)
    fe = (ctypes.c_double * 4)(*synth.C5_FILTER)
    q = (ctypes.c_double * 4)(synth.C5_FILTER[0], synth.C5_FILTER[2], synth.C5_FILTER[1], synth.C5_FILTER[3])
    L, ctx = eng.L, eng.ctx

    def step():
        N.check(L.kd_envelopes(ctx, ctypes.byref(g), fe, bits, match.data_ptr(), enc.data_ptr(), ok.data_ptr(),
                               N.KD_MEM_DEVICE, None), "kd_envelopes")
        N.check(L.kd_env_overlap(ctx, enc.data_ptr(), n, bits, q, ovl.data_ptr(), N.KD_MEM_DEVICE), "kd_env_overlap")

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    if not args.no_check:  # size-independent: an encoded envelope only where the indexer stores one
        assert not (ok.cpu().numpy().astype(bool) & (match.cpu().numpy() == 2)).any(), "enc_ok on a null geometry"
    eng.prof_reset()
    eng.prof_select(None if args.time_all else ["k_envelopes"])
    eng.prof_enable(not args.no_events)
    cnt = torch.zeros(1, dtype=torch.int64, device=D.dev)
    gathered = [torch.empty_like(cnt) for _ in range(D.world)]
    elapsed = D.timed(step, args.steps, lambda: D.dist.all_gather(gathered, cnt))
    eng.prof_enable(False)
    (total,) = D.total(n)
    kern = kernel_times(eng, ("k_envelopes", "k_env_overlap"))
    npt = int(is_pt.sum())
    # algorithmic bytes per k_envelopes launch: offsets (8 B) + GPKG header (8 B) + stored envelope
    # (32 B, polygons) or point WKB (21 B) read; match + enc_ok flags (2 B) + encoded envelope written
    alg = n * (8 + 8 + 2 + nb) + npt * 21 + (n - npt) * 32
    roof = roofline(kern, "k_envelopes", alg, args.traffic_json, "n_geoms", n)
    cpu = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from oracle import oracle as O

        m = min(n, 2_000_000)
        t0 = time.perf_counter()
        reps = 0
        while True:
            om, oe, okk, _ = O.envelope_batch(data[: int(off[m])], off[: m + 1], synth.C5_FILTER, bits)
            if reps == 0 and not args.no_check:  # the baseline's sample doubles as a bit-exact check
                assert np.array_equal(match[:m].cpu().numpy(), om), "k_envelopes match flags differ from the oracle"
                assert np.array_equal(ok[:m].cpu().numpy(), okk), "k_envelopes enc_ok differs from the oracle"
                assert np.array_equal(enc[: m * nb].cpu().numpy().reshape(m, nb), oe), "EnvelopeEncoder bytes differ"
                t0 = time.perf_counter()
            reps += 1
            if time.perf_counter() - t0 >= min(args.cpu_seconds, 5.0):
                break
        dt = time.perf_counter() - t0
        cpu = {"value": round(m * reps / dt / 1e6, 3), "unit": "M geometries/s", "cores": 1, "kind": "port",
               "sample": f"first {m} geometries of the same layer x {reps} reps in {dt:.1f}s: oracle/kd_oracle.c "
                         f"envelope batch (bbox test + index envelope + EnvelopeEncoder), 1 thread"}
    eng.close()
    return {
        "metric": METRIC,
        "value": round(total * args.steps / elapsed / 1e6, 2),
        "unit": "M geometries/s",
        "n_gpus": D.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64 (envelopes, EnvelopeEncoder) + u8",
        "data": "synthetic (seeded GPKG geometries: 30% points, 70% multipolygons, EPSG:4326)",
        "config": {"workload": f"C5 (scaled to {n} geometries per GPU): spatial-filter envelopes + "
                               "EnvelopeEncoder + encoded-envelope overlap",
                   "geoms_per_gpu": n, "points": npt, "bits": bits, "filter": list(synth.C5_FILTER),
                   "parallelism": f"independent shards x{D.world}"},
        "kernels_avg_ms": {k: round(v[1], 5) for k, v in kern.items()},
        "roofline": roof,
        "cpu_baseline": cpu,
    }


# ---------------------------------------------------------------------------------------------
def run_c6(args, D):
    """Writer formatting: hex WKB of every geometry of the C5 layer (kd_hex_encode,
    KD_HEX_GPKG_WKB), the formatting `kart diff -o json` applies per geometry value."""
    import ctypes

    torch = D.torch
    from kart_amd import _native as N
    from kart_amd import synth
    from kart_amd.device import to_dev
    from kart_amd.engine import Engine

    n = args.n
    t0 = time.time()
    data, off, is_pt = synth.geometry_layer(n, seed=synth.SEED + D.rank)
    nbytes = int(off[-1])
    log(f"[rank {D.rank}] generated {n} geometries ({nbytes / 1e9:.2f} GB) in {time.time() - t0:.1f}s")
    eng = Engine(torch.cuda.current_device())
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    d_data, d_off = to_dev(data, D.dev), to_dev(off, D.dev)
    g = N.KdBlobs()
    g.n, g.data, g.off, g.mem, g.size_hint = n, d_data.data_ptr(), d_off.data_ptr(), N.KD_MEM_DEVICE, 0
    hexbuf = torch.empty(2 * nbytes, dtype=torch.uint8, device=D.dev)
    start = torch.empty(n, dtype=torch.int32, device=D.dev)
    status = torch.empty(n, dtype=torch.uint8, device=D.dev)
    L, ctx = eng.L, eng.ctx

    def step():
        N.check(L.kd_hex_encode(ctx, ctypes.byref(g), N.KD_HEX_GPKG_WKB, hexbuf.data_ptr(), start.data_ptr(),
                                status.data_ptr(), N.KD_MEM_DEVICE), "kd_hex_encode")

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle as O

    if not args.no_check:  # every geometry is valid LE GPKG; sampled strings equal the oracle's
        assert int(status.max().item()) == 0, "kd_hex_encode flagged a valid geometry"
        st = start.cpu().numpy()
        for i in list(range(0, n, max(1, n // 2000))) + [n - 1]:
            o, e = int(off[i]), int(off[i + 1])
            got = hexbuf[2 * (o + int(st[i])): 2 * e].cpu().numpy().tobytes().decode()
            assert got == O.hex_wkb(data[o:e].tobytes()), f"hex WKB of geometry {i} differs from the oracle"
    eng.prof_reset()
    eng.prof_select(None if args.time_all else ["k_hex"])
    eng.prof_enable(not args.no_events)
    cnt = torch.zeros(1, dtype=torch.int64, device=D.dev)
    gathered = [torch.empty_like(cnt) for _ in range(D.world)]
    elapsed = D.timed(step, args.steps, lambda: D.dist.all_gather(gathered, cnt))
    eng.prof_enable(False)
    (total,) = D.total(n)
    kern = kernel_times(eng, ("k_hex", "k_wkb_start"))
    # algorithmic bytes per k_hex launch: the geometry arena read once, two hex chars written per byte
    alg = 3 * nbytes
    roof = roofline(kern, "k_hex", alg, args.traffic_json, "n_geoms", n)
    cpu = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline:
        m = min(n, 200_000)
        blobs = [data[int(off[i]):int(off[i + 1])].tobytes() for i in range(m)]
        t0 = time.perf_counter()
        reps = 0
        while True:
            for b in blobs:
                O.hex_wkb(b)
            reps += 1
            if time.perf_counter() - t0 >= min(args.cpu_seconds, 5.0):
                break
        dt = time.perf_counter() - t0
        cpu = {"value": round(m * reps / dt / 1e6, 3), "unit": "M geometries/s", "cores": 1, "kind": "port",
               "sample": f"first {m} geometries of the same layer x {reps} reps in {dt:.1f}s: oracle.hex_wkb "
                         f"(the reference's gpkg_geom_to_hex_wkb restated: slice + hexlify + upper), 1 thread"}
    eng.close()
    return {
        "metric": METRIC,
        "value": round(total * args.steps / elapsed / 1e6, 2),
        "unit": "M geometries/s",
        "n_gpus": D.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded GPKG geometries: 30% points, 70% multipolygons, EPSG:4326)",
        "config": {"workload": f"C6 (SURVEY 8f #2, {n} geometries per GPU): hex WKB of every geometry "
                               "(Geometry.to_hex_wkb for kart diff -o json)",
                   "geoms_per_gpu": n, "points": int(is_pt.sum()), "arena_bytes": nbytes,
                   "parallelism": f"independent shards x{D.world}"},
        "kernels_avg_ms": {k: round(v[1], 5) for k, v in kern.items()},
        "roofline": roof,
        "cpu_baseline": cpu,
    }


# ---------------------------------------------------------------------------------------------
def run_c4(args, D):
    torch = D.torch
    from kart_amd import synth
    from kart_amd.device import MergePipeline
    from kart_amd.engine import Engine

    n = args.n
    t0 = time.time()
    M = synth.table3_layers(n, seed=synth.SEED + D.rank)
    A, O_, T = M.ancestor, M.ours, M.theirs
    log(f"[rank {D.rank}] generated ancestor/ours/theirs {A.n}/{O_.n}/{T.n} string-pk rows in {time.time() - t0:.1f}s "
        f"({M.n_conflict} conflicts planned)")
    eng = Engine(torch.cuda.current_device())
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    pipe = MergePipeline(eng, A, O_, T, D.dev)
    for _ in range(max(1, args.warmup)):
        pipe.step()
    torch.cuda.synchronize()
    n_clean, conf, md = pipe.results()
    if not args.no_check:  # the generator's own plan (libgit2 rule over planned edits)
        assert conf.shape[0] == M.n_conflict, (conf.shape[0], M.n_conflict)
    eng.prof_reset()
    eng.prof_select(None if args.time_all else ["k_join2"])
    eng.prof_enable(not args.no_events)
    cnt = torch.zeros(1, dtype=torch.int64, device=D.dev)
    gathered = [torch.empty_like(cnt) for _ in range(D.world)]
    elapsed = D.timed(pipe.step, args.steps, lambda: D.dist.all_gather(gathered, cnt))
    eng.prof_enable(False)
    (total,) = D.total(A.n + O_.n + T.n)
    kern = kernel_times(eng, ("k_sorted3", "k_partition2", "k_join2", "k_place2", "k_resolve3"))
    nall = A.n + O_.n + T.n
    # classify3 = classify2(ours, theirs) + k_resolve3 over the paths where they differ.
    # Dominant kernel k_join2, algorithmic bytes per launch: every ours/theirs key + OID once (28 B),
    # every ours/theirs filename once (hash keys are verified against the names) and one 8-B record
    # per differing path
    _, io, it = np.intersect1d(O_.key, T.key, assume_unique=True, return_indices=True)
    n_cand = int(O_.n + T.n - 2 * io.size + np.count_nonzero((O_.oid[io] != T.oid[it]).any(axis=1)))
    alg = 28 * (O_.n + T.n) + int(O_.name.size + T.name.size) + 8 * n_cand
    roof = roofline(kern, "k_join2", alg, args.traffic_json, "n_rows", n)
    cpu = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from oracle import oracle as Orc

        t0 = time.perf_counter()
        reps = 0
        while True:
            oc, om, ocl = Orc.classify3(A.key, A.oid, O_.key, O_.oid, T.key, T.oid)
            if reps == 0 and not args.no_check:  # the baseline's run doubles as a bit-exact check
                key = lambda r: sorted(map(tuple, np.asarray(r).tolist()))
                assert key(conf) == key(oc), "classify3 conflicts differ from the oracle"
                assert key(md) == key(om), "classify3 merge deltas differ from the oracle"
                t0 = time.perf_counter()
            reps += 1
            if time.perf_counter() - t0 >= min(args.cpu_seconds, 10.0):
                break
        dt = time.perf_counter() - t0
        cpu = {"value": round(nall * reps / dt / 1e6, 3), "unit": "M entries/s", "cores": 1, "kind": "port",
               "sample": f"the full C4 layer ({nall} entries) x {reps} reps in {dt:.1f}s: oracle/kd_oracle.c classify3, "
                         f"1 thread"}
    eng.close()
    return {
        "metric": METRIC,
        "value": round(total * args.steps / elapsed / 1e6, 2),
        "unit": "M entries/s",
        "n_gpus": D.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u64 (integer)",
        "data": "synthetic (seeded string-PK table: MsgpackHashPathEncoder paths, synthetic OIDs)",
        "config": {"workload": f"C4: {n}-row string-PK table per GPU, three-way merge classification "
                               "(ancestor/ours/theirs join + libgit2 conflict rule)",
                   "rows_per_gpu": n, "entries_per_step": total, "conflicts": int(conf.shape[0]),
                   "merge_deltas": int(md.shape[0]), "differing_paths": n_cand,
                   "parallelism": f"independent shards x{D.world}"},
        "kernels_avg_ms": {k: round(v[1], 5) for k, v in kern.items()},
        "roofline": roof,
        "cpu_baseline": cpu,
    }


def main():
    args = parse()
    D = Dist()
    out = {"c2": run_c2, "c3": lambda a, d: run_c2(a, d, polygons=True), "c4": run_c4,
           "c5": run_c5, "c6": run_c6}[args.workload](args, D)
    if D.rank == 0:
        print(json.dumps(out), flush=True)
    D.close()


if __name__ == "__main__":
    main()
