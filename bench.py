#!/usr/bin/env python3
"""Bench: device-resident two-way feature diff (classify2 + field diff) on MI355X.

Workload (BASELINE.json configs[1], "C2"): a synthetic 10M-point int-PK layer per GPU with seeded
1% updates / 1% deletes / 1% inserts (kart_amd.synth.points_layer; the reference's feature blob
and path encodings, synthetic OIDs).  One *step* = one full pass of the hot path over that layer:
merge-path join + OID compare + key-ordered compaction of the delta set (k_partition2, k_join2,
k_place2), then the msgpack field decode + Python-== column compare of every
update (k_fielddiff) — all on the device, inputs resident in HBM before the timed region.

Multi-GPU (torch.distributed, one process per GPU, RCCL): each rank owns a disjoint dataset3
path-bucket range (its own 10M-point shard; weak scaling); the only collective is the all-gather
of per-rank delta counts each step.  value = feature pairs (union PKs) of all ranks / max-rank time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--n POINTS] [--no-cpu-baseline]
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
    ap.add_argument("--n", type=int, default=10_000_000, help="points per GPU (C2: 10M)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--unordered", action="store_true",
                    help="tile-grouped delta list (per-tile atomic appends, no k_place2); default: key order")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-check", action="store_true", help="profiling variants only: skip the count check")
    ap.add_argument("--no-events", action="store_true", help="no per-kernel HIP events in the timed region")
    ap.add_argument("--time-all", action="store_true",
                    help="HIP events around every kernel of a step (default: only the dominant k_join2, "
                         "so the events do not inflate the step time)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_c2.json"))
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from kart_amd import shard, synth
    from kart_amd.device import DiffPipeline
    from kart_amd.engine import Engine
    from kart_amd.schema import FieldMaps

    n = args.n
    t0 = time.time()
    pk0 = shard.rank_pk_base(rank, n)
    L = synth.points_layer(n, seed=synth.SEED + rank, pk0=pk0)
    log(f"[rank {rank}] generated {n} points in {time.time() - t0:.1f}s "
        f"(+{L.n_insert} ins, ~{L.n_update} upd, -{L.n_delete} del)")
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    eng = Engine(torch.cuda.current_device())
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    pipe = DiffPipeline(eng, L.base, L.target, L.base_blobs, L.target_blobs, maps, dev, ordered=not args.unordered)
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
    counts_t = torch.tensor([counts["inserts"], counts["updates"], counts["deletes"]], device=dev, dtype=torch.int64)

    # ---- timed region ----
    eng.prof_reset()
    eng.prof_select(None if args.time_all else ["k_join2"])
    eng.prof_enable(not args.no_events)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    gathered = None
    for _ in range(args.steps):
        pipe.step()
        if world > 1:
            gathered = [torch.empty_like(counts_t) for _ in range(world)]
            dist.all_gather(gathered, counts_t)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    eng.prof_enable(False)
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        tot = torch.tensor([n_pairs, counts["deltas"]], device=dev, dtype=torch.int64)
        dist.all_reduce(tot)
        total_pairs, total_deltas = int(tot[0].item()), int(tot[1].item())
    else:
        total_pairs, total_deltas = n_pairs, counts["deltas"]

    kern = {}
    for name in ("k_partition2", "k_join2", "k_place2", "k_fielddiff"):  # kernels of a step
        launches, ms = eng.prof_get(name)
        if launches:
            kern[name] = (launches, ms / launches)
    ms_per_step = elapsed / args.steps * 1e3
    value = total_pairs * args.steps / elapsed / 1e6

    # ---- roofline of the dominant kernel (algorithmic bytes per launch) ----
    nA, nB = L.base.n, L.target.n
    ob_off, nb_off = L.base_blobs[1], L.target_blobs[1]
    upd_bytes = int((ob_off[upd[:, 0] + 1] - ob_off[upd[:, 0]]).sum() + (nb_off[upd[:, 1] + 1] - nb_off[upd[:, 1]]).sum())
    alg = {
        "k_join2": 28 * (nA + nB) + 8 * counts["deltas"] + 8 * counts["updates"],
        "k_fielddiff": upd_bytes + counts["updates"] * (8 + 8 * maps.words + 1),
    }
    dom = max(kern, key=lambda k: kern[k][1]) if kern else None
    roof = None
    if dom in alg:
        achieved = alg[dom] / (kern[dom][1] * 1e-3) / 1e9
        traffic = None
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("kernel") == dom and int(tj.get("n_points", -1)) == n:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": alg[dom], "avg_launch_ms": round(kern[dom][1], 5)}

    # ---- CPU baseline: the oracle (C port, 1 thread) on a bounded sample of the same workload ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(L, maps, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "M feature-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/u64 (integer + fp64 compare)",
            "data": "synthetic (seeded points layer: reference blob/path encodings, synthetic OIDs)",
            "config": {"workload": "C2: 10M-point int-PK layer per GPU, 1% upd/del/ins, two-commit diff + field diff",
                       "points_per_gpu": n, "pairs_per_step": total_pairs, "deltas_per_step": total_deltas,
                       "delta_order": "tile-grouped (same delta set)" if args.unordered else "key",
                       "parallelism": f"bucket-range shards x{world}"},
            "kernels_avg_ms": {k: round(v[1], 5) for k, v in kern.items()},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


def cpu_baseline(L, maps, seconds):
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
            "sample": f"full C2 layer ({A.n + L.n_insert} pairs) x {reps} reps in {dt:.1f}s: oracle/kd_oracle.c "
                      f"classify2 + fielddiff, 1 thread"}


if __name__ == "__main__":
    main()
