"""Experiment: does running two halves of the C3 layer on two streams (two contexts on one GPU)
overlap k_join2 (bandwidth) with k_fielddiff (latency)?  Prints sequential vs concurrent step times."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from kart_amd import synth
from kart_amd.engine import Engine
from kart_amd.device import DiffPipeline
from kart_amd.schema import FieldMaps

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
parts = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n_pks = n + n // 100
engs, pipes = [], []
for r in range(parts):
    lo, hi = synth.shard_pk_range(r, parts, n_pks)
    L = synth.polygons_layer(n, lo=lo, hi=hi)
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    e = Engine(0)
    engs.append(e)
    pipes.append(DiffPipeline(e, L.base, L.target, L.base_blobs, L.target_blobs, maps))
    del L
for p in pipes:
    p.step()
for e in engs:
    e.sync()
K = 10
def run(concurrent):
    for e in engs: e.device_sync()
    t0 = time.perf_counter()
    for _ in range(K):
        if concurrent:
            for p in pipes: p.step()
        else:
            for p, e in zip(pipes, engs):
                p.step(); e.sync()
    for e in engs: e.device_sync()
    return (time.perf_counter() - t0) / K * 1e3
for _ in range(2):
    print("sequential ms/step", round(run(False), 3), "concurrent ms/step", round(run(True), 3), flush=True)
