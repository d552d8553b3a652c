#!/usr/bin/env python3
"""kd_sort_side_into on C3-shaped sides (git walk order), per-kernel times — and A/B of probe builds.

    python scripts/sort_bench.py [--n 100000000] [--steps 10] [--libs kart_amd/libkartdiff.so,kart_amd/probe/x.so]

Every library is loaded side by side in this one process (its own context and buffers); the data
is generated once.  Each run is checked bit-exact (sorted keys, OIDs, order) unless --no-check
(probe builds that skip work give wrong results on purpose).  One JSON line per library."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kart_amd import synth  # noqa: E402

KERNELS = ("k_rs_bits", "k_sort_hist", "k_sort_scan", "k_sort_pass", "k_gather_oid", "k_check_sorted")


def bind(path):
    L = ctypes.CDLL(path)
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    sig = {
        "kd_init": [ctypes.c_int, ctypes.POINTER(vp)],
        "kd_malloc": [vp, u64, ctypes.POINTER(vp)],
        "kd_memcpy": [vp, vp, vp, u64, ctypes.c_uint32],
        "kd_sync": [vp],
        "kd_sort_side_into": [vp, vp, vp, vp, vp, vp, u64, vp, vp],  # ..., d_dup, info (kd_keys_info*)
        "kd_prof_enable": [vp, ctypes.c_int],
        "kd_prof_select": [vp, ctypes.c_char_p],
        "kd_prof_get": [vp, ctypes.c_char_p, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_double)],
        "kd_prof_reset": [vp],
        "kd_last_error": [],
    }
    for k, a in sig.items():
        f = getattr(L, k)
        f.argtypes = a
        f.restype = ctypes.c_char_p if k == "kd_last_error" else ctypes.c_int
    return L


def chk(L, rc, what):
    if rc:
        raise RuntimeError(f"{what}: {rc} {L.kd_last_error().decode()}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--libs", default=os.path.join(ROOT, "kart_amd", "libkartdiff.so"))
    ap.add_argument("--kind", default="c3", choices=["c3", "rand64"])
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    t0 = time.time()
    if a.kind == "c3":
        keys = synth._int_keys(np.arange(a.n, dtype=np.int64))
        perm = synth.walk_perm(keys)
    else:
        rng = np.random.default_rng(1)
        keys = np.unique(rng.integers(0, 2**64 - 1, size=a.n + a.n // 16, dtype=np.uint64))[: a.n]
        perm = rng.permutation(keys.shape[0])
    n = keys.shape[0]
    oids = synth.synth_oids(np.arange(n), 0)
    wk, wo = np.ascontiguousarray(keys[perm]), np.ascontiguousarray(oids[perm])
    print(f"# data: {n} keys ({a.kind}) in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    for path in a.libs.split(","):
        L = bind(path)
        ctx = ctypes.c_void_p()
        chk(L, L.kd_init(0, ctypes.byref(ctx)), "kd_init")
        bufs = {}
        for name, nb in (("wk", 8 * n), ("wo", 20 * n), ("ko", 8 * n), ("oo", 20 * n), ("ord", 4 * n)):
            p = ctypes.c_void_p()
            chk(L, L.kd_malloc(ctx, nb, ctypes.byref(p)), "kd_malloc")
            bufs[name] = p.value
        chk(L, L.kd_memcpy(ctx, bufs["wk"], wk.ctypes.data, 8 * n, 1), "H2D")
        chk(L, L.kd_memcpy(ctx, bufs["wo"], wo.ctypes.data, 20 * n, 1), "H2D")

        def sort():
            chk(L, L.kd_sort_side_into(ctx, bufs["wk"], bufs["wo"], bufs["ko"], bufs["oo"], bufs["ord"], n, None, None),
                "kd_sort_side_into")

        sort()
        chk(L, L.kd_sync(ctx), "sync")
        ok = None
        if not a.no_check:
            ko = np.empty(n, np.uint64)
            oo = np.empty((n, 20), np.uint8)
            od = np.empty(n, np.uint32)
            chk(L, L.kd_memcpy(ctx, ko.ctypes.data, bufs["ko"], 8 * n, 2), "D2H")
            chk(L, L.kd_memcpy(ctx, oo.ctypes.data, bufs["oo"], 20 * n, 2), "D2H")
            chk(L, L.kd_memcpy(ctx, od.ctypes.data, bufs["ord"], 4 * n, 2), "D2H")
            chk(L, L.kd_sync(ctx), "sync")
            # sorted, and each output row is the input row the order names (ties keep input order);
            # walk-order keys are not ascending in pk, so the expectation is not `keys` itself
            srt = bool(np.all(ko[1:] > ko[:-1]) or np.all((ko[1:] > ko[:-1]) | ((ko[1:] == ko[:-1]) & (od[1:] > od[:-1]))))
            ok = bool(srt and np.array_equal(ko, wk[od]) and np.array_equal(oo, wo[od])
                      and np.array_equal(np.sort(od), np.arange(n, dtype=np.uint32)))
        # wall time of K sorts, then per-kernel event times of K more
        chk(L, L.kd_sync(ctx), "sync")
        t0 = time.perf_counter()
        for _ in range(a.steps):
            sort()
        chk(L, L.kd_sync(ctx), "sync")
        wall = (time.perf_counter() - t0) / a.steps * 1e3
        chk(L, L.kd_prof_reset(ctx), "prof")
        chk(L, L.kd_prof_select(ctx, None), "prof")
        chk(L, L.kd_prof_enable(ctx, 1), "prof")
        for _ in range(a.steps):
            sort()
        chk(L, L.kd_sync(ctx), "sync")
        chk(L, L.kd_prof_enable(ctx, 0), "prof")
        kern = {}
        for k in KERNELS:
            c, ms = ctypes.c_uint64(), ctypes.c_double()
            chk(L, L.kd_prof_get(ctx, k.encode(), ctypes.byref(c), ctypes.byref(ms)), "prof_get")
            if c.value:
                kern[k] = {"per_sort_ms": round(ms.value / a.steps, 4), "launches_per_sort": c.value // a.steps}
        print(json.dumps({"lib": os.path.relpath(path, ROOT), "n": n, "kind": a.kind, "ok": ok,
                          "wall_ms_per_sort": round(wall, 4), "kernels": kern}), flush=True)


if __name__ == "__main__":
    main()
