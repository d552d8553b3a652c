#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of bench.py runs (profile_gpu.sh layout) per kernel.

usage: pmc_summary.py OUT_DIR [--n POINTS] [--kernel k_join2] [--write-traffic profiles/traffic_c2.json]
Reads OUT_DIR/trace/run_kernel_stats.csv and every OUT_DIR/*/run_counter_collection.csv; prints
per-kernel mean counter values per dispatch.  HBM traffic per launch of --kernel =
2 x FETCH_SIZE (gfx950 tallies wide streaming reads at half their bytes, MI355X_MICROARCH.md
"HBM") + WRITE_SIZE, both reported by rocprofv3 in KB.
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys


def counters(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> ctr -> sum
    with open(path) as f:
        for r in csv.DictReader(f):
            per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--kernel", default="k_join2")
    ap.add_argument("--write-traffic")
    a = ap.parse_args()
    allc = collections.defaultdict(dict)
    for p in sorted(glob.glob(os.path.join(a.out, "*", "run_counter_collection.csv"))):
        for k, cs in counters(p).items():
            allc[k].update(cs)
    stats = {}
    sp = os.path.join(a.out, "trace", "run_kernel_stats.csv")
    if os.path.exists(sp):
        with open(sp) as f:
            for r in csv.DictReader(f):
                stats[r["Name"]] = float(r["AverageNs"])
    for k in sorted(set(allc) | set(stats)):
        short = k.split("(")[0]
        print(f"{short:40s} avg_ns={stats.get(k, float('nan')):10.0f} " +
              " ".join(f"{c}={v:.4g}" for c, v in sorted(allc.get(k, {}).items())))
    if a.write_traffic:
        hit = [k for k in allc if a.kernel in k]
        if not hit:
            sys.exit(f"no counters for {a.kernel}")
        cs = allc[hit[0]]
        fetch_kb, write_kb = cs.get("FETCH_SIZE"), cs.get("WRITE_SIZE")
        if fetch_kb is None or write_kb is None:
            sys.exit("FETCH_SIZE / WRITE_SIZE missing")
        tj = {"kernel": a.kernel, "n_units": a.n, "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
              "hbm_bytes_per_launch": int(round((2 * fetch_kb + write_kb) * 1024)),
              "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH doubled (gfx950)"}
        with open(a.write_traffic, "w") as f:
            json.dump(tj, f, indent=1)
        print(json.dumps(tj))


if __name__ == "__main__":
    main()
