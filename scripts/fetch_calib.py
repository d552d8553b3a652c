#!/usr/bin/env python3
"""FETCH_SIZE calibration summary (scripts/fetch_calib.hip under rocprofv3 --pmc FETCH_SIZE).

usage: fetch_calib.py PATTERNS.jsonl PMC_DIR [--out calib.json]   (PMC_DIR: the rocprofv3 -d directory)
For each pattern: FETCH_SIZE (rocprofv3 reports KB) in bytes, and its ratio to the requested bytes
and to the distinct 32 / 64 / 128-B blocks the pattern touched."""
import argparse
import collections
import csv
import glob
import json
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("patterns")
    ap.add_argument("counters")
    ap.add_argument("--out")
    a = ap.parse_args()
    pats = [json.loads(ln) for ln in open(a.patterns) if ln.startswith("{")]
    # rocprofv3 names the template instances all "k_pat": they run in pattern order, so the k-th
    # k_pat dispatch is pattern k
    per = collections.defaultdict(float)
    for path in glob.glob(os.path.join(a.counters, "**", "run_counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if re.match(r"k_pat\b", r["Kernel_Name"]) and r["Counter_Name"] == "FETCH_SIZE":
                    per[int(r["Dispatch_Id"])] += float(r["Counter_Value"]) * 1024
    fetch = {i: per[d] for i, d in enumerate(sorted(per))}
    out = []
    for i, p in enumerate(pats):
        fb = fetch.get(i)
        row = dict(p, fetch_size_bytes=fb)
        if fb:
            for k in ("bytes", "b32", "b64", "b128"):
                row[f"fetch_over_{k}"] = round(fb / p[k], 4)
        out.append(row)
        print(json.dumps(row))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
