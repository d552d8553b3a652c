"""The reference's own diff path, timed in the build container (where /root/reference exists):
`Dataset3.diff` -> `RichBaseDataset.diff_feature` (kart/rich_base_dataset.py:205-300) consumed
into the DeltaDiff, then every update's old and new feature decoded (`Dataset3.get_feature`,
kart/dataset3.py:185-223) and its fields compared with Python `==` (the text writer's rule,
kart/text_diff_writer.py:135-145) — over the same repositories scripts/e2e_repo_bench.py builds
for the drop-in (N point features, a second commit with the given update / delete / insert
fractions).

MEASUREMENT ONLY, build container only: the reference's hot-path modules are imported through
tests/golden/refshim.py (stubbed pygit2 / osgeo, libgit2's tree diff stood in for by `git diff-tree`
— the same algorithm, in C); nothing here runs on the GPU box.  Object-store I/O is excluded as in
BASELINE.md: a first pass reads every tree and blob the diff touches through the shim's caches, the
timed pass then runs on warm caches (the tree diff itself is the `git diff-tree` subprocess, timed).
usage: python3 -B scripts/ref_path_bench.py --n 1000000 [--edits 0.08,0.01,0.01] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.dont_write_bytecode = True

DS = "nz_points"
_NULL = object()


def run(ds_a, ds_b):
    """the reference path: the feature DeltaDiff (lazy deltas), then each update's values decoded and
    compared (changed-field lists, as TextDiffWriter.write_feature_delta computes them)"""
    t0 = time.perf_counter()
    dd = ds_a.diff(ds_b)
    fdiff = dd.get("feature")
    deltas = list(fdiff.items()) if fdiff is not None else []
    t1 = time.perf_counter()
    changed = 0
    n_upd = 0
    for _, d in deltas:
        if d.type != "update":
            continue
        n_upd += 1
        old, new = d.old_value, d.new_value
        for k in list(old.keys()) + [k for k in new.keys() if k not in old]:
            if k.startswith("__"):
                continue
            if old.get(k, _NULL) != new.get(k, _NULL):
                changed += 1
    t2 = time.perf_counter()
    counts = fdiff.type_counts() if fdiff is not None else {}
    return {"classify_s": t1 - t0, "decode_compare_s": t2 - t1, "total_s": t2 - t0, "deltas": len(deltas),
            "updates": n_upd, "changed_fields": changed, "counts": counts}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--edits", default="0.08,0.01,0.01")
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import e2e_repo_bench as E
    import refshim

    edits = tuple(float(x) for x in a.edits.split(","))
    gitdir = f"/tmp/kart_ref_{a.n}_{a.edits.replace(',', '_')}.git"
    if not os.path.isdir(gitdir):
        t0 = time.perf_counter()
        E.build_parallel(gitdir, a.n, procs=a.procs, edits=edits)
        print(f"built {gitdir} in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    refshim.load_reference()
    repo = refshim.GitRepo(gitdir, index_file=f"/tmp/kart_ref_index_{os.getpid()}")
    ds_a = refshim.dataset3(repo, "main^", DS)
    ds_b = refshim.dataset3(repo, "main", DS)
    warm = run(ds_a, ds_b)  # fills the shim's tree and blob caches (object-store I/O excluded)
    print(f"warm-up pass {warm['total_s']:.1f} s", file=sys.stderr, flush=True)
    runs = [run(ds_a, ds_b) for _ in range(a.reps)]
    best = min(runs, key=lambda r: r["total_s"])
    pairs = a.n + int(a.n * edits[2])  # union pks
    out = {"n": a.n, "edits_update_delete_insert": list(edits), "feature_pairs": pairs,
           "what": "the reference's Dataset3.diff (diff_feature generator consumed into the DeltaDiff) + "
                   "get_feature of both sides of every update + the Python == field compare, 1 thread, warm "
                   "object caches; libgit2's tree diff by `git diff-tree -r` (C)",
           "classify_s": round(best["classify_s"], 3), "decode_compare_s": round(best["decode_compare_s"], 3),
           "total_s": round(best["total_s"], 3),
           "feature_pairs_per_s": round(pairs / best["total_s"], 1),
           "deltas_per_s": round(best["deltas"] / best["total_s"], 1),
           "deltas": best["deltas"], "updates": best["updates"], "changed_fields": best["changed_fields"],
           "counts": best["counts"], "reps": [round(r["total_s"], 3) for r in runs], "cores": 1}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
