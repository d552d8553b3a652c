"""Host walk benchmark (BASELINE.md "host walk cost"): a Kart-shaped repository of
N features (IntPathEncoder paths, 64 branches x 4 levels, one blob per feature) with a second commit
editing 1% of them, then

  git ls-tree -r   of the feature tree (the 0.67 s / 1M baseline BASELINE.md quotes),
  kd_walk          the same listing natively (1 thread, all threads),
  kd_walk pruned   the two commits' changed leaves only (subtree-OID pruning),
  kd_odb_read_batch  the changed blobs, and the key packing of the full listing,

on the fast-import pack and again after `git repack -adf` (trees then delta-chained).  Prints one
JSON object.  CPU only.  usage: python scripts/walk_bench.py [--n 1000000] [--out FILE]
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kart_amd import packing, synth  # noqa: E402
from kart_amd.odb import ObjectDB  # noqa: E402

FEAT = "layer/.table-dataset/feature"


def build(gitdir, n, seed=5):
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    pk = np.arange(1, n + 1, dtype=np.int64)
    arena, off = synth.int_pk_paths(pk)
    paths = [arena[int(off[i]):int(off[i + 1])].tobytes() for i in range(n)]
    rng = np.random.default_rng(seed)
    out = [b"commit refs/heads/c0\ncommitter t <t@t> 1600000000 +0000\ndata 1\nx\n"]
    for i in range(n):
        d = b"\x92\xd9(%040d\x94\xce%08x" % (i, i) + b"v0" * 40
        out.append(b"M 100644 inline %s/%s\ndata %d\n%s\n" % (FEAT.encode(), paths[i], len(d), d))
    out.append(b"\n")
    edit = rng.choice(n, n // 100, replace=False)
    out.append(b"commit refs/heads/c1\ncommitter t <t@t> 1600000001 +0000\ndata 1\ny\nfrom refs/heads/c0\n")
    for i in edit.tolist():
        d = b"\x92\xd9(%040d\x94\xce%08x" % (i, i) + b"v1" * 40
        out.append(b"M 100644 inline %s/%s\ndata %d\n%s\n" % (FEAT.encode(), paths[i], len(d), d))
    out.append(b"\n")
    subprocess.run(["git", "fast-import", "--quiet"], input=b"".join(out), env=dict(os.environ, GIT_DIR=gitdir),
                   check=True)


def best(fn, reps=3):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), r


def measure(gitdir, label):
    rev = {s: subprocess.run(["git", "--git-dir", gitdir, "rev-parse", s], capture_output=True, check=True)
           .stdout.decode().strip() for s in ("c0", "c1")}
    t_git, raw = best(lambda: subprocess.run(["git", "--git-dir", gitdir, "ls-tree", "-r", "-z", "c0", "--", FEAT],
                                             capture_output=True, check=True).stdout, reps=2)
    n_git = raw.count(b"\0")
    db = ObjectDB(gitdir)
    nt = os.cpu_count() or 1
    t1, (lv,) = best(lambda: db.walk([rev["c0"]], FEAT, threads=1))
    tn, (lv,) = best(lambda: db.walk([rev["c0"]], FEAT, threads=0))
    assert lv.n == n_git
    tp, (pa, pb) = best(lambda: db.walk([rev["c0"], rev["c1"]], FEAT, compare=(0, 1)))
    tb, (data, off, st) = best(lambda: db.read_batch(pb.oids))
    assert not st.any()
    enc = packing.PathEncoding.from_dict({"scheme": "int", "branches": 64, "levels": 4, "encoding": "base64"})
    tk, _ = best(lambda: packing.parse_keys(lv.paths, lv.off, enc))
    return {
        "store": label,
        "entries": int(lv.n),
        "git_ls_tree_r_s": round(t_git, 4),
        "kd_walk_1thread_s": round(t1, 4),
        "kd_walk_s": round(tn, 4),
        "kd_walk_threads": min(nt, 16),
        "speedup_vs_git": round(t_git / tn, 1),
        "pruned_walk_s": round(tp, 5),
        "pruned_leaves": [int(pa.n), int(pb.n)],
        "read_batch_s": round(tb, 5),
        "read_batch_blobs": int(pb.n),
        "read_batch_MBps": round(int(off[-1]) / tb / 1e6, 1),
        "pack_keys_s": round(tk, 4),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--repo", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    gitdir = a.repo or f"/tmp/kart_walk_{a.n}.git"
    if not os.path.isdir(gitdir):
        t0 = time.perf_counter()
        build(gitdir, a.n)
        print(f"built {gitdir} in {time.perf_counter() - t0:.1f} s", file=sys.stderr)
    res = {"n": a.n, "cpus": os.cpu_count(), "runs": [measure(gitdir, "fast-import pack")]}
    subprocess.run(["git", "--git-dir", gitdir, "repack", "-adfq", "--depth=50", "--window=10"], check=True)
    res["runs"].append(measure(gitdir, "repacked (-adf --depth=50)"))
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
