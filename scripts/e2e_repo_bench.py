"""End-to-end `kart diff HEAD^ HEAD` of a Kart-shaped git repository through the drop-in path:
object store + walk (gitsource) -> key packing -> kd_diff2 -> Delta objects -> batched blob read +
kd_fielddiff, timed stage by stage, next to `git diff-tree -r` (the tree diff libgit2 does for the
reference).  The reference's own Python path is measured apart, in the build container
(scripts/ref_path_bench.py, on repositories built by this script's build_parallel).

The repository: N points features (IntPathEncoder paths, the reference's feature blob encoding,
EPSG:4326), a second commit with --edits update / delete / insert fractions.  Prints one JSON object.
usage: python scripts/e2e_repo_bench.py [--n 1000000] [--edits 0.08,0.01,0.01] [--out FILE]   (GPU needed)
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kart_amd import synth  # noqa: E402
from kart_amd.schema import Legend  # noqa: E402

DS = "nz_points"


def _import_blobs(args):
    """one worker: write a chunk of blobs with its own `git fast-import` (one pack) and return their
    object ids (sha1 of the loose-object header + content, as git names them)"""
    gitdir, data, off = args
    n = off.shape[0] - 1
    raw = data.tobytes()
    ids = bytearray(20 * n)
    parts = []
    for i in range(n):
        b = raw[int(off[i]):int(off[i + 1])]
        ids[20 * i:20 * i + 20] = hashlib.sha1(b"blob %d\0" % len(b) + b).digest()
        parts.append(b"blob\ndata %d\n%s\n" % (len(b), b))
    subprocess.run(["git", "-c", "fastimport.unpackLimit=0", "fast-import", "--quiet"], input=b"".join(parts),
                   env=dict(os.environ, GIT_DIR=gitdir), check=True)
    return bytes(ids)


def _blob_ids(gitdir, data, off, procs):
    """all blobs of the arena into the repository, `procs` fast-imports in parallel"""
    from multiprocessing import Pool

    n = off.shape[0] - 1
    cuts = np.linspace(0, n, procs + 1).astype(np.int64)
    jobs = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        lo, hi = int(off[a]), int(off[b])
        jobs.append((gitdir, data[lo:hi], (off[a:b + 1] - np.uint64(lo)).astype(np.uint64)))
    with Pool(procs) as pool:
        ids = pool.map(_import_blobs, jobs)
    return np.frombuffer(b"".join(ids), np.uint8).reshape(n, 20)


def build_parallel(gitdir, n, seed=3, procs=16, edits=(0.01, 0.01, 0.01)):
    """the same repository as build(), with the blobs written by parallel fast-imports (packs of
    blobs) and the two commits by one fast-import referencing them by id: for 10M features.
    edits = (update, delete, insert) fractions of n"""
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    legend = Legend(["c-fid"], [c["id"] for c in synth.POINT_SCHEMA[1:]])
    lh = legend.hexhash()
    rng = np.random.default_rng(seed)
    pks = np.arange(1, n + 1, dtype=np.int64)
    perm = rng.permutation(n)
    ku, kd, ki = (int(n * f) for f in edits)
    upd, dele = np.sort(perm[:ku]), np.sort(perm[ku:ku + kd])
    ins = np.arange(n + 1, n + 1 + ki, dtype=np.int64)
    k = kd
    inner = f"{DS}/.table-dataset"
    meta = _meta(inner, lh, legend)
    t0 = time.perf_counter()
    feats = []
    for p, ver in ((pks, 0), (pks[upd], 1), (ins, 2)):
        data, boff = synth.point_blobs(p, np.full(p.shape[0], ver, np.uint64), lh)
        feats.append((p, _blob_ids(gitdir, data, boff, procs)))
        print(f"  blobs of version {ver}: {p.shape[0]} in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)

    def m_lines(p, ids):
        arena, off = synth.int_pk_paths(p)
        hexes = ids.tobytes().hex()
        pre = f"M 100644 ".encode()
        return [pre + hexes[40 * i:40 * i + 40].encode() + b" %s/feature/%s\n" % (
            inner.encode(), arena[int(off[i]):int(off[i + 1])].tobytes()) for i in range(p.shape[0])]

    lines = [b"commit refs/heads/main\ncommitter t <t@t> 1600000000 +0000\ndata 1\nx\n"]
    for path, d in meta.items():
        lines.append(b"M 100644 inline %s\ndata %d\n%s\n" % (path.encode(), len(d), d))
    lines += m_lines(*feats[0])
    lines.append(b"\ncommit refs/heads/main\ncommitter t <t@t> 1600000001 +0000\ndata 1\ny\n")
    lines += m_lines(*feats[1])
    lines += m_lines(*feats[2])
    arena, off = synth.int_pk_paths(pks[dele])
    for i in range(k):
        lines.append(b"D %s/feature/%s\n" % (inner.encode(), arena[int(off[i]):int(off[i + 1])].tobytes()))
    lines.append(b"\n")
    print(f"  tree stream built in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    import threading

    done = threading.Event()

    def heartbeat():  # fast-import builds 10M-entry trees silently for minutes
        while not done.wait(30):
            print(f"  fast-import running, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    try:
        subprocess.run(["git", "fast-import", "--quiet"], input=b"".join(lines), env=dict(os.environ, GIT_DIR=gitdir),
                       check=True)
    finally:
        done.set()
    print(f"  commits written in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    return ku + kd + ki


def _subtree_import(args):
    """one worker: the entries of one two-level path prefix ('A/B/') as a commit of their own whose
    root tree is that prefix's subtree; returns (prefix, tree id)"""
    gitdir, ref, prefix, pks, ids = args
    arena, off = synth.int_pk_paths(pks)
    hexes = ids.tobytes().hex()
    lines = [b"commit %s\ncommitter t <t@t> 1600000000 +0000\ndata 1\ns\n" % ref.encode()]
    for i in range(pks.shape[0]):
        path = arena[int(off[i]):int(off[i + 1])].tobytes()
        assert path[:4] == prefix
        lines.append(b"M 100644 %s %s\n" % (hexes[40 * i:40 * i + 40].encode(), path[4:]))
    lines.append(b"\n")
    env = dict(os.environ, GIT_DIR=gitdir)
    subprocess.run(["git", "fast-import", "--quiet"], input=b"".join(lines), env=env, check=True)
    tree = subprocess.run(["git", "rev-parse", ref + "^{tree}"], env=env, check=True, capture_output=True).stdout.strip()
    return prefix, tree.decode()


def build_sharded(gitdir, n, seed=3, procs=16, edits=(0.08, 0.01, 0.01)):
    """build_parallel for tens of millions of features: the blobs by parallel fast-imports as there,
    and each commit's feature tree too — one fast-import per two-level path prefix (its subtree, as a
    commit of its own; ~4k leaf trees each), the commits then placing those subtrees by id (M 040000).
    One fast-import building a 10M-entry tree alone took ~240 s."""
    from multiprocessing import Pool

    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    legend = Legend(["c-fid"], [c["id"] for c in synth.POINT_SCHEMA[1:]])
    lh = legend.hexhash()
    rng = np.random.default_rng(seed)
    pks = np.arange(1, n + 1, dtype=np.int64)
    perm = rng.permutation(n)
    ku, kd, ki = (int(n * f) for f in edits)
    upd, dele = np.sort(perm[:ku]), np.sort(perm[ku:ku + kd])
    ins = np.arange(n + 1, n + 1 + ki, dtype=np.int64)
    inner = f"{DS}/.table-dataset"
    meta = _meta(inner, lh, legend)
    t0 = time.perf_counter()
    ids = []
    for p, ver in ((pks, 0), (pks[upd], 1), (ins, 2)):
        data, boff = synth.point_blobs(p, np.full(p.shape[0], ver, np.uint64), lh)
        ids.append(_blob_ids(gitdir, data, boff, procs))
        del data, boff
        print(f"  blobs of version {ver}: {p.shape[0]} in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    # the two commits' entries: (pks ascending, blob ids)
    keep = np.ones(n, bool)
    keep[dele] = False
    ids2 = ids[0].copy()
    ids2[upd] = ids[1]
    c1 = (pks, ids[0])
    c2 = (np.concatenate([pks[keep], ins]), np.concatenate([ids2[keep], ids[2]]))
    commits = []
    alpha = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
    for ci, (cp, cid) in enumerate((c1, c2)):
        group = ((cp // 64) % (1 << 24)) >> 12  # the first two path levels (positive pks)
        order = np.argsort(group, kind="stable")
        g_sorted = group[order]
        cuts = np.flatnonzero(np.diff(g_sorted)) + 1
        starts = np.concatenate([[0], cuts])
        ends = np.concatenate([cuts, [g_sorted.shape[0]]])
        jobs = []
        for a, b in zip(starts, ends):
            g = int(g_sorted[a])
            prefix = bytes([alpha[g >> 6], ord("/"), alpha[g & 63], ord("/")])
            rows = order[a:b]
            jobs.append((gitdir, f"refs/heads/s{ci}_{g}", prefix, cp[rows], cid[rows]))
        with Pool(procs) as pool:
            subtrees = pool.map(_subtree_import, jobs)
        commits.append(subtrees)
        print(f"  commit {ci}: {len(subtrees)} subtrees in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    lines = []
    for ci, subtrees in enumerate(commits):
        lines.append(b"commit refs/heads/main\ncommitter t <t@t> %d +0000\ndata 1\nx\n" % (1600000000 + ci))
        if ci:
            lines.append(b"deleteall\n")
        for path, d in meta.items():
            lines.append(b"M 100644 inline %s\ndata %d\n%s\n" % (path.encode(), len(d), d))
        for prefix, tree in subtrees:
            lines.append(b"M 040000 %s %s/feature/%s\n" % (tree.encode(), inner.encode(), prefix[:3]))
        lines.append(b"\n")
    subprocess.run(["git", "fast-import", "--quiet"], input=b"".join(lines), env=dict(os.environ, GIT_DIR=gitdir),
                   check=True)
    print(f"  commits written in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    return ku + kd + ki


def _meta(inner, lh, legend):
    return {f"{inner}/meta/schema.json": json.dumps(synth.POINT_SCHEMA).encode(),
            f"{inner}/meta/path-structure.json": json.dumps(
                {"scheme": "int", "branches": 64, "levels": 4, "encoding": "base64"}).encode(),
            f"{inner}/meta/legend/{lh}": legend.dumps(),
            f"{inner}/meta/crs/EPSG:4326.wkt": b'GEOGCS["WGS 84",AUTHORITY["EPSG","4326"]]',
            ".kart.repostructure.version": b"3\n"}


def build(gitdir, n, seed=3):
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    legend = Legend(["c-fid"], [c["id"] for c in synth.POINT_SCHEMA[1:]])
    lh = legend.hexhash()
    rng = np.random.default_rng(seed)
    pks = np.arange(1, n + 1, dtype=np.int64)
    perm = rng.permutation(n)
    k = n // 100
    upd, dele = np.sort(perm[:k]), np.sort(perm[k:2 * k])
    ins = np.arange(n + 1, n + 1 + k, dtype=np.int64)
    inner = f"{DS}/.table-dataset"
    meta = _meta(inner, lh, legend)

    def feature_lines(p, ver):
        arena, off = synth.int_pk_paths(p)
        data, boff = synth.point_blobs(p, ver, lh)
        out = []
        for i in range(p.shape[0]):
            path = arena[int(off[i]):int(off[i + 1])].tobytes()
            blob = data[int(boff[i]):int(boff[i + 1])].tobytes()
            out.append(b"M 100644 inline %s/feature/%s\ndata %d\n%s\n" % (inner.encode(), path, len(blob), blob))
        return out

    lines = [b"commit refs/heads/main\ncommitter t <t@t> 1600000000 +0000\ndata 1\nx\n"]
    for p, d in meta.items():
        lines.append(b"M 100644 inline %s\ndata %d\n%s\n" % (p.encode(), len(d), d))
    lines += feature_lines(pks, np.zeros(n, np.uint64))
    lines.append(b"\ncommit refs/heads/main\ncommitter t <t@t> 1600000001 +0000\ndata 1\ny\n")
    lines += feature_lines(pks[upd], np.ones(k, np.uint64))
    lines += feature_lines(ins, np.full(k, 2, np.uint64))
    arena, off = synth.int_pk_paths(pks[dele])
    for i in range(k):
        lines.append(b"D %s/feature/%s\n" % (inner.encode(), arena[int(off[i]):int(off[i + 1])].tobytes()))
    lines.append(b"\n")
    subprocess.run(["git", "fast-import", "--quiet"], input=b"".join(lines), env=dict(os.environ, GIT_DIR=gitdir),
                   check=True)
    return k


def fielddiff_split(eng, od, oo, nd, no, old, new):
    """kd_fielddiff on the update arenas split into its parts: H2D of both arenas (pinned staging by
    the library), the device call on resident arenas (synchronised), D2H of the masks"""
    import ctypes

    from kart_amd import _native as N
    from kart_amd.device import DevBlobs, DevBuf
    from kart_amd.schema import FieldMaps

    maps = FieldMaps(old.schema, old.legends, new.schema, new.legends)
    n = int(oo.shape[0]) - 1
    eng.sync()
    t0 = time.perf_counter()
    OB, NB = DevBlobs(eng, od, oo), DevBlobs(eng, nd, no)
    eng.sync()
    t1 = time.perf_counter()
    masks, status = DevBuf(eng, 8 * max(n, 1) * maps.words), DevBuf(eng, max(n, 1))
    ob, nb, km = OB.kd_blobs(), NB.kd_blobs(), maps.kd_maps()
    N.check(eng.L.kd_fielddiff(eng.ctx, ctypes.byref(ob), ctypes.byref(nb), None, n, None, N.KD_MEM_DEVICE,
                               ctypes.byref(km), masks.ptr, status.ptr, N.KD_MEM_DEVICE), "kd_fielddiff")
    eng.sync()
    t2 = time.perf_counter()
    masks.download(np.uint64, n * maps.words)
    t3 = time.perf_counter()
    return {"h2d_s": round(t1 - t0, 4), "device_s": round(t2 - t1, 4), "d2h_s": round(t3 - t2, 4),
            "arena_bytes": int(od.size + nd.size), "updates": n}


def timed(fn):
    t0 = time.perf_counter()
    r = fn()
    return time.perf_counter() - t0, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--repo", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--procs", type=int, default=16, help="parallel blob writers when building the repository")
    ap.add_argument("--edits", default="0.01,0.01,0.01",
                    help="update,delete,insert fractions of n in the second commit (C3's mix: 0.08,0.01,0.01)")
    a = ap.parse_args()
    edits = tuple(float(x) for x in a.edits.split(","))
    gitdir = a.repo or f"/tmp/kart_e2e_{a.n}_{a.edits.replace(',', '_')}.git"
    if not os.path.isdir(gitdir):
        build = build_sharded if a.n > 5_000_000 else build_parallel
        t, k = timed(lambda: build(gitdir, a.n, procs=a.procs, edits=edits))
        print(f"built {gitdir} in {t:.1f} s", file=sys.stderr, flush=True)
    from kart_amd import dataset as D
    from kart_amd.engine import Engine
    from kart_amd.gitsource import GitRepo

    feat = f"{DS}/.table-dataset/feature"
    t_git, out = timed(lambda: subprocess.run(["git", "--git-dir", gitdir, "diff-tree", "-r", "--name-only",
                                               "main^", "main", "--", feat], capture_output=True, check=True).stdout)
    n_git = out.count(b"\n")
    res = {"n": a.n, "edits_update_delete_insert": list(edits), "changed_paths": n_git,
           "git_diff_tree_s": round(t_git, 4),
           "reference_path": "measured in the build container by scripts/ref_path_bench.py (the reference's own "
                             "Dataset3.diff_feature + get_feature loop) at 1M and 3M: profiles/r05/ref_path_*.json"}
    t_eng = time.perf_counter()
    with Engine(0) as eng:
        res["engine_init_s"] = round(time.perf_counter() - t_eng, 4)  # context + the library's code object
        # the first run of a process also loads the GPU code objects and sizes the workspaces:
        # reported as "cold", the repeat as "warm"
        for label, pruned in (("pruned walk (cold)", True), ("pruned walk (warm)", True), ("full walk", False)):
            stages = {}
            t0 = time.perf_counter()
            repo = GitRepo(gitdir)
            if pruned:
                t, (old, new) = timed(lambda: repo.diff_versions("main^", "main", DS))
            else:
                t, (old, new) = timed(lambda: (repo.dataset_version("main^", DS), repo.dataset_version("main", DS)))
            stages["walk_s"] = t
            t, (pa, pb) = timed(lambda: (old.pack(eng), new.pack(eng)))
            stages["pack_s"] = t
            stages["pack_parse_s"] = pa.timing["parse_s"] + pb.timing["parse_s"]
            stages["pack_sort_s"] = pa.timing["sort_s"] + pb.timing["sort_s"]
            stages["sort_on"] = pa.timing["sort_on"]
            D.STAGE_TIMES = {}
            t, ds = timed(lambda: D.get_dataset_diff(eng, old, new))
            stages["diff_s"] = t
            stages["diff_parts_s"] = {k: round(v, 4) for k, v in D.STAGE_TIMES.items()}
            D.STAGE_TIMES = None
            fd = ds["feature"]
            fds = {}
            t, nu = timed(lambda: D.field_diff(eng, fd, old, new, stats=fds))
            stages["field_diff_s"] = t
            stages["field_diff_parts_s"] = {k: round(v, 4) for k, v in fds.items()}
            total = time.perf_counter() - t0
            # the field diff's kernel call split (outside total_s): H2D of the two update arenas, the
            # device call on resident arenas, the masks' D2H
            batch = D._live_batch(fd, old, new)
            if batch is not None and batch.deltas:
                (od, oo), (nd, no) = D._arena_pair(old, new, batch.old_leaf, batch.new_leaf)
                stages["field_diff_split_s"] = fielddiff_split(eng, od, oo, nd, no, old, new)
            counts = fd.type_counts()
            assert sum(counts.values()) == n_git, (counts, n_git)
            assert all(d.changed_fields for d in fd.values() if d.type == "update")
            repo.close()
            res[label] = {**{k: round(v, 4) if isinstance(v, float) else v for k, v in stages.items()},
                          "total_s": round(total, 4),
                          "counts": counts, "leaves": [int(old.n), int(new.n)]}
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
