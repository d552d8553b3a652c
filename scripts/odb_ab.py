"""A/B of the batched blob reader on the e2e repository: the blobs field_diff reads (both sides of
every update), timed per library build (KART_AMD_LIB) and inflater (KD_ODB_ZLIB) in child processes.
usage: python scripts/odb_ab.py N [lib ...]"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

CHILD = r"""
import sys, time, json
sys.path.insert(0, %(root)r); sys.path.insert(0, %(root)r + "/scripts")
import numpy as np
import e2e_repo_bench as E
from kart_amd import dataset as D
from kart_amd.gitsource import GitRepo
repo = GitRepo(%(git)r)
old, new = repo.diff_versions("main^", "main", E.DS)
# the update leaves: paths on both sides (the pruned walk keeps only changed paths)
po = {old.rel_paths[int(old.rel_off[i]):int(old.rel_off[i + 1])].tobytes(): i for i in range(old.n)}
pairs = [(po[p], j) for j in range(new.n) for p in [new.rel_paths[int(new.rel_off[j]):int(new.rel_off[j + 1])].tobytes()] if p in po]
oi = np.array([a for a, _ in pairs]); ni = np.array([b for _, b in pairs])
res = {}
for rep in range(8):
    t0 = time.perf_counter(); d1 = old.read_blobs(oi); t1 = time.perf_counter(); d2 = new.read_blobs(ni); t2 = time.perf_counter()
    res.setdefault("old_ms", []).append(round(1e3 * (t1 - t0), 1)); res.setdefault("new_ms", []).append(round(1e3 * (t2 - t1), 1))
res["old_min"], res["new_min"] = min(res["old_ms"]), min(res["new_ms"])
res["n_updates"] = len(pairs)
res["bytes"] = int(d1[1][-1]) + int(d2[1][-1])
print(json.dumps(res))
"""


def main():
    n = int(sys.argv[1])
    libs = sys.argv[2:] or ["kart_amd/libkartdiff.so"]
    gitdir = f"/tmp/kart_e2e_{n}.git"
    if not os.path.isdir(gitdir):
        import e2e_repo_bench as E

        t0 = time.perf_counter()
        E.build_parallel(gitdir, n, procs=16)
        print(f"built {gitdir} in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    for lib in libs:
        for zlib in (False, True):
            env = dict(os.environ, KART_AMD_LIB=os.path.join(ROOT, lib))
            if zlib:
                env["KD_ODB_ZLIB"] = "1"
            out = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT, "git": gitdir}], env=env,
                                 capture_output=True, text=True, timeout=600)
            if out.returncode:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            print(json.dumps({"lib": lib, "zlib": zlib, **json.loads(out.stdout.strip().splitlines()[-1])}), flush=True)


if __name__ == "__main__":
    main()
