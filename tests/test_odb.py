"""The native object store + leaf walk (kd_odb_* / kd_walk, kart_amd/odb.py) against git itself:
every listing equals `git ls-tree -r`, every object equals `git cat-file`, over packed (fast-import),
repacked (deep OFS delta chains), loose and alternate object stores.  Pruned walks keep exactly
the leaves a tree diff must see.  CPU only (host code)."""
import os
import subprocess

import numpy as np
import pytest

from kart_amd import _native as N
from kart_amd.odb import ObjectDB

FEAT = "ds/.table-dataset/feature"


def _git(gitdir, *args, input=None):
    return subprocess.run(["git", "--git-dir", gitdir, *args], input=input, capture_output=True, check=True).stdout


def _fast_import(gitdir, commits):
    """commits: [(branch, {path: bytes | (mode, bytes)})], each on top of the previous"""
    lines = []
    for ci, (br, files) in enumerate(commits):
        lines.append(b"commit refs/heads/%s\ncommitter t <t@t> %d +0000\ndata 1\nx\n" % (br.encode(), 1600000000 + ci))
        if ci:
            lines.append(b"from refs/heads/%s\n" % commits[ci - 1][0].encode())
        lines.append(b"deleteall\n")
        for p, d in files.items():
            mode, d = d if isinstance(d, tuple) else (0o100644, d)
            lines.append(b"M %o inline %s\ndata %d\n%s\n" % (mode, p.encode(), len(d), d))
        lines.append(b"\n")
    subprocess.run(["git", "fast-import", "--quiet"], input=b"".join(lines), env=dict(os.environ, GIT_DIR=gitdir),
                   check=True)


def _ls(gitdir, spec, pre=""):
    out = _git(gitdir, "ls-tree", "-r", "-z", spec, *(["--", pre] if pre else []))
    res = []
    for rec in out.split(b"\0"):
        if rec:
            meta, path = rec.split(b"\t", 1)
            path = path.decode()
            res.append((path[len(pre) + 1:] if pre else path, meta.split()[2].decode(), int(meta.split()[0], 8)))
    return res


def _rev(gitdir, spec):
    return _git(gitdir, "rev-parse", spec).decode().strip()


def _layer(seed, n=3000, drop=0.0, change=0.0):
    rng = np.random.default_rng(seed)
    files = {}
    for i in range(n):
        if drop and rng.random() < drop:
            continue
        v = int(rng.integers(1, 1000)) if change and rng.random() < change else 0
        files[f"{FEAT}/{i % 7}/{(i // 7) % 13}/f{i}"] = b"feature %d v%d" % (i, v)
    # names that sort around a tree named "0" (git orders a tree as "0/")
    files[f"{FEAT}/0-x"] = b"before 0/"
    files[f"{FEAT}/0.x"] = b"after 0/"
    files[f"{FEAT}/00"] = b"after 0/ too"
    files[f"{FEAT}/exec"] = (0o100755, b"#!/bin/sh\n")
    files[f"{FEAT}/link"] = (0o120000, b"0/0/f0")
    files["ds/.table-dataset/meta/schema.json"] = b"[]"
    files["a b/\xc3\xa9 name"] = b"non-ascii path"
    return files


@pytest.fixture(scope="module")
def repo(tmp_path_factory):
    gitdir = str(tmp_path_factory.mktemp("odb") / "r.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    _fast_import(gitdir, [("c0", _layer(0)), ("c1", _layer(1, drop=0.03, change=0.05)),
                          ("c2", _layer(2, drop=0.05, change=0.10))])
    return gitdir


def _items(lv):
    return [(lv.path(i), lv.oids[i].tobytes().hex(), int(lv.modes[i])) for i in range(lv.n)]


@pytest.mark.parametrize("threads", [1, 8])
def test_walk_equals_ls_tree(repo, threads):
    db = ObjectDB(repo)
    for spec in ("c0", "c1", "c2"):
        (lv,) = db.walk([_rev(repo, spec)], FEAT, threads=threads)
        assert lv.present and _items(lv) == _ls(repo, spec, FEAT)
        (lv,) = db.walk([_rev(repo, spec)], "", threads=threads)
        assert _items(lv) == _ls(repo, spec)
    # a tree OID works as a root as well as a commit; an absent subpath is "not present"
    (lv,) = db.walk([_rev(repo, "c0^{tree}")], "ds")
    assert lv.n == len(_ls(repo, "c0", "ds"))
    (lv,) = db.walk([_rev(repo, "c0")], "no/such/dir")
    assert not lv.present and lv.n == 0


def _changed(repo, a, b):
    A = {p: o for p, o, _ in _ls(repo, a, FEAT)}
    B = {p: o for p, o, _ in _ls(repo, b, FEAT)}
    return A, B, {p for p in set(A) | set(B) if A.get(p) != B.get(p)}


def test_pruned_walk_keeps_every_changed_leaf(repo):
    db = ObjectDB(repo)
    A, B, changed = _changed(repo, "c0", "c2")
    la, lb = db.walk([_rev(repo, "c0"), _rev(repo, "c2")], FEAT, compare=(0, 1))
    pa, pb = {p: o for p, o, _ in _items(la)}, {p: o for p, o, _ in _items(lb)}
    assert changed <= set(pa) | set(pb)
    assert all(A[p] == o for p, o in pa.items()) and all(B[p] == o for p, o in pb.items())
    # subtrees and leaves equal on both sides are skipped: what is left is exactly the changed paths
    assert set(pa) | set(pb) == changed
    assert la.n < len(A) and lb.n < len(B)
    # identical roots: nothing opened
    la, lb = db.walk([_rev(repo, "c1")] * 2, FEAT, compare=(0, 1))
    assert la.n == lb.n == 0


def test_pruned_three_way_walk(repo):
    """merge pruning: compare ours (1) and theirs (2); the ancestor's leaves under the opened
    subtrees come along"""
    db = ObjectDB(repo)
    roots = [_rev(repo, s) for s in ("c0", "c1", "c2")]
    a, o, t = db.walk(roots, FEAT, compare=(1, 2))
    O, T, changed = _changed(repo, "c1", "c2")
    po, pt = {p for p, _, _ in _items(o)}, {p for p, _, _ in _items(t)}
    assert po | pt == changed  # a leaf equal in ours and theirs is skipped even inside an opened tree
    full_a = {p: x for p, x, _ in _ls(repo, "c0", FEAT)}
    assert {p: x for p, x, _ in _items(a)} == {p: x for p, x in full_a.items() if O.get(p) != T.get(p)}


def test_deep_delta_chains_and_batch_reads(tmp_path):
    """40 commits editing a 600-entry tree, repacked with --depth=50: trees reach long OFS_DELTA
    chains; every version's walk and every blob equal git's"""
    gitdir = str(tmp_path / "d.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    base = {f"t/{i // 40}/{i:04d}": b"row %d " % i + b"x" * 200 for i in range(600)}
    commits = []
    for c in range(40):
        files = dict(base)
        for i in range(c * 15, c * 15 + 15):
            files[f"t/{(i % 600) // 40}/{i % 600:04d}"] = b"row %d edit %d " % (i % 600, c) + b"y" * 200
        base = files
        commits.append((f"v{c}", files))
    _fast_import(gitdir, commits)
    _git(gitdir, "repack", "-adfq", "--depth=50", "--window=250")
    packs = [f for f in os.listdir(os.path.join(gitdir, "objects", "pack")) if f.endswith(".idx")]
    vp = _git(gitdir, "verify-pack", "-v", *[os.path.join(gitdir, "objects", "pack", f) for f in packs]).decode()
    depths = [int(ln.split("=")[1].split(":")[0]) for ln in vp.splitlines() if ln.startswith("chain length")]
    assert max(depths) >= 10, vp[-400:]
    db = ObjectDB(gitdir)
    for spec in ("v0", "v17", "v39"):
        (lv,) = db.walk([_rev(gitdir, spec)], "t")
        assert _items(lv) == _ls(gitdir, spec, "t")
        data, off, st = db.read_batch(lv.oids, threads=4)
        assert not st.any()
        want = _git(gitdir, "cat-file", "--batch", input="".join(lv.oids[i].tobytes().hex() + "\n"
                                                                for i in range(lv.n)).encode())
        pos = 0
        for i in range(lv.n):
            nl = want.index(b"\n", pos)
            size = int(want[pos:nl].split()[2])
            assert data[int(off[i]):int(off[i + 1])].tobytes() == want[nl + 1:nl + 1 + size]
            pos = nl + 1 + size + 1
        # shuffled and repeated: read in pack order, the arena stitched back in input order
        pick = np.random.default_rng(5).integers(0, lv.n, 3 * lv.n)
        d2, o2, s2 = db.read_batch(lv.oids[pick], threads=3)
        assert not s2.any() and int(o2[-1]) == int(sum(off[i + 1] - off[i] for i in pick))
        for k, i in enumerate(pick):
            assert d2[int(o2[k]):int(o2[k + 1])].tobytes() == data[int(off[i]):int(off[i + 1])].tobytes()
    # the zlib inflate path (taken when libdeflate.so.0 is absent) reads the same bytes
    import hashlib
    import sys

    prog = ("import hashlib, sys; sys.path.insert(0, %r); from kart_amd.odb import ObjectDB; "
            "db = ObjectDB(%r); (lv,) = db.walk([%r], 't'); d, o, st = db.read_batch(lv.oids); "
            "print(hashlib.sha256(d.tobytes() + o.tobytes()).hexdigest(), int(st.sum()))"
            % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), gitdir, _rev(gitdir, "v39")))
    out = subprocess.run([sys.executable, "-c", prog], env=dict(os.environ, KD_ODB_ZLIB="1"), capture_output=True,
                         check=True, text=True).stdout.split()
    assert out == [hashlib.sha256(data.tobytes() + off.tobytes()).hexdigest(), "0"]
    # the same switch as an option of the open store (kd_odb_set_option), kept across a reopen
    assert db.get_option("zlib") == 0
    db.set_option("zlib", 1)
    db.reopen()
    assert db.get_option("zlib") == 1
    d3, o3, s3 = db.read_batch(lv.oids)
    assert not s3.any() and d3.tobytes() == data.tobytes() and np.array_equal(o3, off)
    db.set_option("zlib", 0)
    with pytest.raises(Exception):
        db.set_option("no_such_option", 1)


def test_loose_objects_missing_and_corrupt(tmp_path, repo):
    gitdir = str(tmp_path / "l.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    big = bytes(range(256)) * 4000
    oid = _git(gitdir, "hash-object", "-w", "--stdin", input=big).decode().strip()
    empty = _git(gitdir, "hash-object", "-w", "--stdin", input=b"").decode().strip()
    db = ObjectDB(gitdir)
    assert db.read(oid) == (3, big)
    assert db.read(empty) == (3, b"")
    # a loose tree (update-index + write-tree) walks like a packed one
    env = dict(os.environ, GIT_DIR=gitdir, GIT_INDEX_FILE=str(tmp_path / "idx"))
    info = b"100644 %s\tx/y/big\x00100644 %s\tx/empty\x00" % (oid.encode(), empty.encode())
    subprocess.run(["git", "update-index", "-z", "--index-info"], input=info, env=env, check=True)
    tree = subprocess.run(["git", "write-tree"], env=env, capture_output=True, check=True).stdout.decode().strip()
    (lv,) = db.walk([tree], "")
    assert [(p, o) for p, o, _ in _items(lv)] == [("x/empty", empty), ("x/y/big", oid)]
    with pytest.raises(N.NotFound):
        db.read("1" * 40)
    data, off, st = db.read_batch(np.frombuffer(bytes.fromhex(oid) + b"\x11" * 20 + bytes.fromhex(tree), np.uint8))
    assert st.tolist() == [0, 1, 2] and int(off[1]) == len(big) and off[1] == off[3]
    with pytest.raises(N.NotFound):
        db.walk(["2" * 40], "")
    # a truncated loose object is an error, never a crash
    p = os.path.join(gitdir, "objects", oid[:2], oid[2:])
    os.chmod(p, 0o644)
    raw = open(p, "rb").read()
    open(p, "wb").write(raw[: len(raw) // 2])
    with pytest.raises(N.KdError):
        ObjectDB(gitdir).read(oid)


def test_alternates(tmp_path, repo):
    gitdir = str(tmp_path / "alt.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    with open(os.path.join(gitdir, "objects", "info", "alternates"), "w") as f:
        f.write(os.path.join(repo, "objects") + "\n")
    db = ObjectDB(gitdir)
    (lv,) = db.walk([_rev(repo, "c1")], FEAT)
    assert _items(lv) == _ls(repo, "c1", FEAT)


def test_gitrepo_refs_and_dataset_paths(repo):
    from kart_amd.gitsource import GitRepo

    r = GitRepo(repo)
    try:
        assert r.rev_parse("c1") == _rev(repo, "c1")
        assert r.rev_parse("refs/heads/c2") == _rev(repo, "c2")
        assert r.rev_parse("c2~1") == _rev(repo, "c1")  # expression: git rev-parse
        assert r.rev_tree("c0") == _rev(repo, "c0^{tree}")
        _git(repo, "pack-refs", "--all")
        assert GitRepo(repo).rev_parse("c0") == _rev(repo, "c0")
        assert r.dataset_paths("c0") == ["ds"]
        assert [e[3] for e in r.ls_tree("c0")] == ["a b", "ds"]
    finally:
        r.close()


def test_ref_delta_pack(tmp_path):
    """a pack written with REF_DELTA bases (repack.useDeltaBaseOffset=false, what older git and
    some servers send) reads like the OFS_DELTA one"""
    gitdir = str(tmp_path / "r.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    base = {f"t/{i // 40}/{i:04d}": b"row %d " % i + b"x" * 200 for i in range(400)}
    commits = []
    for c in range(12):
        files = dict(base)
        for i in range(c * 20, c * 20 + 20):
            files[f"t/{(i % 400) // 40}/{i % 400:04d}"] = b"row %d edit %d " % (i % 400, c) + b"y" * 200
        base = files
        commits.append((f"v{c}", files))
    _fast_import(gitdir, commits)
    subprocess.run(["git", "--git-dir", gitdir, "-c", "repack.useDeltaBaseOffset=false", "repack", "-adfq",
                    "--depth=20", "--window=50"], check=True)
    packs = [f for f in os.listdir(os.path.join(gitdir, "objects", "pack")) if f.endswith(".pack")]
    raw = open(os.path.join(gitdir, "objects", "pack", packs[0]), "rb").read()
    # object type 7 (REF_DELTA) occurs in the pack's entry headers; 6 (OFS_DELTA) does not
    vp = _git(gitdir, "verify-pack", "-v", os.path.join(gitdir, "objects", "pack", packs[0])).decode()
    assert "chain length" in vp
    types = set()
    for ln in vp.splitlines():
        parts = ln.split()
        if len(parts) >= 5 and len(parts[0]) == 40:
            off = int(parts[4])
            types.add((raw[off] >> 4) & 7)
    assert 7 in types and 6 not in types, types
    db = ObjectDB(gitdir)
    for spec in ("v0", "v11"):
        (lv,) = db.walk([_rev(gitdir, spec)], "t")
        assert _items(lv) == _ls(gitdir, spec, "t")
        data, off, st = db.read_batch(lv.oids)
        assert not st.any()
        for i in (0, lv.n // 2, lv.n - 1):
            want = _git(gitdir, "cat-file", "blob", lv.oids[i].tobytes().hex())
            assert data[int(off[i]):int(off[i + 1])].tobytes() == want


def test_corrupt_loose_copy_falls_through_to_alternate(tmp_path, repo):
    """a truncated loose copy in the repository's own object directory does not hide the good copy
    in an alternate"""
    alt = str(tmp_path / "alt_src.git")
    subprocess.run(["git", "init", "-q", "--bare", alt], check=True)
    blob = b"the good copy " * 100
    oid = _git(alt, "hash-object", "-w", "--stdin", input=blob).decode().strip()
    gitdir = str(tmp_path / "main.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    with open(os.path.join(gitdir, "objects", "info", "alternates"), "w") as f:
        f.write(os.path.join(alt, "objects") + "\n")
    good = open(os.path.join(alt, "objects", oid[:2], oid[2:]), "rb").read()
    os.makedirs(os.path.join(gitdir, "objects", oid[:2]), exist_ok=True)
    with open(os.path.join(gitdir, "objects", oid[:2], oid[2:]), "wb") as f:
        f.write(good[: len(good) // 2])
    db = ObjectDB(gitdir)
    assert db.read(oid) == (3, blob)
    data, off, st = db.read_batch(np.frombuffer(bytes.fromhex(oid), np.uint8))
    assert st.tolist() == [0] and data.tobytes() == blob


def test_refresh_only_when_packs_change(tmp_path):
    """a miss with an unchanged pack set does not reopen the store (promised blobs miss on every
    read); a pack written after the open is picked up by the next miss"""
    from kart_amd.gitsource import EOBJECTMISSING, GitRepo

    gitdir = str(tmp_path / "p.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    _fast_import(gitdir, [("a", {"x/one": b"one"})])
    r = GitRepo(gitdir)
    try:
        h = r.odb.n_opens
        with pytest.raises(KeyError) as ei:
            r.cat("3" * 40)
        assert ei.value.subcode == EOBJECTMISSING
        assert r.odb.n_opens == h  # not reopened
        _fast_import(gitdir, [("b", {"x/two": b"two, in a new pack"})])
        _git(gitdir, "repack", "-adq")  # small imports land loose: put everything in a new pack
        oid = _git(gitdir, "rev-parse", "b:x/two").decode().strip()
        assert r.cat(oid) == b"two, in a new pack"
        assert r.odb.n_opens == h + 1
    finally:
        r.close()


def test_refresh_sees_packs_added_to_an_alternate(tmp_path):
    """a pack written into an alternate object directory after the open changes the signature, so the
    next miss reopens and finds the object (alternates' pack dirs were not watched)"""
    from kart_amd.gitsource import GitRepo

    alt = str(tmp_path / "alt.git")
    subprocess.run(["git", "init", "-q", "--bare", alt], check=True)
    _fast_import(alt, [("a", {"x/one": b"one"})])
    gitdir = str(tmp_path / "main.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    with open(os.path.join(gitdir, "objects", "info", "alternates"), "w") as f:
        f.write(os.path.join(alt, "objects") + "\n")
    r = GitRepo(gitdir)
    try:
        h = r.odb.n_opens
        sig = r.odb._pack_signature()
        _fast_import(alt, [("b", {"x/two": b"two, in the alternate's new pack"})])
        _git(alt, "repack", "-adq")
        assert r.odb._pack_signature() != sig
        oid = _git(alt, "rev-parse", "b:x/two").decode().strip()
        assert r.cat(oid) == b"two, in the alternate's new pack"
        assert r.odb.n_opens == h + 1
    finally:
        r.close()


def test_batch_reads_across_several_packs(tmp_path):
    """three fast-imports = three packs (each with its own delta chains): a shuffled batch over all
    of them, read in (pack, offset) order and stitched back, equals git cat-file object by object"""
    gitdir = str(tmp_path / "m.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    for b in range(3):
        files = {f"p{b}/{i:04d}": b"pack %d row %d " % (b, i) + b"z" * (100 + i % 50) for i in range(400)}
        _fast_import(gitdir, [(f"b{b}", files)])
    packs = [f for f in os.listdir(os.path.join(gitdir, "objects", "pack")) if f.endswith(".idx")]
    assert len(packs) == 3
    db = ObjectDB(gitdir)
    oids = np.concatenate([db.walk([_rev(gitdir, f"b{b}")], f"p{b}")[0].oids for b in range(3)])
    pick = np.random.default_rng(7).permutation(np.concatenate([np.arange(oids.shape[0])] * 2))
    data, off, st = db.read_batch(oids[pick], threads=4)
    assert not st.any()
    want = _git(gitdir, "cat-file", "--batch", input="".join(oids[i].tobytes().hex() + "\n" for i in pick).encode())
    pos = 0
    for k in range(pick.size):
        nl = want.index(b"\n", pos)
        size = int(want[pos:nl].split()[2])
        assert data[int(off[k]):int(off[k + 1])].tobytes() == want[nl + 1:nl + 1 + size]
        pos = nl + 1 + size + 1
