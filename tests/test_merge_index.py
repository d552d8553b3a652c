"""The three-way merge boundary: MergeIndex-shaped results (kart/merge_util.py:67-103),
list_conflicts summaries (kart/conflicts.py:22-132), write_tree, and the KeyError subcodes of
missing / promised blobs (kart/base_dataset.py:256-265, kart/promisor_utils.py:10-29).

Goldens: tests/golden/conflicts_* (generated from the reference repos; the polygons merge index
has 237 entries and 4 conflicts, PKs 98001, 1452332, 1456853, 1456912 — tests/test_conflicts.py).
Each test runs against the HIP engine (-m gpu) and, on CPU, against the oracle stand-in (host
logic only).
"""
import json
import os
import subprocess

import numpy as np
import pytest

from checks import NONE
from fixtures import MERGE_FIXTURES, load
from kart_amd import merge as M
from kart_amd.engine import Diff2Result, Merge3Result
from test_dropin import version


class OracleEngine:
    """test-only stand-in with the Engine interface, computed by the CPU oracle"""

    def diff2(self, A, B):
        from oracle import oracle as O

        delta, c = O.classify2(A.key, A.oid, B.key, B.oid)
        upd = delta[(delta[:, 0] != NONE) & (delta[:, 1] != NONE)]
        return Diff2Result(c["inserts"], c["updates"], c["deletes"], delta, upd)

    def merge3(self, A, O_, T):
        from oracle import oracle as O

        conf, md, n_clean = O.classify3(A.key, A.oid, O_.key, O_.oid, T.key, T.oid)
        return Merge3Result(n_clean, conf, md)


@pytest.fixture(params=["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def eng(request):
    if request.param == "oracle":
        yield OracleEngine()
    else:
        yield request.getfixturevalue("engine")


def _decode(fx):
    """RepoStructure.decode_path for the fixture's dataset: (ds, "feature", pk)"""
    ds = fx.meta["ds_path"]
    v = None

    def decode(path):
        nonlocal v
        pre = ds + "/.table-dataset/feature/"
        assert path.startswith(pre)
        v = v or version(fx, "ours")
        return (ds, "feature", v.decode_path_to_1pk(path[len(pre):]))

    return decode


@pytest.mark.parametrize("name", MERGE_FIXTURES)
def test_merge_trees_golden(eng, name):
    fx = load(name)
    (case,) = fx.cases("merge3")
    ds = fx.meta["ds_path"]
    pre = ds + "/.table-dataset/feature/"
    vers = [version(fx, k) for k in case["sides"]]
    mi = M.merge_trees(eng, *vers, prefix=pre)
    # conflicts: the golden set, keyed "0".. in path (libgit2 index) order
    want = [c for c in case["conflicts"] if c["path"].startswith(pre)]
    got = [(next(e for e in c if e).path, *(e.id if e else None for e in c)) for c in mi.conflicts.values()]
    assert got == sorted(((c["path"], c["ancestor"], c["ours"], c["theirs"]) for c in want), key=lambda r: r[0].encode())
    assert list(mi.conflicts) == [str(i) for i in range(len(want))]
    for c in mi.conflicts.values():
        assert all(e is None or (e.mode == M.FILEMODE_BLOB and e.path == next(x for x in c if x).path) for e in c)
    # entries: every merged feature path, a conflicted one at its last stage (pygit2 index iteration)
    want_entries = {p: oid for p, oid in case["entries_sha"] if p.startswith(pre)}
    assert {p: e.id for p, e in mi.entries.items()} == want_entries
    assert len(mi.unresolved_conflicts) == len(want)
    assert sorted(e.path for e in mi) == sorted(want_entries)
    if name == "conflicts_polygons":
        assert len(mi.conflicts) == 4 and mi.automerge_candidates == []  # geometry blobs hold NUL


def test_list_conflicts_polygons(eng):
    """kart conflicts -s / -ss (tests/test_conflicts.py:55-92)"""
    fx = load("conflicts_polygons")
    vers = [version(fx, k) for k in ("ancestor", "ours", "theirs")]
    mi = M.merge_trees(eng, *vers, prefix=fx.meta["ds_path"] + "/.table-dataset/feature/")
    dec = _decode(fx)
    assert M.list_conflicts(mi, dec, summarise=2) == {"nz_waca_adjustments": {"feature": 4}}
    assert M.list_conflicts(mi, dec, summarise=1) == {"nz_waca_adjustments": {"feature": [98001, 1452332, 1456853, 1456912]}}
    # resolving one conflict removes it from the unresolved set (merge_util.py add_resolve)
    k = next(iter(mi.conflicts))
    mi.add_resolve(k, [mi.conflicts[k].ours])
    assert M.list_conflicts(mi, dec, summarise=2) == {"nz_waca_adjustments": {"feature": 3}}
    with pytest.raises(TypeError):
        mi.add_resolve(0, [])


def _fast_import_repo(tmp_path, fx, keys, branches):
    """a bare git repo with one commit per fixture side, built from the fixture's own blobs"""
    gitdir = str(tmp_path / "repo.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    ds = fx.meta["ds_path"]
    inner = f"{ds}/.table-dataset"
    lines, mark = [], 0
    for key, br in zip(keys, branches):
        files = {}
        idx = fx.a[f"{key}_blob"]
        for name, bi in zip(fx.names(key), idx):
            files[f"{inner}/feature/{name}"] = fx.blob(int(bi))
        files[f"{inner}/meta/schema.json"] = json.dumps(fx.meta["sides"][key]["schema"]).encode()
        files[f"{inner}/meta/path-structure.json"] = json.dumps(fx.meta["sides"][key]["path_structure"]).encode()
        for h, lg in fx.legends.items():
            files[f"{inner}/meta/legend/{h}"] = lg.dumps()
        files[".kart.repostructure.version"] = b"3\n"
        marks = {}
        for p, data in files.items():
            mark += 1
            marks[p] = mark
            lines.append(b"blob\nmark :%d\ndata %d\n" % (mark, len(data)) + data + b"\n")
        lines.append(b"commit refs/heads/%s\ncommitter t <t@t> 1600000000 +0000\ndata 1\nx\n" % br.encode())
        lines.append(b"deleteall\n")
        for p in files:
            lines.append(b"M 100644 :%d %s\n" % (marks[p], p.encode()))
        lines.append(b"\n")
    subprocess.run(["git", "fast-import", "--quiet"], input=b"".join(lines), env=dict(os.environ, GIT_DIR=gitdir),
                   check=True)
    return gitdir


def test_merge_repo_and_write_tree(eng, tmp_path):
    """merge_repo over whole commits (feature trees on the engine, meta paths on the host) == the
    golden feature entries/conflicts; a conflict-free merge writes ours' tree"""
    from kart_amd.gitsource import GitRepo

    fx = load("conflicts_polygons")
    (case,) = fx.cases("merge3")
    gitdir = _fast_import_repo(tmp_path, fx, case["sides"], ["anc", "ours", "theirs"])
    repo = GitRepo(gitdir)
    try:
        mi = M.merge_repo(eng, repo, "anc", "ours", "theirs")
        pre = fx.meta["ds_path"] + "/.table-dataset/feature/"
        want = sorted((c["path"] for c in case["conflicts"] if c["path"].startswith(pre)), key=str.encode)
        assert [next(e for e in c if e).path for c in mi.conflicts.values()] == want
        feat = {p: e.id for p, e in mi.entries.items() if p.startswith(pre)}
        assert feat == {p: oid for p, oid in case["entries_sha"] if p.startswith(pre)}
        assert ".kart.repostructure.version" in mi.entries
        with pytest.raises(ValueError):
            mi.write_tree(repo)
        clean = M.merge_repo(eng, repo, "anc", "ours", "ours")
        assert not clean.conflicts
        assert clean.write_tree(repo) == repo.rev_tree("ours")
    finally:
        repo.close()


def test_missing_and_promised_blob_subcodes(tmp_path):
    """KeyError.subcode: EOBJECTMISSING, or EOBJECTPROMISED when the repo has a promisor remote"""
    from kart_amd import gitsource as G

    gitdir = str(tmp_path / "r.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    repo = G.GitRepo(gitdir)
    try:
        with pytest.raises(KeyError) as ei:
            repo.cat("0" * 40)
        assert ei.value.subcode == G.EOBJECTMISSING
    finally:
        repo.close()
    subprocess.run(["git", "--git-dir", gitdir, "config", "remote.origin.url", "file:///nowhere"], check=True)
    subprocess.run(["git", "--git-dir", gitdir, "config", "remote.origin.promisor", "true"], check=True)
    repo = G.GitRepo(gitdir)
    try:
        with pytest.raises(KeyError) as ei:
            repo.cat("1" * 40)
        assert ei.value.subcode == G.EOBJECTPROMISED
    finally:
        repo.close()


@pytest.mark.skipif(not os.path.isdir("/root/reference/kart"), reason="build container only (reads /root/reference)")
def test_engine_returns_the_references_own_diff_structs():
    """Inside Kart the engine hands back kart.diff_structs objects: with the reference's own module
    (imported through tests/golden/refshim.py, in a child interpreter so its stub modules stay out of
    this one), get_dataset_diff on the points fixture yields its DatasetDiff / DeltaDiff / Delta,
    whose sorted_items, type_counts and lazy values match the golden"""
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    code = f"""
import importlib, sys
sys.dont_write_bytecode = True
sys.path[:0] = [{os.path.dirname(here)!r}, {here!r}, {os.path.join(here, "golden")!r}]
import refshim
refshim.load_reference()
ref = importlib.import_module("kart.diff_structs")
from kart_amd import adaptor, dataset as D
from fixtures import load, pk_of
from test_merge_index import OracleEngine
from test_dropin import version
adaptor.use_structs(ref)
fx = load("repo_points")
(case,) = [c for c in fx.cases("diff2") if c["base"] == "head1" and c["target"] == "head"]
ds = D.get_dataset_diff(OracleEngine(), version(fx, "head1"), version(fx, "head"))
assert type(ds) is ref.DatasetDiff and type(ds["feature"]) is ref.DeltaDiff
fd = ds["feature"]
assert all(type(d) is ref.Delta for d in fd.values())
assert [k for k, _ in fd.sorted_items()] == [pk_of(d["old_pk"]) for d in case["deltas"]] == [1095, 1166, 1168, 1181, 1182]
assert fd.type_counts() == {{"updates": 5}}
k, d = fd.sorted_items()[0]
assert d.old_value["fid"] == k and callable(d.old.value) and d.old.value.args[0].id.hex
print("REF-STRUCTS-OK")
"""
    r = subprocess.run([sys.executable, "-B", "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "REF-STRUCTS-OK" in r.stdout, r.stdout + r.stderr
