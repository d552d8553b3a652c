"""The drop-in boundary: get_dataset_diff / diff_feature / field_diff return the reference's
delta sets, values, changed fields and streaming behaviour (tests/golden, from the reference).

Each test runs twice: against the HIP engine (-m gpu) and, on CPU, against a test-only engine
whose diff2/fielddiff are the oracle — that CPU run checks the host adaptor logic (swap/reverse,
pk decoding, lazy values, key filter), never the kernels.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from checks import NONE
from fixtures import DIFF_FIXTURES, load, pk_of
from kart_amd import dataset as D
from kart_amd.adaptor import structs
from kart_amd.engine import Diff2Result


class OracleEngine:
    """test-only stand-in with the Engine interface, computed by the CPU oracle"""

    def diff2(self, A, B):
        from oracle import oracle as O

        delta, c = O.classify2(A.key, A.oid, B.key, B.oid)
        upd = delta[(delta[:, 0] != NONE) & (delta[:, 1] != NONE)]
        return Diff2Result(c["inserts"], c["updates"], c["deletes"], delta, upd)

    def fielddiff(self, od, oo, nd, no, pairs, maps):
        from oracle import oracle as O

        return O.fielddiff(od, oo, nd, no, pairs, maps)


@pytest.fixture(params=["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def eng(request):
    if request.param == "oracle":
        yield OracleEngine()
    else:
        yield request.getfixturevalue("engine")


def version(fx, key):
    if fx.n(key) == 0:
        return None
    idx = fx.a[f"{key}_blob"]
    from kart_amd import meta as M

    return D.DatasetVersion(fx.meta["ds_path"], fx.schema(key), fx.legends, fx.encoding(key), fx.a[f"{key}_names"],
                            fx.a[f"{key}_name_off"].astype(np.uint64), fx.oids(key), lambda i: fx.blob(int(idx[i])),
                            meta=M.meta_items(fx.meta_files(key), fx.attachments(key)))


def meta_diff_rows(ds):
    """a DatasetDiff's meta DeltaDiff as sorted [key, old, new] rows (the golden form)"""
    return sorted([k, d.old_value, d.new_value] for k, d in ds.get("meta", {}).items())


def _jv(v):
    """engine value -> golden json_safe form"""
    if v is None:
        return None
    if isinstance(v, bool):
        return {"bool": v}
    if isinstance(v, int):
        return {"int": str(v)}
    if isinstance(v, float):
        return {"float": v.hex()}
    if isinstance(v, str):
        return {"str": v}
    if isinstance(v, (bytes, bytearray)):
        return {"bytes": bytes(v).hex(), "geom": isinstance(v, D.Geometry)}
    return {"repr": repr(v)}


@pytest.mark.parametrize("name", DIFF_FIXTURES)
def test_get_dataset_diff_golden(eng, name):
    fx = load(name)
    for case in fx.cases("diff2"):
        base, target = version(fx, case["base"]), version(fx, case["target"])
        ds = D.get_dataset_diff(eng, base, target)
        # diff_meta: the meta items' DeltaDiff equals the reference's (normalised schema.json and CRS
        # WKT, the metadata.xml attachment, non-standard meta files left out)
        assert meta_diff_rows(ds) == case["meta"], (name, case["base"], case["target"])
        fd = ds.get("feature") or structs().DeltaDiff()
        got = {(d.type, d.old_key, d.new_key) for d in fd.values()}
        want = {(d["type"], pk_of(d["old_pk"]), pk_of(d["new_pk"])) for d in case["deltas"]}
        assert got == want
        assert fd.type_counts() if fd else {} == {k: v for k, v in case["counts"].items() if v}
        # sorted_items order == the golden (reference DeltaDiff.sorted_items) order
        assert [k for k, _ in fd.sorted_items()] == [pk_of(d["old_pk"]) if d["old_pk"] is not None
                                                     else pk_of(d["new_pk"]) for d in case["deltas"]]
        if any("old" in d for d in case["deltas"]):
            for (k, delta), gd in zip(fd.sorted_items(), case["deltas"]):
                if "old" in gd:
                    assert {a: _jv(b) for a, b in delta.old_value.items()} == gd["old"]
                    assert {a: _jv(b) for a, b in delta.new_value.items()} == gd["new"]
        # field diff attached in one batch equals the reference text writer's decision
        n = D.field_diff(eng, fd, base or target, target or base) if fd else 0
        for (k, delta), gd in zip(fd.sorted_items() if fd else [], case["deltas"]):
            if gd["type"] == "update":
                assert delta.changed_fields == gd["changed"]
        assert n == sum(1 for d in case["deltas"] if d["type"] == "update")


def test_diff_streaming_contract(eng):
    """tests/test_diff.py:1656-1685: diffing calls get_feature zero times; each value access once."""
    fx = load("repo_points")
    old, new = version(fx, "head1"), version(fx, "head")
    calls = {"n": 0}
    for v in (old, new):
        orig = v.get_feature

        def counted(*a, _orig=orig, **k):
            calls["n"] += 1
            return _orig(*a, **k)

        v.get_feature = counted
    reads = {"n": 0}
    for v in (old, new):
        rb = v.read_blob

        def counted_read(i, _rb=rb):
            reads["n"] += 1
            return _rb(i)

        v.read_blob = counted_read
    fd = D.dataset_diff(eng, old, new)["feature"]
    assert calls["n"] == 0 and reads["n"] == 0
    expected = 0
    for key, delta in sorted(fd.items()):
        delta.old_value
        delta.new_value
        expected += 2
        assert calls["n"] == expected
        delta.old_value  # cached
        assert calls["n"] == expected
    # DeltaFetcher reads the blob id from the promise (base_diff_writer.py:505-507)
    d = next(iter(fd.values()))
    assert len(d.old.value.args[0].id.hex) == 40


def test_key_filter(eng):
    fx = load("repo_points")
    old, new = version(fx, "head1"), version(fx, "head")

    class F(set):
        match_all = False

    fd = structs().DeltaDiff(D.diff_feature(eng, old, new, F({"1166", "1182", "999999"})))
    assert sorted(fd.keys()) == [1166, 1182]


def test_reverse_and_missing_dataset(eng):
    fx = load("repo_points")
    head = version(fx, "head")
    ins = D.get_dataset_diff(eng, None, head)["feature"]
    dels = D.get_dataset_diff(eng, head, None)["feature"]
    assert ins.type_counts() == {"inserts": 2143}
    assert dels.type_counts() == {"deletes": 2143}
    inv = ~ins
    assert {k: (d.type, d.old_key, d.new_key) for k, d in inv.items()} == \
        {k: (d.type, d.old_key, d.new_key) for k, d in dels.items()}


def test_gitsource_walk(eng, tmp_path):
    """host tree walker over a real git repository built from the fixture's own blobs"""
    fx = load("repo_points")
    gitdir = str(tmp_path / "repo.git")
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    ds = fx.meta["ds_path"]
    inner = f"{ds}/.table-dataset"
    lines = []
    mark = 0
    for ci, key in enumerate(("head1", "head")):
        files = {}
        idx = fx.a[f"{key}_blob"]
        for name, bi in zip(fx.names(key), idx):
            files[f"{inner}/feature/{name}"] = fx.blob(int(bi))
        files[f"{inner}/meta/schema.json"] = json.dumps(fx.meta["sides"][key]["schema"]).encode()
        files[f"{inner}/meta/path-structure.json"] = json.dumps(fx.meta["sides"][key]["path_structure"]).encode()
        for h, lg in fx.legends.items():
            files[f"{inner}/meta/legend/{h}"] = lg.dumps()
        marks = {}
        for p, data in files.items():
            mark += 1
            marks[p] = mark
            lines.append(b"blob\nmark :%d\ndata %d\n" % (mark, len(data)) + data + b"\n")
        lines.append(b"commit refs/heads/c%d\ncommitter t <t@t> %d +0000\ndata 1\nx\n" % (ci, 1600000000 + ci))
        if ci:
            lines.append(b"from refs/heads/c0\n")
        lines.append(b"deleteall\n")
        for p in files:
            lines.append(b"M 100644 :%d %s\n" % (marks[p], p.encode()))
        lines.append(b"\n")
    subprocess.run(["git", "fast-import", "--quiet"], input=b"".join(lines), env=dict(os.environ, GIT_DIR=gitdir),
                   check=True)
    from kart_amd.gitsource import GitRepo

    repo = GitRepo(gitdir)
    assert repo.dataset_paths("refs/heads/c1") == [ds]
    old = repo.dataset_version("refs/heads/c0", ds)
    new = repo.dataset_version("refs/heads/c1", ds)
    fd = D.get_dataset_diff(eng, old, new)["feature"]
    assert sorted(fd.keys()) == [1095, 1166, 1168, 1181, 1182]
    D.field_diff(eng, fd, old, new)
    assert sum(len(d.changed_fields) for d in fd.values()) == 13
    # the pruned walk (only subtrees whose OIDs differ are opened) gives the same diff
    old_p, new_p = repo.diff_versions("refs/heads/c0", "refs/heads/c1", ds)
    assert old_p.partial and new_p.partial and old_p.n == new_p.n == 5 < old.n
    fdp = D.get_dataset_diff(eng, old_p, new_p)["feature"]
    assert sorted(fdp.keys()) == [1095, 1166, 1168, 1181, 1182]
    D.field_diff(eng, fdp, old_p, new_p)
    assert {k: d.changed_fields for k, d in fdp.items()} == {k: d.changed_fields for k, d in fd.items()}
    assert {k: d.new_value for k, d in fdp.items()} == {k: d.new_value for k, d in fd.items()}
    repo.close()


@pytest.mark.parametrize("name", DIFF_FIXTURES)
def test_exact_feature_counts(eng, name):
    """get_exact_diff_blob_count / estimate_diff_feature_counts (kart/diff_estimation.py:51-184):
    the changed-path count of every golden diff (reference counts), and of one-sided diffs"""
    fx = load(name)
    for case in fx.cases("diff2"):
        base, target = version(fx, case["base"]), version(fx, case["target"])
        want = sum(case["counts"].values())
        assert D.get_exact_diff_blob_count(eng, base, target) == want
        path = fx.meta["ds_path"]
        got = D.estimate_diff_feature_counts(eng, {path: base} if base else {}, {path: target} if target else {},
                                             accuracy="exact")
        assert got == ({path: want} if want else {})
        if base is not None:  # dataset deleted in the target: every feature is a changed path
            assert D.get_exact_diff_blob_count(eng, base, None) == base.n
    assert D.get_exact_diff_blob_count(eng, None, None) == 0


def test_field_diff_batch_path(eng):
    """field_diff on a DeltaDiff from dataset_diff reads each side's update blobs in one batched
    read by leaf index (no per-delta blob object) and keeps the arena: the values the writer reads
    afterwards come from it, with no further object read.  A diff changed after dataset_diff (a
    delta removed) goes through the lazy blobs and gives the same fields."""
    fx = load("repo_points")
    old, new = version(fx, "head1"), version(fx, "head")
    batches = {"n": 0}
    reads = {"n": 0}
    for v in (old, new):
        rb = v.read_blob

        def counted_read(i, _rb=rb):
            reads["n"] += 1
            return _rb(i)

        def batch_read(idx, _rb=rb):
            batches["n"] += 1
            bs = [bytes(_rb(int(i))) for i in idx]
            off = np.zeros(len(bs) + 1, np.uint64)
            off[1:] = np.cumsum([len(b) for b in bs])
            return np.frombuffer(b"".join(bs), np.uint8).copy(), off, np.zeros(len(bs), np.uint8)

        v.read_blob = counted_read
        v._read_blobs = batch_read
    fd = D.dataset_diff(eng, old, new)["feature"]
    assert fd._kd_updates.n_total == len(fd) == 5
    assert D.field_diff(eng, fd, old, new) == 5
    assert batches["n"] == 2 and reads["n"] == 0
    fields = {k: d.changed_fields for k, d in fd.items()}
    assert sum(len(v) for v in fields.values()) == 13
    vals = {k: (d.old_value, d.new_value) for k, d in fd.items()}
    assert reads["n"] == 0  # every value came from the field diff's arenas
    # a mutated diff: the recorded batch no longer describes it -> the lazy-blob path
    fd2 = D.dataset_diff(eng, version(fx, "head1"), version(fx, "head"))["feature"]
    gone = sorted(fd2.keys())[0]
    del fd2[gone]
    assert D._live_batch(fd2, fd2._kd_updates.old_v, fd2._kd_updates.new_v) is None
    assert D.field_diff(eng, fd2, fd2._kd_updates.old_v, fd2._kd_updates.new_v) == 4
    assert {k: d.changed_fields for k, d in fd2.items()} == {k: v for k, v in fields.items() if k != gone}
    assert {k: (d.old_value, d.new_value) for k, d in fd2.items()} == {k: v for k, v in vals.items() if k != gone}


def test_field_diff_prefetched_arenas(eng, monkeypatch):
    """diffs over PREFETCH_MIN_UPDATES updates of two versions read from one repository start the
    updates' batched blob read on a worker thread before the deltas are built: field_diff takes
    those arenas (no second read) and attaches the same fields"""
    from kart_amd import packing

    fx = load("repo_points")
    want = D.dataset_diff(eng, version(fx, "head1"), version(fx, "head"))["feature"]
    assert D.field_diff(eng, want, want._kd_updates.old_v, want._kd_updates.new_v) == 5
    monkeypatch.setattr(D, "PREFETCH_MIN_UPDATES", 1)
    old, new = version(fx, "head1"), version(fx, "head")
    reads = {"batch": 0, "one": 0}

    class Source:  # one repository's batched reader (what gitsource's read_blobs.source is)
        def __init__(self, versions):
            self.where = {}
            for v in versions:
                for i in range(v.n):
                    self.where[v.oids[i].tobytes()] = (v, i)

        def read_blobs(self, oids):
            reads["batch"] += 1
            bs = [bytes(v.read_blob(i)) for v, i in (self.where[o.tobytes()] for o in np.asarray(oids))]
            data, off = packing._arena(bs)
            return data, off, np.zeros(len(bs), np.uint8)

    src = Source([old, new])
    for v in (old, new):
        def rbs(idx, _v=v):
            return src.read_blobs(_v.oids[np.asarray(idx, np.int64)])

        rbs.source = src
        v._read_blobs = rbs
    fd = D.dataset_diff(eng, old, new)["feature"]
    assert fd._kd_updates.prefetch is not None
    fd._kd_updates.prefetch.fut.result()  # the read is done: field_diff must not read again
    assert reads["batch"] == 1
    for v in (old, new):
        rb = v.read_blob

        def counted(i, _rb=rb):
            reads["one"] += 1
            return _rb(i)

        v.read_blob = counted
    assert D.field_diff(eng, fd, old, new) == 5
    assert reads == {"batch": 1, "one": 0} and fd._kd_updates.prefetch is None
    assert {k: d.changed_fields for k, d in fd.items()} == {k: d.changed_fields for k, d in want.items()}


def test_changed_names_rows_matches_per_row():
    """the batch decode (one np.unique over the rows' words) equals changed_names row by row, for
    one- and multi-word masks, with a fresh list per row"""
    from kart_amd.schema import FieldMaps

    rng = np.random.default_rng(3)
    for n_keys in (5, 64, 65, 130):
        fm = object.__new__(FieldMaps)
        fm.keys = [f"k{i}" for i in range(n_keys)]
        fm.n_keys, fm.words = n_keys, max(1, (n_keys + 63) // 64)
        distinct = rng.integers(0, 2**63, (7, fm.words), dtype=np.uint64) | np.uint64(1 << 63)
        if n_keys % 64:
            distinct[:, -1] &= np.uint64((1 << (n_keys % 64)) - 1)
        masks = distinct[rng.integers(0, 7, 500)]
        rows = fm.changed_names_rows(masks)
        assert rows == [fm.changed_names(r) for r in masks]
        assert len({id(r) for r in rows}) == len(rows)
    assert fm.changed_names_rows(np.zeros((0, fm.words), np.uint64)) == []


def test_attach_fields_matches_per_row():
    """the native attach (kd_pystr.c attach_fields) gives every update changed_names of its row as
    a fresh list, None where the status is not 0, for Delta slots and for plain objects (setattr),
    one- and multi-word masks, and more distinct masks than its first table holds (growth)"""
    from kart_amd import _kd_pystr as P
    from kart_amd.deltas import Delta
    from kart_amd.schema import FieldMaps

    class Plain:
        pass

    rng = np.random.default_rng(5)
    for n_keys, n_distinct in ((5, 7), (64, 300), (130, 40)):
        fm = object.__new__(FieldMaps)
        fm.keys = [f"k{i}" for i in range(n_keys)]
        fm.n_keys, fm.words = n_keys, max(1, (n_keys + 63) // 64)
        distinct = rng.integers(0, 2**63, (n_distinct, fm.words), dtype=np.uint64)
        if n_keys % 64:
            distinct[:, -1] &= np.uint64((1 << (n_keys % 64)) - 1)
        masks = np.ascontiguousarray(distinct[rng.integers(0, n_distinct, 2000)])
        status = (rng.random(2000) < 0.1).astype(np.uint8)
        objs = [Delta.__new__(Delta) if i % 3 else Plain() for i in range(2000)]
        calls = []

        def names_of(i):
            calls.append(i)
            return list(fm.changed_names(masks[i]))

        used = P.attach_fields(objs, masks, status, fm.words, names_of, Delta)
        assert used == len(calls) == len({masks[i].tobytes() for i in range(2000) if not status[i]})
        for o, m, s in zip(objs, masks, status):
            assert o.changed_fields == (None if s else fm.changed_names(m))
        lists = [o.changed_fields for o in objs if o.changed_fields is not None]
        assert len({id(x) for x in lists}) == len(lists)
    with pytest.raises(ValueError):
        P.attach_fields([Plain()], masks[:1], np.zeros(1, np.int32), fm.words, names_of, Delta)
    with pytest.raises(ValueError):
        P.attach_fields([Plain(), Plain()], masks[:1], np.zeros(2, np.uint8), fm.words, names_of, Delta)


def test_field_diff_one_read_for_both_sides(tmp_path, eng):
    """versions of one git repository: field_diff reads both sides' update blobs in ONE batched
    read, split into two arenas over the same buffer; the changed fields are those whose values
    differ, and every value the writer reads afterwards comes from the arenas"""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import e2e_repo_bench as E
    from kart_amd.gitsource import GitRepo

    gitdir = str(tmp_path / "r.git")
    k = E.build(gitdir, 3000)
    repo = GitRepo(gitdir)
    try:
        old, new = repo.diff_versions("main^", "main", E.DS)
        calls, orig = [], repo.read_blobs
        repo.read_blobs = lambda oids, *a, **kw: (calls.append(len(oids)), orig(oids, *a, **kw))[1]
        fd = D.get_dataset_diff(eng, old, new)["feature"]
        assert D.field_diff(eng, fd, old, new) == k
        assert calls == [2 * k]
        cats = []
        old.read_blob = new.read_blob = lambda i: cats.append(i)  # no single-object read may happen
        for d in fd.values():
            if d.type != "update":
                continue
            a, b = d.old_value, d.new_value
            assert sorted(d.changed_fields) == sorted(f for f in a if a[f] != b.get(f))
        assert not cats and calls == [2 * k]
    finally:
        repo.close()


def test_gc_pause_leaves_collector_state():
    """the bulk-construction pause re-enables the collector, promotes what it built without a
    young-generation pass, and leaves objects the host froze itself frozen"""
    import gc

    assert gc.isenabled()
    with D._gc_paused():
        assert not gc.isenabled()
        built = [[i] for i in range(1000)]
    assert gc.isenabled() and gc.get_freeze_count() == 0
    gc.freeze()
    try:
        n = gc.get_freeze_count()
        with D._gc_paused():
            more = [[i] for i in range(1000)]
        assert gc.isenabled() and gc.get_freeze_count() == n  # the host's frozen set untouched
    finally:
        gc.unfreeze()
    gc.disable()
    try:
        with D._gc_paused():
            pass
        assert not gc.isenabled()  # a collector the host had disabled stays disabled
    finally:
        gc.enable()
    assert len(built) == len(more) == 1000


def _delta_view(fd):
    out = {}
    for k, d in fd.items():
        halves = []
        for kv in (d.old, d.new):
            if kv is None:
                halves.append(None)
                continue
            blob = kv.value.args[0]
            halves.append((kv.key, type(blob).__name__, blob._i, blob._src is not None, kv.value.func.__name__))
        out[k] = (d.type, d.flags, tuple(halves))
    return out


@pytest.mark.parametrize("name", ["repo_points", "repo_string_pks", "synth_str", "conflicts_table"])
def test_native_delta_builder_matches_python_loop(eng, name, monkeypatch):
    """the C delta builder (kart_amd/csrc/kd_pystr.c build_deltas) yields the deltas the Python
    loop builds: same keys, types, flags, KeyValue halves, partial(get_feature_from_blob, LazyBlob)
    promises over the same leaves and the same update batch; values equal and stay lazy"""
    assert D._pystr is not None, "kart_amd/_kd_pystr was not built (make -C kart_amd/csrc)"
    fx = load(name)
    for case in fx.cases("diff2")[:3]:
        got = {}
        for native in (True, False):
            if not native:
                monkeypatch.setattr(D, "_pystr", None)
            base, target = version(fx, case["base"]), version(fx, case["target"])
            ds = D.get_dataset_diff(eng, base, target)
            fd = ds.get("feature") or structs().DeltaDiff()
            b = getattr(fd, "_kd_updates", None)
            got[native] = (_delta_view(fd), [(k, d.old_value, d.new_value) for k, d in fd.sorted_items()][:50],
                           None if b is None else (b.keys, [id(x) in {id(y) for y in fd.values()} for x in b.deltas],
                                                   b.old_leaf.tolist(), b.new_leaf.tolist(), b.n_total))
            monkeypatch.undo()
        assert got[True] == got[False]
    # generator form (diff_feature without _collect) and reverse through the builder
    old, new = version(fx, fx.cases("diff2")[0]["base"]), version(fx, fx.cases("diff2")[0]["target"])
    if old is not None and new is not None:
        fwd = structs().DeltaDiff(D.diff_feature(eng, old, new))
        rev = structs().DeltaDiff(D.diff_feature(eng, new, old, reverse=True))
        assert _delta_view(fwd) == _delta_view(rev)


def test_native_delta_builder_kart_structs_path(monkeypatch):
    """own=False: halves handed to the Delta constructor as (pk, promise) tuples, as for
    kart.diff_structs"""
    import functools

    from kart_amd import _kd_pystr as P
    from kart_amd import deltas as DL

    calls = []

    class KD:
        def __init__(self, old, new):
            calls.append((old, new))
            self.old, self.new = old, new

    class V:
        def get_feature_from_blob(self, blob):
            return blob._i

    ov, nv = V(), V()
    ol = np.array([3, -1, 5], np.int64)
    nl = np.array([-1, 4, 6], np.int64)
    r = P.build_deltas(KD, DL.KeyValue, D.LazyBlob, functools.partial, ov.get_feature_from_blob,
                       nv.get_feature_from_blob, ov, nv, ol, nl, ["a", None, "c"], [None, "b", "c"], False)
    keys, deltas, rows, upd, ukeys = r
    assert keys == ["a", "b", "c"] and np.frombuffer(rows, np.int64).tolist() == [2]
    assert ukeys == ["c"] and upd == [deltas[2]]
    assert calls[0][1] is None and calls[1][0] is None
    assert [c[0][0] if c[0] else None for c in calls] == ["a", None, "c"]
    assert [c[1][1]() if c[1] else None for c in calls] == [None, 4, 6]
    with pytest.raises(ValueError):
        P.build_deltas(DL.Delta, DL.KeyValue, D.LazyBlob, functools.partial, None, None, ov, nv,
                       np.array([-1], np.int64), np.array([-1], np.int64), np.zeros(1, np.int64),
                       np.zeros(1, np.int64), True)


def test_promise_acts_as_partial():
    """_kd_pystr.Promise: partial(func, LazyBlob(src, i)) with the blob made on first use — called
    once per value access, .args[0] the same blob object every time, .func / .keywords as a partial,
    extra call arguments passed after the blob"""
    import functools

    from kart_amd import _kd_pystr as P
    from kart_amd import deltas as DL

    made = []

    class Blob(D.LazyBlob):
        __slots__ = ()

        def __init__(self, src, i):
            made.append(i)
            super().__init__(src, i)

    class V:
        def get(self, blob, *extra, **kw):
            return ("feat", blob._i, extra, kw)

    v = V()
    _, deltas, *_ = P.build_deltas(DL.Delta, DL.KeyValue, Blob, P.Promise, v.get, v.get, v, v,
                                   np.array([7, -1], np.int64), np.array([9, 4], np.int64),
                                   np.array([1, 0], np.int64), np.array([1, 2], np.int64), True)
    assert made == []  # nothing materialised by the diff
    pr = deltas[0].old.value
    assert pr() == ("feat", 7, (), {}) and made == [7]
    assert pr.args[0] is pr.args[0] and pr.args[0]._i == 7 and made == [7]
    assert pr.func == v.get and pr.keywords == {}
    assert pr(1, k=2) == ("feat", 7, (1,), {"k": 2})
    assert repr(pr).startswith("functools.partial(")
    ref = functools.partial(v.get, Blob(v, 9))
    assert deltas[0].new.value() == ref() and deltas[1].new.value.args[0]._i == 4
    assert deltas[0].old_value == ("feat", 7, (), {})  # KeyValue.get_lazy_value caches
