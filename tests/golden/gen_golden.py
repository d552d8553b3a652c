#!/usr/bin/env python3 -B
"""Generate the committed golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Run here (the build container), never on the GPU box:

    python -B tests/golden/gen_golden.py

What it does (all outputs are data — inputs and expected outputs — never reference source):

* Extracts the reference's own test repos (``tests/data/{points,polygons,table,string-pks}.tgz``
  and ``tests/data/conflicts/*.tgz``) into /tmp and flattens every commit's feature tree into
  packed leaf arrays (filename, 20-byte blob OID) plus the feature blobs.
* Runs the reference's ``kart.diff_util.get_dataset_diff`` -> ``Dataset3.diff`` ->
  ``RichBaseDataset.diff_feature`` (kart/rich_base_dataset.py:205-300) over a git-CLI pygit2
  shim (refshim.py) and records the delta set; for every update it records the changed field
  names exactly as ``TextDiffWriter.write_feature_delta`` decides them
  (kart/text_diff_writer.py:135-145 with ``BaseDiffWriter._all_feature_keys``,
  kart/base_diff_writer.py:181-187).
* Three-way: libgit2 is absent here, so the conflict set is the libgit2 OID rule applied to
  ``git ls-tree -r`` of ancestor/ours/theirs; it reproduces the pinned
  tests/test_conflicts.py:27-30,60-92 numbers (asserted below).
* Builds two seeded synthetic repos (int PK and string PK) with the reference's own
  ``Legend``/``Schema``/``msg_pack``/path encoders and edge-case values (NaN, -0.0, int/float/bool
  equality, 2**53+1, bin vs ext 'G', schema change with added/dropped columns, negative and
  wrapped PKs) and diffs them with the reference as above.
* EnvelopeEncoder / union_of_envelopes / bbox / GPKG envelope vectors straight from the
  reference functions (kart/spatial_filter/index.py:485-548,835-867; __init__.py:709-734;
  kart/geometry.py:638-700), including the 9 KATs of tests/test_spatial_filter_index.py:191-222.
"""
import binascii
import json
import math
import os
import random
import shutil
import struct
import subprocess
import sys
import tarfile

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402

REF = refshim.REF
WORK = "/tmp/kart_amd_golden"
OUT = HERE

d3m = refshim.ref("dataset3")
diff_util = refshim.ref("diff_util")
su = refshim.ref("serialise_util")
schema_m = refshim.ref("schema")
paths_m = refshim.ref("dataset3_paths")
bdw = refshim.ref("base_diff_writer")
geom_m = refshim.ref("geometry")
sf_init = refshim.ref("spatial_filter")
sf_index = refshim.ref("spatial_filter.index")
structure_m = refshim.ref("structure")

_NULL = object()


# ---------------------------------------------------------------------------------------------
def extract(tgz, name):
    dst = os.path.join(WORK, name)
    if os.path.exists(dst):
        shutil.rmtree(dst)
    os.makedirs(dst)
    with tarfile.open(tgz) as t:
        t.extractall(dst)
    # the archive holds one top-level dir whose .git file points at .kart
    (top,) = [d for d in os.listdir(dst)]
    return os.path.join(dst, top, ".kart")


def json_safe(v):
    """Encode a decoded feature value for the golden JSON (type-tagged, lossless)."""
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
    if isinstance(v, bytes):
        return {"bytes": v.hex(), "geom": isinstance(v, geom_m.Geometry)}
    return {"repr": repr(v)}


def changed_fields(old, new):
    """The field-diff decision of kart/text_diff_writer.py:135-145 (reference functions)."""
    out = []
    for k in bdw.BaseDiffWriter._all_feature_keys(old, new):
        if k.startswith("__"):
            continue
        if old.get(k, _NULL) == new.get(k, _NULL):
            continue
        out.append(k)
    return out


class Side:
    """Packed leaf arrays of one commit's dataset feature tree."""

    def __init__(self, repo, spec, ds_path):
        self.spec = spec
        self.repo = repo
        self.ds = refshim.dataset3(repo, spec, ds_path) if spec else None
        self.names, self.oids = [], []
        if self.ds is not None:
            inner = f"{ds_path}/.table-dataset/feature/"
            for path, oid in repo.ls_tree_r(spec, inner):
                self.names.append(path[len(inner):])
                self.oids.append(oid)

    def schema_json(self):
        if self.ds is None:
            return None
        return self.ds.get_meta_item("schema.json")

    def meta_files(self):
        """{path relative to the meta tree: raw bytes} (legends left out: they are stored apart)"""
        if self.ds is None:
            return None
        pre = f"{self.ds.path}/.table-dataset/meta/"
        return {p[len(pre):]: self.repo.blob_data(o) for p, o in self.repo.ls_tree_r(self.spec, pre)
                if not p[len(pre):].startswith("legend/")}

    def attachments(self):
        """{name: raw bytes} of the blobs beside .table-dataset (the metadata.xml attachment)"""
        if self.ds is None:
            return None
        return {b.name: bytes(b.data) for b in self.ds.tree if b.type_str == "blob"}

    def path_structure(self):
        if self.ds is None:
            return None
        return self.ds.feature_path_encoder.to_dict()


class Fixture:
    """Collects several sides + a shared blob arena into one compressed npz + one JSON."""

    def __init__(self, name, repo):
        self.name = name
        self.repo = repo
        self.blob_index = {}
        self.blob_data = []
        self.arrays = {}
        self.meta = {"name": name, "sides": {}, "cases": []}
        self.legends = {}

    def _blob(self, oid):
        if oid not in self.blob_index:
            self.blob_index[oid] = len(self.blob_data)
            self.blob_data.append(self.repo.blob_data(oid))
        return self.blob_index[oid]

    def add_side(self, key, side):
        names = [n.encode() for n in side.names]
        off = np.zeros(len(names) + 1, np.int64)
        if names:
            off[1:] = np.cumsum([len(n) for n in names])
        self.arrays[f"{key}_names"] = np.frombuffer(b"".join(names), np.uint8)
        self.arrays[f"{key}_name_off"] = off
        self.arrays[f"{key}_oid"] = np.array(
            [list(bytes.fromhex(o)) for o in side.oids], np.uint8
        ).reshape(-1, 20)
        self.arrays[f"{key}_blob"] = np.array(
            [self._blob(o) for o in side.oids], np.int64
        )
        if side.ds is not None:
            for name in side.names:
                pass
            # legends referenced by this side's blobs
            for oid in side.oids:
                data = self.repo.blob_data(oid)
                lh = su.msg_unpack(data)[0]
                if lh not in self.legends:
                    lg = side.ds.get_legend(lh)
                    self.legends[lh] = [list(lg.pk_columns), list(lg.non_pk_columns)]
        self.meta["sides"][key] = {
            "spec": side.spec,
            "n": len(names),
            "schema": side.schema_json(),
            "path_structure": side.path_structure(),
            "meta_files": {k: v.hex() for k, v in (side.meta_files() or {}).items()},
            "attachments": {k: v.hex() for k, v in (side.attachments() or {}).items()},
        }

    def save(self):
        off = np.zeros(len(self.blob_data) + 1, np.int64)
        if self.blob_data:
            off[1:] = np.cumsum([len(b) for b in self.blob_data])
        self.arrays["blob_data"] = np.frombuffer(b"".join(self.blob_data), np.uint8)
        self.arrays["blob_off"] = off
        self.meta["legends"] = self.legends
        np.savez_compressed(os.path.join(OUT, f"{self.name}.npz"), **self.arrays)
        with open(os.path.join(OUT, f"{self.name}.json"), "w") as f:
            json.dump(self.meta, f, indent=1, sort_keys=True)
        print(f"  wrote {self.name}: {len(self.blob_data)} blobs, {len(self.meta['cases'])} cases")


def golden_diff2(fx, base_key, target_key, base_side, target_side, ds_path, with_values=False):
    """Reference two-way diff via diff_util.get_dataset_diff semantics (swap+reverse)."""
    base_ds, target_ds = base_side.ds, target_side.ds
    params = {}
    if not base_ds:
        base_ds, target_ds = target_ds, base_ds
        params["reverse"] = True
    ds_diff = base_ds.diff(target_ds, **params)
    # diff_meta (kart/rich_base_dataset.py:183-195): the meta items' DeltaDiff, (key, old, new)
    meta_diff = sorted([k, d.old_value, d.new_value] for k, d in ds_diff.get("meta", {}).items())
    fdiff = ds_diff.get("feature")
    deltas = []
    counts = {}
    if fdiff:
        counts = fdiff.type_counts()
        for key, delta in fdiff.sorted_items():
            rec = {
                "type": delta.type,
                "old_pk": json_safe(delta.old_key),
                "new_pk": json_safe(delta.new_key),
            }
            if delta.type == "update":
                old, new = delta.old_value, delta.new_value
                rec["changed"] = changed_fields(old, new)
                if with_values:
                    rec["old"] = {k: json_safe(v) for k, v in old.items()}
                    rec["new"] = {k: json_safe(v) for k, v in new.items()}
            deltas.append(rec)
    fx.meta["cases"].append(
        {
            "kind": "diff2",
            "base": base_key,
            "target": target_key,
            "counts": counts,
            "deltas": deltas,
            "meta": meta_diff,
        }
    )
    return deltas


def golden_merge3(fx, repo, keys, specs, expect_conflicts=None, expect_entries=None):
    """libgit2 three-way OID rule over full trees (see module docstring)."""
    trees = [dict(repo.ls_tree_r(s)) for s in specs]
    paths = sorted(set().union(*[t.keys() for t in trees]), key=lambda p: p.encode())
    entries, conflicts = {}, []
    for p in paths:
        a, o, t = (tr.get(p) for tr in trees)
        if o == t:
            res = o
        elif a == o:
            res = t
        elif a == t:
            res = o
        else:
            conflicts.append({"path": p, "ancestor": a, "ours": o, "theirs": t})
            # pygit2 index iteration yields every stage; the dict keeps the last one.
            entries[p] = t or o or a
            continue
        if res is not None:
            entries[p] = res
    if expect_conflicts is not None:
        assert len(conflicts) == expect_conflicts, (fx.name, len(conflicts))
    if expect_entries is not None:
        assert len(entries) == expect_entries, (fx.name, len(entries))
    fx.meta["cases"].append(
        {
            "kind": "merge3",
            "sides": keys,
            "specs": specs,
            "n_entries": len(entries),
            "conflicts": conflicts,
            "entries_sha": sorted(entries.items()),
        }
    )
    return conflicts


# ---------------------------------------------------------------------------------------------
def real_repos():
    cases = [
        ("points", "nz_pa_points_topo_150k"),
        ("polygons", "nz_waca_adjustments"),
        ("table", "countiestbl"),
        ("string-pks", "nz_waca_adjustments"),
    ]
    for name, ds_path in cases:
        gitdir = extract(f"{REF}/tests/data/{name}.tgz", name)
        repo = refshim.GitRepo(gitdir)
        fx = Fixture(f"repo_{name.replace('-', '_')}", repo)
        head = Side(repo, "HEAD", ds_path)
        empty = Side(repo, None, ds_path)
        fx.add_side("head", head)
        fx.add_side("empty", empty)
        fx.meta["ds_path"] = ds_path
        ins = golden_diff2(fx, "empty", "head", empty, head, ds_path)
        assert all(d["type"] == "insert" for d in ins)
        golden_diff2(fx, "head", "empty", head, empty, ds_path)
        if name == "points":
            head1 = Side(repo, "HEAD^", ds_path)
            fx.add_side("head1", head1)
            fwd = golden_diff2(fx, "head1", "head", head1, head, ds_path, with_values=True)
            # tests/test_diff.py:1061-1084 pins exactly these 5 updates
            assert sorted(int(d["old_pk"]["int"]) for d in fwd) == [1095, 1166, 1168, 1181, 1182]
            golden_diff2(fx, "head", "head1", head, head1, ds_path, with_values=True)
            spatial_goldens(fx, head1, head)
        fx.save()


def conflict_repos():
    pinned = {
        "polygons": dict(expect_conflicts=4, expect_entries=237),
        "points": dict(expect_conflicts=4),
        "table": dict(expect_conflicts=4),
    }
    ds_paths = {"points": "nz_pa_points_topo_150k", "polygons": "nz_waca_adjustments", "table": "countiestbl"}
    for name in ("points", "polygons", "table"):
        gitdir = extract(f"{REF}/tests/data/conflicts/{name}.tgz", f"conflicts_{name}")
        repo = refshim.GitRepo(gitdir)
        ds_path = ds_paths[name]
        fx = Fixture(f"conflicts_{name}", repo)
        fx.meta["ds_path"] = ds_path
        sides = {}
        for key in ("ancestor", "ours", "theirs"):
            sides[key] = Side(repo, f"{key}_branch", ds_path)
            fx.add_side(key, sides[key])
        for a, b in (("ancestor", "ours"), ("ancestor", "theirs"), ("ours", "theirs"), ("theirs", "ours")):
            golden_diff2(fx, a, b, sides[a], sides[b], ds_path, with_values=True)
        conf = golden_merge3(
            fx, repo, ["ancestor", "ours", "theirs"],
            ["ancestor_branch", "ours_branch", "theirs_branch"], **pinned[name]
        )
        if name == "polygons":
            d3 = sides["ancestor"].ds
            pks = sorted(
                d3.decode_path_to_1pk(c["path"]) for c in conf
            )
            assert pks == [98001, 1452332, 1456853, 1456912], pks  # tests/test_conflicts.py:79-82
        fx.save()


# ---------------------------------------------------------------------------------------------
# Synthetic repos built with the reference's own encoders.
def _fast_import(gitdir, commits):
    """commits: list of (message, {path: bytes or None}) applied cumulatively; returns refs."""
    if os.path.exists(gitdir):
        shutil.rmtree(gitdir)
    subprocess.run(["git", "init", "-q", "--bare", gitdir], check=True)
    lines = []
    mark = 0
    for ci, (msg, files) in enumerate(commits):
        fmarks = {}
        for p, data in files.items():
            if data is None:
                continue
            mark += 1
            fmarks[p] = mark
            lines.append(b"blob\nmark :%d\ndata %d\n" % (mark, len(data)) + data + b"\n")
        m = msg.encode()
        lines.append(
            b"commit refs/heads/c%d\ncommitter golden <g@x> %d +0000\ndata %d\n%s\n"
            % (ci, 1600000000 + ci, len(m), m)
        )
        if ci > 0:
            lines.append(b"from refs/heads/c%d\n" % (ci - 1))
        for p, data in files.items():
            if data is None:
                lines.append(b"D %s\n" % p.encode())
            else:
                lines.append(b"M 100644 :%d %s\n" % (fmarks[p], p.encode()))
        lines.append(b"\n")
    subprocess.run(
        ["git", "fast-import", "--quiet"],
        input=b"".join(lines),
        env=dict(os.environ, GIT_DIR=gitdir),
        check=True,
    )


def _ds_meta_files(ds_path, schema, encoder, extra_legends=()):
    inner = f"{ds_path}/.table-dataset"
    files = {
        f"{inner}/meta/schema.json": schema.dumps(),
        f"{inner}/meta/title": b"synthetic",
        f"{inner}/meta/path-structure.json": json.dumps(encoder.to_dict()).encode(),
    }
    for lg in (schema.legend, *extra_legends):
        files[f"{inner}/meta/legend/{lg.hexhash()}"] = lg.dumps()
    return files


def _rand_value(rng, kind):
    if kind == "int":
        return rng.choice([0, 1, -1, 7, 2**31 - 1, -(2**31), 2**53 + 1, 2**63 - 1, -(2**63), 2**64 - 1, rng.randrange(-10**6, 10**6)])
    if kind == "float":
        return rng.choice([0.0, -0.0, 1.0, 0.5, float("nan"), float("inf"), -float("inf"), 1e308, 5e-324, float(2**53), rng.uniform(-1e3, 1e3)])
    if kind == "text":
        return rng.choice(["", "a", "abc", "Rākairoa", "x" * 40, "y" * 300, "z" * 70000 if rng.random() < 0.01 else "zz", None])
    if kind == "bool":
        return rng.choice([True, False, None])
    if kind == "blob":
        return rng.choice([b"", b"\x00", b"abc", bytes(range(40)), None])
    raise ValueError(kind)


def _point(rng):
    x = rng.uniform(-180, 180)
    y = rng.uniform(-90, 90)
    return geom_m.Geometry(b"GP\x00\x01\xe6\x10\x00\x00" + struct.pack("<bIdd", 1, 1, x, y))


# pairs of values that are equal under Python == but differ in msgpack bytes (and vice versa)
_EDGE_PAIRS = [
    ("int_vs_float", "mixed", 1, 1.0),
    ("bool_vs_int", "mixed", True, 1),
    ("false_vs_zero", "mixed", False, 0),
    ("negzero", "mixed", -0.0, 0.0),
    ("nan_nan", "mixed", float("nan"), float("nan")),
    ("big_int_float", "mixed", 2**53 + 1, float(2**53)),
    ("exact_big", "mixed", 2**53, float(2**53)),
    ("u64_vs_float", "mixed", 2**64 - 1, float(2**64)),
    ("i64min_float", "mixed", -(2**63), float(-(2**63))),
    ("str_vs_bytes", "mixed", "abc", b"abc"),
    ("none_vs_zero", "mixed", None, 0),
    ("none_none", "mixed", None, None),
    ("inf_inf", "mixed", float("inf"), float("inf")),
    ("f32_widen", "mixed", 0.5, 0.5),
    ("empty_str_vs_none", "mixed", "", None),
    ("int_vs_str", "mixed", 1, "1"),
    ("large_uint_eq", "mixed", 2**64 - 1, 2**64 - 1),
    ("float_vs_int_frac", "mixed", 2.5, 2),
]


def synthetic_int(schema_change=True):
    rng = random.Random(0x4B415254 + (0 if schema_change else 1))
    ds_path = "synth/points"
    enc = paths_m.PathEncoder.INT_PK_ENCODER
    cols_v1 = [
        {"name": "fid", "dataType": "integer", "size": 64, "id": "c-fid", "primaryKeyIndex": 0},
        {"name": "geom", "dataType": "geometry", "id": "c-geom", "geometryType": "POINT", "geometryCRS": "EPSG:4326"},
        {"name": "ival", "dataType": "integer", "size": 64, "id": "c-ival"},
        {"name": "fval", "dataType": "float", "size": 64, "id": "c-fval"},
        {"name": "txt", "dataType": "text", "id": "c-txt"},
        {"name": "flag", "dataType": "boolean", "id": "c-flag"},
        {"name": "raw", "dataType": "blob", "id": "c-raw"},
        {"name": "mixed", "dataType": "text", "id": "c-mixed"},
        {"name": "dropped", "dataType": "text", "id": "c-dropped"},
    ]
    # v2 drops "dropped", adds "added", reorders ival/fval, renames txt -> text2 (same id)
    cols_v2 = [cols_v1[0], cols_v1[1], cols_v1[3], cols_v1[2],
               dict(cols_v1[4], name="text2"), cols_v1[5], cols_v1[6], cols_v1[7],
               {"name": "added", "dataType": "integer", "size": 32, "id": "c-added"}]
    if not schema_change:
        cols_v2 = cols_v1
    s1 = schema_m.Schema.from_column_dicts(cols_v1)
    s2 = schema_m.Schema.from_column_dicts(cols_v2)
    ds1 = d3m.Dataset3.new_dataset_for_writing(ds_path, s1)
    kinds = {"ival": "int", "fval": "float", "txt": "text", "text2": "text", "flag": "bool", "raw": "blob", "added": "int", "dropped": "text"}

    pks = list(range(0, 600)) + [-1, -2, -64, -65, -4096, 64**5, -(64**5), 64**5 + 1,
                                 2**30, 2**30 + 63, -(2**30), 2**40 + 7, 2**62, -(2**63), 2**63 - 1]
    def feat(schema, pk, edge=None, side=0):
        f = {"fid": pk, "geom": _point(rng)}
        for c in schema.columns:
            if c.name in ("fid", "geom"):
                continue
            if c.name == "mixed":
                f[c.name] = edge[2 + side] if edge else None
            else:
                f[c.name] = _rand_value(rng, kinds[c.name])
        return f

    def encode(ds, schema, f):
        raw = schema.feature_to_raw_dict(f)
        path, data = ds.encode_raw_feature_dict(raw, schema.legend, relative=True, schema=schema)
        return f"{ds_path}/.table-dataset/{path}", data

    base_files = dict(_ds_meta_files(ds_path, s1, enc))
    feats1 = {}
    for i, pk in enumerate(pks):
        edge = _EDGE_PAIRS[i % len(_EDGE_PAIRS)] if i < 200 else None
        f = feat(s1, pk, edge, 0)
        feats1[pk] = (f, edge)
        p, d = encode(ds1, s1, f)
        base_files[p] = d
    # commit 2: schema v2; updates / deletes / inserts / identical rewrites
    ds2 = d3m.Dataset3.new_dataset_for_writing(ds_path, s2)
    target_files = dict(_ds_meta_files(ds_path, s2, enc, extra_legends=[s1.legend] if schema_change else []))
    del target_files[f"{ds_path}/.table-dataset/meta/title"]
    for i, pk in enumerate(pks):
        f1, edge = feats1[pk]
        r = rng.random()
        p1, _ = encode(ds1, s1, f1)
        if i < 200:
            # edge-pair column flips from value[0] to value[1]; everything else copied
            f2 = {c.name: f1.get("txt" if c.name == "text2" else c.name) for c in s2.columns}
            f2["mixed"] = edge[3]
            f2["added"] = None if rng.random() < 0.5 else 5
            p2, d2 = encode(ds2, s2, f2)
            target_files[p2] = d2
        elif r < 0.1:
            target_files[p1] = None  # delete
        elif r < 0.4:
            f2 = {c.name: f1.get("txt" if c.name == "text2" else c.name) for c in s2.columns}
            col = rng.choice(["geom", "ival", "fval", "text2", "flag", "raw", "added", None])
            if col == "geom":
                f2["geom"] = _point(rng)
            elif col is not None:
                f2[col] = _rand_value(rng, kinds[col])
            p2, d2 = encode(ds2, s2, f2)
            target_files[p2] = d2
        elif r < 0.5:
            # same values rewritten under the new legend: an update whose fields may all be equal
            f2 = {c.name: f1.get("txt" if c.name == "text2" else c.name) for c in s2.columns}
            p2, d2 = encode(ds2, s2, f2)
            target_files[p2] = d2
        # else: unchanged (old legend blob kept)
    for pk in list(range(10**6, 10**6 + 40)) + [-(10**9), 3 * 64**5 + 5]:
        f = feat(s2, pk)
        p, d = encode(ds2, s2, f)
        target_files[p] = d
    name = "synth_int" if schema_change else "synth_int_same"
    gitdir = os.path.join(WORK, name + ".git")
    _fast_import(gitdir, [("base", base_files), ("target", target_files)])
    repo = refshim.GitRepo(gitdir)
    fx = Fixture(name, repo)
    fx.meta["ds_path"] = ds_path
    base = Side(repo, "refs/heads/c0", ds_path)
    target = Side(repo, "refs/heads/c1", ds_path)
    fx.add_side("base", base)
    fx.add_side("target", target)
    golden_diff2(fx, "base", "target", base, target, ds_path, with_values=True)
    golden_diff2(fx, "target", "base", target, base, ds_path, with_values=True)
    fx.save()


def synthetic_str():
    rng = random.Random(0x53545250)
    ds_path = "synth/strtable"
    enc = paths_m.PathEncoder.GENERAL_ENCODER
    cols = [
        {"name": "code", "dataType": "text", "id": "c-code", "primaryKeyIndex": 0},
        {"name": "n", "dataType": "integer", "size": 64, "id": "c-n"},
        {"name": "label", "dataType": "text", "id": "c-label"},
    ]
    s1 = schema_m.Schema.from_column_dicts(cols)
    ds1 = d3m.Dataset3.new_dataset_for_writing(ds_path, s1)

    def encode(pk, n, label):
        raw = s1.feature_to_raw_dict({"code": pk, "n": n, "label": label})
        path, data = ds1.encode_raw_feature_dict(raw, s1.legend, relative=True, schema=s1)
        return f"{ds_path}/.table-dataset/{path}", data

    alphabet = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 _-ĀāēŌ日本"
    pks = set(["", "Dave", "a", "A", "é", "日本語", "x" * 200])
    while len(pks) < 700:
        pks.add("".join(rng.choice(alphabet) for _ in range(rng.randint(1, 24))))
    pks = sorted(pks)
    base_files = dict(_ds_meta_files(ds_path, s1, enc))
    target_files = {}
    vals = {}
    for pk in pks:
        vals[pk] = (rng.randint(-5, 5), rng.choice(["x", "y", None]))
        p, d = encode(pk, *vals[pk])
        base_files[p] = d
    for pk in pks:
        r = rng.random()
        p, _ = encode(pk, *vals[pk])
        if r < 0.1:
            target_files[p] = None
        elif r < 0.3:
            n, label = vals[pk]
            if rng.random() < 0.5:
                n = float(n) if rng.random() < 0.5 else n + 1
            else:
                label = rng.choice(["x", "y", "z", None])
            p2, d2 = encode(pk, n, label)
            target_files[p2] = d2
    for i in range(60):
        pk = f"new-{i}-" + "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 10)))
        p, d = encode(pk, i, "new")
        target_files[p] = d
    gitdir = os.path.join(WORK, "synth_str.git")
    _fast_import(gitdir, [("base", base_files), ("target", target_files)])
    repo = refshim.GitRepo(gitdir)
    fx = Fixture("synth_str", repo)
    fx.meta["ds_path"] = ds_path
    base = Side(repo, "refs/heads/c0", ds_path)
    target = Side(repo, "refs/heads/c1", ds_path)
    fx.add_side("base", base)
    fx.add_side("target", target)
    golden_diff2(fx, "base", "target", base, target, ds_path, with_values=True)
    fx.save()


# ---------------------------------------------------------------------------------------------
def spatial_goldens(fx, head1, head):
    """Envelope + bbox goldens for the points repo with the 'points-edit' filter.

    filter_env follows SpatialFilter.__init__ (kart/spatial_filter/__init__.py:520-531):
    OGR GetEnvelope of the bbox polygon -> (minx, maxx, miny, maxy).
    tests/test_spatial_filter.py:151 bbox_as_wkt_polygon(175.8, 175.9, -36.9, -37.1).
    """
    filter_env = (175.8, 175.9, -37.1, -36.9)
    out = []
    for side_key, side in (("head1", head1),):
        for name, oid in zip(side.names, side.oids):
            blob = fx.repo.blob_data(oid)
            feat = side.ds.get_feature(path=name, data=memoryview(blob))
            g = feat["geom"]
            env = g.envelope(only_2d=True) if g is not None else None
            if env is None and g is not None:
                # OGR GetEnvelope of a point = (x, x, y, y) (geometry.py:679-687 fallback)
                flags = g[3]
                off = 8 + geom_m.gpkg_envelope_size(flags)
                le = g[off] == 1
                x, y = struct.unpack_from("<dd" if le else ">dd", g, off + 5)
                env = (x, x, y, y)
            hit = sf_init.bbox_intersects_fast(filter_env, env) if env is not None else True
            if hit:
                out.append(name)
    assert len(out) == 13, len(out)  # tests/test_spatial_filter.py:682
    fx.meta["spatial"] = {"filter_env": filter_env, "side": "head1", "matching_names": out}


def envelope_goldens():
    rng = random.Random(0x454E56)
    E = sf_index.EnvelopeEncoder()
    kats = [
        ((0, 0, 0, 0), "7ffff7ffff8000080000"),
        ((1e-10, 1e-10, 1e-10, 1e-10), "7ffff7ffff8000080000"),
        ((-1e-10, -1e-10, -1e-10, -1e-10), "7ffff7ffff8000080000"),
        ((-180, -90, 180, 90), "0000000000ffffffffff"),
        ((-90, -10, 90, 10), "3ffff71c71c00008e38e"),
        ((90, -20, -90, 20), "bffff638e3400009c71c"),
        ((-45.830, 65.173, -43.232, 65.745), "5f68edcb0b6141edd810"),
        ((174.958, -37.198, 174.992, -37.190), "fc6a14b189fc7054b1b9"),
        ((178.723, 0.148, -175.234, 2.538), "ff1778035d0363a839c1"),
    ]
    for env, hx in kats:  # tests/test_spatial_filter_index.py:191-222
        assert E.encode(env).hex() == hx
    encode_vectors = [[list(map(float, env)), hx] for env, hx in kats]
    edge_vals = [-180.0, 180.0, -90.0, 90.0, 0.0, -0.0, 179.99999999999997, -179.99999999999997,
                 1e-300, -1e-300, 89.99999999, 45.0, 12.345678901234567]
    for i in range(3000):
        if i % 10 == 0:
            w, e = rng.choice(edge_vals), rng.choice(edge_vals)
            s, n = rng.choice(edge_vals), rng.choice(edge_vals)
            w = max(-180.0, min(180.0, w)); e = max(-180.0, min(180.0, e))
            s = max(-90.0, min(90.0, s)); n = max(-90.0, min(90.0, n))
        else:
            w, e = rng.uniform(-180, 180), rng.uniform(-180, 180)
            s, n = sorted([rng.uniform(-90, 90), rng.uniform(-90, 90)])
        encode_vectors.append([[w, s, e, n], E.encode((w, s, e, n)).hex()])
    bits_vectors = []
    for bits in (8, 16, 20, 24, 32):
        Eb = sf_index.EnvelopeEncoder(bits)
        for i in range(200):
            w, e = rng.uniform(-180, 180), rng.uniform(-180, 180)
            s, n = sorted([rng.uniform(-90, 90), rng.uniform(-90, 90)])
            enc = Eb.encode((w, s, e, n))
            bits_vectors.append([bits, [w, s, e, n], enc.hex(), [x.hex() for x in Eb.decode(enc)]])
    # decode + cyclic overlap (spatial_filter.cpp:170-208 semantics; decode per index.py:532-548)
    overlap_vectors = []
    queries = [(175.8, -37.1, 175.9, -36.9), (170.0, -50.0, -170.0, 50.0), (-10.0, -10.0, 10.0, 10.0),
               (-180.0, -90.0, 180.0, 90.0), (179.0, 0.0, -179.0, 1.0)]
    for i in range(2000):
        w, e = rng.uniform(-180, 180), rng.uniform(-180, 180)
        if rng.random() < 0.7:
            e = min(180.0, w + abs(rng.gauss(0, 5)))
        s, n = sorted([rng.uniform(-90, 90), rng.uniform(-90, 90)])
        enc = E.encode((w, s, e, n))
        overlap_vectors.append([enc.hex(), [x.hex() for x in E.decode(enc)]])
    # union_of_envelopes (index.py:835-867) incl. tests/test_spatial_filter_index.py:525-543
    union_vectors = []
    ukats = [((1, 2, 3, 4), (5, 6, 7, 8)), ((3, 2, 7, 8), (1, 4, 5, 6)), ((-10, -1, 10, 1), (-1, -10, 1, 10)),
             ((170, 2, 175, 4), (-165, 6, -160, 8)), ((0, 2, 10, 6), (170, 4, -150, 8)), ((0, 2, 10, 6), (160, 4, -160, 8))]
    for a, b in ukats:
        union_vectors.append([list(map(float, a)), list(map(float, b)), list(map(float, sf_index.union_of_envelopes(a, b)))])
    for i in range(500):
        a = [rng.uniform(-180, 180), rng.uniform(-90, 0), rng.uniform(-180, 180), rng.uniform(0, 90)]
        b = [rng.uniform(-180, 180), rng.uniform(-90, 0), rng.uniform(-180, 180), rng.uniform(0, 90)]
        union_vectors.append([a, b, [float(x) for x in sf_index.union_of_envelopes(tuple(a), tuple(b))]])
    # bbox_intersects_fast (spatial_filter/__init__.py:709-734)
    bbox_vectors = []
    base = [-1.0, 0.0, 1.0, 2.0, 3.0]
    for i in range(3000):
        if i < 1500:
            a1, a2 = sorted(rng.choices(base, k=2)); a3, a4 = sorted(rng.choices(base, k=2))
            b1, b2 = sorted(rng.choices(base, k=2)); b3, b4 = sorted(rng.choices(base, k=2))
        else:
            a1, a2 = sorted([rng.uniform(-5, 5), rng.uniform(-5, 5)]); a3, a4 = sorted([rng.uniform(-5, 5), rng.uniform(-5, 5)])
            b1, b2 = sorted([rng.uniform(-5, 5), rng.uniform(-5, 5)]); b3, b4 = sorted([rng.uniform(-5, 5), rng.uniform(-5, 5)])
        a, b = (a1, a2, a3, a4), (b1, b2, b3, b4)
        bbox_vectors.append([list(a), list(b), bool(sf_init.bbox_intersects_fast(a, b))])
    # identity-CRS get_envelope_for_indexing pieces: _wrap_lon, _buffer_minmax_envelope via
    # transform_minmax_envelope with an identity transform stand-in (index.py:639-707)
    class IdentityTransform:
        desc = "identity"
        def TransformPoint(self, x, y, z=0):
            return (x, y, z)
    wrap_vectors = []
    for x in [-540.0, -360.0, -180.0, -179.5, -0.0, 0.0, 179.9, 180.0, 180.1, 359.0, 360.0, 540.0, 1e-300, -1e-300] + [rng.uniform(-720, 720) for _ in range(500)]:
        wrap_vectors.append([x.hex(), sf_index._wrap_lon(x).hex()])
    buffer_vectors = []
    for i in range(1000):
        minx = rng.uniform(-179, 179); miny = rng.uniform(-89, 89)
        w = 10 ** rng.uniform(-7, 1.5); h = 10 ** rng.uniform(-7, 1.5)
        if i % 7 == 0:
            w = 0.0
        env = (minx, miny, minx + w, min(90.0, miny + h))
        width, height = env[2] - env[0], env[3] - env[1]
        if env[0] == env[2] and env[1] == env[3]:
            res = sf_index.transform_minmax_envelope(env, IdentityTransform())
        elif width >= 180:
            res = None
        elif max(width, height) < 1.0:
            t = sf_index._buffer_minmax_envelope(env, 0.1 * max(width, height))
            res = (sf_index._wrap_lon(t[0]), t[1], sf_index._wrap_lon(t[2]), t[3])
        else:
            t = sf_index._buffer_minmax_envelope(env, 0.1)  # identity: segmented ring env == env
            res = (sf_index._wrap_lon(t[0]), t[1], sf_index._wrap_lon(t[2]), t[3])
        buffer_vectors.append([[v.hex() for v in env], None if res is None else [float(v).hex() for v in res]])
    # GPKG header envelope (geometry.py:638-700) over hand-built headers (LE/BE, XY/XYZ/XYM/XYZM, empty, NaN)
    gpkg_vectors = []
    for i in range(400):
        etype = rng.choice([0, 1, 2, 3, 4])
        le = rng.random() < 0.8
        empty = rng.random() < 0.05
        flags = (1 if le else 0) | (etype << 1) | (0x10 if empty else 0)
        n = {0: 0, 1: 4, 2: 6, 3: 6, 4: 8}[etype]
        vals = [rng.uniform(-200, 200) for _ in range(n)]
        if n and rng.random() < 0.05:
            vals[rng.randrange(n)] = float("nan")
        bo = "<" if le else ">"
        hdr = b"GP\x00" + bytes([flags]) + struct.pack(bo + "i", 4326) + struct.pack(bo + "d" * n, *vals)
        wkb = struct.pack("<bIdd", 1, 1, rng.uniform(-180, 180), rng.uniform(-90, 90))
        g = hdr + wkb
        env = geom_m.geom_envelope(g, only_2d=True)
        gpkg_vectors.append([g.hex(), None if env is None else [float(v).hex() for v in env]])
    out = {
        "encode": encode_vectors,
        "bits": bits_vectors,
        "decode": overlap_vectors,
        "queries": queries,
        "union": union_vectors,
        "bbox": bbox_vectors,
        "wrap_lon": wrap_vectors,
        "identity_env": buffer_vectors,
        "gpkg_env": gpkg_vectors,
    }
    with open(os.path.join(OUT, "envelopes.json"), "w") as f:
        json.dump(out, f)
    print("  wrote envelopes.json")


def path_goldens():
    """IntPathEncoder / MsgpackHashPathEncoder KATs + seeded vectors (dataset3_paths.py)."""
    rng = random.Random(0x50415448)
    out = {"int": [], "hash": [], "legacy": []}
    ie = paths_m.PathEncoder.INT_PK_ENCODER
    ge = paths_m.PathEncoder.GENERAL_ENCODER
    le = paths_m.PathEncoder.LEGACY_ENCODER
    ints = [0, 1, -1, 1181, 64**5, -(64**5), 2**63 - 1, -(2**63), 2**30, -(2**30) - 1]
    ints += [rng.randrange(-(2**63), 2**63) for _ in range(300)] + [rng.randrange(-10**7, 10**7) for _ in range(300)]
    for pk in ints:
        out["int"].append([str(pk), ie.encode_pks_to_path([pk])])
        out["legacy"].append([str(pk), le.encode_pks_to_path([pk])])
    strs = ["", "Dave", "a", "é", "日本語"] + ["".join(chr(rng.randrange(32, 0x3000)) for _ in range(rng.randint(1, 20))) for _ in range(200)]
    for s in strs:
        out["hash"].append([s, ge.encode_pks_to_path([s])])
        out["legacy"].append(["s:" + s, le.encode_pks_to_path([s])])
    assert ie.encode_pks_to_path([1181]) == "A/A/A/S/kc0EnQ=="  # tests/test_structure.py:915
    assert ge.encode_pks_to_path(["Dave"]) == "s/v/7/j/kaREYXZl"  # tests/test_structure.py:884
    with open(os.path.join(OUT, "paths.json"), "w") as f:
        json.dump(out, f, ensure_ascii=False)
    print("  wrote paths.json")


WKT_A = ('GEOGCS["WGS 84",DATUM["WGS_1984", SPHEROID["WGS 84",6378137,298.257223563,AUTHORITY["EPSG","7030"]],'
         'AUTHORITY["EPSG","6326"]],\n  PRIMEM["Greenwich",0,AUTHORITY["EPSG","8901"]],UNIT["degree",0.0174532925199433,'
         'AUTHORITY["EPSG","9122"]],AXIS["Latitude",NORTH],AXIS["Longitude",EAST],AUTHORITY["EPSG","4326"]]')
WKT_B = ('PROJCS["NZGD2000 / New Zealand Transverse Mercator 2000",GEOGCS["NZGD2000",DATUM["New_Zealand_Geodetic_Datum_2000",'
         'SPHEROID["GRS 1980",6378137,298.257222101]],PRIMEM["Greenwich",0],UNIT["degree",0.0174532925199433]],'
         'PROJECTION["Transverse_Mercator"],PARAMETER["latitude_of_origin",0],PARAMETER["central_meridian",173],'
         'PARAMETER["scale_factor",0.9996],PARAMETER["false_easting",1600000],PARAMETER["false_northing",10000000],'
         'UNIT["metre",1],AUTHORITY["EPSG","2193"]]')


WKT_CASES = ['GEOGCS["a",DATUM["b"]]', '  A [ 1 ,2.5e3, "x""y" ] ', 'A[B[1],C[2,D[3]],E]', 'A[1,]]',
             'A[1,]]\nB[2,C[3]]', 'x\r\ny', '1.5.3,[$', '\n\nA(1 , -0.5E+3 ,B("q"))\n\n', 'A[007,-0,1e5]', WKT_A, WKT_B,
             'A["unterminated, B[1]]', 'Ω[1,Ж[2]]', '\ufeffA[1]', '\tA[\t1,\r2]']


def wkt_goldens():
    """crs_util.normalise_wkt (kart/crs_util.py:204-209) on crafted WKT: whitespace, nesting, error
    characters, unbalanced brackets, newlines, non-ASCII keywords"""
    cu = refshim.ref("crs_util")
    out = [[w, cu.normalise_wkt(w)] for w in WKT_CASES]
    with open(os.path.join(OUT, "wkt.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"  wrote wkt.json: {len(out)} cases")


def meta_edits():
    """A dataset whose meta items change: title, description, CRS definitions (odd whitespace,
    nested, added, removed), the metadata.xml attachment, a schema.json that only changes its
    formatting (normalised: no item change), and non-standard meta files (never items)."""
    schema = schema_m.Schema.from_column_dicts([
        {"id": "m-fid", "name": "fid", "dataType": "integer", "primaryKeyIndex": 0, "size": 64},
        {"id": "m-geom", "name": "geom", "dataType": "geometry", "geometryType": "POINT", "geometryCRS": "EPSG:4326"},
        {"id": "m-name", "name": "name", "dataType": "text", "length": None},
    ])
    enc = paths_m.PathEncoder.INT_PK_ENCODER
    ds = "mds"
    inner = f"{ds}/.table-dataset"
    base = _ds_meta_files(ds, schema, enc)
    raw_schema = json.loads(schema.dumps())
    feats = {}
    rng = random.Random(11)
    for pk in range(20):
        feats[f"{inner}/feature/{enc.encode_pks_to_path([pk])}"] = su.msg_pack(
            [schema.legend.hexhash(), [_point(rng), f"n{pk}"]])
    c0 = dict(base, **feats)
    c0[f"{inner}/meta/title"] = b"Title A"
    c0[f"{inner}/meta/crs/EPSG:4326.wkt"] = WKT_A.encode()
    c0[f"{inner}/meta/custom.json"] = b'{"x": 1}'
    c0[f"{ds}/metadata.xml"] = b"<gmd:MD_Metadata>one</gmd:MD_Metadata>"
    c1 = {
        f"{inner}/meta/title": b"Title B",
        f"{inner}/meta/description": "A longer description \u2014 with non-ASCII".encode(),
        f"{inner}/meta/crs/EPSG:4326.wkt": (WKT_A.replace(",", ",  ") + "\r\n").encode(),  # same tokens
        f"{inner}/meta/crs/EPSG:2193.wkt": WKT_B.encode(),
        f"{inner}/meta/custom.json": b'{"x": 2}',
        f"{ds}/metadata.xml": b"<gmd:MD_Metadata>two</gmd:MD_Metadata>",
        # the same columns with explicit nulls and another key order: normalised to the same item
        f"{inner}/meta/schema.json": json.dumps([dict(reversed(list(c.items())), extra=None) for c in raw_schema]).encode(),
    }
    c2 = {
        f"{inner}/meta/title": b"",
        f"{inner}/meta/crs/EPSG:4326.wkt": None,
        f"{inner}/meta/crs/nested/EPSG:3857.wkt": b'PROJCS["Pseudo",GEOGCS["WGS 84"],UNIT["metre",1]]',
        f"{ds}/metadata.xml": None,
        f"{inner}/meta/description": None,
    }
    gitdir = os.path.join(WORK, "meta_edits.git")
    _fast_import(gitdir, [("c0", c0), ("c1", c1), ("c2", c2)])
    repo = refshim.GitRepo(gitdir)
    fx = Fixture("meta_edits", repo)
    fx.meta["ds_path"] = ds
    sides = {k: Side(repo, f"c{i}", ds) for i, k in enumerate(("c0", "c1", "c2"))}
    sides["empty"] = Side(repo, None, ds)
    for k, sd in sides.items():
        fx.add_side(k, sd)
    for a, b in (("c0", "c1"), ("c1", "c2"), ("c0", "c2"), ("c2", "c0"), ("empty", "c0"), ("c1", "empty")):
        golden_diff2(fx, a, b, sides[a], sides[b], ds)
    (c01,) = [c for c in fx.meta["cases"] if c["base"] == "c0" and c["target"] == "c1"]
    assert {k for k, _, _ in c01["meta"]} == {"title", "description", "crs/EPSG:2193.wkt", "metadata.xml"}, c01["meta"]
    fx.save()


if __name__ == "__main__":
    os.makedirs(WORK, exist_ok=True)
    which = sys.argv[1:] or ["paths", "envelopes", "real", "conflicts", "synth", "meta"]
    if "paths" in which:
        path_goldens()
    if "envelopes" in which:
        envelope_goldens()
    if "real" in which:
        real_repos()
    if "conflicts" in which:
        conflict_repos()
    if "synth" in which:
        synthetic_int(True)
        synthetic_int(False)
        synthetic_str()
    if "meta" in which:
        meta_edits()
        wkt_goldens()
