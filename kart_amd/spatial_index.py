"""Spatial-filter index of a repository's history: the feature envelopes Kart's
spatial-filtered clone / fetch serve from, computed for every feature blob of the commits to index.

Mirrors ``update_spatial_filter_index`` (kart/spatial_filter/index.py:273-371):

* which blobs — ``iter_feature_oids`` runs ``git rev-list --objects`` over the commits to index
  ``--not`` the already-indexed ones (:193-206); here the commit graph is read from the object
  store and each commit's feature trees are walked against each of its parents with ``kd_walk``'s
  tree-OID pruning, so unchanged subtrees are never opened;
* the geometry of each blob — ``get_geometry`` (:463-483): the legend's geometry value;
* its envelope — ``get_envelope_for_indexing`` + ``EnvelopeEncoder.encode`` (:485-579) for an
  identity CRS (EPSG:4326), computed on the GPU for all blobs in one ``kd_geom_filter`` call (the
  new-side index envelopes), empty and null geometries skipped as the reference skips them;
* the ``feature_envelopes`` / ``commits`` tables of ``feature_envelopes.db`` (:175-191, :340-371),
  with ``_build_on_last_index`` (:232-263): the commits table holds the minimal description of
  everything indexed, and a later run stops at those commits.

Datasets whose CRS is not EPSG:4326 need PROJ (out of scope): they are skipped and reported.

``CloneFilter`` is the other end: the clone-time decision git's spatial-filter extension makes per
object from this index (sf_filter_blob, vendor/spatial-filter/spatial_filter.cpp:212-260), for a
whole batch of objects per GPU call.
"""
import ctypes
import json
import os
import re
import sqlite3

import numpy as np

from . import _native as N
from .gitsource import GitRepo, _HEX40
from .odb import OBJ_COMMIT
from .schema import Legend, Schema

DS_FEATURE = re.compile(r"^(.+)/\.(sno|table)-dataset/feature/.+$")
FEATURE_ENVELOPES_DB = "feature_envelopes.db"
WORLD = (-180.0, 180.0, -90.0, 90.0)


# ---- the commit graph ---------------------------------------------------------------------------
def commit_info(repo, oid):
    """(tree hex, [parent hex]) of a commit, read from the object store"""
    t, data = repo._read(oid)
    if t != OBJ_COMMIT:
        raise ValueError(f"{oid} is not a commit")
    tree, parents = None, []
    for line in data.split(b"\n"):
        if not line:
            break
        if line.startswith(b"tree "):
            tree = line[5:45].decode()
        elif line.startswith(b"parent "):
            parents.append(line[7:47].decode())
    return tree, parents


def _ancestors(repo, commits, cache):
    seen, stack = set(), list(commits)
    while stack:
        c = stack.pop()
        if c in seen:
            continue
        seen.add(c)
        if c not in cache:
            cache[c] = commit_info(repo, c)
        stack.extend(cache[c][1])
    return seen


def commits_to_index(repo, start, stop, cache=None):
    """the commits reachable from ``start`` and not from ``stop`` (rev-list START --not STOP),
    parents before children"""
    cache = {} if cache is None else cache
    done = _ancestors(repo, stop, cache)
    order, seen = [], set()
    for s in start:
        stack = [(s, False)]
        while stack:
            c, expanded = stack.pop()
            if c in done or (c in seen and not expanded):
                continue
            if expanded:
                order.append(c)
                continue
            seen.add(c)
            if c not in cache:
                cache[c] = commit_info(repo, c)
            stack.append((c, True))
            stack.extend((p, False) for p in cache[c][1] if p not in seen and p not in done)
    return order


def minimal_description(repo, commits, cache=None):
    """the commits of the set that are not ancestors of another commit of the set
    (git merge-base --independent, :209-229)"""
    cache = {} if cache is None else cache
    commits = set(commits)
    out = set()
    for c in commits:
        others = commits - {c}
        if not others or c not in _ancestors(repo, others, cache):
            out.add(c)
    return out


def iter_feature_oids(repo, start, stop, cache=None):
    """{(dataset path, blob oid hex)} of every feature blob reachable from ``start`` and not from
    ``stop`` (iter_feature_oids, :193-206): per commit, the feature blobs at paths where it differs
    from every one of its parents (a blob a merge takes from one parent is that parent's, not
    new), from pruned walks of the commit against each parent"""
    cache = {} if cache is None else cache
    out = set()

    def tree_of(c):
        if c not in cache:
            cache[c] = commit_info(repo, c)
        return cache[c][0]

    def feature_leaves(lv):
        got = set()
        for i in range(lv.n):
            m = DS_FEATURE.match(lv.path(i))
            if m:
                got.add((lv.path(i), m.group(1), lv.oids[i].tobytes().hex()))
        return got

    for c in commits_to_index(repo, start, stop, cache):
        tree, parents = cache[c]
        if not parents:
            (lv,) = repo.odb.walk([tree], "")
            new = feature_leaves(lv)
        else:
            new = None
            for p in parents:
                _, lv = repo.odb.walk([tree_of(p), tree], "", compare=(0, 1))
                changed = feature_leaves(lv)
                new = changed if new is None else new & changed
                if not new:
                    break
        out.update((d, o) for _, d, o in new)
    return out


# ---- per-dataset geometry columns and CRS ----------------------------------------------------------
def _dataset_meta(repo, commits, ds_paths, cache):
    """per dataset: the legends and geometry column ids seen in the given commits, and whether every
    CRS it carries is EPSG:4326 (identity to the index's CRS)"""
    info = {d: {"legends": {}, "geom_ids": set(), "crs": set()} for d in ds_paths}
    for c in commits:
        tree = cache[c][0] if c in cache else commit_info(repo, c)[0]
        for d in ds_paths:
            for kind in ("table", "sno"):
                (lv,) = repo.odb.walk([tree], f"{d}/.{kind}-dataset/meta")
                if not lv.present:
                    continue
                for rel, oid in lv.items():
                    if rel.startswith("legend/"):
                        h = rel[len("legend/"):]
                        if h not in info[d]["legends"]:
                            info[d]["legends"][h] = Legend.loads(repo.cat(oid))
                    elif rel == "schema.json":
                        sch = Schema.from_column_dicts(json.loads(repo.cat(oid)))
                        info[d]["geom_ids"].update(col.id for col in sch.geometry_columns)
                    elif rel.startswith("crs/"):
                        info[d]["crs"].add((rel[len("crs/"):], repo.cat(oid)))
    return info


def is_identity_crs(name, wkt):
    """EPSG:4326, the index's own CRS (CrsHelper.target_crs): no transform needed"""
    if name.upper().startswith("EPSG:4326"):
        return True
    t = wkt.decode(errors="replace") if isinstance(wkt, bytes) else wkt
    m = re.findall(r'AUTHORITY\["EPSG",\s*"(\d+)"\]\s*\]\s*$', t.strip())
    return bool(m) and m[-1] == "4326"


def _geom_cols(info):
    """a kd_geom_cols stand-in whose new side lists every legend of the dataset with the value
    index of its first geometry column (get_geometry's legend -> column cache, :463-483)"""
    from .spatial import GeomCols

    hashes = sorted(info["legends"])
    gidx = []
    for h in hashes:
        nonpk = list(info["legends"][h].non_pk_columns)
        gidx.append(next((i for i, cid in enumerate(nonpk) if cid in info["geom_ids"]), -1))
    gc = GeomCols.__new__(GeomCols)
    hexarr = np.frombuffer(b"".join(h.encode() for h in hashes), np.uint8).copy() if hashes else np.zeros(40, np.uint8)
    gc.old_hex = gc.new_hex = hexarr
    gc.old_gidx = gc.new_gidx = np.asarray(gidx or [0], np.int16)
    gc.old_map = gc.new_map = dict(zip(hashes, gidx))
    return gc


# ---- the index ---------------------------------------------------------------------------------
def _open_db(path, clear_existing):
    db = sqlite3.connect(path)
    if clear_existing:
        db.execute("DROP TABLE IF EXISTS commits;")
        db.execute("DROP TABLE IF EXISTS feature_envelopes;")
    db.execute("CREATE TABLE IF NOT EXISTS commits (commit_id BLOB NOT NULL PRIMARY KEY) WITHOUT ROWID;")
    db.execute("CREATE TABLE IF NOT EXISTS feature_envelopes (blob_id BLOB NOT NULL PRIMARY KEY, "
               "envelope BLOB NOT NULL) WITHOUT ROWID;")
    return db


def _index_envelopes(engine, data, off, pairs, cols, bits):
    """(codes, enc, enc_ok) of the blobs pairs[:, 1] of a host arena: the blob reader's 48-byte
    geometry heads (kd_geom_heads, host threads) are all that goes to the GPU
    (kd_geom_filter_heads); the few blobs whose head cannot decide (XYZ/XYM envelopes, NaN
    envelopes, unusual layouts) are sent whole through kd_geom_filter, so the result is the
    blob-arena kernel's on every row"""
    from .spatial import GEOM_HEAD, geom_filter, geom_filter_heads, geom_heads

    empty = (np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    heads = geom_heads(data, off, cols.new_hex, cols.new_gidx, len(cols.new_map))
    codes, _, enc, ok = geom_filter_heads(engine, np.zeros(0, GEOM_HEAD), heads, pairs, WORLD, False, bits)
    redo = np.nonzero(codes[:, 1] == 3)[0]
    if redo.size:
        rows = pairs[redo, 1].astype(np.int64)
        lens = (off[rows + 1] - off[rows]).astype(np.int64)
        sub_off = np.zeros(rows.size + 1, np.uint64)
        np.cumsum(lens, out=sub_off[1:])
        sub = np.concatenate([data[int(off[r]):int(off[r + 1])] for r in rows.tolist()]) if rows.size else empty[0]
        sp = np.full((rows.size, 2), N.KD_NONE, np.uint32)
        sp[:, 1] = np.arange(rows.size, dtype=np.uint32)
        c2, _, e2, o2 = geom_filter(engine, empty, (sub, sub_off), sp, cols, WORLD, False, bits)
        codes[redo], enc[redo], ok[redo] = c2, e2, o2
    return codes, enc, ok


def update_spatial_filter_index(engine, repo, commits, db_path=None, clear_existing=False, bits=None):
    """Index the feature envelopes of ``commits`` (revisions; their ancestors implicitly) into
    ``db_path`` (default <gitdir>/feature_envelopes.db), building on what is already indexed.
    Returns {"features": rows written, "commits": commits walked, "skipped": {dataset: reason},
    "fallback": blobs whose envelope needs OGR}."""
    if not isinstance(repo, GitRepo):
        raise TypeError("repo: a kart_amd.gitsource.GitRepo")
    db_path = db_path or os.path.join(repo.gitdir, FEATURE_ENVELOPES_DB)
    db = _open_db(db_path, clear_existing)
    cache = {}
    start = {repo.rev_parse(c) if not _HEX40.match(c) else c.lower() for c in commits}
    stop = {bytes(r[0]).hex() for r in db.execute("SELECT commit_id FROM commits;")}
    everything = minimal_description(repo, start | stop, cache)
    start = everything - stop
    out = {"features": 0, "commits": 0, "skipped": {}, "fallback": 0}
    if not start:
        db.close()
        return out
    if bits is None:
        ln = db.execute("SELECT length(envelope) FROM feature_envelopes LIMIT 1;").fetchone()
        bits = ln[0] * 8 // 4 if ln else 20
    walked = commits_to_index(repo, start, stop, cache)
    out["commits"] = len(walked)
    blobs = iter_feature_oids(repo, start, stop, cache)
    by_ds = {}
    for d, oid in blobs:
        by_ds.setdefault(d, []).append(oid)
    meta = _dataset_meta(repo, walked, list(by_ds), cache)
    rows = []
    for d, oids in sorted(by_ds.items()):
        info = meta[d]
        if not info["crs"]:
            out["skipped"][d] = "no CRS"  # CrsHelper finds no transform: the reference skips it
            continue
        if not all(is_identity_crs(n, w) for n, w in info["crs"]):
            out["skipped"][d] = "non-identity CRS (needs PROJ)"
            continue
        oids = sorted(oids)
        raw = np.frombuffer(b"".join(bytes.fromhex(o) for o in oids), np.uint8).reshape(-1, 20)
        data, off, status = repo.read_blobs(raw)
        present = np.nonzero(status == 0)[0]  # promised blobs: not indexable here (the reference skips them too)
        pairs = np.full((present.size, 2), N.KD_NONE, np.uint32)
        pairs[:, 1] = present.astype(np.uint32)
        codes, enc, ok = _index_envelopes(engine, data, off, pairs, _geom_cols(info), bits)
        out["fallback"] += int(np.count_nonzero(codes[:, 1] == 3))
        for j in np.nonzero(ok)[0].tolist():
            rows.append((raw[present[j]].tobytes(), enc[j].tobytes()))
    with db:
        db.executemany("INSERT OR REPLACE INTO feature_envelopes (blob_id, envelope) VALUES (?, ?);", rows)
        db.execute("DELETE FROM commits;")
        db.executemany("INSERT INTO commits (commit_id) VALUES (?);", [(bytes.fromhex(c),) for c in sorted(everything)])
    db.close()
    out["features"] = len(rows)
    return out


def read_index(db_path):
    """{blob oid hex: envelope bytes} and the indexed commits of an index database"""
    db = sqlite3.connect(db_path)
    try:
        env = {bytes(b).hex(): bytes(e) for b, e in db.execute("SELECT blob_id, envelope FROM feature_envelopes;")}
        commits = {bytes(c).hex() for (c,) in db.execute("SELECT commit_id FROM commits;")}
    finally:
        db.close()
    return env, commits


# ---- clone-time filtering: sf_filter_blob over batches -----------------------------------------
FEATURE_PATH_MARKERS = ("/.sno-dataset/feature/", "/.table-dataset/feature/")
SF_MATCH, SF_NOT_MATCHED, SF_ERROR = 0, 1, 2  # spatial_filter.cpp:154-158 (enum match_result)


_NUM = re.compile(r"\s*([+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?)")


def parse_filter_arg(filter_arg):
    """sf_init's bounds argument (spatial_filter.cpp:266-285): `while (ss >> d) { push(d); if (peek
    == ',') ignore(); }` — numbers with optional leading whitespace, each optionally followed by one
    comma; the first thing that is not a number ends the list (trailing text is ignored); exactly
    four numbers -> (w, s, e, n), else the reference's error."""
    text, pos, rect = str(filter_arg), 0, []
    while True:
        m = _NUM.match(text, pos)
        if m is None:
            break
        rect.append(float(m.group(1)))
        pos = m.end()
        if text[pos:pos + 1] == ",":
            pos += 1
    if len(rect) != 4:
        raise ValueError("spatial-filter: Error: invalid bounds, expected '<lng_w>,<lat_s>,<lng_e>,<lat_n>'")
    return tuple(rect)


class CloneFilter:
    """The git filter extension's per-object decision (sf_filter_blob,
    vendor/spatial-filter/spatial_filter.cpp:212-260) for batches of objects: feature_envelopes is
    loaded into HBM once (kd_sf_index_build), then every batch is one kd_sf_filter call.

    ``available`` is False when the repository has no index database: the reference then omits
    nothing (sf_init, :287-292), and so every object matches."""

    def __init__(self, engine, db_path, filter_arg):
        self.engine = engine
        self.q = parse_filter_arg(filter_arg)
        self._ix = ctypes.c_void_p()
        self.available = os.path.isfile(db_path)
        self.n_index = 0
        if not self.available:
            return
        db = sqlite3.connect(f"file:{db_path}?mode=ro", uri=True)
        try:
            rows = db.execute("SELECT blob_id, envelope FROM feature_envelopes;").fetchall()
        finally:
            db.close()
        self.n_index = len(rows)
        nbytes = len(rows[0][1]) if rows else 10
        if any(len(e) != nbytes for _, e in rows) or any(len(b) != 20 for b, _ in rows):
            raise ValueError("feature_envelopes: rows of different widths")
        self.bits = nbytes * 8 // 4  # sf_filter_blob: bits_per_value = num_bytes * 8 / 4
        oid = np.frombuffer(b"".join(bytes(b) for b, _ in rows), np.uint8) if rows else np.zeros(20, np.uint8)
        env = np.frombuffer(b"".join(bytes(e) for _, e in rows), np.uint8) if rows else np.zeros(nbytes, np.uint8)
        N.check(engine.L.kd_sf_index_build(engine.ctx, N.ptr(oid), N.ptr(env), len(rows), self.bits, N.KD_MEM_HOST,
                                            ctypes.byref(self._ix)), "kd_sf_index_build")

    def close(self):
        if self._ix:
            N.check(self.engine.L.kd_sf_index_free(self._ix), "kd_sf_index_free")
            self._ix = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def feature_paths(paths):
        """1 where the path is a feature blob's (the only objects the filter may omit)"""
        return np.fromiter((any(m in p for m in FEATURE_PATH_MARKERS) for p in paths), np.uint8, len(paths))

    def filter(self, oids, paths=None, is_feature=None):
        """MR codes (SF_MATCH / SF_NOT_MATCHED / SF_ERROR) of objects ``oids`` [m, 20]; ``paths``
        (their paths in the traversal) or ``is_feature`` flags decide which are feature blobs
        (neither: all are)"""
        oids = np.ascontiguousarray(oids, np.uint8).reshape(-1, 20)
        m = oids.shape[0]
        if is_feature is None and paths is not None:
            is_feature = self.feature_paths(paths)
        if not self.available or m == 0:
            return np.zeros(m, np.uint8)
        feat = None if is_feature is None else np.ascontiguousarray(is_feature, np.uint8)
        out = np.zeros(m, np.uint8)
        q = (ctypes.c_double * 4)(*self.q)
        N.check(self.engine.L.kd_sf_filter(self.engine.ctx, self._ix, N.ptr(oids), N.ptr(feat) if feat is not None else None,
                                           m, q, N.ptr(out), N.KD_MEM_HOST), "kd_sf_filter")
        return out
