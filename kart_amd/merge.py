"""Three-way merge classification behind Kart's merge boundary.

Mirrors, behind the same object shapes, what ``kart merge`` consumes from libgit2:

* ``merge_trees(engine, ancestor, ours, theirs)`` <- ``repo.merge_trees(ancestor, ours, theirs,
  flags={"find_renames": False})`` (kart/merge.py:99-100) for one dataset's feature tree: the GPU
  classify3 (kd_merge3) applies libgit2's per-path rule (o == t -> o; a == o -> t; a == t -> o; else
  conflict) and the result is a ``MergeIndex``.
* ``MergeIndex`` <- ``MergeIndex.from_pygit2_index`` (kart/merge_util.py:67-103): ``entries``
  ``{path: Entry(path, id, mode)}`` (every merged path; a conflicted path keeps its last stage, as
  iterating a pygit2 index does), ``conflicts`` ``{"0": AncestorOursTheirs(Entry | None x 3), ...}``
  in libgit2's (path) order, ``resolves``, iteration over entries, ``write_tree(repo)``.
* ``merge_repo(engine, repo, ancestor, ours, theirs)``: the whole-repository form — every dataset's
  feature tree through the GPU, the few other paths (meta items, repo structure files) by the same
  rule on the host.
* ``list_conflicts(merge_index, decode_path, summarise)`` <- kart/conflicts.py:22-132 for the
  summaries ``kart conflicts -s`` / ``-ss`` print (the per-value outputs need GDAL: out of scope).

The libgit2 text-automerge of a modify/modify pair whose blobs are both NUL-free (SURVEY §7 hard
part 6) is not reproduced: such conflicts are reported in ``MergeIndex.automerge_candidates`` so the
caller can send those paths through libgit2 (every GPKG geometry blob contains NUL; aspatial rows
may not).
"""
import subprocess
from collections import namedtuple

import numpy as np

from . import _native as N
from . import packing

FILEMODE_BLOB = 0o100644


class Entry(namedtuple("Entry", ("path", "id", "mode"))):
    """MergeIndex.Entry (kart/merge_util.py:82): path, hex blob id, file mode"""


class AncestorOursTheirs(namedtuple("AncestorOursTheirs", ("ancestor", "ours", "theirs"))):
    """kart/merge_util.py:28-65: the three versions of a conflict, always in this order"""

    NAMES = ("ancestor", "ours", "theirs")

    @staticmethod
    def partial(*, ancestor=None, ours=None, theirs=None):
        return AncestorOursTheirs(ancestor, ours, theirs)

    def map(self, fn, skip_nones=True):
        f = (lambda x: fn(x) if x else None) if skip_nones else fn
        return AncestorOursTheirs(*map(f, self))

    def as_dict(self):
        return dict(zip(self.NAMES, self))


AncestorOursTheirs.EMPTY = AncestorOursTheirs(None, None, None)


class _LazyEntries(dict):
    """{path: Entry} built on first use: a merge of 100M-feature layers should not pay for a Python
    dict of every path unless a caller asks for one"""

    def __init__(self, build):
        super().__init__()
        self._build = build

    def _fill(self):
        if self._build is not None:
            build, self._build = self._build, None
            for e in build():
                dict.__setitem__(self, e.path, e)

    def __len__(self):
        self._fill()
        return dict.__len__(self)

    def __iter__(self):
        self._fill()
        return dict.__iter__(self)

    def __getitem__(self, k):
        self._fill()
        return dict.__getitem__(self, k)

    def __contains__(self, k):
        self._fill()
        return dict.__contains__(self, k)

    def get(self, k, default=None):
        self._fill()
        return dict.get(self, k, default)

    def items(self):
        self._fill()
        return dict.items(self)

    def values(self):
        self._fill()
        return dict.values(self)

    def keys(self):
        self._fill()
        return dict.keys(self)

    def __eq__(self, other):
        self._fill()
        return dict.__eq__(self, other)

    def __setitem__(self, k, v):
        self._fill()
        dict.__setitem__(self, k, v)

    def __delitem__(self, k):
        self._fill()
        dict.__delitem__(self, k)


class MergeIndex:
    """The shape of kart.merge_util.MergeIndex as from_pygit2_index builds it."""

    Entry = Entry

    def __init__(self, entries, conflicts, resolves=None):
        self.entries = entries
        self.conflicts = conflicts
        self.resolves = dict(resolves or {})
        self.automerge_candidates = []  # conflict keys libgit2 might text-merge (NUL-free blobs)

    def __iter__(self):
        return iter(self.entries.values())

    def __getitem__(self, path):
        return self.entries[path]

    def __eq__(self, other):
        return isinstance(other, MergeIndex) and (self.entries, self.conflicts, self.resolves) == \
            (other.entries, other.conflicts, other.resolves)

    @property
    def unresolved_conflicts(self):
        return {k: c for k, c in self.conflicts.items() if k not in self.resolves}

    def add_resolve(self, key, resolve):
        if not isinstance(key, str):
            raise TypeError("resolve key must be str", type(key))
        self.resolves[key] = list(resolve)

    def write_tree(self, repo):
        """index.write_tree(repo) (kart/merge.py:122): the merged tree's id; like libgit2, refuses an
        index with unresolved conflicts.  ``repo``: kart_amd.gitsource.GitRepo."""
        if self.unresolved_conflicts:
            raise ValueError("cannot write a tree from an index with unresolved conflicts")
        lines = b"".join(b"%o %s\t%s\0" % (e.mode, e.id.encode(), e.path.encode()) for e in self.entries.values())
        return repo.write_index_tree(lines)


# ---------------------------------------------------------------------------------------------
def _side(version, encoding, engine=None):
    if version is None or version.n == 0:
        return packing.empty_side(encoding)
    return version.pack(engine)


def merge_trees(engine, ancestor, ours, theirs, prefix="", ours_all=None):
    """Three-way classification of one dataset's feature tree (DatasetVersion or None for each of
    ancestor / ours / theirs) -> MergeIndex of its feature paths (``prefix`` + relative path, e.g.
    "<ds>/.table-dataset/feature/").  Entries and conflicts follow libgit2's rule exactly.

    Versions from a pruned walk (``.partial``: only the subtrees where ours and theirs differ,
    gitsource.merge_versions) classify the same; ``ours_all() -> [(rel path, oid hex)]`` then lists
    every leaf of ours, for the merged entries outside those subtrees (ours == theirs there)."""
    present = next((v for v in (ours, theirs, ancestor) if v is not None), None)
    if present is None:
        return MergeIndex({}, {})
    vers = (ancestor, ours, theirs)
    sides = [_side(v, present.encoding, engine) for v in vers]
    r = engine.merge3(*sides)

    def entry(s, i):
        v, side = vers[s], sides[s]
        orig = int(side.order[i])
        return Entry(prefix + v.rel_path(orig), v.oids[orig].tobytes().hex(), FILEMODE_BLOB)

    rows = r.conflict.tolist()
    conf = [AncestorOursTheirs(*(entry(s, int(i)) if i != N.KD_NONE else None for s, i in enumerate(row)))
            for row in rows]
    mm = [all(i != N.KD_NONE for i in row) and _nul_free(vers, sides, row) for row in rows]
    order = sorted(range(len(conf)), key=lambda k: next(e for e in conf[k] if e).path.encode())  # libgit2: path bytes
    conflicts = {str(k): conf[j] for k, j in enumerate(order)}
    conf = [conf[j] for j in order]

    def build():
        if ours_all is not None and ours is not None and ours.partial:
            # outside the opened subtrees ours == theirs: the merge keeps ours
            opened = {ours.rel_path(i) for i in range(ours.n)}
            for rel, oid in ours_all():
                if rel not in opened:
                    yield Entry(prefix + rel, oid, FILEMODE_BLOB)
        # ours, then the merge deltas (take theirs) ...
        o = sides[1]
        skip = np.zeros(o.n, bool)
        md = r.mdelta
        if md.size:
            ro = md[:, 0][md[:, 0] != N.KD_NONE].astype(np.int64)
            skip[ro] = True
        for i in np.nonzero(~skip)[0].tolist():
            yield entry(1, i)
        for t in md[:, 1][md[:, 1] != N.KD_NONE].tolist():
            yield entry(2, int(t))
        # ... and every conflicted path with its last stage (theirs, else ours, else ancestor)
        for c in conf:
            yield c.theirs or c.ours or c.ancestor

    mi = MergeIndex(_LazyEntries(build), conflicts)
    mi.n_clean = r.n_clean
    mi.automerge_candidates = [str(k) for k, j in enumerate(order) if mm[j]]
    return mi


def _nul_free(vers, sides, row):
    """a modify/modify conflict whose ours and theirs blobs are both NUL-free in their first 8000
    bytes (libgit2's binary test): libgit2 would try a text merge there"""
    for s in (1, 2):
        try:
            data = vers[s].read_blob(int(sides[s].order[int(row[s])]))
        except KeyError:  # missing / promised: cannot tell, leave it to the caller
            return True
        if b"\0" in bytes(data[:8000]):
            return False
    return True


def merge_rule(a, o, t):
    """libgit2's per-path rule (kart/merge.py:99-100): (result, conflict?)"""
    if o == t:
        return o, False
    if a == o:
        return t, False
    if a == t:
        return o, False
    return None, True


def merge_repo(engine, repo, ancestor, ours, theirs):
    """repo.merge_trees for whole commits of a kart_amd.gitsource.GitRepo: every dataset's feature
    tree through merge_trees (GPU), the other paths (meta items, structure files) by the same rule on
    the host.  Conflict keys follow path order over the whole index."""
    specs = (ancestor, ours, theirs)
    ds_paths = sorted(set().union(*[repo.dataset_paths(s) for s in specs]))
    other = [repo.non_feature_entries(s) for s in specs]  # {path: (mode, oid)}
    entries, conf = {}, []
    for p in sorted(set().union(*[x.keys() for x in other]), key=lambda p: p.encode()):
        a, o, t = (x.get(p) for x in other)
        res, clash = merge_rule(a, o, t)
        ent = [Entry(p, x[1], x[0]) if x else None for x in (a, o, t)]
        if clash:
            conf.append(AncestorOursTheirs(*ent))
            last = ent[2] or ent[1] or ent[0]
            entries[p] = last
        elif res is not None:
            entries[p] = Entry(p, res[1], res[0])
    parts = []
    for ds in ds_paths:
        pre = f"{ds}/.table-dataset/feature/"
        vers = repo.merge_versions(*specs, ds)  # pruned to the subtrees where ours and theirs differ

        def ours_all(pre=pre):
            (lv,) = repo.walk([ours], pre.rstrip("/"))
            return lv.items()

        parts.append(merge_trees(engine, *vers, prefix=pre, ours_all=ours_all))
    for mi in parts:
        conf.extend(mi.conflicts.values())
    conf.sort(key=lambda c: next(e for e in c if e).path.encode())
    conflicts = {str(k): c for k, c in enumerate(conf)}

    def build():
        yield from entries.values()
        for mi in parts:
            yield from mi.entries.values()

    out = MergeIndex(_LazyEntries(build), conflicts)
    keys = {id(c): k for k, c in conflicts.items()}
    out.automerge_candidates = [keys[id(mi.conflicts[k])] for mi in parts for k in mi.automerge_candidates]
    return out


# ---------------------------------------------------------------------------------------------
# kart conflicts -s / -ss (kart/conflicts.py:22-132, summarise 1 and 2)
def _path_part_sort_key(part):
    if isinstance(part, str) and part.isdigit():
        part = int(part)
    if part == "meta":
        return ("A", part)
    if part == "feature":
        return ("B", part)
    if isinstance(part, str) and "," in part:
        return ("Z", part)
    if isinstance(part, int):
        return ("N", "", part)
    return ("N", part)


def _path_sort_key(path):
    if isinstance(path, str) and ":" in path:
        return tuple(_path_part_sort_key(p) for p in path.split(":"))
    return _path_part_sort_key(path)


def list_conflicts(merge_index, decode_path, summarise=2):
    """{dataset: {"feature": n}} (summarise=2) or {dataset: {"feature": [pk, ...]}} (summarise=1) of
    the unresolved conflicts.  ``decode_path(path) -> (dataset, "feature" | "meta", key)`` is
    RepoStructure.decode_path (kart/structure.py:155-166); a conflict whose versions decode to
    different keys (renames) is labelled "ancestor=..,ours=..,theirs=.." as RichConflict does."""
    if summarise not in (1, 2):
        raise ValueError("summarise: 1 (keys) or 2 (counts); the full output needs the feature values")
    out = {}
    for c in merge_index.unresolved_conflicts.values():
        decoded = [(name, decode_path(e.path)) for name, e in zip(AncestorOursTheirs.NAMES, c) if e]
        parts = []
        for i in range(3):
            vals = {d[i] for _, d in decoded}
            parts.append(next(iter(vals)) if len(vals) == 1 else ",".join(f"{n}={d[i]}" for n, d in decoded))
        node = out.setdefault(parts[0], {}).setdefault(parts[1], {})
        node[parts[2]] = None
    for ds in out.values():
        for kind, node in ds.items():
            ds[kind] = len(node) if summarise >= 2 else sorted(node.keys(), key=_path_sort_key)
    return out
