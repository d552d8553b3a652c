"""Host side of the drop-in: a Kart repository's dataset versions, read natively.

Stand-in for the libgit2/pygit2 object reads under Dataset3 (kart/dataset3.py:225-231,
kart/base_dataset.py:230-283) on machines without pygit2 (this image).  Objects come from
libkartdiff's own reader (kart_amd.odb: loose + packed objects, delta chains); a dataset's feature
leaves come from one multithreaded ``kd_walk`` of ``<ds>/.table-dataset/feature`` — for a diff or
a merge of two (three) commits, a pruned walk that never opens a subtree whose OID the compared
commits share (what libgit2's tree diff does, kart/rich_base_dataset.py:212-232).  Feature blobs
are read lazily (one object per value access) or in one batch (``read_blobs``) for the field diff.

The git CLI is used only to write (``write_index_tree``: a merged index's tree) and to resolve
revision expressions beyond plain refs and OIDs (``HEAD^``, ``@{u}`` ...).
"""
import json
import os
import re
import subprocess

import numpy as np

from . import _native as N
from .dataset import DatasetVersion
from .odb import OBJ_BLOB, OBJ_COMMIT, OBJ_TAG, OBJ_TREE, ObjectDB, oid_bytes
from .packing import PathEncoding
from .schema import Legend, Schema

DATASET_DIRNAME = ".table-dataset"
# libgit2 error subcodes Kart's pygit2 attaches to a KeyError (kart/promisor_utils.py:10-22)
ENOSUCHPATH, EOBJECTMISSING, EOBJECTPROMISED = -3001, -3002, -3003
_HEX40 = re.compile(r"^[0-9a-fA-F]{40}$")


class GitRepo:
    def __init__(self, gitdir, index_file=None):
        self.gitdir = gitdir
        self.env = dict(os.environ, GIT_DIR=gitdir)
        # Kart's index carries a "kart" extension stock git rejects; never touch it
        self.env["GIT_INDEX_FILE"] = index_file or os.path.join(gitdir, "kart_amd.index")
        self.odb = ObjectDB(gitdir)
        self._promisor = None

    def git(self, *args):
        return subprocess.run(["git", *args], env=self.env, check=True, capture_output=True).stdout

    def close(self):
        self.odb.close()

    # ---- references -----------------------------------------------------------------------------
    def _ref(self, name, depth=0):
        """a ref's OID (loose file, then packed-refs; symbolic refs followed), or None"""
        if depth > 5:
            return None
        path = os.path.join(self.gitdir, name)
        if os.path.isfile(path):
            val = open(path).read().strip()
            if val.startswith("ref: "):
                return self._ref(val[5:].strip(), depth + 1)
            return val if _HEX40.match(val) else None
        packed = os.path.join(self.gitdir, "packed-refs")
        if os.path.isfile(packed):
            for line in open(packed):
                parts = line.split()
                if len(parts) == 2 and parts[1] == name and _HEX40.match(parts[0]):
                    return parts[0]
        return None

    def rev_parse(self, spec):
        """the object a revision names: a 40-hex id, a ref (git's lookup order), else `git rev-parse`"""
        if _HEX40.match(spec):
            return spec.lower()
        for name in (spec, f"refs/{spec}", f"refs/tags/{spec}", f"refs/heads/{spec}", f"refs/remotes/{spec}",
                     f"refs/remotes/{spec}/HEAD"):
            oid = self._ref(name)
            if oid:
                return oid
        return self.git("rev-parse", "--verify", spec).decode().strip()

    def rev_tree(self, spec):
        """the tree a revision names (commits and tags peeled)"""
        oid = self.rev_parse(spec)
        for _ in range(8):
            t, data = self._read(oid)
            if t == OBJ_TREE:
                return oid
            key = b"tree " if t == OBJ_COMMIT else b"object " if t == OBJ_TAG else None
            if key is None or not data.startswith(key):
                raise ValueError(f"{spec} does not name a tree")
            oid = data[len(key):len(key) + 40].decode()
        raise ValueError(f"{spec}: tag chain too long")

    # ---- objects --------------------------------------------------------------------------------
    def promisor_remote(self):
        """the promisor remote of a partial clone, or None (promisor_utils.get_promisor_remote)"""
        if self._promisor is None:
            out = subprocess.run(["git", "config", "--get-regexp", r"^remote\..*\.promisor$"], env=self.env,
                                 capture_output=True).stdout.decode().split("\n")
            names = [ln.split()[0][len("remote."):-len(".promisor")] for ln in out
                     if ln.strip() and ln.split()[-1].lower() in ("true", "1", "yes", "on")]
            self._promisor = names[0] if names else ""
        return self._promisor or None

    def _missing(self, oid_hex):
        # kart/base_dataset.py:256-265 + promisor_utils.py:10-29: a KeyError with the libgit2
        # subcode — promised (partial clone: DeltaFetcher fetches it) or missing
        promised = self.promisor_remote() is not None
        e = KeyError(f"object {oid_hex} {'promised' if promised else 'missing'}")
        e.subcode = EOBJECTPROMISED if promised else EOBJECTMISSING
        return e

    def _read(self, oid):
        try:
            return self.odb.read(oid)
        except N.NotFound:
            # packs written since the store was opened (a miss with an unchanged pack set does
            # not reopen: promised blobs of a partial clone miss on every read)
            if not self.odb.refresh():
                raise self._missing(oid_bytes(oid).hex()) from None
            try:
                return self.odb.read(oid)
            except N.NotFound:
                raise self._missing(oid_bytes(oid).hex()) from None

    def cat(self, oid_hex):
        """a blob's content; KeyError (with .subcode) when it is not in the repository"""
        t, data = self._read(oid_hex)
        if t != OBJ_BLOB:
            raise ValueError(f"{oid_hex} is not a blob")
        return data

    def read_blobs(self, oids):
        """(data, off, status) of blobs [n, 20] in one batched native read"""
        data, off, status = self.odb.read_batch(oids)
        if status.any() and self.odb.refresh():
            data, off, status = self.odb.read_batch(oids)
        return data, off, status

    # ---- trees ----------------------------------------------------------------------------------
    def ls_tree(self, treeish):
        """one tree level: [(mode, type, oid hex, name)]"""
        oid = treeish if _HEX40.match(treeish) else self.rev_tree(treeish)
        t, data = self._read(oid)
        if t != OBJ_TREE:
            oid = self.rev_tree(oid)
        return self.odb.tree_entries(oid)

    def walk(self, specs, subpath, compare=None):
        """leaves under ``subpath`` of each revision (odb.Leaves), optionally pruned by ``compare``"""
        roots = [self.rev_parse(s) for s in specs]
        try:
            return self.odb.walk(roots, subpath, compare)
        except N.NotFound:
            if not self.odb.refresh():
                raise
            return self.odb.walk(roots, subpath, compare)

    def ls_tree_r(self, treeish, prefix):
        """[(path, oid hex)] of every blob under ``prefix`` (full paths)"""
        (lv,) = self.walk([treeish], prefix)
        pre = prefix.rstrip("/") + "/" if prefix else ""
        return [(pre + p, o) for p, o in lv.items()]

    def non_feature_entries(self, spec):
        """{path: (mode, oid hex)} of every blob of a commit outside the datasets' feature trees
        (meta items, structure files): the walk never enters a .table-dataset/feature tree"""
        out = {}
        stack = [(self.rev_tree(spec), "")]
        while stack:
            tree, pre = stack.pop()
            for mode, typ, oid, name in self.odb.tree_entries(tree):
                path = pre + name
                if typ == "tree":
                    if not path.endswith("/" + DATASET_DIRNAME + "/feature") and path != DATASET_DIRNAME + "/feature":
                        stack.append((oid, path + "/"))
                elif typ == "blob":
                    out[path] = (mode, oid)
        return out

    def dataset_paths(self, spec):
        """dataset paths of a commit (dirs containing .table-dataset); a dataset's own tree is
        never descended into"""
        out = []
        stack = [(self.rev_tree(spec), "")]
        while stack:
            tree, pre = stack.pop()
            ents = self.odb.tree_entries(tree)
            if any(typ == "tree" and name == DATASET_DIRNAME for _, typ, _, name in ents):
                out.append(pre.rstrip("/"))
            for _, typ, oid, name in ents:
                if typ == "tree" and name != DATASET_DIRNAME:
                    stack.append((oid, pre + name + "/"))
        return sorted(p for p in out if p)

    def write_index_tree(self, index_info):
        """a tree from '<mode> <oid>\\t<path>\\0' records (git update-index -z --index-info into a
        scratch index, then write-tree): what libgit2's index.write_tree does"""
        import tempfile

        with tempfile.TemporaryDirectory() as td:
            env = dict(self.env, GIT_INDEX_FILE=os.path.join(td, "index"))
            subprocess.run(["git", "update-index", "-z", "--index-info"], input=index_info, env=env, check=True,
                           capture_output=True)
            return subprocess.run(["git", "write-tree"], env=env, check=True, capture_output=True).stdout.decode().strip()

    # ---- dataset versions -----------------------------------------------------------------------
    def tree_at(self, spec, path):
        """the OID of the tree at ``path`` in revision ``spec``, or None"""
        tree = self.rev_tree(spec)
        for part in [p for p in path.split("/") if p]:
            nxt = None
            for _, typ, oid, name in self.odb.tree_entries(tree):
                if name == part and typ == "tree":
                    nxt = oid
                    break
            if nxt is None:
                return None
            tree = nxt
        return tree

    def _meta(self, spec, ds_path):
        """(meta items, legends, schema, path structure) of a dataset version: the meta tree's files
        read once; the items as Dataset3.meta_items yields them (kart_amd/meta.py), the
        ``metadata.xml`` attachment taken from the dataset's own tree"""
        from . import meta as M

        inner = f"{ds_path}/{DATASET_DIRNAME}/meta"
        (lv,) = self.walk([spec], inner)
        if not lv.present or lv.n == 0:
            return None
        files, legends, schema, path_structure = {}, {}, None, None
        for rel, oid in lv.items():
            data = self.cat(oid)
            if rel.startswith("legend/"):
                legends[rel[len("legend/"):]] = Legend.loads(data)
                continue
            files[rel] = data
            if rel == "schema.json":
                schema = Schema.from_column_dicts(json.loads(data))
            elif rel == "path-structure.json":
                path_structure = json.loads(data)
        attachments = {}
        ds_tree = self.tree_at(spec, ds_path)
        if ds_tree is not None:
            for _, typ, oid, name in self.odb.tree_entries(ds_tree):
                if typ == "blob" and name in M.ATTACHMENT_META_ITEMS:
                    attachments[name] = self.cat(oid)
        return M.meta_items(files, attachments), legends, schema, path_structure

    def _version(self, ds_path, m, leaves, partial):
        meta, legends, schema, path_structure = m
        oid_arr = leaves.oids
        repo = self

        def read_blob(i):
            return repo.cat(oid_arr[i].tobytes().hex())

        def read_blobs(idx):
            return repo.read_blobs(oid_arr[np.asarray(idx, np.int64)])

        read_blobs.source = repo  # versions of one repository can share a batched read

        v = DatasetVersion(ds_path, schema, legends, PathEncoding.from_dict(path_structure), leaves.paths,
                           leaves.off, oid_arr, read_blob, meta, read_blobs=read_blobs)
        v.partial = partial
        return v

    def dataset_versions(self, specs, ds_path, compare=None):
        """DatasetVersion (or None when absent) of ``ds_path`` at each revision, the feature leaves
        from one walk.  ``compare=(i, j)``: prune to the subtrees where revisions i and j differ —
        the versions then hold only those leaves (``.partial``), which is all a diff or merge
        classification of them needs: every leaf outside is identical on the compared sides."""
        metas = [self._meta(s, ds_path) for s in specs]
        prune = compare is not None and all(metas[i] is not None for i in compare)
        if prune:
            prune = metas[compare[0]][3] == metas[compare[1]][3]  # same path structure: same leaf paths
        leaves = self.walk(specs, f"{ds_path}/{DATASET_DIRNAME}/feature", compare if prune else None)
        return [self._version(ds_path, m, lv, prune) if m is not None else None for m, lv in zip(metas, leaves)]

    def dataset_version(self, spec, ds_path):
        """DatasetVersion of ``ds_path`` at commit/tree ``spec``, or None if absent."""
        return self.dataset_versions([spec], ds_path)[0]

    def diff_versions(self, base, target, ds_path):
        """(old, new) DatasetVersions for a diff of two revisions, pruned to their changed subtrees"""
        return tuple(self.dataset_versions([base, target], ds_path, compare=(0, 1)))

    def merge_versions(self, ancestor, ours, theirs, ds_path):
        """(ancestor, ours, theirs) DatasetVersions pruned to the subtrees where ours and theirs
        differ (elsewhere libgit2's rule takes ours unchanged)"""
        return tuple(self.dataset_versions([ancestor, ours, theirs], ds_path, compare=(1, 2)))
