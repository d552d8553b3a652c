"""Host tree walker: a Kart repository's dataset version -> DatasetVersion, via the git CLI.

Stand-in for the libgit2/pygit2 tree walk of Dataset3 (kart/dataset3.py:225-231,
kart/base_dataset.py:230-283) on machines without pygit2 (this image): ``git ls-tree -r -z``
lists the feature leaves of ``<ds>/.table-dataset/feature`` (the packer sorts them by join key),
meta items and legends are read once, and feature blobs are read lazily through one persistent
``git cat-file --batch`` process — classification itself never reads a blob.

A native pack/loose-object reader with leaf-tree pruning is SURVEY.md §8f's next step #1.
"""
import json
import os
import subprocess

import numpy as np

from . import packing
from .dataset import DatasetVersion
from .schema import Legend, Schema

DATASET_DIRNAME = ".table-dataset"
# libgit2 error subcodes Kart's pygit2 attaches to a KeyError (kart/promisor_utils.py:10-22)
ENOSUCHPATH, EOBJECTMISSING, EOBJECTPROMISED = -3001, -3002, -3003


class GitRepo:
    def __init__(self, gitdir, index_file=None):
        self.gitdir = gitdir
        self.env = dict(os.environ, GIT_DIR=gitdir)
        # Kart's index carries a "kart" extension stock git rejects; never touch it
        self.env["GIT_INDEX_FILE"] = index_file or os.path.join(gitdir, "kart_amd.index")
        self._cat = None
        self._promisor = None

    def git(self, *args):
        return subprocess.run(["git", *args], env=self.env, check=True, capture_output=True).stdout

    def rev_tree(self, spec):
        return self.git("rev-parse", spec + "^{tree}").decode().strip()

    def promisor_remote(self):
        """the promisor remote of a partial clone, or None (promisor_utils.get_promisor_remote)"""
        if self._promisor is None:
            out = subprocess.run(["git", "config", "--get-regexp", r"^remote\..*\.promisor$"], env=self.env,
                                 capture_output=True).stdout.decode().split("\n")
            names = [ln.split()[0][len("remote."):-len(".promisor")] for ln in out
                     if ln.strip() and ln.split()[-1].lower() in ("true", "1", "yes", "on")]
            self._promisor = names[0] if names else ""
        return self._promisor or None

    def cat(self, oid_hex):
        if self._cat is None:
            self._cat = subprocess.Popen(["git", "cat-file", "--batch"], env=self.env, stdin=subprocess.PIPE,
                                         stdout=subprocess.PIPE)
        self._cat.stdin.write(oid_hex.encode() + b"\n")
        self._cat.stdin.flush()
        hdr = self._cat.stdout.readline().split()
        if len(hdr) < 3 or hdr[1] == b"missing":
            # kart/base_dataset.py:256-265 + promisor_utils.py:10-29: a KeyError with the libgit2
            # subcode — promised (partial clone: DeltaFetcher fetches it) or missing
            promised = self.promisor_remote() is not None
            e = KeyError(f"object {oid_hex} {'promised' if promised else 'missing'}")
            e.subcode = EOBJECTPROMISED if promised else EOBJECTMISSING
            raise e
        data = self._cat.stdout.read(int(hdr[2]))
        self._cat.stdout.read(1)
        return data

    def close(self):
        if self._cat is not None:
            self._cat.stdin.close()
            self._cat.wait()
            self._cat = None

    def ls_tree_r(self, treeish, prefix):
        raw = self.git("ls-tree", "-r", "-z", "--full-tree", treeish, "--", prefix)
        names, oids = [], []
        for rec in raw.split(b"\0"):
            if not rec:
                continue
            meta, path = rec.split(b"\t", 1)
            names.append(path)
            oids.append(meta.split(b" ")[2])
        return names, oids

    def ls_tree(self, treeish):
        """one tree level: [(mode, type, oid hex, name)]"""
        out = []
        for rec in self.git("ls-tree", "-z", treeish).split(b"\0"):
            if rec:
                meta, name = rec.split(b"\t", 1)
                mode, typ, oid = meta.split(b" ")
                out.append((int(mode, 8), typ.decode(), oid.decode(), name.decode()))
        return out

    def non_feature_entries(self, spec):
        """{path: (mode, oid hex)} of every blob of a commit outside the datasets' feature trees
        (meta items, structure files): the walk never enters a .table-dataset/feature tree"""
        out = {}
        stack = [(self.rev_tree(spec), "")]
        while stack:
            tree, pre = stack.pop()
            for mode, typ, oid, name in self.ls_tree(tree):
                path = pre + name
                if typ == "tree":
                    if not path.endswith("/" + DATASET_DIRNAME + "/feature") and path != DATASET_DIRNAME + "/feature":
                        stack.append((oid, path + "/"))
                elif typ == "blob":
                    out[path] = (mode, oid)
        return out

    def write_index_tree(self, index_info):
        """a tree from '<mode> <oid>\\t<path>\\0' records (git update-index -z --index-info into a
        scratch index, then write-tree): what libgit2's index.write_tree does"""
        import tempfile

        with tempfile.TemporaryDirectory() as td:
            env = dict(self.env, GIT_INDEX_FILE=os.path.join(td, "index"))
            subprocess.run(["git", "update-index", "-z", "--index-info"], input=index_info, env=env, check=True,
                           capture_output=True)
            return subprocess.run(["git", "write-tree"], env=env, check=True, capture_output=True).stdout.decode().strip()

    def dataset_paths(self, spec):
        """dataset paths of a commit (dirs containing .table-dataset)"""
        raw = self.git("ls-tree", "-r", "-d", "-z", "--name-only", spec)
        out = []
        for p in raw.split(b"\0"):
            p = p.decode()
            if p.endswith("/" + DATASET_DIRNAME):
                out.append(p[: -len(DATASET_DIRNAME) - 1])
        return sorted(out)

    def dataset_version(self, spec, ds_path):
        """DatasetVersion of ``ds_path`` at commit/tree ``spec``, or None if absent."""
        inner = f"{ds_path}/{DATASET_DIRNAME}/"
        meta_names, meta_oids = self.ls_tree_r(spec, inner + "meta")
        if not meta_names:
            return None
        meta, legends = {}, {}
        schema = None
        path_structure = None
        for p, o in zip(meta_names, meta_oids):
            rel = p.decode()[len(inner) + len("meta/"):]
            data = self.cat(o.decode())
            if rel.startswith("legend/"):
                lg = Legend.loads(data)
                legends[rel[len("legend/"):]] = lg
            elif rel == "schema.json":
                cols = json.loads(data)
                schema = Schema.from_column_dicts(cols)
                meta[rel] = cols
            elif rel == "path-structure.json":
                path_structure = json.loads(data)
            elif rel.endswith(".json"):
                meta[rel] = json.loads(data)
            else:
                meta[rel] = data.decode()
        names, oids = self.ls_tree_r(spec, inner + "feature")
        fp = len(inner) + len("feature/")
        rel = [n[fp:] for n in names]
        arena, off = packing._arena(rel)
        oid_arr = np.frombuffer(b"".join(bytes.fromhex(o.decode()) for o in oids), np.uint8).reshape(-1, 20) \
            if oids else np.zeros((0, 20), np.uint8)
        oid_hex = [o.decode() for o in oids]
        return DatasetVersion(ds_path, schema, legends, packing.PathEncoding.from_dict(path_structure), arena, off,
                              oid_arr, lambda i: self.cat(oid_hex[i]), meta)
