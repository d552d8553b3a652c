"""Loader for the reference's hot-path modules + a pygit2-shaped shim over the git CLI.

GOLDEN-VECTOR GENERATION ONLY.  This file is executed in the build container (where
/root/reference exists) by ``tests/golden/gen_golden.py``; nothing on the GPU box, in the
product package, in ``bench.py`` or in ``smoke()`` imports it.  It contains no reference source:
it imports the reference modules from /root/reference (read-only, no bytecode written) with
four third-party modules stubbed (pygit2, osgeo, jsonschema, pysqlite3), exactly as SURVEY.md
Appendix A describes, and stands in for libgit2's tree diff with ``git diff-tree -r``.
"""
import hashlib
import importlib
import os
import subprocess
import sys
import types

sys.dont_write_bytecode = True

REF = "/root/reference"

GIT_DELTA_ADDED, GIT_DELTA_DELETED, GIT_DELTA_MODIFIED = 1, 2, 3
EMPTY_TREE = "4b825dc642cb6eb9a060e54bf8d69288fbee4904"


def _stub(name, **kw):
    m = types.ModuleType(name)
    m.__dict__.update(kw)
    sys.modules[name] = m
    return m


class _Any:
    def __getattr__(self, k):
        return _Any()

    def __call__(self, *a, **k):
        return _Any()


_loaded = False


def load_reference():
    """Install stubs and a bare ``kart`` namespace package pointing at /root/reference/kart."""
    global _loaded
    if _loaded:
        return
    pg = _stub(
        "pygit2",
        GIT_DELTA_ADDED=GIT_DELTA_ADDED,
        GIT_DELTA_MODIFIED=GIT_DELTA_MODIFIED,
        GIT_DELTA_DELETED=GIT_DELTA_DELETED,
        GIT_DIFF_SKIP_BINARY_CHECK=1 << 30,
    )
    classes = {}

    def pg_getattr(k):
        if k.startswith("GIT_"):
            return hash(k) & 0xFFFF
        if k[:1].isupper():
            return classes.setdefault(k, type(k, (), {}))
        return _Any()

    pg.__getattr__ = pg_getattr
    pg.hash = lambda d: types.SimpleNamespace(
        raw=hashlib.sha1(b"blob %d\0" % len(d) + d).digest()
    )
    # Make the shim's Blob/Tree the pygit2 types so isinstance() checks in the reference work.
    pg.Blob = Blob
    pg.Tree = Tree
    o = _stub("osgeo")
    o.ogr = o.osr = o.gdal = _Any()
    sys.modules["osgeo.ogr"] = o.ogr
    sys.modules["osgeo.osr"] = o.osr
    sys.modules["osgeo.gdal"] = o.gdal
    js = _stub("jsonschema")
    js.__getattr__ = lambda k: _Any()
    _stub("pysqlite3", dbapi2=_Any())
    sys.modules["pysqlite3.dbapi2"] = _Any()
    k = types.ModuleType("kart")
    k.__path__ = [REF + "/kart"]
    k.is_windows = False
    k.is_darwin = False
    k.is_linux = True
    sys.modules["kart"] = k
    _loaded = True


def ref(modname):
    load_reference()
    return importlib.import_module("kart." + modname)


# ---------------------------------------------------------------------------------------------
# git CLI shim (just enough of pygit2 for Dataset3.diff_feature / get_feature)
# ---------------------------------------------------------------------------------------------


class GitRepo:
    def __init__(self, gitdir, index_file="/tmp/kart_amd_golden_index"):
        self.gitdir = gitdir
        self.env = dict(os.environ, GIT_DIR=gitdir, GIT_INDEX_FILE=index_file)
        self._trees = {}
        self._maps = {}
        self._children = {}
        self._blobs = {}
        self._cat = None

    def git(self, *args, text=False):
        out = subprocess.run(
            ["git", *args], env=self.env, check=True, capture_output=True
        ).stdout
        return out.decode() if text else out

    def rev(self, spec):
        return self.git("rev-parse", spec, text=True).strip()

    def tree(self, spec):
        return Tree(self, self.rev(spec + "^{tree}"), "")

    def entry_map(self, oid):
        """{name: entry} of a tree (libgit2 finds an entry by binary search in C; a dict keeps the shim's
        lookups from dominating timings of the reference path)"""
        m = self._maps.get(oid)
        if m is None:
            m = self._maps[oid] = {e[0]: e for e in self.ls_tree(oid)}
        return m

    def child(self, tree_oid, name):
        """the Tree / Blob object of entry ``name`` of a tree, made once (pygit2 hands out C-backed
        objects; the shim keeps its Python ones so a path lookup costs dict hits, not object builds)"""
        key = (tree_oid, name)
        c = self._children.get(key)
        if c is None:
            ent = self.entry_map(tree_oid).get(name)
            if ent is None:
                return None
            c = self._children[key] = (Tree(self, ent[2], name) if ent[1] == "tree" else Blob(self, ent[2], name))
        return c

    def ls_tree(self, oid):
        if oid not in self._trees:
            raw = self.git("ls-tree", "-z", oid)
            ents = []
            for rec in raw.split(b"\0"):
                if not rec:
                    continue
                meta, name = rec.split(b"\t", 1)
                mode, typ, eoid = meta.split(b" ")
                ents.append((name.decode(), typ.decode(), eoid.decode(), mode.decode()))
            self._trees[oid] = ents
        return self._trees[oid]

    def blob_data(self, oid):
        if oid not in self._blobs:
            if self._cat is None:
                self._cat = subprocess.Popen(
                    ["git", "cat-file", "--batch"],
                    env=self.env,
                    stdin=subprocess.PIPE,
                    stdout=subprocess.PIPE,
                )
            self._cat.stdin.write(oid.encode() + b"\n")
            self._cat.stdin.flush()
            hdr = self._cat.stdout.readline().split()
            size = int(hdr[2])
            data = self._cat.stdout.read(size)
            self._cat.stdout.read(1)
            self._blobs[oid] = data
        return self._blobs[oid]

    def ls_tree_r(self, treeish, prefix=""):
        """All leaf blobs under ``treeish`` (optionally a sub-path) as [(path, oid_hex)]."""
        args = ["ls-tree", "-r", "-z", treeish]
        if prefix:
            args.append(prefix)
        raw = self.git(*args)
        out = []
        for rec in raw.split(b"\0"):
            if not rec:
                continue
            meta, name = rec.split(b"\t", 1)
            out.append((name.decode(), meta.split(b" ")[2].decode()))
        return out


class _Oid(str):
    @property
    def hex(self):
        return str(self)

    @property
    def raw(self):
        return bytes.fromhex(self)


class Blob(bytes):
    type_str = "blob"

    def __new__(cls, repo, oid, name):
        self = super().__new__(cls, repo.blob_data(oid))
        self.id = self.oid = _Oid(oid)
        self.name = name
        return self

    @property
    def data(self):
        return bytes(self)

    @property
    def size(self):
        return len(self)


class _File:
    def __init__(self, path):
        self.path = path


class _Delta:
    _chars = {GIT_DELTA_ADDED: "A", GIT_DELTA_DELETED: "D", GIT_DELTA_MODIFIED: "M"}

    def __init__(self, status, path):
        self.status = status
        self.old_file = _File(path)
        self.new_file = _File(path)

    def status_char(self):
        return self._chars[self.status]


class _Diff:
    def __init__(self, deltas):
        self.deltas = deltas

    def __len__(self):
        return len(self.deltas)


class Tree:
    type_str = "tree"

    def __init__(self, repo, oid, name):
        self.repo = repo
        self.id = self.oid = _Oid(oid)
        self.name = name

    def _entries(self):
        return self.repo.ls_tree(self.id)

    def _child(self, ent):
        name, typ, oid, _ = ent
        return Tree(self.repo, oid, name) if typ == "tree" else Blob(self.repo, oid, name)

    def __iter__(self):
        for ent in self._entries():
            yield self._child(ent)

    def __len__(self):
        return len(self._entries())

    def __bool__(self):
        return True

    def __contains__(self, path):
        try:
            self / path
            return True
        except KeyError:
            return False

    def __getitem__(self, name):
        return self / name

    def __truediv__(self, path):
        node = self
        for part in [p for p in str(path).split("/") if p]:
            if not isinstance(node, Tree):
                raise KeyError(path)
            nxt = node.repo.child(node.id, part)
            if nxt is None:
                raise KeyError(path)
            node = nxt
        return node

    def diff_to_tree(self, other=None, flags=0, swap=False):
        a = self.id
        b = other.id if other is not None else EMPTY_TREE
        if swap:
            a, b = b, a
        raw = self.repo.git("diff-tree", "-r", "-z", "--no-renames", a, b)
        toks = [t for t in raw.split(b"\0")]
        deltas = []
        i = 0
        while i < len(toks):
            t = toks[i]
            if not t.startswith(b":"):
                i += 1
                continue
            status = t.split(b" ")[-1].decode()
            path = toks[i + 1].decode()
            st = {"A": GIT_DELTA_ADDED, "D": GIT_DELTA_DELETED, "M": GIT_DELTA_MODIFIED}[status]
            deltas.append(_Delta(st, path))
            i += 2
        return _Diff(deltas)


def dataset3(repo, commit_spec, ds_path):
    """Reference Dataset3 at ``<commit>:<ds_path>`` backed by the shim."""
    d3 = ref("dataset3")
    root = repo.tree(commit_spec)
    try:
        tree = root / ds_path
    except KeyError:
        return None
    return d3.Dataset3(tree, ds_path, repo=repo)
