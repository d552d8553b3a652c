"""The git object database through libkartdiff's native reader (kd_odb_* / kd_walk).

What Kart gets from libgit2 on the diff path (kart/dataset3.py:26-35,225-231 tree iteration,
kart/base_dataset.py:230-265 blob reads, Tree.diff_to_tree's subtree pruning at
kart/rich_base_dataset.py:212-232), read natively: loose objects, packs with delta chains,
a multithreaded leaf walk that never opens a subtree whose OID two roots share.
"""
import ctypes
import os
import threading
import weakref

import numpy as np

from . import _native as N

OBJ_COMMIT, OBJ_TREE, OBJ_BLOB, OBJ_TAG = 1, 2, 3, 4
TYPE_NAMES = {OBJ_COMMIT: "commit", OBJ_TREE: "tree", OBJ_BLOB: "blob", OBJ_TAG: "tag"}
MODE_TREE = 0o40000


def oid_bytes(oid):
    """20 raw bytes from raw bytes, a 40-char hex str/bytes, or a uint8[20] array"""
    if isinstance(oid, np.ndarray):
        return oid.astype(np.uint8).tobytes()
    if isinstance(oid, (bytes, bytearray)) and len(oid) == 20:
        return bytes(oid)
    if isinstance(oid, bytes):
        oid = oid.decode()
    if isinstance(oid, str) and len(oid) == 40:
        return bytes.fromhex(oid)
    raise ValueError(f"not an object id: {oid!r}")


class Leaves:
    """One root's leaves of a walk: path arena + offsets (relative to the walked tree), OIDs
    [n, 20], git modes; ``present`` False when the walked tree is absent from that root."""

    __slots__ = ("paths", "off", "oids", "modes", "present")

    def __init__(self, paths, off, oids, modes, present):
        self.paths, self.off, self.oids, self.modes, self.present = paths, off, oids, modes, present

    @property
    def n(self):
        return int(self.off.shape[0]) - 1

    def path(self, i):
        return self.paths[int(self.off[i]):int(self.off[i + 1])].tobytes().decode()

    def items(self):
        """[(path, oid hex)] (small walks / tests)"""
        return [(self.path(i), self.oids[i].tobytes().hex()) for i in range(self.n)]


def _copy_out(addr, dtype, shape):
    a = np.empty(shape, dtype)
    if a.nbytes:
        ctypes.memmove(a.ctypes.data, addr, a.nbytes)
    return a


def _take_leaves(L, p):
    """copy one kd_leaves block into numpy arrays, then free it"""
    try:
        x = p.contents
        n = int(x.n)
        off = _copy_out(ctypes.cast(x.path_off, ctypes.c_void_p).value, np.uint64, n + 1)
        paths = _copy_out(ctypes.cast(x.path, ctypes.c_void_p).value, np.uint8, int(off[-1]))
        oids = _copy_out(ctypes.cast(x.oid, ctypes.c_void_p).value, np.uint8, (n, 20))
        modes = _copy_out(ctypes.cast(x.mode, ctypes.c_void_p).value, np.uint32, n)
        return Leaves(paths, off, oids, modes, bool(x.present))
    finally:
        L.kd_free(ctypes.cast(p, ctypes.c_void_p))


class ObjectDB:
    """A repository's object store (``gitdir`` = the .git directory or a bare repo).  The pack
    set is read at open; ``refresh()`` reopens when packs were written since (``reopen()``
    unconditionally).  Native calls and reopening share one lock, so a thread never closes the
    handle under another thread's GIL-released native call."""

    def __init__(self, gitdir):
        self.gitdir = gitdir
        self.L = N.lib()
        self._h = None
        self._lock = threading.RLock()
        self._sig = None
        self._opts = {}
        self.n_opens = 0
        self.reopen()

    def set_option(self, name, value):
        """an option of the object store (kd_odb_set_option: ``zlib`` 1 inflates with zlib even when
        libdeflate is present); kept across reopens"""
        with self._lock:
            N.check(self.L.kd_odb_set_option(self._h, name.encode(), int(value)), "kd_odb_set_option")
            self._opts[name] = int(value)

    def get_option(self, name):
        with self._lock:
            v = ctypes.c_int64()
            N.check(self.L.kd_odb_get_option(self._h, name.encode(), ctypes.byref(v)), "kd_odb_get_option")
            return int(v.value)

    def _alternate_dirs(self):
        """objects directories named by objects/info/alternates (recursively, as git follows them)"""
        out, todo, seen = [], [os.path.join(self.gitdir, "objects")], set()
        while todo:
            d = os.path.realpath(todo.pop())
            if d in seen:
                continue
            seen.add(d)
            out.append(d)
            try:
                with open(os.path.join(d, "info", "alternates")) as f:
                    for line in f:
                        line = line.strip()
                        if line and not line.startswith("#"):
                            todo.append(line if os.path.isabs(line) else os.path.join(d, line))
            except OSError:
                pass
        return out

    def _pack_signature(self):
        """what a reopen would see differently: every objects directory's pack files (this repository's
        and each alternate's) and the alternates files themselves"""
        sig = []
        for d in self._alternate_dirs():
            for rel in ("pack", "info/alternates"):
                path = os.path.join(d, rel)
                try:
                    st = os.stat(path)
                except OSError:
                    sig.append((path, None))
                    continue
                sig.append((path, st.st_mtime_ns, st.st_size,
                            tuple(sorted(os.listdir(path))) if os.path.isdir(path) else ()))
        return tuple(sig)

    def reopen(self):
        with self._lock:
            self.close()
            sig = self._pack_signature()
            h = ctypes.c_void_p()
            N.check(self.L.kd_odb_open(self.gitdir.encode(), ctypes.byref(h)), "kd_odb_open")
            self._h = h
            self._sig = sig
            self.n_opens += 1
            for name, value in self._opts.items():
                N.check(self.L.kd_odb_set_option(h, name.encode(), value), "kd_odb_set_option")

    def refresh(self):
        """reopen if packs or alternates changed since the last open; True when it reopened"""
        with self._lock:
            if self._h is not None and self._pack_signature() == self._sig:
                return False
            self.reopen()
            return True

    def close(self):
        with self._lock:
            if self._h is not None and self._h.value:
                self.L.kd_odb_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def read(self, oid):
        """(type, content bytes); raises N.NotFound when absent"""
        raw = oid_bytes(oid)
        t = ctypes.c_int()
        data = N.c_u8p()
        n = ctypes.c_uint64()
        with self._lock:
            N.check(self.L.kd_odb_read(self._h, raw, ctypes.byref(t), ctypes.byref(data), ctypes.byref(n)),
                    "kd_odb_read")
        try:
            return t.value, ctypes.string_at(data, n.value)
        finally:
            self.L.kd_free(ctypes.cast(data, ctypes.c_void_p))

    def read_batch(self, oids, threads=0):
        """blobs of ``oids`` [n, 20] into one arena: (data uint8, off uint64[n+1], status uint8[n])
        — status 0 ok, 1 missing, 2 corrupt / not a blob"""
        oids = np.ascontiguousarray(oids, np.uint8).reshape(-1, 20)
        n = oids.shape[0]
        off = np.zeros(n + 1, np.uint64)
        status = np.zeros(max(n, 1), np.uint8)
        data = N.c_u8p()
        with self._lock:
            N.check(self.L.kd_odb_read_batch(self._h, oids.ctypes.data if n else None, n, threads, ctypes.byref(data),
                                             off.ctypes.data, status.ctypes.data), "kd_odb_read_batch")
        total = int(off[-1])
        addr = ctypes.cast(data, ctypes.c_void_p).value
        if not total:
            self.L.kd_free(ctypes.c_void_p(addr))
            return np.zeros(0, np.uint8), off, status[:n]
        # the library's buffer itself, freed when the last array over it goes (no copy)
        buf = (ctypes.c_uint8 * total).from_address(addr)
        weakref.finalize(buf, self.L.kd_free, ctypes.c_void_p(addr))
        return np.frombuffer(buf, np.uint8), off, status[:n]

    def walk(self, roots, subpath="", compare=None, threads=0):
        """Leaves under ``subpath`` of each root (commit/tag/tree ids), one Leaves per root.
        ``compare=(i, j)``: skip every entry identical in roots i and j (tree-OID pruning)."""
        roots = [oid_bytes(r) for r in roots]
        k = len(roots)
        c0, c1 = compare if compare is not None else (N.KD_WALK_ALL, N.KD_WALK_ALL)
        outs = (ctypes.POINTER(N.KdLeaves) * k)()
        with self._lock:
            N.check(self.L.kd_walk(self._h, b"".join(roots), k, subpath.encode(), c0, c1, threads, outs), "kd_walk")
        return [_take_leaves(self.L, outs[i]) for i in range(k)]

    def tree_entries(self, oid):
        """one tree level: [(mode, type name, oid hex, name)] in git order"""
        t, data = self.read(oid)
        if t != OBJ_TREE:
            raise ValueError(f"{oid_bytes(oid).hex()} is a {TYPE_NAMES.get(t, t)}, not a tree")
        return parse_tree(data)


def parse_tree(data):
    """[(mode, "tree" | "blob" | "commit", oid hex, name)] of a raw tree object"""
    out, i, n = [], 0, len(data)
    while i < n:
        sp = data.index(b" ", i)
        nul = data.index(b"\0", sp)
        mode = int(data[i:sp], 8)
        oid = data[nul + 1:nul + 21].hex()
        typ = "tree" if mode == MODE_TREE else "commit" if mode == 0o160000 else "blob"
        out.append((mode, typ, oid, data[sp + 1:nul].decode()))
        i = nul + 21
    return out
