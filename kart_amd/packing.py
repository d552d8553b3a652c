"""Packing one commit's dataset feature tree into the engine's flat, key-sorted side arrays.

A *side* is what ``RichBaseDataset.diff_feature`` hands to libgit2 implicitly: the leaves under
``<ds>/.table-dataset/feature/`` of one commit (kart/rich_base_dataset.py:212-232).  Here they
become SoA arrays in join-key order (DESIGN.md "join key"):

* ``KD_KEY_INT`` (IntPathEncoder, kart/dataset3_paths.py:283-299): the filename is
  ``b64(msgpack([pk]))``; key = rank24(bucket) | wrap34 | frank(pk) (kart_amd/walkkey.py) —
  bijective with the pk, so equal keys are equal paths and the pk is recovered from the key without
  touching the filename again, and ascending in git's tree order: the leaves the tree walk lists are
  a key-ordered side already, with no sort (a leaf tree mixing 2**30 pk wraps is the exception:
  kd_keys_scan reports it and the side is sorted).
* ``KD_KEY_HASH`` (MsgpackHashPathEncoder, :202-215, and the 2x256 hex legacy layout): key = the
  tree levels as a (rank-mapped) bucket number | FNV-1a bits of the filename; the GPU verifies
  filenames of matched keys, a collision returns KD_EUNSUPPORTED.  Walk order is ascending in the
  bucket bits only: each bucket's few entries are sorted.

Packing runs on the CPU in the native library (kd_pack_*, kd_keys_scan), multithreaded.
"""
import time
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _native as N

# placeholder a native call gets for an empty host array: a module-level array, alive for every call
_PAD = np.zeros(16, np.uint8)


@dataclass
class PathEncoding:
    """The dataset's path-structure.json (kart/dataset3_paths.py:121-130,474-486)."""

    scheme: str = "int"  # "int" | "msgpack/hash"
    levels: int = 4
    branches: int = 64
    encoding: str = "base64"  # "base64" | "hex"

    @classmethod
    def from_dict(cls, d):
        if d is None:  # no path-structure.json -> LEGACY_ENCODER (kart/dataset3.py:233-248)
            return cls("msgpack/hash", 2, 256, "hex")
        return cls(d["scheme"], int(d["levels"]), int(d["branches"]), d["encoding"])

    @property
    def key_mode(self):
        return N.KD_KEY_INT if self.scheme == "int" else N.KD_KEY_HASH

    def to_dict(self):
        return {"scheme": self.scheme, "branches": self.branches, "levels": self.levels, "encoding": self.encoding}


INT_PK_ENCODING = PathEncoding("int", 4, 64, "base64")
GENERAL_ENCODING = PathEncoding("msgpack/hash", 4, 64, "base64")
LEGACY_ENCODING = PathEncoding("msgpack/hash", 2, 256, "hex")


def _arena(strings):
    """list[bytes|str] -> (uint8 arena, int64 offsets[n+1])"""
    bs = [s.encode() if isinstance(s, str) else s for s in strings]
    off = np.zeros(len(bs) + 1, np.uint64)
    if bs:
        off[1:] = np.cumsum(np.fromiter((len(b) for b in bs), np.uint64, len(bs)))
    data = np.frombuffer(b"".join(bs), np.uint8) if bs else np.zeros(0, np.uint8)
    return data, off


@dataclass
class PackedSide:
    """Key-sorted side arrays (host memory).  ``order[k]`` = index of sorted entry k in the
    caller's original entry order, so results map back to the caller's paths/blobs."""

    key: np.ndarray  # uint64 [n], strictly ascending
    oid: np.ndarray  # uint8 [n, 20]
    key_mode: int
    order: np.ndarray  # int64 [n]
    name: Optional[np.ndarray] = None  # uint8 arena (KD_KEY_HASH: relative paths, sorted order)
    name_off: Optional[np.ndarray] = None  # uint64 [n+1]
    encoding: PathEncoding = field(default_factory=lambda: INT_PK_ENCODING)
    dev: Optional[tuple] = None  # (key, oid) DevBufs when the side was packed on the GPU
    timing: Optional[dict] = None  # pack_side's stage times (parse_s, sort_s, sort_on)
    info: Optional[object] = None  # kd_keys_scan of the walk-order keys (_native.KdKeysInfo)
    # GPU pack of a side whose walk order is not key order: keys sorted (``key``, and in HBM), but
    # ``oid`` / ``name`` / ``name_off`` still in walk order (row ``order[k]`` for sorted entry k) and
    # the join reads them through the order (device.DevPermSide)
    dperm: Optional[object] = None

    @property
    def walk_rows(self):
        return self.dperm is not None

    @property
    def n(self):
        return int(self.key.shape[0])

    def kd_side(self):
        if self.walk_rows:
            raise ValueError("a late-materialised side joins through its order (engine *_perm paths); "
                             "materialised() gives the sorted form")
        s = N.KdSide()
        s.n = self.n
        if self.dev is not None and self.key_mode == N.KD_KEY_INT:  # already in HBM (GPU pack)
            s.key, s.oid, s.mem, s.key_mode = self.dev[0].ptr, self.dev[1].ptr, N.KD_MEM_DEVICE, self.key_mode
            s.name = s.name_off = None
            return s
        s.key = N.ptr(self.key)
        s.oid = N.ptr(self.oid)
        s.name = N.ptr(self.name) if self.name is not None and self.name.size else None
        s.name_off = N.ptr(self.name_off) if self.name_off is not None else None
        s.mem = N.KD_MEM_HOST
        s.key_mode = self.key_mode
        return s

    def rel_path(self, k):
        """relative path ('c/c/c/c/<filename>') of sorted entry k (KD_KEY_HASH sides)"""
        r = int(self.order[k]) if self.walk_rows else k
        a, b = int(self.name_off[r]), int(self.name_off[r + 1])
        return self.name[a:b].tobytes().decode()

    def materialised(self):
        """the sorted form of a late-materialised side (OIDs and filenames gathered into key order),
        for the host-form entry points (sharding, kd_diff2 / kd_merge3 on host arrays)"""
        if not self.walk_rows:
            return self
        out = PackedSide(key=self.key, oid=np.ascontiguousarray(self.oid[self.order]), key_mode=self.key_mode,
                         order=self.order, encoding=self.encoding, timing=self.timing, info=self.info)
        if self.name is not None:
            out.name, out.name_off = _gather_names(self.name, self.name_off, self.order)
        return out


class PackError(ValueError):
    pass


def parse_keys(paths, off, encoding: PathEncoding):
    """join keys of a relative-path arena, in arena order (native, multithreaded); PackError on a
    path the encoding cannot pack"""
    n = len(off) - 1
    keys = np.empty(n, np.uint64)
    status = np.empty(n, np.uint8)
    L = N.lib()
    pp = N.ptr(paths) if paths.size else N.ptr(_PAD)
    if encoding.key_mode == N.KD_KEY_INT:  # the native packer decodes each path's filename
        bad = L.kd_pack_int_keys(pp, N.ptr(off), n, N.ptr(keys), N.ptr(status))
    else:
        hex_ = 1 if encoding.encoding == "hex" else 0
        if (hex_ and encoding.branches != 256) or (not hex_ and encoding.branches != 64):
            raise PackError(f"unsupported path structure {encoding}")
        bad = L.kd_pack_hash_keys(pp, N.ptr(off), n, encoding.levels, hex_, N.ptr(keys), N.ptr(status))
    if bad < 0:
        N.check(int(bad), "pack")
    if bad:
        i = int(np.nonzero(status)[0][0])
        raise PackError(f"{bad} feature paths not packable, first: {paths[int(off[i]):int(off[i+1])].tobytes()!r}")
    return keys


def keys_scan(keys, key_mode):
    """kd_keys_scan: (vary bits, key0, pk range, already strictly ascending?) of a key array"""
    import ctypes

    keys = np.ascontiguousarray(keys, np.uint64)
    info = N.KdKeysInfo()
    N.check(N.lib().kd_keys_scan(N.ptr(keys) if keys.size else N.ptr(_PAD), keys.shape[0], int(key_mode),
                                 ctypes.byref(info)), "kd_keys_scan")
    return info


def _gather_names(paths, off, order, chunk=1 << 20):
    """the filename arena with rows in ``order`` (vectorised gathers, ``chunk`` rows at a time so
    the byte index stays small)"""
    n = order.shape[0]
    lens = (off[1:] - off[:-1])[order]
    noff = np.zeros(n + 1, np.uint64)
    noff[1:] = np.cumsum(lens)
    out = np.empty(int(noff[-1]), np.uint8)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        ln = lens[a:b].astype(np.int64)
        base = int(noff[a])
        idx = np.arange(int(noff[b]) - base, dtype=np.int64) + np.repeat(
            off[:-1][order[a:b]].astype(np.int64) - (noff[a:b].astype(np.int64) - base), ln)
        out[base:int(noff[b])] = paths[idx]
    return out, noff


SEG_SORT_MAX = 512  # the longest leaf tree kd_sort_segmented_into orders (err 4 beyond)


def sort_on_device_perm(engine, keys, oids, info, encoding, paths, off):
    """GPU pack of a side whose walk order is not key order, late-materialised as bench.py times it:
    the per-leaf-tree sort (kd_sort_segmented_into, one kernel) — KD_KEY_HASH sides always try it (a
    leaf tree lists its entries in filename order, not FNV order), KD_KEY_INT sides when the host's
    kd_keys_scan finds their leaf trees short (seg_max <= 512: a walk mixing pk wraps inside leaf
    trees) — else, or when a bucket is long or the buckets descend, the full radix sort of the
    compacted varying key bits (kd_sort_side_into, passes from kd_keys_scan, no OIDs moved).
    Returns (DevPermSide, sorted keys, order) — OIDs and filenames stay in walk order.  PackError on
    duplicate keys."""
    import ctypes

    from . import shard
    from .device import DevBuf, DevPermSide

    n = keys.shape[0]
    dk_in = DevBuf.from_numpy(engine, keys)
    dk, dord, flag = DevBuf(engine, 8 * n), DevBuf(engine, 4 * n), DevBuf(engine, 8)
    sorted_ok = False
    if encoding.key_mode == N.KD_KEY_HASH or 0 < info.seg_max <= SEG_SORT_MAX:
        flag.zero()
        bits = shard.bucket_bits(encoding.key_mode, encoding)
        N.check(engine.L.kd_sort_segmented_into(engine.ctx, dk_in.ptr, dk.ptr, dord.ptr, n, bits,
                                                info.seg_max if bits == 24 else 0, flag.ptr),
                "kd_sort_segmented_into")
        sorted_ok = int(flag.download(np.uint32, 1)[0]) == 0
    if not sorted_ok:
        flag.zero()
        N.check(engine.L.kd_sort_side_into(engine.ctx, dk_in.ptr, None, dk.ptr, None, dord.ptr, n, flag.ptr,
                                           ctypes.byref(info)), "kd_sort_side_into")
        if int(flag.download(np.uint32, 1)[0]):
            raise PackError("duplicate join keys within one side")
    dk_in.free()
    flag.free()
    do = DevBuf.from_numpy(engine, oids.reshape(-1))
    name = name_off = None
    if encoding.key_mode == N.KD_KEY_HASH:
        name = DevBuf.from_numpy(engine, paths if paths.size else np.zeros(1, np.uint8))
        name_off = DevBuf.from_numpy(engine, off)
    dp = DevPermSide(engine, n, encoding.key_mode, dk, do, dord, name, name_off)
    return dp, dk.download(np.uint64, n), dord.download(np.uint32, n).astype(np.int64)


def sort_on_device(engine, keys, oids):
    """GPU pack: (arena-order keys, oids) -> device-resident sorted side (kd_sort_side, LDS-ranked
    LSD radix sort) + host copies (sorted keys, sorted oids, order).  PackError on duplicate keys."""
    import ctypes

    from .device import DevBuf

    n = keys.shape[0]
    dk = DevBuf.from_numpy(engine, keys if n else np.zeros(1, np.uint64))
    do = DevBuf.from_numpy(engine, oids.reshape(-1) if n else np.zeros(20, np.uint8))
    dord = DevBuf(engine, 4 * max(n, 1))
    dup = ctypes.c_uint32(0)
    N.check(engine.L.kd_sort_side(engine.ctx, dk.ptr, do.ptr, dord.ptr, n, ctypes.byref(dup)), "kd_sort_side")
    if dup.value:
        raise PackError("duplicate join keys within one side")
    return dk, do, dord


def pack_side(rel_paths, oids, encoding: PathEncoding, rel_off=None, engine=None):
    """Pack leaves: rel_paths = list[str] (relative to feature/) or a uint8 arena with
    ``rel_off``; oids = uint8 [n, 20].  Returns PackedSide.  Raises PackError on paths that are
    not valid for the encoding (the caller falls back to the reference path).

    With an ``engine`` the sort runs on the GPU (kd_sort_side) and the side keeps its device copy
    (``side.dev``), which the engine's diffs then use without another upload."""
    if rel_off is None:
        paths, off = _arena(rel_paths)
    else:
        paths, off = np.ascontiguousarray(rel_paths, np.uint8), np.ascontiguousarray(rel_off, np.uint64)
    n = len(off) - 1
    oids = np.ascontiguousarray(oids, np.uint8).reshape(n, 20)
    t0 = time.perf_counter()
    keys = parse_keys(paths, off, encoding)
    info = keys_scan(keys, encoding.key_mode)
    t1 = time.perf_counter()
    dev = dperm = None
    if info.ascending:  # git walk order is key order already (int keys of one pk wrap per leaf tree)
        order = np.arange(n, dtype=np.int64)
        sorted_oids = oids
        sort_on = "none"
    elif engine is not None:
        # late materialisation: only the keys are sorted, OIDs and filenames stay in walk order
        dperm, keys, order = sort_on_device_perm(engine, keys, oids, info, encoding, paths, off)
        sorted_oids = oids
        sort_on = "gpu"
    else:
        order = np.argsort(keys, kind="stable")
        keys = keys[order]
        if n > 1 and not np.all(keys[1:] > keys[:-1]):
            raise PackError("duplicate join keys within one side")
        sorted_oids = oids[order]
        sort_on = "host"
    side = PackedSide(key=np.ascontiguousarray(keys), oid=np.ascontiguousarray(sorted_oids),
                      key_mode=encoding.key_mode, order=order.astype(np.int64), encoding=encoding)
    side.dev = dev
    side.info = info
    side.timing = {"parse_s": t1 - t0, "sort_s": time.perf_counter() - t1, "sort_on": sort_on}
    if sort_on == "gpu":
        side.dperm = dperm
        if encoding.key_mode == N.KD_KEY_HASH:  # the walk-order arena: the join reads it through the order
            side.name, side.name_off = paths, off
        return side
    if encoding.key_mode == N.KD_KEY_HASH:
        # sorted relative-path arena (needed for collision verification + pk decode)
        lens = (off[1:] - off[:-1])[order]
        noff = np.zeros(n + 1, np.uint64)
        noff[1:] = np.cumsum(lens)
        # byte j of sorted path k comes from off[order[k]] + j: one vectorised gather
        lens_i = lens.astype(np.int64)
        idx = np.arange(int(noff[-1]), dtype=np.int64) + np.repeat(off[:-1][order].astype(np.int64) - noff[:-1].astype(np.int64), lens_i)
        side.name = np.ascontiguousarray(paths[idx]) if n else np.zeros(0, np.uint8)
        side.name_off = noff
    return side


def empty_side(encoding: PathEncoding):
    s = PackedSide(key=np.zeros(0, np.uint64), oid=np.zeros((0, 20), np.uint8), key_mode=encoding.key_mode,
                   order=np.zeros(0, np.int64), encoding=encoding)
    if encoding.key_mode == N.KD_KEY_HASH:
        s.name = np.zeros(0, np.uint8)
        s.name_off = np.zeros(1, np.uint64)
    return s


def int_keys_to_pks(keys):
    keys = np.ascontiguousarray(keys, np.uint64)
    out = np.empty(keys.shape[0], np.int64)
    N.check(N.lib().kd_int_keys_to_pks(N.ptr(keys), keys.shape[0], N.ptr(out)), "int_keys_to_pks")
    return out


def pk_to_int_key(pk):
    """Python-int pk -> KD_KEY_INT key (same formula as the native packer, kart_amd/walkkey.py)."""
    from . import walkkey

    try:
        return walkkey.pk_to_int_key(pk)
    except ValueError as e:
        raise PackError(str(e)) from None
