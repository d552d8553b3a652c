"""Engine-backed dataset versions and the drop-in diff entry points.

Mirrors, behind the same call shapes, the reference's hot path:

* ``diff_feature(old, new, ...)``  <- RichBaseDataset.diff_feature (kart/rich_base_dataset.py:205-300)
* ``dataset_diff(base, target)``   <- RichBaseDataset.diff (:170-181) incl. diff_meta (:183-195)
* ``get_dataset_diff(...)``        <- diff_util.get_dataset_diff (kart/diff_util.py:51-95): swap +
                                      reverse when the base version is missing, prune.
* ``field_diff(feature_diff, ...)``<- the update loop of TextDiffWriter.write_feature_delta
                                      (kart/text_diff_writer.py:135-145), batched on the GPU.

Values stay lazy exactly as in the reference: every half-delta is
``(pk, functools.partial(version.get_feature_from_blob, blob))`` — classification reads no blob and
calls ``get_feature`` zero times; each value access calls it once (tests/test_diff.py:1656-1685);
``value.args[0]`` is the blob (base_diff_writer.py:505-507, DeltaFetcher).
"""
import base64
import contextlib
import functools
import gc
import operator
import os
import time

import msgpack
import numpy as np

from . import _native as N
from . import deltas as _deltas
from . import packing
from .adaptor import structs
from .schema import FieldMaps, Legend, Schema

try:
    from . import _kd_pystr as _pystr  # built with libkartdiff (kart_amd/csrc/Makefile)
except ImportError:  # pragma: no cover - the helper is optional host code
    _pystr = None

FEATURE_PATH = "feature/"
# stage timings of the last dataset_diff when set to a dict (scripts/e2e_repo_bench.py reads them)
STAGE_TIMES = None


def _lap(name, t0):
    t1 = time.perf_counter()
    if STAGE_TIMES is not None:
        STAGE_TIMES[name] = STAGE_TIMES.get(name, 0.0) + (t1 - t0)
    return t1
GPU_SORT_MIN = 1 << 20  # sides at least this long are sorted on the GPU when an engine is at hand


class Geometry(bytes):
    """A StandardGeoPackageBinary value (kart/geometry.py:111-122): bytes starting with b'GP'."""

    @classmethod
    def of(cls, b):
        if isinstance(b, Geometry):
            return b
        return Geometry(b) if b else None

    def __new__(cls, b):
        self = super().__new__(cls, b)
        if not self.startswith(b"GP"):
            raise ValueError(f"Invalid StandardGeoPackageBinary geometry: {bytes(self[:100])!r}")
        return self

    def __repr__(self):
        return f"Geometry({bytes.__repr__(self)})"


def _ext_hook(code, data):
    if code == ord("G"):
        return Geometry.of(data)
    return msgpack.ExtType(code, data)


def msg_unpack(b):
    """serialise_util.msg_unpack (kart/serialise_util.py:44-48)"""
    return msgpack.unpackb(b, raw=False, ext_hook=_ext_hook)


class Oid(str):
    """hex OID with the pygit2.Oid attributes the writers use (.hex, .raw)"""

    @property
    def hex(self):
        return str(self)

    @property
    def raw(self):
        return bytes.fromhex(self)


class LazyBlob:
    """What get_blob_at returns (a pygit2.Blob in Kart): .name / .id / content, each computed on
    first use from (dataset version, leaf index) — so classification reads no blob and builds no
    name or OID string, and a missing (promised) blob raises KeyError only when its value is
    accessed, as in the reference (DeltaFetcher relies on that)."""

    __slots__ = ("_src", "_i", "_data")
    type_str = "blob"

    def __init__(self, src, i):
        self._src = src
        self._i = i
        self._data = None

    @property
    def name(self):
        return self._src.blob_name(self._i)

    @property
    def id(self):
        return Oid(self._src.oids[self._i].tobytes().hex())

    oid = id

    @property
    def data(self):
        if self._data is None:
            d = self._src.cached_blob(self._i) if self._src._arenas else None
            self._data = d if d is not None else self._src.read_blob(self._i)
        return self._data

    def __bytes__(self):
        return self.data

    def __len__(self):
        return len(self.data)


class DatasetVersion:
    """One commit's version of one dataset (the state Dataset3 wraps): leaves + meta.

    ``rel_paths``: uint8 arena + offsets of the leaf paths relative to ``feature/``;
    ``oids`` [n, 20]; ``read_blob(i)`` -> bytes of leaf i (original order); ``read_blobs(idx)``
    (optional) -> (data, off, status) of many leaves in one batched read.  ``partial``: the leaves
    are only those under the subtrees a pruned walk opened (gitsource.dataset_versions).
    """

    partial = False

    def __init__(self, path, schema, legends, encoding, rel_paths, rel_off, oids, read_blob, meta=None,
                 read_blobs=None):
        self.path = path
        self.schema = schema
        self.legends = dict(legends)
        self.encoding = encoding
        self.rel_paths = np.ascontiguousarray(rel_paths, np.uint8)
        self.rel_off = np.ascontiguousarray(rel_off, np.uint64)
        self.oids = np.ascontiguousarray(oids, np.uint8).reshape(-1, 20)
        self.read_blob = read_blob
        self._read_blobs = read_blobs
        self.meta = dict(meta or {})
        self._packed = None
        self._packed_by = None  # the engine whose buffers a GPU-packed side holds
        self._arenas = []

    @property
    def n(self):
        return int(self.rel_off.shape[0]) - 1

    @property
    def packed(self):
        return self.pack()

    def pack(self, engine=None):
        """the side packed for the join (cached).  With a GPU engine and a large side the sort runs
        on the GPU (kd_sort_side); the host parses the keys either way.  A GPU-packed side holds device
        buffers of the engine that packed it: another engine, or that engine once closed, re-packs."""
        if self._packed is not None and self._packed.dperm is not None and engine is not None:
            own = self._packed_by
            if own is not engine or not getattr(own, "ctx", None):
                self._packed = None
        if self._packed is None:
            self._packed_by = None
            if self.n == 0:
                self._packed = packing.empty_side(self.encoding)
            else:
                gpu = engine if self.n >= GPU_SORT_MIN and hasattr(engine, "ctx") else None
                self._packed = packing.pack_side(self.rel_paths, self.oids, self.encoding, rel_off=self.rel_off,
                                                 engine=gpu)
                self._packed_by = gpu
        return self._packed

    # ---- Dataset3 API used by the diff path ----------------------------------------------------
    def rel_path(self, i):
        return self.rel_paths[int(self.rel_off[i]):int(self.rel_off[i + 1])].tobytes().decode()

    def meta_items(self):
        return dict(self.meta)

    def decode_path_to_1pk(self, path):
        """Dataset3.decode_path_to_1pk (kart/dataset3.py:250-259)"""
        pks = msg_unpack(base64.urlsafe_b64decode(os.path.basename(path)))
        if len(pks) != 1:
            raise ValueError(f"Expected a single pk_value, got {pks}")
        return pks[0]

    def get_blob(self, i):
        """leaf i (original order) as a lazy blob (BaseDataset.get_blob_at); a batch of them is read
        in one call (prefetch_blobs)"""
        return LazyBlob(self, int(i))

    def blob_name(self, i):
        """the leaf's filename (the last path component)"""
        a, b = int(self.rel_off[i]), int(self.rel_off[i + 1])
        seg = self.rel_paths[a:b].tobytes()
        return seg[seg.rfind(b"/") + 1:].decode()

    def get_blobs(self, idx):
        """LazyBlobs of many leaves (original order)"""
        return [LazyBlob(self, i) for i in np.asarray(idx, np.int64).tolist()]

    def get_feature(self, pk_values=None, *, path=None, data=None):
        """Dataset3.get_feature (kart/dataset3.py:185-223)"""
        if pk_values is None:
            pk_values = [self.decode_path_to_1pk(path)]
        legend_hash, non_pk = msg_unpack(data)
        legend = self.legends[legend_hash]
        raw = legend.value_tuples_to_raw_dict(tuple(pk_values), non_pk)
        return self.schema.feature_from_raw_dict(raw)

    def get_feature_from_blob(self, blob):
        """BaseDataset.get_feature_from_blob (kart/base_dataset.py:506-507)"""
        return self.get_feature(path=blob.name, data=memoryview(blob.data))

    def read_blobs(self, idx):
        """(data, off, status) of leaves ``idx`` (original order) as one arena; status 1 = the blob
        is not in the repository (its bytes are empty; reading it alone raises the KeyError)"""
        if self._read_blobs is not None:
            return self._read_blobs(idx)
        bs, status = [], np.zeros(len(idx), np.uint8)
        for k, i in enumerate(idx):
            try:
                bs.append(bytes(self.read_blob(int(i))))
            except KeyError:
                bs.append(b"")
                status[k] = 1
        data, off = packing._arena(bs)
        return data, off, status

    def blob_arena_leaves(self, leaf_idx):
        """contiguous (data, off) of the blobs of leaves ``leaf_idx`` (original order), one batched
        read; KeyError when one is missing.  The arena is remembered, so a later value access of
        one of these leaves slices it instead of reading the object again."""
        idx = np.asarray(leaf_idx, np.int64)
        data, off, status = self.read_blobs(idx)
        if status.any():
            self.read_blob(int(idx[int(np.nonzero(status)[0][0])]))  # raises the reference's KeyError
        self._remember_arena(idx, data, off)
        return data, off

    ARENAS_KEPT = 2  # the latest batched reads (a field diff reads both sides once): a bounded cache

    def _remember_arena(self, idx, data, off):
        order = np.argsort(idx, kind="stable")
        self._arenas.append((idx[order], order, data, off))
        del self._arenas[:-self.ARENAS_KEPT]

    def cached_blob(self, i):
        """leaf i's bytes from an arena blob_arena_leaves read, or None"""
        for idx, order, data, off in self._arenas:
            p = int(np.searchsorted(idx, i))
            if p < idx.shape[0] and idx[p] == i:
                r = int(order[p])
                return data[int(off[r]):int(off[r + 1])].tobytes()
        return None

    def blob_arena(self, sorted_idx):
        """contiguous (data, off) of the blobs at the given sorted indices (host packing for
        kd_fielddiff); KeyError when one is missing"""
        order = self.packed.order
        idx = order[np.asarray(sorted_idx, np.int64)]
        data, off, status = self.read_blobs(idx)
        if status.any():
            self.read_blob(int(idx[int(np.nonzero(status)[0][0])]))  # raises the reference's KeyError
        return data, off


def _pks(version, sorted_idx):
    """pk values of sorted entries (KD_KEY_INT: straight from the keys, vectorised)"""
    side = version.packed
    if side.key_mode == N.KD_KEY_INT:
        return packing.int_keys_to_pks(side.key[sorted_idx]).tolist()
    order = side.order
    return [version.decode_path_to_1pk(version.rel_path(int(order[k]))) for k in sorted_idx]


class UpdateBatch:
    """The update deltas one diff_feature run yielded, with both sides' leaf indices (original
    order): what field_diff needs to read the blobs straight into one arena per side, without
    walking the DeltaDiff or touching a blob object.  ``prefetch``: a future of those two arenas,
    read while the deltas were being built (or None)"""

    __slots__ = ("old_v", "new_v", "old_leaf", "new_leaf", "deltas", "keys", "n_total", "prefetch")

    def __init__(self):
        self.old_v = self.new_v = None
        self.old_leaf = self.new_leaf = None
        self.deltas, self.keys, self.n_total = [], [], -1
        self.prefetch = None


# diffs with at least this many updates read the updates' blobs while their deltas are built
PREFETCH_MIN_UPDATES = 10_000
_PREFETCH_POOL = None


def _prefetch_pool():
    global _PREFETCH_POOL
    if _PREFETCH_POOL is None:
        import concurrent.futures

        _PREFETCH_POOL = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="kd-prefetch")
    return _PREFETCH_POOL


class _Prefetch:
    """the update blobs of both sides being read by one native batched read on a worker thread; the
    caller does not return before the worker is inside that (GIL-free) call, so the delta
    construction that follows — one long C call holding the GIL — cannot starve it"""

    def __init__(self, old_v, new_v, oi, ni):
        import threading

        self.old_v, self.new_v, self.oi, self.ni = old_v, new_v, oi, ni
        src = old_v._read_blobs.source
        oids = np.concatenate([old_v.oids[oi], new_v.oids[ni]])
        started = threading.Event()

        def work():
            started.set()  # the read below releases the GIL within microseconds
            return src.read_blobs(oids)

        self.fut = _prefetch_pool().submit(work)
        started.wait()

    def result(self):
        """the two update-order arenas, as _arena_pair returns them"""
        data, off, status = self.fut.result()
        oi, ni = self.oi, self.ni
        if status.any():  # the per-side reads raise the reference's KeyError for the first missing blob
            return self.old_v.blob_arena_leaves(oi), self.new_v.blob_arena_leaves(ni)
        k = oi.size
        cut = int(off[k])
        arenas = ((data[:cut], off[:k + 1]), (data[cut:], off[k:] - off[k]))
        self.old_v._remember_arena(oi, *arenas[0])
        self.new_v._remember_arena(ni, *arenas[1])
        return arenas


def _start_prefetch(old_v, new_v, old_leaf, new_leaf):
    """a _Prefetch of the updates' blobs when both versions read from one repository (else None:
    the per-side reads happen in field_diff)"""
    src = getattr(old_v._read_blobs, "source", None)
    if src is None or src is not getattr(new_v._read_blobs, "source", None):
        return None
    return _Prefetch(old_v, new_v, np.asarray(old_leaf, np.int64), np.asarray(new_leaf, np.int64))


def diff_feature(engine, base, target, feature_filter=None, reverse=False, updates=None, _collect=None):
    """Generator of Delta with lazy values (RichBaseDataset.diff_feature semantics).

    base / target: DatasetVersion or None (a missing dataset diffs against the empty tree).
    updates: an UpdateBatch that receives the yielded update deltas (set once the generator is
    exhausted).  _collect=dict: the deltas are stored there at their keys instead of
    yielded (dataset_diff's bulk path)."""
    present = base if base is not None else target
    if present is None:
        return
    S = structs()
    t = time.perf_counter()
    empty = packing.empty_side(present.encoding)
    A = base.pack(engine) if base is not None else empty
    B = target.pack(engine) if target is not None else empty
    t = _lap("pack", t)
    res = engine.diff2(A, B)
    t = _lap("classify2", t)
    old_v, new_v = (target, base) if reverse else (base, target)
    d = res.delta
    if reverse:
        d = d[:, ::-1]
        A, B = B, A
    a_idx, b_idx = d[:, 0], d[:, 1]
    has_a, has_b = a_idx != N.KD_NONE, b_idx != N.KD_NONE
    ia, ib = np.nonzero(has_a)[0], np.nonzero(has_b)[0]
    n = d.shape[0]
    old_leaf = np.full(n, -1, np.int64)
    new_leaf = np.full(n, -1, np.int64)
    old_leaf[ia] = A.order[a_idx[ia]]
    new_leaf[ib] = B.order[b_idx[ib]]
    match_all = feature_filter is None or getattr(feature_filter, "match_all", False)
    if updates is not None and match_all and old_v is not None and new_v is not None:
        # the updates' blobs are read on a worker thread (native, GIL released) while the deltas
        # are built here: field_diff then takes the arenas from updates.prefetch
        both = np.nonzero(has_a & has_b)[0]
        if both.size >= PREFETCH_MIN_UPDATES:
            updates.prefetch = _start_prefetch(old_v, new_v, old_leaf[both], new_leaf[both])
    old_pks, new_pks = _pk_column(old_v, a_idx, ia, n), _pk_column(new_v, b_idx, ib, n)
    t = _lap("pks", t)
    # this module's own Delta / KeyValue: built field by field (the constructor's argument
    # normalisation is most of a delta's host cost); Kart's classes through their constructor
    own = S.Delta is _deltas.Delta
    old_get, new_get = (old_v.get_feature_from_blob if old_v is not None else None,
                        new_v.get_feature_from_blob if new_v is not None else None)
    if match_all and _pystr is not None:
        # the whole delta list built in C (kart_amd/csrc/kd_pystr.c build_deltas): the same lazy
        # blobs, partial promises, KeyValue halves and Delta objects the loop below builds
        # (the promises are _kd_pystr.Promise: partial(get_feature_from_blob, LazyBlob(version, leaf))
        # with the blob made on first use — one object per half instead of blob + partial + args)
        keys, dl, upd_rows, upd_deltas, upd_keys = _pystr.build_deltas(
            S.Delta, _deltas.KeyValue, LazyBlob, _pystr.Promise, old_get, new_get, old_v, new_v,
            old_leaf, new_leaf, old_pks, new_pks, own, _collect)
        n_total = len(dl)
        t = _lap("build_deltas", t)
        if _collect is None:
            yield from dl
    else:
        if isinstance(old_pks, np.ndarray):
            old_pks = old_pks.tolist()
        if isinstance(new_pks, np.ndarray):
            new_pks = new_pks.tolist()
        upd_rows, upd_deltas, upd_keys, n_total = [], [], [], 0
        store = _collect.__setitem__ if _collect is not None else None
        Delta, KeyValue, new_obj, partial = _deltas.Delta, _deltas.KeyValue, object.__new__, functools.partial
        olist, nlist = old_leaf.tolist(), new_leaf.tolist()
        for i in range(n):
            opk, npk = old_pks[i], new_pks[i]
            ol, nl = olist[i], nlist[i]
            if not match_all and (ol < 0 or str(opk) not in feature_filter) and (nl < 0 or str(npk) not in feature_filter):
                continue
            ob = LazyBlob(old_v, ol) if ol >= 0 else None
            nb = LazyBlob(new_v, nl) if nl >= 0 else None
            if own:
                delta = new_obj(Delta)
                delta.old = KeyValue(opk, partial(old_get, ob)) if ob is not None else None
                delta.new = KeyValue(npk, partial(new_get, nb)) if nb is not None else None
                delta.type = "insert" if ob is None else ("delete" if nb is None else "update")
                delta.flags = 0
            else:
                old_half = (opk, partial(old_get, ob)) if ob is not None else None
                new_half = (npk, partial(new_get, nb)) if nb is not None else None
                delta = S.Delta(old_half, new_half)
            if ob is not None and nb is not None:
                upd_rows.append(i)
                upd_deltas.append(delta)
                upd_keys.append(opk)
            n_total += 1
            if _collect is None:
                yield delta
            else:
                store(opk if ob is not None else npk, delta)
    if updates is not None:
        rows = np.frombuffer(upd_rows, np.int64) if isinstance(upd_rows, bytes) else np.asarray(upd_rows, np.int64)
        updates.old_v, updates.new_v = old_v, new_v
        updates.old_leaf = old_leaf[rows]
        updates.new_leaf = new_leaf[rows]
        updates.deltas, updates.keys, updates.n_total = upd_deltas, upd_keys, n_total


def _pk_column(version, idx, present, n):
    """the pk of every delta row on one side (rows ``present`` hold an entry): an int64 array for
    KD_KEY_INT sides (straight from the keys), else a list (None where absent)"""
    if version is None or not present.size:
        return np.zeros(n, np.int64)
    sorted_idx = idx[present]
    side = version.packed
    if side.key_mode == N.KD_KEY_INT:
        out = np.zeros(n, np.int64)
        out[present] = packing.int_keys_to_pks(side.key[sorted_idx])
        return out
    out = [None] * n
    for i, pk in zip(present.tolist(), _pks(version, sorted_idx)):
        out[i] = pk
    return out


def dataset_diff(engine, base, target, ds_filter=None, reverse=False):
    """RichBaseDataset.diff (kart/rich_base_dataset.py:170-181): {"meta": dict diff, "feature": DeltaDiff}"""
    S = structs()
    t = time.perf_counter()
    out = S.DatasetDiff()
    old, new = (target, base) if reverse else (base, target)
    out["meta"] = S.DeltaDiff.diff_dicts(old.meta_items() if old else {}, new.meta_items() if new else {})
    t = _lap("meta", t)
    ffilter = None
    if ds_filter is not None and not getattr(ds_filter, "match_all", False):
        # a filter without a "feature" entry matches no feature (the reference falls back to an empty
        # child filter: ds_filter.get("feature", ds_filter.child_type()), :177)
        ffilter = ds_filter.get("feature", _NoKeys())
    batch = UpdateBatch()
    with _gc_paused():
        if S.DeltaDiff is _deltas.DeltaDiff:  # this module's own DeltaDiff: its dict filled in place
            fd = S.DeltaDiff()
            for _ in diff_feature(engine, base, target, ffilter, reverse=reverse, updates=batch, _collect=fd.data):
                pass
        else:
            fd = S.DeltaDiff(diff_feature(engine, base, target, ffilter, reverse=reverse, updates=batch))
    fd._kd_updates = batch
    out["feature"] = fd
    return out


@contextlib.contextmanager
def _gc_paused():
    """Bulk construction of deltas (about ten small objects each, none of them cyclic garbage):
    with the cyclic collector running, its generation-2 passes rescan the whole heap several times
    per 100K deltas, which doubled the host cost of a diff"""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            # the objects built while paused go straight to the oldest generation (freeze moves every
            # tracked object to the permanent generation, unfreeze back into the oldest one): without
            # this, the first young-generation pass after enable() walks all of them (~0.15 s per
            # 300k deltas).  Skipped when the host keeps frozen objects of its own.
            if gc.get_freeze_count() == 0:
                gc.freeze()
                gc.unfreeze()
            gc.enable()


class _NoKeys(frozenset):
    """an empty, non-match-all key filter"""

    match_all = False


def get_dataset_diff(engine, base, target, ds_filter=None):
    """diff_util.get_dataset_diff for one dataset present in either commit (kart/diff_util.py:51-95)"""
    params = {}
    if base is None:
        base, target = target, base
        params["reverse"] = True
    if base is None:
        return structs().DatasetDiff()
    ds = dataset_diff(engine, base, target, ds_filter, **params)
    ds.prune()
    return ds


# ---------------------------------------------------------------------------------------------
# diff_estimation: exact counts straight from classify2
# ---------------------------------------------------------------------------------------------
ACCURACY_CHOICES = ("veryfast", "fast", "medium", "good", "exact")  # kart/diff_estimation.py:50


def get_exact_diff_blob_count(engine, base, target):
    """diff_estimation.get_exact_diff_blob_count (kart/diff_estimation.py:51-76) for one dataset's
    feature trees: the number of paths `git diff --name-only --no-renames` lists = inserts +
    updates + deletes of classify2, with no blob read and no git subprocess.

    base / target: DatasetVersion or None (the empty tree)."""
    present = base if base is not None else target
    if present is None:
        return 0
    empty = packing.empty_side(present.encoding)
    A = base.pack(engine) if base is not None else empty
    B = target.pack(engine) if target is not None else empty
    r = engine.diff2(A, B)
    return int(r.n_insert + r.n_update + r.n_delete)


def estimate_diff_feature_counts(engine, base_datasets, target_datasets, *, accuracy):
    """diff_estimation.estimate_diff_feature_counts (kart/diff_estimation.py:96-184) without a
    working copy: {dataset path: changed feature count}, datasets with no change left out.

    base_datasets / target_datasets: {path: DatasetVersion} of the two commits.  Every accuracy
    is answered with the exact count: the join costs less than the reference's subtree sampling,
    so "veryfast".."good" (estimates by contract) return the exact value too."""
    assert accuracy in ACCURACY_CHOICES
    counts = {}
    for path in sorted(set(base_datasets) | set(target_datasets)):
        n = get_exact_diff_blob_count(engine, base_datasets.get(path), target_datasets.get(path))
        if n:
            counts[path] = n
    return counts


def field_diff(engine, feature_diff, old_version, new_version, stats=None):
    """Attach ``changed_fields`` (names, in _all_feature_keys order) to every update delta of
    ``feature_diff``, computed by kd_fielddiff in one batch.  Updates the GPU cannot handle
    (status != 0) get None and the caller uses the reference loop for them.

    A DeltaDiff that dataset_diff built carries its updates' leaf indices: each side's blobs are
    read by one kd_odb_read_batch straight into the arena kd_fielddiff takes (no per-blob Python
    object), and the arena is kept for later value reads.  Any other DeltaDiff (built by hand,
    combined with ``+``) goes through its lazy blobs.  ``stats`` (a dict) receives the seconds of
    the blob reads, the kernel call and the name attachment."""
    import time

    t0 = time.perf_counter()
    with _gc_paused():
        batch = _live_batch(feature_diff, old_version, new_version)
        if batch is not None:
            ups = batch.deltas
            if not ups:
                return 0
            if batch.prefetch is not None:  # read while the deltas were built (diff_feature)
                fut, batch.prefetch = batch.prefetch, None
                (od, oo), (nd, no) = fut.result()
            else:
                (od, oo), (nd, no) = _arena_pair(old_version, new_version, batch.old_leaf, batch.new_leaf)
        else:
            ups = [d for d in feature_diff.values() if d.type == "update"]
            if not ups:
                return 0
            od, oo = _blob_arena([d.old.value.args[0] for d in ups])
            nd, no = _blob_arena([d.new.value.args[0] for d in ups])
        t1 = time.perf_counter()
        maps = FieldMaps(old_version.schema, old_version.legends, new_version.schema, new_version.legends)
        masks, status = engine.fielddiff(od, oo, nd, no, None, maps)
        t2 = time.perf_counter()
        masks = masks[:len(ups)]
        if _pystr is not None and isinstance(ups, list):
            # kart_amd/csrc/kd_pystr.c attach_fields: each distinct mask decoded once, a fresh
            # list per update written into Delta's slot
            _pystr.attach_fields(ups, masks, status, maps.words,
                                 lambda i: list(maps.changed_names(masks[i])), _deltas.Delta)
        else:
            names = maps.changed_names_rows(masks)
            for d, nm, s in zip(ups, names, status.tolist()):
                d.changed_fields = nm if s == 0 else None
        if stats is not None:
            stats.update(read_s=t1 - t0, kernel_s=t2 - t1, attach_s=time.perf_counter() - t2)
        return len(ups)


def _arena_pair(old_v, new_v, old_leaf, new_leaf):
    """blob_arena_leaves of both sides; versions read from one repository take ONE batched read (one
    thread pool over both sides' delta chains: the old side's deep chains and the new side's short
    ones balance), split into two arenas over the same buffer"""
    src = getattr(old_v._read_blobs, "source", None)
    if src is None or src is not getattr(new_v._read_blobs, "source", None):
        return old_v.blob_arena_leaves(old_leaf), new_v.blob_arena_leaves(new_leaf)
    oi, ni = np.asarray(old_leaf, np.int64), np.asarray(new_leaf, np.int64)
    data, off, status = src.read_blobs(np.concatenate([old_v.oids[oi], new_v.oids[ni]]))
    if status.any():  # the per-side reads raise the reference's KeyError for the first missing blob
        return old_v.blob_arena_leaves(old_leaf), new_v.blob_arena_leaves(new_leaf)
    k = oi.size
    cut = int(off[k])
    arenas = ((data[:cut], off[:k + 1]), (data[cut:], off[k:] - off[k]))
    old_v._remember_arena(oi, *arenas[0])
    new_v._remember_arena(ni, *arenas[1])
    return arenas


def _live_batch(feature_diff, old_version, new_version):
    """the UpdateBatch of a DeltaDiff that still holds exactly the deltas dataset_diff put there:
    same size, and every recorded update still stored under its key (C-level loops, no walk of the
    whole diff)"""
    batch = getattr(feature_diff, "_kd_updates", None)
    if batch is None or batch.old_v is not old_version or batch.new_v is not new_version:
        return None
    if len(feature_diff) != batch.n_total:
        return None
    if not all(map(operator.is_, map(feature_diff.get, batch.keys), batch.deltas)):
        return None
    return batch


def prefetch_blobs(blobs):
    """Read the not-yet-read LazyBlobs of ``blobs`` with one batched read per dataset version
    (kd_odb_read_batch under gitsource).  Returns ok[] — False where the blob is not in the
    repository (reading it alone raises the reference's KeyError)."""
    groups = {}
    for k, b in enumerate(blobs):
        if type(b) is LazyBlob and b._data is None:
            groups.setdefault(id(b._src), (b._src, []))[1].append(k)
    ok = np.ones(len(blobs), bool)
    for v, ks in groups.values():
        data, off, status = v.read_blobs([blobs[k]._i for k in ks])
        raw, offs, st = data.tobytes(), off.tolist(), status.tolist()
        for j, k in enumerate(ks):
            if st[j] == 0:
                blobs[k]._data = raw[offs[j]:offs[j + 1]]
            else:
                ok[k] = False
    return ok


def _blob_arena(blobs):
    """(data, off) of LazyBlobs, read in batches; a missing blob raises its KeyError as a single
    read does"""
    ok = prefetch_blobs(blobs)
    if not ok.all():
        blobs[int(np.nonzero(~ok)[0][0])].data  # raises the reference's KeyError
    return packing._arena([b.data for b in blobs])
