"""Device-resident pipelines on libkartdiff's own memory API (kd_malloc / kd_memcpy): sides and blob
arenas held in HBM, classify2 -> fielddiff launched back to back on the context stream with no host
round trip.  No GPU framework is involved.

This is the path bench.py times: inputs already resident, outputs stay resident (the delta list,
update list, per-update changed-field masks).
"""
import ctypes

import numpy as np

from . import _native as N


class DevBuf:
    """One HBM allocation of the engine's device (freed with the object or by ``free()``)."""

    def __init__(self, engine, nbytes):
        self.eng = engine
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        N.check(engine.L.kd_malloc(engine.ctx, max(self.nbytes, 16), ctypes.byref(p)), "kd_malloc")
        self.ptr = p.value

    @classmethod
    def from_numpy(cls, engine, a):
        """device copy of a numpy array (synchronous; pinned staging is the caller's choice)"""
        a = np.ascontiguousarray(a)
        b = cls(engine, a.nbytes)
        b.upload(a)
        return b

    def upload(self, a, offset=0, sync=True):
        a = np.ascontiguousarray(a)
        assert offset + a.nbytes <= self.nbytes
        if a.nbytes:
            N.check(self.eng.L.kd_memcpy(self.eng.ctx, self.ptr + offset, a.ctypes.data, a.nbytes, N.KD_COPY_H2D),
                    "kd_memcpy H2D")
            if sync:
                self.eng.sync()

    def download(self, dtype, count, offset=0):
        """host numpy copy of `count` items of `dtype` at byte `offset` (synchronous)"""
        dt = np.dtype(dtype)
        out = np.empty(int(count), dt)
        if out.nbytes:
            assert offset + out.nbytes <= self.nbytes
            N.check(self.eng.L.kd_memcpy(self.eng.ctx, out.ctypes.data, self.ptr + offset, out.nbytes, N.KD_COPY_D2H),
                    "kd_memcpy D2H")
            self.eng.sync()
        return out

    def zero(self):
        N.check(self.eng.L.kd_memset(self.eng.ctx, self.ptr, 0, self.nbytes), "kd_memset")

    def free(self):
        if self.ptr and self.eng.ctx:
            self.eng.L.kd_mfree(self.eng.ctx, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _nonempty(a, dtype, width=1):
    return a if a is not None and a.size else np.zeros(width, dtype)


class DevSide:
    """A PackedSide's arrays in HBM."""

    def __init__(self, engine, side, keys_only=False):
        """keys_only: only the keys go to HBM (OIDs / filenames: a zero placeholder), for entry points
        that read keys alone (kd_delta_pk_order) — any side form"""
        if keys_only:
            self.n, self.key_mode = side.n, side.key_mode
            self.key = DevBuf.from_numpy(engine, _nonempty(side.key, np.uint64))
            self.oid = DevBuf.from_numpy(engine, np.zeros(20, np.uint8))
            self.name = self.name_off = None
            return
        if getattr(side, "walk_rows", False):
            # (sorted keys beside walk-order OIDs / filenames: uploaded as one side, each key would be
            # paired with another entry's OID — such sides join through their order, DevPermSide)
            raise ValueError("DevSide needs a key-ordered side; a late-materialised side joins through its order "
                             "(side.materialised() gives the sorted form)")
        self.n = side.n
        self.key_mode = side.key_mode
        self.key = DevBuf.from_numpy(engine, _nonempty(side.key, np.uint64))
        self.oid = DevBuf.from_numpy(engine, _nonempty(side.oid.reshape(-1) if side.n else None, np.uint8, 20))
        self.name = self.name_off = None
        if side.name is not None:
            self.name = DevBuf.from_numpy(engine, _nonempty(side.name, np.uint8))
            self.name_off = DevBuf.from_numpy(engine, side.name_off)

    def kd_side(self):
        s = N.KdSide()
        s.n = self.n
        s.key = self.key.ptr
        s.oid = self.oid.ptr
        s.name = self.name.ptr if self.name is not None else None
        s.name_off = self.name_off.ptr if self.name_off is not None else None
        s.mem = N.KD_MEM_DEVICE
        s.key_mode = self.key_mode
        return s


class DevPermSide:
    """A side packed on the GPU for the late-materialised join (packing.pack_side with an engine, when
    the walk order is not key order): keys sorted in HBM, OIDs and (KD_KEY_HASH) the filename arena
    left in walk order, ``order[k]`` = walk row of sorted entry k — what kd_diff2_device_perm /
    kd_merge3_device_perm read through (bench.py's fallback_sort times the same path)."""

    def __init__(self, engine, n, key_mode, key, oid, order, name=None, name_off=None):
        self.n, self.key_mode = int(n), key_mode
        self.key, self.oid, self.order, self.name, self.name_off = key, oid, order, name, name_off

    def kd_side(self):
        s = N.KdSide()
        s.n = self.n
        s.key, s.oid = self.key.ptr, self.oid.ptr
        s.name = self.name.ptr if self.name is not None else None
        s.name_off = self.name_off.ptr if self.name_off is not None else None
        s.mem = N.KD_MEM_DEVICE
        s.key_mode = self.key_mode
        return s


def perm_dev(engine, side):
    """(kd_side, order DevBuf, keep-alive) of a PackedSide for the *_perm entry points: its DevPermSide,
    or a sorted-form side uploaded with an identity order"""
    if side.dperm is not None:
        return side.dperm.kd_side(), side.dperm.order, side.dperm
    ds = DevSide(engine, side)
    order = DevBuf.from_numpy(engine, np.arange(max(side.n, 1), dtype=np.uint32))
    return ds.kd_side(), order, (ds, order)


class _WalkSide:
    """a side's arrays in another order (what DevSide uploads): keys, OIDs and (KD_KEY_HASH) the
    filename arena with rows in that order"""

    def __init__(self, side, perm):
        self.key, self.oid = np.ascontiguousarray(side.key[perm]), np.ascontiguousarray(side.oid[perm])
        self.n = int(side.n)
        self.key_mode = side.key_mode
        self.name = self.name_off = None
        if side.name is not None:
            lens = (side.name_off[1:] - side.name_off[:-1])[perm]
            off = np.zeros(self.n + 1, np.uint64)
            np.cumsum(lens, out=off[1:])
            src = side.name_off[:-1][perm].astype(np.int64)
            idx = np.arange(int(off[-1]), dtype=np.int64) + np.repeat(src - off[:-1].astype(np.int64), lens.astype(np.int64))
            self.name, self.name_off = np.ascontiguousarray(side.name[idx]), off


class DevBlobs:
    """A blob arena (uint8 data, uint64 off[n+1]) in HBM."""

    def __init__(self, engine, data, off):
        self.n = int(off.shape[0]) - 1
        self.data = DevBuf.from_numpy(engine, _nonempty(data, np.uint8))
        self.off = DevBuf.from_numpy(engine, off)
        self.nbytes = int(data.size)
        # typical blob = mean over the non-empty blobs (an arena may hold only the blobs a diff reads)
        nz = int(np.count_nonzero(off[1:] != off[:-1])) if self.n else 0
        self.mean_len = int((int(off[-1]) - int(off[0]) + nz - 1) // nz) if nz else 0

    def kd_blobs(self):
        b = N.KdBlobs()
        b.n = self.n
        b.data = self.data.ptr
        b.off = self.off.ptr
        b.mem = N.KD_MEM_DEVICE
        b.size_hint = min(self.mean_len, 0xFFFFFFFF)  # typical (mean) blob size: picks the window shape
        return b


class DiffPipeline:
    """classify2 + fielddiff (+ the deltas in pk order) over device-resident sides (one GPU), back to
    back on one stream.

    The sides are as the tree walk lists them: for int pks that is ascending key order already
    (kart_amd/walkkey.py), so a step is the join on the walk-order arrays, the field diff of its
    updates and (``pk_order``) the radix sort of the delta and update records into pk order
    (kd_delta_pk_order: DeltaDiff.sorted_items) — no side sort.

    ``unsorted=(base_perm, target_perm)``: the fallback for a side whose walk order is not key order
    (a leaf tree mixing pk wraps, or a hash-key side): the sides are held with rows ``side.key[perm]``
    and every step first sorts their keys on the GPU (kd_sort_side_into, passes sized by
    kd_keys_scan, no read-back); the join reads the OIDs (and filenames) through the sort orders
    (kd_diff2_device_perm), or — ``late=False`` — the sort gathers the OIDs into key order.

    ``gather=(base_off, target_off)``: this GPU holds one bucket-range shard of a larger diff (its
    entries start at those global sorted indices); each step then runs kd_diff2_gather — the shard's
    join, its delta records rebased to global indices and all-gathered with every rank's counts over
    the library's RCCL communicator (``engine.comm_init`` first) — and field-diffs the shard's own
    updates."""

    def __init__(self, engine, base, target, base_blobs, target_blobs, maps, ordered=True, gather=None, unsorted=None,
                 late=True, pk_order=True, radix=False):
        """``unsorted`` (the fallback): both sides in that row order instead, sorted on the device inside
        every step — per leaf tree (kd_sort_segmented_into) when the host's kd_keys_scan finds the
        leaf trees short, else (or ``radix``) the onesweep radix sort (kd_sort_side_into)"""
        from . import packing

        self.eng = engine
        self.flags = 0 if ordered else N.KD_DIFF_UNORDERED
        self.A = DevSide(engine, base)
        self.B = DevSide(engine, target)
        self.walk = None
        self.late = bool(late) and gather is None
        self.seg_err = None
        if unsorted is not None:
            self.walk = []
            for side, perm in zip((base, target), unsorted):
                w = _WalkSide(side, perm)
                info = packing.keys_scan(w.key, side.key_mode)
                self.walk.append((DevSide(engine, w), DevBuf(engine, 4 * max(side.n, 1)), side.n, info))
            # per leaf tree when every side's leaf trees are short (no read-back: the plan is the host scan's)
            self.segmented = self.late and not radix and all(0 < x[3].seg_max <= packing.SEG_SORT_MAX for x in self.walk)
            if self.segmented:
                self.seg_err = DevBuf(engine, 8)
                self.seg_err.zero()
        self.OB = DevBlobs(engine, *base_blobs)
        self.NB = DevBlobs(engine, *target_blobs)
        self.OB_off_host, self.NB_off_host = base_blobs[1], target_blobs[1]
        self.OB_data_host, self.NB_data_host = base_blobs[0], target_blobs[0]
        self._ob_u = None  # use_update_arenas: update-order arenas (no pairs)
        self.maps = maps
        cap = base.n + target.n + 1
        self.cap = cap
        self.cap_upd = min(base.n, target.n)  # updates <= matched keys
        self.delta = DevBuf(engine, 8 * cap)
        self.upd = DevBuf(engine, 8 * cap)
        self.counts = DevBuf(engine, 64)  # [0..3] counts, [4] error word
        self.counts.zero()
        self.masks = DevBuf(engine, 8 * cap * maps.words)
        self.status = DevBuf(engine, cap)
        self._sa, self._sb = self.A.kd_side(), self.B.kd_side()
        self._ob, self._nb = self.OB.kd_blobs(), self.NB.kd_blobs()
        self._km = maps.kd_maps()
        self._perm_sides = None
        # pk order of the deltas and updates (KD_KEY_INT): the passes sized by the pk range
        self.pk_order = bool(pk_order) and base.key_mode == N.KD_KEY_INT and gather is None
        if self.pk_order:
            lo, hi = [], []
            for side in (base, target):
                info = side.info if side.info is not None else packing.keys_scan(side.key, side.key_mode)
                if side.n:
                    lo.append(int(info.pk_min))
                    hi.append(int(info.pk_max))
            self.pk_range = (min(lo), max(hi)) if lo else (0, 0)
            self.d_pk = DevBuf(engine, 8 * cap)
            self.d_perm = DevBuf(engine, 4 * cap)
            # the join writes every delta's / update's key beside it (kd_diff2_device_ex): the pk
            # order reads them in order instead of gathering them from the sides
            self.dkey = DevBuf(engine, 8 * cap)
            self.ukey = DevBuf(engine, 8 * cap)
            self.u_pk = DevBuf(engine, 8 * max(self.cap_upd, 1))
            self.u_perm = DevBuf(engine, 4 * max(self.cap_upd, 1))
        self.gather = gather
        if gather is not None:
            self.world = engine.nranks
            self.all_counts = DevBuf(engine, 64 * self.world)
            self.h_counts = np.zeros(8 * self.world, np.uint64)
            self.all_cap = cap * self.world  # until reserve_gather() knows the largest shard's deltas
            self.all_delta = DevBuf(engine, 8 * self.all_cap)
        engine.reserve(max(base.n, target.n))
        engine.sync()

    def use_update_arenas(self, upd):
        """field-diff from update-order arenas (the drop-in's form: the blob reader writes update i's
        blobs at arena index i) instead of the per-entry arenas through the join's pairs.  When the
        per-entry arenas hold the updated entries' blobs only, back to back in key (= update) order
        (the synthetic C3 layers), the update-order arenas are the same bytes with one offset per
        update and only those offsets are uploaded; otherwise the updates' blobs are gathered on the
        host into new arenas.  ``upd`` = the join's update list [m, 2] (the same every step)."""
        m = int(upd.shape[0])
        self._u_arenas = []
        blobs = []
        for side, off_h, dev in ((0, self.OB_off_host, self.OB), (1, self.NB_off_host, self.NB)):
            idx = np.asarray(upd[:, side], np.int64)
            start = off_h[idx]
            lens = off_h[idx + 1] - start
            off = np.zeros(m + 1, np.uint64)
            np.cumsum(lens, out=off[1:])
            if m == 0 or np.array_equal(start, start[0] + off[:-1]):  # contiguous: same bytes, new offsets
                u = DevBuf.from_numpy(self.eng, off + (np.uint64(start[0]) if m else np.uint64(0)))
                self._u_arenas.append(u)
                b = dev.kd_blobs()
                b.n, b.off = m, u.ptr
            else:  # gather the updates' blobs into an update-order arena
                data = (self.OB_data_host, self.NB_data_host)[side]
                pos = np.repeat(start.astype(np.int64) - off[:-1].astype(np.int64), lens.astype(np.int64)) + \
                    np.arange(int(off[-1]), dtype=np.int64)
                arena = DevBlobs(self.eng, np.ascontiguousarray(data[pos]), off)
                self._u_arenas.append(arena)
                b = arena.kd_blobs()
            blobs.append(b)
        self._ob_u, self._nb_u = blobs

    def reserve_gather(self, max_deltas_per_rank):
        """size the gathered-record buffer for at most this many deltas on any rank"""
        self.all_delta.free()
        self.all_cap = max(int(max_deltas_per_rank), 1) * self.world
        self.all_delta = DevBuf(self.eng, 8 * self.all_cap)

    def sort_step(self):
        """(fallback) the two GPU side sorts into the sorted side buffers"""
        L, ctx = self.eng.L, self.eng.ctx
        for (w, order, n, info), S in zip(self.walk, (self.A, self.B)):
            if self.segmented:
                N.check(L.kd_sort_segmented_into(ctx, w.key.ptr, S.key.ptr, order.ptr, n, 24, info.seg_max, self.seg_err.ptr),
                        "kd_sort_segmented_into")
            elif self.late:
                N.check(L.kd_sort_side_into(ctx, w.key.ptr, None, S.key.ptr, None, order.ptr, n, None,
                                            ctypes.byref(info)), "kd_sort_side_into")
            else:
                N.check(L.kd_sort_side_into(ctx, w.key.ptr, w.oid.ptr, S.key.ptr, S.oid.ptr, order.ptr, n, None,
                                            ctypes.byref(info)), "kd_sort_side_into")

    def orders(self):
        """(fallback) host copies of the two sort orders: walk index of sorted entry k"""
        return [order.download(np.uint32, n) for _, order, n, _ in self.walk]

    def step(self):
        """one pass of the hot path: (fallback) both side sorts, then the diff + field diff (+ pk order)"""
        if self.walk is not None:
            self.sort_step()
        self._diff(self.walk is not None and self.late)

    def diff_step(self):
        """classify2 + fielddiff (+ pk order) over the key-ordered side buffers"""
        self._diff(False)

    def _diff(self, perm):
        L, ctx = self.eng.L, self.eng.ctx
        keys = self.pk_order and self.flags == 0
        if perm:  # sorted keys; OIDs and filenames read through the sort orders from the walk-order rows
            if self._perm_sides is None:
                self._perm_sides = []
                for S, (w, _, _, _) in zip((self.A, self.B), self.walk):
                    k = S.kd_side()
                    k.oid = w.oid.ptr
                    if w.name is not None:
                        k.name, k.name_off = w.name.ptr, w.name_off.ptr
                    self._perm_sides.append(k)
            N.check(L.kd_diff2_device_ex(ctx, ctypes.byref(self._perm_sides[0]), ctypes.byref(self._perm_sides[1]),
                                         self.walk[0][1].ptr, self.walk[1][1].ptr, self.flags, self.delta.ptr,
                                         self.upd.ptr, self.dkey.ptr if keys else None, self.ukey.ptr if keys else None,
                                         self.counts.ptr, self.counts.ptr + 32), "kd_diff2_device_ex")
        elif self.gather is None:
            N.check(L.kd_diff2_device_ex(ctx, ctypes.byref(self._sa), ctypes.byref(self._sb), None, None, self.flags,
                                         self.delta.ptr, self.upd.ptr, self.dkey.ptr if keys else None,
                                         self.ukey.ptr if keys else None, self.counts.ptr, self.counts.ptr + 32),
                    "kd_diff2_device_ex")
        else:
            # the join, rebase and counts' all-gather; the field diff is queued before anything waits
            # for the counts, and the records' all-gather (communication stream) overlaps it
            N.check(L.kd_diff2_gather_begin(ctx, ctypes.byref(self._sa), ctypes.byref(self._sb), self.gather[0],
                                            self.gather[1], self.flags, self.delta.ptr, self.upd.ptr, self.counts.ptr,
                                            self.counts.ptr + 32, self.all_counts.ptr), "kd_diff2_gather_begin")
        if self._ob_u is not None:  # update-order arenas: update i's blobs at index i, no pairs
            N.check(L.kd_fielddiff(ctx, ctypes.byref(self._ob_u), ctypes.byref(self._nb_u), None, self.cap_upd,
                                   ctypes.cast(self.counts.ptr + 8, N.c_u64p), N.KD_MEM_DEVICE,
                                   ctypes.byref(self._km), self.masks.ptr, self.status.ptr, N.KD_MEM_DEVICE),
                    "kd_fielddiff")
        else:
            N.check(L.kd_fielddiff(ctx, ctypes.byref(self._ob), ctypes.byref(self._nb), self.upd.ptr, self.cap_upd,
                               ctypes.cast(self.counts.ptr + 8, N.c_u64p), N.KD_MEM_DEVICE,
                                   ctypes.byref(self._km), self.masks.ptr, self.status.ptr, N.KD_MEM_DEVICE),
                    "kd_fielddiff")
        if keys:
            lo, hi = self.pk_range
            N.check(L.kd_delta_pk_order(ctx, ctypes.byref(self._sa), ctypes.byref(self._sb), self.delta.ptr,
                                        self.dkey.ptr, self.cap, self.counts.ptr + 24, lo, hi, self.d_pk.ptr,
                                        self.d_perm.ptr), "kd_delta_pk_order")
            N.check(L.kd_delta_pk_order(ctx, ctypes.byref(self._sa), ctypes.byref(self._sb), self.upd.ptr,
                                        self.ukey.ptr, max(self.cap_upd, 1), self.counts.ptr + 8, lo, hi, self.u_pk.ptr,
                                        self.u_perm.ptr), "kd_delta_pk_order")
        if self.gather is not None:
            N.check(L.kd_diff2_gather_end(ctx, self.delta.ptr, self.all_delta.ptr, self.all_cap,
                                          self.h_counts.ctypes.data), "kd_diff2_gather_end")

    def results(self):
        """host copies (synchronous): counts dict, delta [n,2], upd [m,2], masks, status"""
        c = self.counts.download(np.uint64, 8)
        if c[4]:
            raise N.Unsupported(N.KD_EUNSUPPORTED, f"device error flag {int(c[4])}")
        if self.seg_err is not None and int(self.seg_err.download(np.uint32, 1)[0]):
            raise N.Unsupported(N.KD_EUNSUPPORTED, "per-leaf-tree sort flagged a long or descending leaf tree")
        nd, nu = int(c[3]), int(c[1])
        delta = self.delta.download(np.uint32, 2 * nd).reshape(nd, 2)
        upd = self.upd.download(np.uint32, 2 * nu).reshape(nu, 2)
        masks = self.masks.download(np.uint64, nu * self.maps.words).reshape(nu, self.maps.words)
        status = self.status.download(np.uint8, nu)
        return {"inserts": int(c[0]), "updates": nu, "deletes": int(c[2]), "deltas": nd}, delta, upd, masks, status

    def pk_results(self):
        """(pk_order) host copies: (pks of the deltas ascending, delta index of each), and the same for
        the updates (update index: the row of masks / status)"""
        c = self.counts.download(np.uint64, 8)
        nd, nu = int(c[3]), int(c[1])
        return (self.d_pk.download(np.int64, nd), self.d_perm.download(np.uint32, nd),
                self.u_pk.download(np.int64, nu), self.u_perm.download(np.uint32, nu))

    def gathered(self):
        """(gather mode, after a step + sync) the whole diff: global delta records in key order and
        the summed counts of every rank"""
        stride = int(self.h_counts.reshape(self.world, 8)[:, 3].max())
        rec = self.all_delta.download(np.uint32, 2 * stride * self.world)
        return assemble_gathered(self.h_counts, rec, self.world)


def assemble_gathered(h_counts, records, world):
    """The whole diff from kd_diff2_gather's outputs: h_counts [world * 8] (rank r's inserts,
    updates, deletes, deltas, error word, ...) and the all-gathered records [world * stride * 2]
    (rank r's rebased records at 2 * r * stride, stride = the largest rank's delta count, the tail
    of each slot padding).  Ranks hold consecutive bucket ranges, so their records in rank order are
    the key-ordered delta list.  Returns (summed counts, delta [n, 2])."""
    c = np.asarray(h_counts, np.uint64).reshape(world, 8)
    if c[:, 4].any():
        raise N.Unsupported(N.KD_EUNSUPPORTED, f"device error flags {c[:, 4].tolist()}")
    stride = int(c[:, 3].max())
    rec = np.asarray(records, np.uint32)[:2 * stride * world].reshape(world, stride, 2)
    delta = np.concatenate([rec[r, :int(c[r, 3])] for r in range(world)]) if stride else np.zeros((0, 2), np.uint32)
    return {"inserts": int(c[:, 0].sum()), "updates": int(c[:, 1].sum()), "deletes": int(c[:, 2].sum()),
            "deltas": int(c[:, 3].sum())}, delta


class FilterPipeline:
    """The spatially filtered diff over device-resident sides (one GPU): classify2's key-ordered
    delta list feeds kd_geom_filter directly (the delta count stays on the device), which tests
    every delta's old and new geometry against the filter, compacts the deltas that may match and
    encodes the new side's index envelopes — BaseDiffWriter.filtered_ds_feature_deltas's work for a
    whole layer in one stream."""

    def __init__(self, engine, base, target, base_blobs, target_blobs, geom_cols, filt_env, rectangle=False, bits=20,
                 heads=False, delta_order=False, gather=False):
        """heads: filter from 48-B geometry heads (the blob reader's host pass) instead of the blob
        arenas; delta_order (with heads): the heads in delta order, as the drop-in's blob reader lays
        them out after classification (it reads the deltas' blobs) — built once on the host from the
        deltas of a first diff (``delta_heads_s``), then every step is classify2 + the filter over them
        (kd_geom_filter_deltas, KD_GF_DELTA_HEADS; the blob fallback through the step's delta pairs);
        gather (with delta_order): the per-entry heads are instead gathered into delta order on the
        device inside every step (k_gh_gather)"""
        import ctypes as _c

        self.eng = engine
        self.A, self.B = DevSide(engine, base), DevSide(engine, target)
        self.OB, self.NB = DevBlobs(engine, *base_blobs), DevBlobs(engine, *target_blobs)
        cap = base.n + target.n + 1
        self.cap = cap
        self.bits = bits
        self.delta = DevBuf(engine, 8 * cap)
        self.upd = DevBuf(engine, 8 * cap)
        self.counts = DevBuf(engine, 64)
        self.counts.zero()
        self.match = DevBuf(engine, 2 * cap)
        self.keep = DevBuf(engine, 4 * cap)
        self.n_keep = DevBuf(engine, 8)
        self.enc = DevBuf(engine, cap * max(bits // 2, 1)) if bits else None
        self.enc_ok = DevBuf(engine, cap) if bits else None
        self._sa, self._sb = self.A.kd_side(), self.B.kd_side()
        self._ob, self._nb = self.OB.kd_blobs(), self.NB.kd_blobs()
        self.cols = geom_cols
        self._kc = geom_cols.kd_cols()
        self._fe = (_c.c_double * 4)(*[float(x) for x in filt_env])
        self.flags = N.KD_GF_RECT if rectangle else 0
        self.heads = None
        self.heads_s = None
        self.heads_host = None
        self.delta_order = bool(delta_order) and heads
        self.gather = bool(gather) and self.delta_order
        self.dheads = None
        self.delta_heads_s = None
        if heads:  # the blob reader's host pass, then 48 bytes per blob in HBM (kd_geom_filter_heads)
            import time

            from .spatial import geom_heads

            t0 = time.perf_counter()
            hs = [geom_heads(*base_blobs, geom_cols.old_hex, geom_cols.old_gidx, len(geom_cols.old_map)),
                  geom_heads(*target_blobs, geom_cols.new_hex, geom_cols.new_gidx, len(geom_cols.new_map))]
            self.heads_s = time.perf_counter() - t0
            self.heads_host = hs
            self.heads = [(DevBuf.from_numpy(engine, h.view(np.uint8).reshape(-1)) if h.size else DevBuf(engine, 48), h.size)
                          for h in hs]
        engine.reserve(max(base.n, target.n))
        engine.sync()
        if self.delta_order and not self.gather:
            self._build_delta_heads()

    def _classify(self):
        L, ctx = self.eng.L, self.eng.ctx
        N.check(L.kd_diff2_device(ctx, ctypes.byref(self._sa), ctypes.byref(self._sb), 0, self.delta.ptr, self.upd.ptr,
                                  self.counts.ptr, self.counts.ptr + 32), "kd_diff2_device")

    def _build_delta_heads(self):
        """the deltas' heads in delta order (slot d: delta d's old / new head, absent sides zero), as
        the blob reader leaves them when it reads the deltas' blobs after classification: from the
        per-entry heads of the host pass and the deltas of one classify2 (host work, outside a step)"""
        import time

        self._classify()
        c = self.counts.download(np.uint64, 8)
        nd = int(c[3])
        delta = self.delta.download(np.uint32, 2 * nd).reshape(nd, 2)
        t0 = time.perf_counter()
        slots = max((self.cap + 63) // 64 * 64, 64)
        self.dheads = []
        for s in range(2):
            col = delta[:, s]
            pres = np.nonzero(col != N.KD_NONE)[0]
            h = np.zeros(slots, self.heads_host[s].dtype)
            h[pres] = self.heads_host[s][col[pres].astype(np.int64)]
            self.dheads.append((DevBuf.from_numpy(self.eng, h.view(np.uint8).reshape(-1)), slots))
        self.delta_heads_s = time.perf_counter() - t0
        self.eng.sync()

    def step(self):
        L, ctx = self.eng.L, self.eng.ctx
        self._classify()
        if self.delta_order:
            if self.gather:  # per-entry heads gathered into delta order on the device
                (ho, no), (hn, nn) = self.heads
                flags = self.flags
            else:
                (ho, no), (hn, nn) = self.dheads
                flags = self.flags | N.KD_GF_DELTA_HEADS
            N.check(L.kd_geom_filter_deltas(ctx, ho.ptr, no, hn.ptr, nn, ctypes.byref(self._ob), ctypes.byref(self._nb),
                                            self.delta.ptr, self.cap, ctypes.cast(self.counts.ptr + 24, N.c_u64p),
                                            self._fe, flags, self.bits, self.match.ptr, self.keep.ptr,
                                            ctypes.cast(self.n_keep.ptr, N.c_u64p), self.enc.ptr if self.enc else None,
                                            self.enc_ok.ptr if self.enc_ok else None), "kd_geom_filter_deltas")
            return
        if self.heads is not None:
            (ho, no), (hn, nn) = self.heads
            N.check(L.kd_geom_filter_heads(ctx, ho.ptr, no, hn.ptr, nn, N.KD_MEM_DEVICE, ctypes.byref(self._ob),
                                           ctypes.byref(self._nb), self.delta.ptr, self.cap,
                                           ctypes.cast(self.counts.ptr + 24, N.c_u64p), N.KD_MEM_DEVICE, self._fe,
                                           self.flags, self.bits, self.match.ptr, self.keep.ptr,
                                           ctypes.cast(self.n_keep.ptr, N.c_u64p), self.enc.ptr if self.enc else None,
                                           self.enc_ok.ptr if self.enc_ok else None, N.KD_MEM_DEVICE),
                    "kd_geom_filter_heads")
            return
        N.check(L.kd_geom_filter(ctx, ctypes.byref(self._ob), ctypes.byref(self._nb), self.delta.ptr, self.cap,
                                 ctypes.cast(self.counts.ptr + 24, N.c_u64p), N.KD_MEM_DEVICE, ctypes.byref(self._kc),
                                 self._fe, self.flags, self.bits, self.match.ptr, self.keep.ptr,
                                 ctypes.cast(self.n_keep.ptr, N.c_u64p), self.enc.ptr if self.enc else None,
                                 self.enc_ok.ptr if self.enc_ok else None, N.KD_MEM_DEVICE), "kd_geom_filter")

    def results(self):
        """host copies: counts, delta [n, 2], codes [n, 2], keep [k], enc [n, bits/2], enc_ok [n]"""
        c = self.counts.download(np.uint64, 8)
        if c[4]:
            raise N.Unsupported(N.KD_EUNSUPPORTED, f"device error flag {int(c[4])}")
        nd = int(c[3])
        k = int(self.n_keep.download(np.uint64, 1)[0])
        nb = self.bits // 2
        return ({"inserts": int(c[0]), "updates": int(c[1]), "deletes": int(c[2]), "deltas": nd, "kept": k},
                self.delta.download(np.uint32, 2 * nd).reshape(nd, 2), self.match.download(np.uint8, 2 * nd).reshape(nd, 2),
                self.keep.download(np.uint32, k),
                self.enc.download(np.uint8, nd * nb).reshape(nd, nb) if self.enc else None,
                self.enc_ok.download(np.uint8, nd) if self.enc_ok else None)


class MergePipeline:
    """classify3 (three-way merge classification) over device-resident sides (one GPU).

    ``segmented``: KD_KEY_HASH sides in git tree order (what the walk lists: keys ascending in the
    bucket bits, each leaf tree's few entries in filename order).  Every step first orders each bucket
    (kd_sort_segmented_into, one kernel per side) and the merge reads OIDs and filenames through the
    orders from the walk-order rows (kd_merge3_device_perm)."""

    def __init__(self, engine, ancestor, ours, theirs, segmented=False):
        from . import shard

        self.eng = engine
        self.S = [DevSide(engine, x) for x in (ancestor, ours, theirs)]
        self._s = [x.kd_side() for x in self.S]
        self.segmented = bool(segmented)
        if self.segmented:
            from . import packing

            self.seg_bits = shard.bucket_bits(ancestor.key_mode, ancestor.encoding)
            # the longest leaf tree of each side (the host's key scan; a halo plan, not a check)
            self.seg_max = [packing.keys_scan(x.key, x.key_mode).seg_max if self.seg_bits == 24 else 0
                            for x in (ancestor, ours, theirs)]
            self.skey = [DevBuf(engine, 8 * max(x.n, 1)) for x in (ancestor, ours, theirs)]
            self.order = [DevBuf(engine, 4 * max(x.n, 1)) for x in (ancestor, ours, theirs)]
            for k, sb in zip(self._s, self.skey):
                k.key = sb.ptr
        na, no, nt = ancestor.n, ours.n, theirs.n
        self.conf = DevBuf(engine, 12 * (na + no + nt + 1))
        self.md = DevBuf(engine, 8 * (no + nt + 1))
        self.counts = DevBuf(engine, 64)  # [0..3] counts, [4] error word, [5] the segmented sorts' error word
        self.counts.zero()
        engine.sync()

    def sort_step(self):
        """(segmented) each side's buckets ordered by key"""
        L, ctx = self.eng.L, self.eng.ctx
        for S, sk, od, segmax in zip(self.S, self.skey, self.order, self.seg_max):
            N.check(L.kd_sort_segmented_into(ctx, S.key.ptr, sk.ptr, od.ptr, S.n, self.seg_bits, segmax, self.counts.ptr + 40),
                    "kd_sort_segmented_into")

    def step(self):
        L, ctx = self.eng.L, self.eng.ctx
        if self.segmented:
            self.sort_step()
            N.check(L.kd_merge3_device_perm(ctx, ctypes.byref(self._s[0]), ctypes.byref(self._s[1]),
                                            ctypes.byref(self._s[2]), self.order[0].ptr, self.order[1].ptr,
                                            self.order[2].ptr, 0, self.conf.ptr, self.md.ptr, self.counts.ptr,
                                            self.counts.ptr + 32), "kd_merge3_device_perm")
            return
        N.check(L.kd_merge3_device(ctx, ctypes.byref(self._s[0]), ctypes.byref(self._s[1]), ctypes.byref(self._s[2]), 0,
                                   self.conf.ptr, self.md.ptr, self.counts.ptr, self.counts.ptr + 32),
                "kd_merge3_device")

    def results(self):
        """host copies (synchronous): n_clean, conflicts [n,3], merge deltas [m,2] (indices of the
        key-ordered sides)"""
        c = self.counts.download(np.uint64, 8)
        if c[4] or c[5]:
            raise N.Unsupported(N.KD_EUNSUPPORTED, f"device error flags {int(c[4])}, {int(c[5])}")
        nc, nm = int(c[1]), int(c[2])
        conf = self.conf.download(np.uint32, 3 * nc).reshape(nc, 3)
        md = self.md.download(np.uint32, 2 * nm).reshape(nm, 2)
        return int(c[0]), conf, md

    def orders(self):
        """(segmented) walk row of sorted entry k, per side"""
        return [o.download(np.uint32, S.n) for o, S in zip(self.order, self.S)]
