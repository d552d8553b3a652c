"""Engine: one libkartdiff context per GPU, with numpy-in / numpy-out calls.

Every method goes through the HIP library; there is no CPU implementation here.  Device-resident
pipelines (bench.py) keep their buffers in HBM through the library's own allocator
(``kart_amd.device``).
"""
import ctypes
import os
import sys
import time
from dataclasses import dataclass

import numpy as np

from . import _native as N

_TRACE = os.environ.get("KD_TRACE_HOST") == "1"  # (diagnosis: host phase times to stderr)

# placeholder a native call gets for an empty host array: a module-level array, alive for every call
_PAD = np.zeros(16, np.uint8)


@dataclass
class Diff2Result:
    n_insert: int
    n_update: int
    n_delete: int
    delta: np.ndarray  # uint32 [n_delta, 2] (base sorted index | NONE, target sorted index | NONE)
    upd: np.ndarray  # uint32 [n_update, 2]

    def type_counts(self):
        out = {}
        for name, v in (("inserts", self.n_insert), ("updates", self.n_update), ("deletes", self.n_delete)):
            if v:
                out[name] = v
        return out


@dataclass
class Merge3Result:
    n_clean: int
    conflict: np.ndarray  # uint32 [n, 3] (ancestor, ours, theirs) sorted indices | NONE
    mdelta: np.ndarray  # uint32 [n, 2] (ours | NONE, theirs | NONE): take theirs


class Engine:
    def __init__(self, device=0):
        self.L = N.lib()
        self.ctx = ctypes.c_void_p()
        N.check(self.L.kd_init(int(device), ctypes.byref(self.ctx)), "kd_init")
        self.device = device

    def set_option(self, name, value):
        """a tuning option of the context (kd_set_option: the A/B switches of kartdiff.h)"""
        N.check(self.L.kd_set_option(self.ctx, name.encode(), int(value)), "kd_set_option")

    def get_option(self, name):
        v = ctypes.c_int64()
        N.check(self.L.kd_get_option(self.ctx, name.encode(), ctypes.byref(v)), "kd_get_option")
        return int(v.value)

    def close(self):
        if self.ctx:
            self.L.kd_fini(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---------------------------------------------------------------------------------------
    def set_stream(self, stream_handle):
        N.check(self.L.kd_set_stream(self.ctx, stream_handle), "kd_set_stream")

    def sync(self):
        N.check(self.L.kd_sync(self.ctx), "kd_sync")

    def device_sync(self):
        """hipDeviceSynchronize (every stream of the device) + profiling flush"""
        N.check(self.L.kd_device_sync(self.ctx), "kd_device_sync")

    # ---- multi-GPU (RCCL owned by the library) ---------------------------------------------
    @staticmethod
    def comm_unique_id():
        buf = (ctypes.c_uint8 * N.KD_COMM_ID_BYTES)()
        N.check(N.lib().kd_comm_unique_id(buf), "kd_comm_unique_id")
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        buf = (ctypes.c_uint8 * N.KD_COMM_ID_BYTES).from_buffer_copy(uid)
        N.check(self.L.kd_comm_init(self.ctx, int(nranks), int(rank), buf), "kd_comm_init")
        self.nranks, self.rank = int(nranks), int(rank)

    def comm_info(self):
        """{"count": ncclCommCount, "rank": ncclCommUserRank, "device": ncclCommCuDevice} of the
        library's communicator"""
        out = (ctypes.c_int32 * 3)()
        N.check(self.L.kd_comm_info(self.ctx, out), "kd_comm_info")
        return {"count": int(out[0]), "rank": int(out[1]), "device": int(out[2])}

    def comm_fini(self):
        N.check(self.L.kd_comm_fini(self.ctx), "kd_comm_fini")

    def reserve(self, max_entries, max_updates=0):
        N.check(self.L.kd_reserve(self.ctx, int(max_entries), int(max_updates)), "kd_reserve")

    def prof_enable(self, on=True):
        N.check(self.L.kd_prof_enable(self.ctx, 1 if on else 0), "kd_prof_enable")

    def prof_select(self, names=None):
        """time only these kernels (iterable of names; None = all)"""
        arg = ",".join(names).encode() if names else None
        N.check(self.L.kd_prof_select(self.ctx, arg), "kd_prof_select")

    def prof_reset(self):
        N.check(self.L.kd_prof_reset(self.ctx), "kd_prof_reset")

    def prof_get(self, name):
        launches = ctypes.c_uint64()
        ms = ctypes.c_double()
        N.check(self.L.kd_prof_get(self.ctx, name.encode(), ctypes.byref(launches), ctypes.byref(ms)), "kd_prof_get")
        return int(launches.value), float(ms.value)

    # ---------------------------------------------------------------------------------------
    def diff2(self, base, target, flags=0) -> Diff2Result:
        """base/target: PackedSide (host) -> key-ordered delta set (kd_diff2).  A side packed on the
        GPU with its rows in walk order (PackedSide.dperm) joins through its order on the device
        (kd_diff2_device_perm: no OID or filename gather)."""
        if base.walk_rows or target.walk_rows:
            return self._diff2_perm(base, target, flags)
        t0 = time.perf_counter() if _TRACE else 0
        sa, sb = base.kd_side(), target.kd_side()
        res = ctypes.POINTER(N.KdDiffResult)()
        if _TRACE:
            print(f"[kd] engine.diff2 kd_side    {1e3 * (time.perf_counter() - t0):9.3f} ms", file=sys.stderr)
        N.check(self.L.kd_diff2(self.ctx, ctypes.byref(sa), ctypes.byref(sb), flags, ctypes.byref(res)), "kd_diff2")
        if _TRACE:
            print(f"[kd] engine.diff2 call       {1e3 * (time.perf_counter() - t0):9.3f} ms", file=sys.stderr)
        try:
            r = res.contents
            nd, nu = int(r.n_delta), int(r.n_update)
            delta = np.ctypeslib.as_array(r.delta, (nd * 2,)).reshape(nd, 2).copy() if nd else np.zeros((0, 2), np.uint32)
            upd = np.ctypeslib.as_array(r.upd, (nu * 2,)).reshape(nu, 2).copy() if nu else np.zeros((0, 2), np.uint32)
            return Diff2Result(int(r.n_insert), nu, int(r.n_delete), delta, upd)
        finally:
            self.L.kd_free(res)

    def _diff2_perm(self, base, target, flags):
        from .device import DevBuf, perm_dev

        (sa, oa, ka), (sb, ob, kb) = perm_dev(self, base), perm_dev(self, target)
        n = base.n + target.n
        d_delta, d_upd, d_c = DevBuf(self, 8 * (n + 1)), DevBuf(self, 8 * (n + 1)), DevBuf(self, 64)
        N.check(self.L.kd_diff2_device_perm(self.ctx, ctypes.byref(sa), ctypes.byref(sb), oa.ptr, ob.ptr, flags,
                                            d_delta.ptr, d_upd.ptr, d_c.ptr, d_c.ptr + 32), "kd_diff2_device_perm")
        c = d_c.download(np.uint64, 5)
        err = int(c[4]) & 0xFFFFFFFF
        if err:
            raise N.Unsupported("kd_diff2: " + ("side keys not strictly ascending" if err & 1 else
                                               "hash key collision between different filenames"))
        nd, nu = int(c[3]), int(c[1])
        delta = d_delta.download(np.uint32, 2 * nd).reshape(nd, 2)
        upd = d_upd.download(np.uint32, 2 * nu).reshape(nu, 2)
        del ka, kb
        return Diff2Result(int(c[0]), nu, int(c[2]), delta, upd)

    def _merge3_perm(self, ancestor, ours, theirs, flags):
        from .device import DevBuf, perm_dev

        ds = [perm_dev(self, s) for s in (ancestor, ours, theirs)]
        n = ancestor.n + ours.n + theirs.n
        d_conf, d_md, d_c = DevBuf(self, 12 * (n + 1)), DevBuf(self, 8 * (ours.n + theirs.n + 1)), DevBuf(self, 64)
        N.check(self.L.kd_merge3_device_perm(self.ctx, *(ctypes.byref(d[0]) for d in ds), *(d[1].ptr for d in ds),
                                             flags, d_conf.ptr, d_md.ptr, d_c.ptr, d_c.ptr + 32),
                "kd_merge3_device_perm")
        c = d_c.download(np.uint64, 5)
        err = int(c[4]) & 0xFFFFFFFF
        if err:
            raise N.Unsupported("kd_merge3: err=0x%x (%s)" % (err, "keys not strictly ascending" if err & 1 else
                                                               "hash key collision" if err & 2 else "tile overflow"))
        nc, nm = int(c[1]), int(c[2])
        conf = d_conf.download(np.uint32, 3 * nc).reshape(nc, 3)
        md = d_md.download(np.uint32, 2 * nm).reshape(nm, 2)
        return Merge3Result(int(c[0]), conf, md)

    @staticmethod
    def diff2_sharded(engines, base, target, bucket_bits, flags=0) -> Diff2Result:
        """One process, len(engines) GPUs: kd_diff2_sharded cuts base/target (host PackedSides) into
        bucket ranges, diffs each on its GPU and all-gathers the records over RCCL."""
        ctxs = (ctypes.c_void_p * len(engines))(*[e.ctx.value for e in engines])
        sa, sb = base.kd_side(), target.kd_side()
        L = engines[0].L
        res = ctypes.POINTER(N.KdDiffResult)()
        N.check(L.kd_diff2_sharded(ctxs, len(engines), ctypes.byref(sa), ctypes.byref(sb), int(bucket_bits), flags,
                                   ctypes.byref(res)), "kd_diff2_sharded")
        try:
            r = res.contents
            nd, nu = int(r.n_delta), int(r.n_update)
            delta = np.ctypeslib.as_array(r.delta, (nd * 2,)).reshape(nd, 2).copy() if nd else np.zeros((0, 2), np.uint32)
            upd = np.ctypeslib.as_array(r.upd, (nu * 2,)).reshape(nu, 2).copy() if nu else np.zeros((0, 2), np.uint32)
            return Diff2Result(int(r.n_insert), nu, int(r.n_delete), delta, upd)
        finally:
            L.kd_free(res)

    def delta_pk_order(self, base, target, records):
        """records uint32 [n, 2] (classify2's (base | NONE, target | NONE) deltas or updates) of two
        KD_KEY_INT PackedSides -> (pks ascending int64 [n], record index of each uint32 [n]): the
        order DeltaDiff.sorted_items yields (kd_delta_pk_order; the sides' keys are uploaded)"""
        from . import packing
        from .device import DevBuf, DevSide

        records = np.ascontiguousarray(records, np.uint32).reshape(-1, 2)
        n = records.shape[0]
        if n == 0:
            return np.zeros(0, np.int64), np.zeros(0, np.uint32)
        lo, hi = [], []
        for side in (base, target):
            if side.n:
                info = side.info if side.info is not None else packing.keys_scan(side.key, side.key_mode)
                lo.append(int(info.pk_min))
                hi.append(int(info.pk_max))
        A, B = DevSide(self, base, keys_only=True), DevSide(self, target, keys_only=True)  # (the pass reads keys only)
        sa, sb = A.kd_side(), B.kd_side()
        d_rec = DevBuf.from_numpy(self, records.reshape(-1))
        d_n = DevBuf.from_numpy(self, np.array([n], np.uint64))
        d_pk, d_perm = DevBuf(self, 8 * n), DevBuf(self, 4 * n)
        N.check(self.L.kd_delta_pk_order(self.ctx, ctypes.byref(sa), ctypes.byref(sb), d_rec.ptr, None, n, d_n.ptr,
                                         min(lo), max(hi), d_pk.ptr, d_perm.ptr), "kd_delta_pk_order")
        return d_pk.download(np.int64, n), d_perm.download(np.uint32, n)

    def fielddiff(self, old_data, old_off, new_data, new_off, pairs, maps):
        """Blob arenas (uint8 data, uint64 off[n+1]) per side; pairs uint32 [n, 2] (old blob,
        new blob) or None (blob u on both sides); maps: schema.FieldMaps.
        Returns (masks uint64 [n, words], status uint8 [n])."""
        old_data = np.ascontiguousarray(old_data, np.uint8)
        new_data = np.ascontiguousarray(new_data, np.uint8)
        old_off = np.ascontiguousarray(old_off, np.uint64)
        new_off = np.ascontiguousarray(new_off, np.uint64)
        n = int(pairs.shape[0]) if pairs is not None else int(old_off.shape[0]) - 1
        if pairs is not None:
            pairs = np.ascontiguousarray(pairs, np.uint32)
        ob, nb = N.KdBlobs(), N.KdBlobs()
        for b, d, o in ((ob, old_data, old_off), (nb, new_data, new_off)):
            b.n = int(o.shape[0]) - 1
            b.data = N.ptr(d) if d.size else N.ptr(_PAD)
            b.off = N.ptr(o)
            b.mem = N.KD_MEM_HOST
        masks = np.zeros((max(n, 1), maps.words), np.uint64)
        status = np.zeros(max(n, 1), np.uint8)
        km = maps.kd_maps()
        N.check(
            self.L.kd_fielddiff(self.ctx, ctypes.byref(ob), ctypes.byref(nb), N.ptr(pairs), n, None, N.KD_MEM_HOST,
                                ctypes.byref(km), N.ptr(masks), N.ptr(status), N.KD_MEM_HOST),
            "kd_fielddiff",
        )
        return masks[:n], status[:n]

    def merge3(self, ancestor, ours, theirs, flags=0) -> Merge3Result:
        """three PackedSides -> conflicts / merge deltas in path order (kd_merge3; sides packed on the
        GPU with walk-order rows through kd_merge3_device_perm)"""
        if ancestor.walk_rows or ours.walk_rows or theirs.walk_rows:
            return self._merge3_perm(ancestor, ours, theirs, flags)
        sa, so, st = ancestor.kd_side(), ours.kd_side(), theirs.kd_side()
        res = ctypes.POINTER(N.KdMergeResult)()
        N.check(self.L.kd_merge3(self.ctx, ctypes.byref(sa), ctypes.byref(so), ctypes.byref(st), flags,
                                 ctypes.byref(res)), "kd_merge3")
        try:
            r = res.contents
            nc, nm = int(r.n_conflict), int(r.n_mdelta)
            conf = np.ctypeslib.as_array(r.conflict, (nc * 3,)).reshape(nc, 3).copy() if nc else np.zeros((0, 3), np.uint32)
            md = np.ctypeslib.as_array(r.mdelta, (nm * 2,)).reshape(nm, 2).copy() if nm else np.zeros((0, 2), np.uint32)
            return Merge3Result(int(r.n_clean), conf, md)
        finally:
            self.L.kd_free(res)

    def envelopes(self, data, off, filt_env, bits=20):
        """GPKG geometry blobs -> (match u8[n], enc u8[n, bits/2], enc_ok u8[n], n_candidates)."""
        data = np.ascontiguousarray(data, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        n = int(off.shape[0]) - 1
        g = N.KdBlobs()
        g.n = n
        g.data = N.ptr(data) if data.size else N.ptr(_PAD)
        g.off = N.ptr(off)
        g.mem = N.KD_MEM_HOST
        nb = bits // 2
        match = np.zeros(max(n, 1), np.uint8)
        enc = np.zeros((max(n, 1), nb), np.uint8)
        ok = np.zeros(max(n, 1), np.uint8)
        fe = (ctypes.c_double * 4)(*[float(x) for x in filt_env])
        ncand = ctypes.c_uint64()
        N.check(self.L.kd_envelopes(self.ctx, ctypes.byref(g), fe, int(bits), N.ptr(match), N.ptr(enc), N.ptr(ok),
                                    N.KD_MEM_HOST, ctypes.byref(ncand)), "kd_envelopes")
        return match[:n], enc[:n], ok[:n], int(ncand.value)

    def hex_encode(self, data, off, mode):
        """Blob arena -> (hex u8[2*off[n]], start u32[n], status u8[n]) via kd_hex_encode (host buffers).
        Blob i's string is hex[2*(off[i] + start[i]) : 2*off[i+1]]."""
        data = np.ascontiguousarray(data, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        n = int(off.shape[0]) - 1
        g = N.KdBlobs()
        g.n = n
        g.data = N.ptr(data) if data.size else N.ptr(_PAD)
        g.off = N.ptr(off)
        g.mem = N.KD_MEM_HOST
        nbytes = int(off[-1]) if n >= 0 and off.size else 0
        hexbuf = np.zeros(max(2 * nbytes, 1), np.uint8)
        start = np.zeros(max(n, 1), np.uint32)
        status = np.zeros(max(n, 1), np.uint8)
        N.check(self.L.kd_hex_encode(self.ctx, ctypes.byref(g), int(mode), N.ptr(hexbuf), N.ptr(start), N.ptr(status),
                                     N.KD_MEM_HOST), "kd_hex_encode")
        return hexbuf[: 2 * nbytes], start[:n], status[:n]

    def env_overlap(self, enc, bits, q):
        enc = np.ascontiguousarray(enc, np.uint8)
        n = enc.shape[0]
        out = np.zeros(max(n, 1), np.uint8)
        qq = (ctypes.c_double * 4)(*[float(x) for x in q])
        N.check(self.L.kd_env_overlap(self.ctx, N.ptr(enc) if enc.size else N.ptr(_PAD), n, int(bits),
                                      qq, N.ptr(out), N.KD_MEM_HOST), "kd_env_overlap")
        return out[:n]
