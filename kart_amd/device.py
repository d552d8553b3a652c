"""Device-resident pipeline: sides and blob arenas held in HBM (torch allocations as plumbing),
classify2 -> fielddiff launched back to back on one stream with no host round trip.

This is the path bench.py times: inputs already resident, outputs stay resident (the delta list,
update list, per-update changed-field masks).  torch only allocates memory and provides the
stream; every kernel is libkartdiff's.
"""
import ctypes

import numpy as np
import torch

from . import _native as N


def to_dev(a, device):
    """numpy -> torch device tensor with the same bytes (uint64 stored as int64)"""
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    t = torch.from_numpy(a)
    return t.to(device, non_blocking=False)


class DevSide:
    def __init__(self, side, device):
        self.n = side.n
        self.key_mode = side.key_mode
        self.key = to_dev(side.key if side.n else np.zeros(1, np.uint64), device)
        self.oid = to_dev(side.oid.reshape(-1) if side.n else np.zeros(20, np.uint8), device)
        self.name = self.name_off = None
        if side.name is not None:
            self.name = to_dev(side.name if side.name.size else np.zeros(1, np.uint8), device)
            self.name_off = to_dev(side.name_off, device)

    def kd_side(self):
        s = N.KdSide()
        s.n = self.n
        s.key = self.key.data_ptr()
        s.oid = self.oid.data_ptr()
        s.name = self.name.data_ptr() if self.name is not None else None
        s.name_off = self.name_off.data_ptr() if self.name_off is not None else None
        s.mem = N.KD_MEM_DEVICE
        s.key_mode = self.key_mode
        return s


class DevBlobs:
    def __init__(self, data, off, device):
        self.n = int(off.shape[0]) - 1
        self.data = to_dev(data if data.size else np.zeros(1, np.uint8), device)
        self.off = to_dev(off, device)
        self.nbytes = int(data.size)
        self.max_len = int((off[1:] - off[:-1]).max()) if self.n else 0
        # typical blob = mean over the non-empty blobs (an arena may hold only the blobs a diff reads)
        nz = int(np.count_nonzero(off[1:] != off[:-1])) if self.n else 0
        self.mean_len = int((int(off[-1]) - int(off[0]) + nz - 1) // nz) if nz else 0

    def kd_blobs(self):
        b = N.KdBlobs()
        b.n = self.n
        b.data = self.data.data_ptr()
        b.off = self.off.data_ptr()
        b.mem = N.KD_MEM_DEVICE
        b.size_hint = min(self.mean_len, 0xFFFFFFFF)  # typical (mean) blob size: sizes the LDS pool
        return b


class DiffPipeline:
    """classify2 + fused-by-stream fielddiff over device-resident sides (one GPU)."""

    def __init__(self, engine, base, target, base_blobs, target_blobs, maps, device, ordered=True):
        self.eng = engine
        self.flags = 0 if ordered else N.KD_DIFF_UNORDERED
        self.device = device
        self.A = DevSide(base, device)
        self.B = DevSide(target, device)
        self.OB = DevBlobs(*base_blobs, device)
        self.NB = DevBlobs(*target_blobs, device)
        self.maps = maps
        cap = base.n + target.n + 1
        self.cap_upd = min(base.n, target.n)  # updates <= matched keys
        self.delta = torch.empty(2 * cap, dtype=torch.int32, device=device)
        self.upd = torch.empty(2 * cap, dtype=torch.int32, device=device)
        self.counts = torch.zeros(8, dtype=torch.int64, device=device)  # [0..3] counts, [4] err
        self.masks = torch.empty(cap * maps.words, dtype=torch.int64, device=device)
        self.status = torch.empty(cap, dtype=torch.uint8, device=device)
        self._sa, self._sb = self.A.kd_side(), self.B.kd_side()
        self._ob, self._nb = self.OB.kd_blobs(), self.NB.kd_blobs()
        self._km = maps.kd_maps()
        engine.reserve(max(base.n, target.n))

    def step(self):
        L, ctx = self.eng.L, self.eng.ctx
        err_ptr = self.counts.data_ptr() + 4 * 8
        N.check(L.kd_diff2_device(ctx, ctypes.byref(self._sa), ctypes.byref(self._sb), self.flags, self.delta.data_ptr(),
                                  self.upd.data_ptr(), self.counts.data_ptr(), err_ptr), "kd_diff2_device")
        N.check(L.kd_fielddiff(ctx, ctypes.byref(self._ob), ctypes.byref(self._nb), self.upd.data_ptr(), self.cap_upd,
                               ctypes.cast(self.counts.data_ptr() + 8, N.c_u64p), N.KD_MEM_DEVICE,
                               ctypes.byref(self._km), self.masks.data_ptr(), self.status.data_ptr(),
                               N.KD_MEM_DEVICE), "kd_fielddiff")

    def results(self):
        """host copies (after a sync): counts dict, delta [n,2], upd [m,2], masks, status"""
        c = self.counts.cpu().numpy()
        if c[4]:
            raise N.Unsupported(N.KD_EUNSUPPORTED, f"device error flag {int(c[4])}")
        nd, nu = int(c[3]), int(c[1])
        delta = self.delta[: 2 * nd].cpu().numpy().view(np.uint32).reshape(nd, 2)
        upd = self.upd[: 2 * nu].cpu().numpy().view(np.uint32).reshape(nu, 2)
        masks = self.masks[: nu * self.maps.words].cpu().numpy().view(np.uint64).reshape(nu, self.maps.words)
        status = self.status[:nu].cpu().numpy()
        return {"inserts": int(c[0]), "updates": nu, "deletes": int(c[2]), "deltas": nd}, delta, upd, masks, status


class MergePipeline:
    """classify3 (three-way merge classification) over device-resident sides (one GPU)."""

    def __init__(self, engine, ancestor, ours, theirs, device):
        self.eng = engine
        self.S = [DevSide(x, device) for x in (ancestor, ours, theirs)]
        self._s = [x.kd_side() for x in self.S]
        na, no, nt = ancestor.n, ours.n, theirs.n
        self.conf = torch.empty(3 * (na + no + nt + 1), dtype=torch.int32, device=device)
        self.md = torch.empty(2 * (no + nt + 1), dtype=torch.int32, device=device)
        self.counts = torch.zeros(8, dtype=torch.int64, device=device)  # [0..3] counts, [4] err

    def step(self):
        L, ctx = self.eng.L, self.eng.ctx
        N.check(L.kd_merge3_device(ctx, ctypes.byref(self._s[0]), ctypes.byref(self._s[1]), ctypes.byref(self._s[2]), 0,
                                   self.conf.data_ptr(), self.md.data_ptr(), self.counts.data_ptr(),
                                   self.counts.data_ptr() + 4 * 8), "kd_merge3_device")

    def results(self):
        """host copies (after a sync): n_clean, conflicts [n,3], merge deltas [m,2]"""
        c = self.counts.cpu().numpy()
        if c[4]:
            raise N.Unsupported(N.KD_EUNSUPPORTED, f"device error flag {int(c[4])}")
        nc, nm = int(c[1]), int(c[2])
        conf = self.conf[: 3 * nc].cpu().numpy().view(np.uint32).reshape(nc, 3)
        md = self.md[: 2 * nm].cpu().numpy().view(np.uint32).reshape(nm, 2)
        return int(c[0]), conf, md
