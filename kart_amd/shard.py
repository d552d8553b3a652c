"""Bucket-range sharding of the diff across GPUs.

A feature's path is ``<bucket levels>/<filename>`` and equal PKs share a path, so every side's
entries split on the same bucket cut points into independent shards: no key can match across
shards.  The join key's top bits *are* the bucket (packing.py), so a cut on bucket b is a
``searchsorted`` of ``b << (64 - bucket_bits)`` in each side's sorted keys.

The cuts balance ``n_base + n_target`` per shard (the same idea as the reference's parallel
import, kart/fast_import.py:289-337, at bucket granularity).  After the per-shard diffs the only
exchange is an all-gather of each shard's counts and compacted delta records: on GPUs inside the
library over RCCL (xGMI), ``ShardRank`` / ``Engine.diff2_sharded``; on CPU (tests) over gloo.
"""
import numpy as np

from . import _native as N


def bucket_bits(key_mode, encoding=None):
    if key_mode == N.KD_KEY_INT:
        return 24
    if encoding is not None and encoding.encoding == "hex":
        return 4 * 2 * encoding.levels
    return 6 * (encoding.levels if encoding is not None else 4)


def cut_points(key_sides, shards, bits):
    """Bucket cut points [shards+1] splitting the bucket space so each shard holds about the same
    number of entries summed over all sides.  key_sides: list of sorted uint64 key arrays."""
    total = sum(k.shape[0] for k in key_sides)
    nb = 1 << bits
    shift = np.uint64(64 - bits)
    if total == 0:
        return np.linspace(0, nb, shards + 1).astype(np.int64)
    buckets = np.concatenate([(k >> shift).astype(np.int64) for k in key_sides])
    buckets.sort()
    cuts = [0]
    for s in range(1, shards):
        b = int(buckets[min(total - 1, (total * s) // shards)])
        cuts.append(max(cuts[-1], b))
    cuts.append(nb)
    return np.array(cuts, np.int64)


def slice_bounds(keys, cuts, bits):
    """index ranges [shards+1] of one sorted side for the given bucket cuts"""
    shift = 64 - bits
    lo = np.array([min(int(c), (1 << bits)) for c in cuts], dtype=object)
    edge = np.array([(int(c) << shift) if int(c) < (1 << bits) else None for c in lo], dtype=object)
    out = np.zeros(len(cuts), np.int64)
    for i, e in enumerate(edge):
        out[i] = keys.shape[0] if e is None else int(np.searchsorted(keys, np.uint64(e), side="left"))
    return out


def shard_side(side, lo, hi):
    """view of a PackedSide restricted to sorted entries [lo, hi) (indices re-based at 0)"""
    from .packing import PackedSide

    side = side.materialised()
    s = PackedSide(key=side.key[lo:hi], oid=side.oid[lo:hi], key_mode=side.key_mode, order=side.order[lo:hi],
                   encoding=side.encoding)
    if side.name is not None:
        a, b = int(side.name_off[lo]), int(side.name_off[hi])
        s.name = side.name[a:b]
        s.name_off = side.name_off[lo:hi + 1] - np.uint64(a)
    return s


def rank_pk_base(rank, n_per_rank):
    """First pk of a rank's synthetic int-PK shard: disjoint, 64-aligned pk ranges give disjoint
    bucket ranges (bucket = (pk // 64) % 2**24) as long as the whole job stays below 2**30 pks."""
    span = ((int(n_per_rank * 1.05) + 64) // 64) * 64
    base = rank * span
    if base + span >= (1 << 30):
        raise ValueError("synthetic job exceeds one bucket wrap (2**30 pks)")
    return base


def diff2_sharded(base, target, shards, run_shard, rank=0, world=1, exchange=None):
    """Split (base, target) into ``shards`` bucket ranges, run ``run_shard(b, t) -> Diff2Result``
    on the shards this rank owns (shard s -> rank s % world), and gather the results.

    Returns the merged (delta [n,2] in global sorted indices, counts) on every rank.  With
    world > 1, ``exchange(local) -> list`` all-gathers the per-shard ``(shard id, records,
    (inserts, updates, deletes))`` tuples of every rank (the GPU path does this inside the library
    over RCCL: ``ShardRank``; CPU tests pass a gloo all-gather)."""
    bits = bucket_bits(base.key_mode, base.encoding)
    cuts = cut_points([base.key, target.key], shards, bits)
    ba, tb = slice_bounds(base.key, cuts, bits), slice_bounds(target.key, cuts, bits)
    local = []
    for s in range(shards):
        if s % world != rank:
            continue
        r = run_shard(shard_side(base, ba[s], ba[s + 1]), shard_side(target, tb[s], tb[s + 1]))
        d = r.delta.astype(np.int64)
        # re-base shard-local indices to global sorted indices (NONE stays NONE)
        da = np.where(d[:, 0] == N.KD_NONE, N.KD_NONE, d[:, 0] + ba[s])
        db = np.where(d[:, 1] == N.KD_NONE, N.KD_NONE, d[:, 1] + tb[s])
        local.append((s, np.stack([da, db], 1).astype(np.uint32) if d.size else np.zeros((0, 2), np.uint32),
                      (r.n_insert, r.n_update, r.n_delete)))
    if world > 1:
        if exchange is None:
            raise ValueError("world > 1 needs an exchange (all-gather) callable")
        local = exchange(local)
    local.sort(key=lambda x: x[0])
    delta = np.concatenate([x[1] for x in local]) if local else np.zeros((0, 2), np.uint32)
    c = np.sum([x[2] for x in local], axis=0) if local else np.zeros(3, np.int64)
    return delta, {"inserts": int(c[0]), "updates": int(c[1]), "deletes": int(c[2])}


class ShardRank:
    """One rank (one GPU, one process) of a bucket-range sharded two-way diff.

    The rank holds its slice of both sides in HBM (``base`` / ``target`` PackedSides of the rank's
    bucket range, starting at global sorted indices ``base_off`` / ``target_off``); ``step()`` runs
    kd_diff2_gather: the device join of the slice, its delta records rebased to global indices, and
    the all-gather of every rank's counts and records over the library's RCCL communicator
    (``engine.comm_init`` first).  The gathered records, in rank order, are the whole diff in key
    order."""

    def __init__(self, engine, base, target, base_off, target_off, flags=0):
        from .device import DevBuf, DevSide

        self.eng = engine
        self.flags = flags
        self.world = engine.nranks
        self.A, self.B = DevSide(engine, base), DevSide(engine, target)
        self._sa, self._sb = self.A.kd_side(), self.B.kd_side()
        self.base_off, self.target_off = int(base_off), int(target_off)
        cap = base.n + target.n + 1
        self.cap = cap
        self.delta = DevBuf(engine, 8 * cap)
        self.upd = DevBuf(engine, 8 * cap)
        self.counts = DevBuf(engine, 64)
        self.counts.zero()
        self.all_counts = DevBuf(engine, 64 * self.world)
        self.h_counts = np.zeros(8 * self.world, np.uint64)
        self.all_cap = 0
        self.all_delta = None
        engine.reserve(max(base.n, target.n))
        engine.sync()

    def reserve_gather(self, max_deltas_per_rank):
        """size the gathered-record buffer for up to this many deltas on any rank"""
        need = int(max_deltas_per_rank) * self.world
        if need > self.all_cap:
            from .device import DevBuf

            self.all_delta = DevBuf(self.eng, 8 * max(need, 1))
            self.all_cap = need

    def step(self):
        import ctypes

        if self.all_delta is None:
            self.reserve_gather(self.cap)
        N.check(self.eng.L.kd_diff2_gather(
            self.eng.ctx, ctypes.byref(self._sa), ctypes.byref(self._sb), self.base_off, self.target_off, self.flags,
            self.delta.ptr, self.upd.ptr, self.counts.ptr, self.counts.ptr + 32, self.all_delta.ptr, self.all_cap,
            self.all_counts.ptr, self.h_counts.ctypes.data), "kd_diff2_gather")

    def results(self):
        """(delta [n, 2] global sorted indices in key order, counts) of the whole diff (sync)"""
        self.eng.sync()
        c = self.h_counts.reshape(self.world, 8)
        if c[:, 4].any():
            raise N.Unsupported(N.KD_EUNSUPPORTED, f"device error flags {c[:, 4].tolist()}")
        stride = int(c[:, 3].max()) if self.world else 0
        allrec = self.all_delta.download(np.uint32, 2 * stride * self.world).reshape(self.world, stride, 2)
        delta = np.concatenate([allrec[r, :int(c[r, 3])] for r in range(self.world)]) if stride else \
            np.zeros((0, 2), np.uint32)
        return delta, {"inserts": int(c[:, 0].sum()), "updates": int(c[:, 1].sum()), "deletes": int(c[:, 2].sum())}
