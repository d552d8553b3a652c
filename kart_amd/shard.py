"""Bucket-range sharding of the diff across GPUs.

A feature's path is ``<bucket levels>/<filename>`` and equal PKs share a path, so every side's
entries split on the same bucket cut points into independent shards: no key can match across
shards.  The join key's top bits *are* the bucket (packing.py), so a cut on bucket b is a
``searchsorted`` of ``b << (64 - bucket_bits)`` in each side's sorted keys.

The cuts balance ``n_base + n_target`` per shard (the same idea as the reference's parallel
import, kart/fast_import.py:289-337, at bucket granularity).  After the per-shard diffs the only
exchange is an all-gather of each shard's counts and compacted delta records (RCCL over xGMI on
GPUs, gloo on CPU).
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


def diff2_sharded(base, target, shards, run_shard, rank=0, world=1, group=None):
    """Split (base, target) into ``shards`` bucket ranges, run ``run_shard(b, t) -> Diff2Result``
    on the shards this rank owns (shard s -> rank s % world), and all-gather results.

    Returns the merged (delta [n,2] in global sorted indices, counts) on every rank.  With
    world > 1 ``torch.distributed`` must be initialised (nccl on GPUs, gloo on CPU)."""
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
        local = _all_gather(local, group)
    local.sort(key=lambda x: x[0])
    delta = np.concatenate([x[1] for x in local]) if local else np.zeros((0, 2), np.uint32)
    c = np.sum([x[2] for x in local], axis=0) if local else np.zeros(3, np.int64)
    return delta, {"inserts": int(c[0]), "updates": int(c[1]), "deletes": int(c[2])}


def _all_gather(local, group):
    """all-gather of per-shard (id, delta records, counts): counts first, then records padded to
    the max count (RCCL has no all-gatherv)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    flat = [(s, d, c) for s, d, c in local]
    hdr = torch.tensor([len(flat)] + [int(d.shape[0]) for _, d, _ in flat] + [0] * 0, dtype=torch.int64)
    n_local = torch.tensor([len(flat), sum(int(d.shape[0]) for _, d, _ in flat)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n_local, group=group)
    max_sh = max(int(x[0]) for x in sizes)
    max_rec = max(int(x[1]) for x in sizes)
    # per-shard headers: id, n_records, inserts, updates, deletes
    h = torch.zeros((max(max_sh, 1), 5), dtype=torch.int64, device=dev)
    recs = torch.zeros((max(max_rec, 1), 2), dtype=torch.int64, device=dev)
    pos = 0
    for i, (s, d, c) in enumerate(flat):
        h[i] = torch.tensor([s, d.shape[0], c[0], c[1], c[2]], dtype=torch.int64)
        if d.shape[0]:
            recs[pos:pos + d.shape[0]] = torch.from_numpy(d.astype(np.int64)).to(dev)
        pos += d.shape[0]
    hs = [torch.empty_like(h) for _ in range(world)]
    rs = [torch.empty_like(recs) for _ in range(world)]
    dist.all_gather(hs, h, group=group)
    dist.all_gather(rs, recs, group=group)
    out = []
    for r in range(world):
        nsh = int(sizes[r][0])
        hr = hs[r].cpu().numpy()
        rr = rs[r].cpu().numpy()
        p = 0
        for i in range(nsh):
            s, nrec, ci, cu, cd = (int(x) for x in hr[i])
            out.append((s, rr[p:p + nrec].astype(np.uint32), (ci, cu, cd)))
            p += nrec
    del hdr
    return out
