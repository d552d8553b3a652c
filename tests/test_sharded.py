"""Bucket-range sharding of the two-way diff (kart_amd/shard.py).

A side's entries split on dataset3 path-bucket cut points into independent shards (equal PKs share a
path, so no key matches across shards).  Sharded results, re-based to global indices and gathered,
must equal the unsharded diff exactly — delta set, order and counts:

* CPU, one process: shards run by the CPU oracle (test-only stand-in for the per-GPU engine);
* CPU, world_size 2 over gloo: each rank diffs its shards and the ranks all-gather the records —
  the same exchange the GPU path does over RCCL;
* GPU (-m gpu): the shards run through the HIP engine.
"""
import os
import socket

import numpy as np
import pytest

from checks import NONE
from kart_amd import shard, synth
from kart_amd.engine import Diff2Result


def _oracle_run(A, B):
    from oracle import oracle as O

    delta, c = O.classify2(A.key, A.oid, B.key, B.oid)
    upd = delta[(delta[:, 0] != NONE) & (delta[:, 1] != NONE)]
    return Diff2Result(c["inserts"], c["updates"], c["deletes"], delta, upd)


def _layer(n, seed):
    return synth.points_layer(n, seed=seed)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_cut_points_partition_buckets():
    L = _layer(200_000, 11)
    bits = shard.bucket_bits(L.base.key_mode, L.base.encoding)
    cuts = shard.cut_points([L.base.key, L.target.key], 5, bits)
    assert cuts[0] == 0 and cuts[-1] == 1 << bits and np.all(np.diff(cuts) >= 0)
    for side in (L.base, L.target):
        b = shard.slice_bounds(side.key, cuts, bits)
        assert b[0] == 0 and b[-1] == side.n and np.all(np.diff(b) >= 0)
        buckets = (side.key >> np.uint64(64 - bits)).astype(np.int64)
        for s in range(5):  # every entry of shard s lies in [cuts[s], cuts[s+1])
            seg = buckets[b[s]:b[s + 1]]
            assert seg.size == 0 or (seg.min() >= cuts[s] and seg.max() < cuts[s + 1])
    # balanced: no shard holds more than twice its share of entries
    tot = L.base.n + L.target.n
    bA, bB = shard.slice_bounds(L.base.key, cuts, bits), shard.slice_bounds(L.target.key, cuts, bits)
    per = np.diff(bA) + np.diff(bB)
    assert per.max() <= 2 * tot / 5


@pytest.mark.parametrize("n,shards", [(0, 3), (1000, 1), (50_000, 4), (300_000, 7)])
def test_sharded_equals_unsharded_cpu(n, shards):
    L = _layer(n, 5 + shards)
    ref = _oracle_run(L.base, L.target)
    delta, counts = shard.diff2_sharded(L.base, L.target, shards, _oracle_run)
    assert np.array_equal(delta, ref.delta)
    assert (counts["inserts"], counts["updates"], counts["deletes"]) == (ref.n_insert, ref.n_update, ref.n_delete)


def _gloo_exchange(local):
    """all-gather of the per-shard (id, records, counts) tuples over gloo (CPU stand-in for the
    library's RCCL all-gather)"""
    import torch.distributed as dist

    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, local)
    return [x for part in out for x in part]


def _gloo_worker(rank, world, port, n, shards, out_dir):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = _layer(n, 23)
        delta, counts = shard.diff2_sharded(L.base, L.target, shards, _oracle_run, rank=rank, world=world,
                                            exchange=_gloo_exchange)
        np.save(os.path.join(out_dir, f"delta_{rank}.npy"), delta)
        np.save(os.path.join(out_dir, f"counts_{rank}.npy"),
                np.array([counts["inserts"], counts["updates"], counts["deletes"]], np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shards", [2, 5])
def test_sharded_gloo_world2(tmp_path, shards):
    import torch.multiprocessing as mp

    n = 120_000
    mp.start_processes(_gloo_worker, args=(2, _free_port(), n, shards, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    L = _layer(n, 23)
    ref = _oracle_run(L.base, L.target)
    for r in range(2):  # every rank holds the whole, globally ordered delta set
        d = np.load(tmp_path / f"delta_{r}.npy")
        c = np.load(tmp_path / f"counts_{r}.npy")
        assert np.array_equal(d, ref.delta)
        assert tuple(c) == (ref.n_insert, ref.n_update, ref.n_delete)


@pytest.mark.gpu
@pytest.mark.parametrize("n,shards", [(400_000, 4), (1_000_000, 8)])
def test_sharded_gpu(engine, n, shards):
    L = _layer(n, 31)
    whole = engine.diff2(L.base, L.target)
    delta, counts = shard.diff2_sharded(L.base, L.target, shards, engine.diff2)
    assert np.array_equal(delta, whole.delta)
    assert (counts["inserts"], counts["updates"], counts["deletes"]) == (whole.n_insert, whole.n_update, whole.n_delete)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 5000, 600_000])
def test_diff2_sharded_library_g1(engine, n):
    """kd_diff2_sharded (the library cuts the sides, owns the RCCL communicator) with one GPU"""
    from kart_amd.engine import Engine

    L = _layer(n, 41)
    ref = _oracle_run(L.base, L.target)
    r = Engine.diff2_sharded([engine], L.base, L.target, shard.bucket_bits(L.base.key_mode, L.base.encoding))
    assert np.array_equal(r.delta, ref.delta) and np.array_equal(r.upd, ref.upd)
    assert (r.n_insert, r.n_update, r.n_delete) == (ref.n_insert, ref.n_update, ref.n_delete)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [3000, 400_000])
def test_shard_rank_gather_world1(engine, n):
    """ShardRank / kd_diff2_gather on a one-rank communicator: rebased records + counts through RCCL"""
    from kart_amd.engine import Engine

    L = _layer(n, 43)
    ref = _oracle_run(L.base, L.target)
    engine.comm_init(1, 0, Engine.comm_unique_id())
    try:
        bits = shard.bucket_bits(L.base.key_mode, L.base.encoding)
        cuts = shard.cut_points([L.base.key, L.target.key], 3, bits)  # one rank owning the middle shard
        ba, tb = shard.slice_bounds(L.base.key, cuts, bits), shard.slice_bounds(L.target.key, cuts, bits)
        rk = shard.ShardRank(engine, shard.shard_side(L.base, ba[1], ba[2]), shard.shard_side(L.target, tb[1], tb[2]),
                             ba[1], tb[1])
        for _ in range(2):
            rk.step()
        delta, counts = rk.results()
        sel = ((ref.delta[:, 0] >= ba[1]) & (ref.delta[:, 0] < ba[2])) | ((ref.delta[:, 1] >= tb[1]) & (ref.delta[:, 1] < tb[2]))
        assert np.array_equal(delta, ref.delta[sel])
        assert counts["inserts"] + counts["updates"] + counts["deletes"] == int(sel.sum())
    finally:
        engine.comm_fini()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [5000, 300_000])
def test_diff_pipeline_gather_world1(engine, n):
    """bench.py's N>1 step on a one-rank communicator: kd_diff2_gather_begin, the shard's field diff
    queued before the counts are waited for, kd_diff2_gather_end (records all-gathered on the
    communication stream) — gathered records, counts, masks and statuses against the oracle"""
    from kart_amd import synth
    from kart_amd.device import DiffPipeline
    from kart_amd.engine import Engine
    from kart_amd.schema import FieldMaps
    from oracle import oracle as O

    L = synth.polygons_layer(n, seed=17)
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    engine.comm_init(1, 0, Engine.comm_unique_id())
    try:
        pipe = DiffPipeline(engine, L.base, L.target, L.base_blobs, L.target_blobs, maps, gather=(0, 0))
        for _ in range(3):  # repeated steps: the next join waits for the previous records' gather
            pipe.step()
        engine.sync()
        g_counts, g_delta = pipe.gathered()
        counts, delta, upd, masks, status = pipe.results()
    finally:
        engine.comm_fini()
    od, oc = O.classify2(L.base.key, L.base.oid, L.target.key, L.target.oid)
    assert np.array_equal(g_delta, od) and np.array_equal(delta, od)
    assert (g_counts["inserts"], g_counts["updates"], g_counts["deletes"]) == (oc["inserts"], oc["updates"], oc["deletes"])
    om, ost = O.fielddiff(*L.base_blobs, *L.target_blobs, upd, maps)
    assert np.array_equal(masks, om) and np.array_equal(status, ost)


# ---------------------------------------------------------------------------------------------
# the library's cut (kd_shard_cuts, what kd_diff2_sharded runs) and the gathered-record layout of
# kd_diff2_gather (device.assemble_gathered, what DiffPipeline.gathered returns), on the CPU
def _lib_cuts(ka, kb, g, bits):
    from kart_amd import _native as N

    cut, alo, blo = (np.zeros(g + 1, np.uint64) for _ in range(3))
    pad = np.zeros(1, np.uint64)
    N.check(N.lib().kd_shard_cuts(N.ptr(ka if ka.size else pad), ka.size, N.ptr(kb if kb.size else pad), kb.size, g, bits,
                                  N.ptr(cut), N.ptr(alo), N.ptr(blo)), "kd_shard_cuts")
    return cut.astype(np.int64), alo.astype(np.int64), blo.astype(np.int64)


@pytest.mark.parametrize("n,g,skew", [(0, 3, False), (1, 4, False), (50_000, 1, False), (200_000, 8, False),
                                      (120_000, 5, True), (7, 8, False)])
def test_library_shard_cuts(n, g, skew):
    """kd_shard_cuts: a partition of the bucket space, each cut the smallest bucket with at least
    total*s/g entries before it (restated with numpy), side ranges = the cut edges' lower bounds"""
    L = _layer(n, 61 + g)
    A, B = L.base.key, L.target.key
    if skew:  # most entries in a few buckets: empty shards, repeated cuts
        A = np.sort(np.concatenate([A[: n // 10], (np.uint64(7) << np.uint64(40)) + np.arange(n, dtype=np.uint64)]))
        B = A.copy()
    bits = 24
    cut, alo, blo = _lib_cuts(A, B, g, bits)
    assert cut[0] == 0 and cut[-1] == 1 << bits and np.all(np.diff(cut) >= 0)
    bA = (A >> np.uint64(64 - bits)).astype(np.int64)
    bB = (B >> np.uint64(64 - bits)).astype(np.int64)
    total = A.size + B.size
    for s in range(1, g):
        want = total * s // g
        before = lambda b: int(np.searchsorted(bA, b)) + int(np.searchsorted(bB, b))
        assert before(cut[s]) >= want or cut[s] == 1 << bits
        assert cut[s] == cut[s - 1] or before(cut[s] - 1) < want  # the smallest such bucket
    assert np.array_equal(alo, [np.searchsorted(bA, c) if c < 1 << bits else A.size for c in cut])
    assert np.array_equal(blo, [np.searchsorted(bB, c) if c < 1 << bits else B.size for c in cut])


def _rank_records(L, ref, world, rank, cuts):
    """rank r's part of kd_diff2_gather: its shard's delta records in global sorted indices and its
    counts row (inserts, updates, deletes, deltas, error word)"""
    cut, alo, blo = cuts
    d = ref.delta
    a, b = d[:, 0], d[:, 1]
    mine = ((a != NONE) & (a >= alo[rank]) & (a < alo[rank + 1])) | ((b != NONE) & (b >= blo[rank]) & (b < blo[rank + 1]))
    rec = d[mine]
    ins = int(((rec[:, 0] == NONE)).sum())
    dele = int(((rec[:, 1] == NONE)).sum())
    return rec, np.array([ins, rec.shape[0] - ins - dele, dele, rec.shape[0], 0, 0, 0, 0], np.uint64)


def _padded(recs, counts, world):
    """the all-gather layout: rank r's records at 2 * r * stride, stride = the largest rank's count,
    the rest of each slot junk"""
    stride = max(int(c[3]) for c in counts)
    out = np.full((world, max(stride, 1), 2), 0xDEADBEEF, np.uint32)
    for r, rec in enumerate(recs):
        out[r, :rec.shape[0]] = rec
    return np.concatenate(counts), out.reshape(-1)


@pytest.mark.parametrize("n,world", [(0, 2), (30_000, 2), (200_000, 3), (100_000, 8)])
def test_assemble_gathered_world_gt1(n, world):
    """assemble_gathered over fabricated per-rank counts and padded records (ranks = the library's
    bucket-range cuts, uneven, some empty): the summed counts and the global key-ordered delta list
    equal the unsharded diff; a rank's error word raises Unsupported"""
    from kart_amd import _native as N
    from kart_amd.device import assemble_gathered

    L = _layer(n, 71 + world)
    ref = _oracle_run(L.base, L.target)
    cuts = _lib_cuts(L.base.key, L.target.key, world, 24)
    parts = [_rank_records(L, ref, world, r, cuts) for r in range(world)]
    h, rec = _padded([p[0] for p in parts], [p[1] for p in parts], world)
    counts, delta = assemble_gathered(h, rec, world)
    assert np.array_equal(delta, ref.delta)
    assert (counts["inserts"], counts["updates"], counts["deletes"], counts["deltas"]) == \
        (ref.n_insert, ref.n_update, ref.n_delete, ref.delta.shape[0])
    h2 = h.copy()
    h2[8 * (world - 1) + 4] = 1
    with pytest.raises(N.Unsupported):
        assemble_gathered(h2, rec, world)


def _gather_worker(rank, world, port, n, out_dir):
    """one rank of the N>1 flow with gloo standing in for RCCL: the library's cut, this rank's shard
    diffed (oracle), counts then padded records all-gathered, reassembled"""
    import torch
    import torch.distributed as dist

    from kart_amd.device import assemble_gathered

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = _layer(n, 83)
        cut, alo, blo = _lib_cuts(L.base.key, L.target.key, world, 24)
        A = shard.shard_side(L.base, alo[rank], alo[rank + 1])
        B = shard.shard_side(L.target, blo[rank], blo[rank + 1])
        r = _oracle_run(A, B)
        rec = r.delta.astype(np.int64)  # rebase to global sorted indices (k_rebase)
        rec[:, 0] = np.where(r.delta[:, 0] == NONE, NONE, rec[:, 0] + alo[rank])
        rec[:, 1] = np.where(r.delta[:, 1] == NONE, NONE, rec[:, 1] + blo[rank])
        rec = rec.astype(np.uint32)
        mine = torch.tensor([r.n_insert, r.n_update, r.n_delete, rec.shape[0], 0, 0, 0, 0], dtype=torch.int64)
        allc = [torch.zeros(8, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allc, mine)
        h = torch.cat(allc).numpy().astype(np.uint64)
        stride = int(h.reshape(world, 8)[:, 3].max())
        send = np.full((max(stride, 1), 2), 0xDEADBEEF, np.uint32)
        send[:rec.shape[0]] = rec
        parts = [torch.zeros(send.size, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(send.reshape(-1).astype(np.int64)))
        records = torch.cat(parts).numpy().astype(np.uint32)
        counts, delta = assemble_gathered(h, records, world)
        np.save(os.path.join(out_dir, f"g_delta_{rank}.npy"), delta)
    finally:
        dist.destroy_process_group()


def test_gather_flow_gloo_world2(tmp_path):
    """the kd_diff2_gather flow at world 2 (gloo for RCCL, the oracle for the shard diff): every rank
    reassembles the whole key-ordered delta list from the library's cuts and the padded layout"""
    import torch.multiprocessing as mp

    n = 150_000
    mp.start_processes(_gather_worker, args=(2, _free_port(), n, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    ref = _oracle_run(_layer(n, 83).base, _layer(n, 83).target)
    for r in range(2):
        assert np.array_equal(np.load(tmp_path / f"g_delta_{r}.npy"), ref.delta)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [3, 20_000, 500_000])
def test_diff2_sharded_library_g1_hash(engine, n):
    """kd_diff2_sharded in KD_KEY_HASH mode (string PKs: the shards share the name arena, their
    filename offsets stay absolute): equal to the oracle and to kd_diff2"""
    from kart_amd.engine import Engine

    M = synth.table3_layers(n, seed=n + 5)
    A, B = M.ours, M.theirs
    bits = shard.bucket_bits(A.key_mode, A.encoding)
    ref = _oracle_run(A, B)
    r = Engine.diff2_sharded([engine], A, B, bits)
    assert np.array_equal(r.delta, ref.delta) and np.array_equal(r.upd, ref.upd)
    assert (r.n_insert, r.n_update, r.n_delete) == (ref.n_insert, ref.n_update, ref.n_delete)
    assert np.array_equal(engine.diff2(A, B).delta, ref.delta)
