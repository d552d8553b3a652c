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
