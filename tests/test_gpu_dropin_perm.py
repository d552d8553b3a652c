"""The drop-in's GPU pack of sides whose walk order is not key order (packing.pack_side with an
engine): late materialisation as bench.py's fallback_sort times it — keys sorted on the device
(KD_KEY_HASH: kd_sort_segmented_into, falling back to kd_sort_side_into for a bucket of more than
512 entries; KD_KEY_INT: kd_sort_side_into), OIDs and filenames left in walk order, and
engine.diff2 / engine.merge3 joining through the order (kd_diff2_device_perm /
kd_merge3_device_perm).  Results must equal the oracle on the key-sorted sides bit for bit."""
import numpy as np
import pytest

from checks import NONE
from kart_amd import packing, synth
from kart_amd import _native as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _walk_int_side(pks, oids):
    """relative paths of int pks in git tree order (path bytes), with their OIDs"""
    arena, off = synth.int_pk_paths(pks)
    paths = [arena[int(off[i]):int(off[i + 1])].tobytes() for i in range(pks.size)]
    order = sorted(range(pks.size), key=lambda i: paths[i])
    return [paths[i].decode() for i in order], np.ascontiguousarray(oids[order])


def _sorted_ref(side):
    """the key-sorted form (host) the oracle classifies"""
    return side.materialised()


def test_gpu_pack_int_mixed_wraps_late_materialised(engine):
    """leaf trees mixing pks of two 2^30 wraps: the walk is not key order, the side is sorted on the
    device (keys only), and the diff through the orders equals the oracle's"""
    rng = np.random.default_rng(5)
    n = 200_000
    pks = np.concatenate([np.arange(n), np.arange(n) + (1 << 30)]).astype(np.int64)
    base_oid = synth.synth_oids(pks, np.zeros(pks.size, np.uint64))
    edit = rng.random(pks.size)
    keep = edit >= 0.01
    tgt_pk = np.concatenate([pks[keep], np.arange(5000) + (3 << 30)])
    ver = np.where(edit[keep] < 0.05, 1, 0).astype(np.uint64)
    tgt_oid = np.concatenate([synth.synth_oids(pks[keep], ver), synth.synth_oids(np.arange(5000) + (3 << 30),
                                                                                  np.zeros(5000, np.uint64))])
    sides = []
    for p, o in ((pks, base_oid), (tgt_pk, tgt_oid)):
        paths, oids = _walk_int_side(p, o)
        s = packing.pack_side(paths, oids, packing.INT_PK_ENCODING, engine=engine)
        assert s.walk_rows and s.timing["sort_on"] == "gpu" and not s.info.ascending
        assert np.all(s.key[1:] > s.key[:-1])
        sides.append(s)
    A, B = sides
    r = engine.diff2(A, B)
    Am, Bm = _sorted_ref(A), _sorted_ref(B)
    od, oc = O.classify2(Am.key, Am.oid, Bm.key, Bm.oid)
    assert np.array_equal(r.delta, od)
    assert (r.n_insert, r.n_update, r.n_delete) == (oc["inserts"], oc["updates"], oc["deletes"])
    assert r.n_insert == 5000 and r.n_delete == int((~keep).sum())
    # pk order of the deltas (DeltaDiff.sorted_items) from the device-sorted keys
    pk, perm = engine.delta_pk_order(A, B, r.delta)
    assert np.all(np.diff(pk) > 0)


@pytest.mark.parametrize("n", [20_000, 300_000])  # (enough rows that some leaf trees hold several)
def test_gpu_pack_hash_walk_late_materialised(engine, n):
    """C4's string-PK sides as the tree walk lists them: the per-bucket sort on the device, filenames
    and OIDs in walk order; merge3 and diff2 through the orders equal the oracle on the sorted layers"""
    W = synth.table3_layers(n, seed=9, walk=True)
    S = synth.table3_layers(n, seed=9, walk=False)
    sides = []
    for w, ref in zip((W.ancestor, W.ours, W.theirs), (S.ancestor, S.ours, S.theirs)):
        s = packing.pack_side(w.name, w.oid, packing.GENERAL_ENCODING, rel_off=w.name_off, engine=engine)
        assert s.walk_rows and np.array_equal(s.key, ref.key)
        m = s.materialised()
        assert np.array_equal(m.oid, ref.oid) and np.array_equal(m.name, ref.name)
        assert s.rel_path(7) == ref.rel_path(7)
        sides.append(s)
    r = engine.merge3(*sides)
    oc, om, ocl = O.classify3(S.ancestor.key, S.ancestor.oid, S.ours.key, S.ours.oid, S.theirs.key, S.theirs.oid)
    assert np.array_equal(r.conflict.reshape(-1, 3), np.asarray(oc).reshape(-1, 3))
    assert np.array_equal(r.mdelta.reshape(-1, 2), np.asarray(om).reshape(-1, 2))
    assert r.n_clean == ocl and r.conflict.shape[0] == W.n_conflict
    d = engine.diff2(sides[1], sides[2])
    od, _ = O.classify2(S.ours.key, S.ours.oid, S.theirs.key, S.theirs.oid)
    assert np.array_equal(d.delta, od)
    # a perm side against a sorted-form one (identity order on the device)
    d2 = engine.diff2(sides[1], S.theirs)
    assert np.array_equal(d2.delta, od)


def test_gpu_pack_hash_long_bucket_falls_back(engine):
    """a leaf tree of 2000 entries (longer than the per-bucket sort takes): the full key sort"""
    rng = np.random.default_rng(2)
    names = sorted({rng.integers(0, 2**62).item() for _ in range(2100)})[:2000]
    files = [f"A/A/A/A/f{v:x}" for v in names] + [f"A/A/A/B/g{v:x}" for v in names[:100]]
    files.sort()
    oids = rng.integers(0, 256, size=(len(files), 20), dtype=np.uint8)
    s = packing.pack_side(files, oids, packing.GENERAL_ENCODING, engine=engine)
    h = packing.pack_side(files, oids, packing.GENERAL_ENCODING)  # host sort
    assert s.walk_rows and np.array_equal(s.key, h.key) and np.array_equal(s.order, h.order)
    r = engine.diff2(s, h)
    assert r.delta.shape[0] == 0 and r.n_update == 0
    with pytest.raises(ValueError):
        s.kd_side()  # a walk-row side joins only through its order


def test_gpu_merge_trees_uses_device_pack(engine, monkeypatch):
    """merge_trees packs large versions on the device (late-materialised sides) and gives the same
    index as the host-packed sides"""
    from kart_amd import dataset as D
    from kart_amd import merge as M

    monkeypatch.setattr(D, "GPU_SORT_MIN", 1)
    W = synth.table3_layers(30_000, seed=4, walk=True)  # (enough rows that some leaf trees hold several)

    def version(side):
        return D.DatasetVersion("ds", None, {}, packing.GENERAL_ENCODING, side.name, side.name_off, side.oid,
                                lambda i: b"")

    vers = [version(x) for x in (W.ancestor, W.ours, W.theirs)]
    idx = M.merge_trees(engine, *vers)
    assert all(v.packed.walk_rows for v in vers)
    monkeypatch.setattr(D, "GPU_SORT_MIN", 1 << 40)
    host = M.merge_trees(engine, *[version(x) for x in (W.ancestor, W.ours, W.theirs)])
    assert {k: (c.ancestor, c.ours, c.theirs) for k, c in idx.conflicts.items()} == \
        {k: (c.ancestor, c.ours, c.theirs) for k, c in host.conflicts.items()}
    assert len(idx.conflicts) == W.n_conflict
    _ = NONE, N
