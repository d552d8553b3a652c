"""C3 generator (CPU): the polygon layer's blobs decode as the reference's feature encoding and its
edit counts follow the plan; geometry edits change only the geometry, attribute edits only the
attributes (checked with the oracle's fielddiff, the CPU restatement of the reference's compare)."""
import numpy as np

from kart_amd import synth
from kart_amd.schema import FieldMaps
from oracle import oracle as O


def test_polygons_layer_plan_and_encoding():
    import msgpack

    L = synth.polygons_layer(20_000, seed=5)
    plan = synth.c3_plan(np.arange(20_000), 20_000)
    assert (L.n_update, L.n_insert, L.n_delete) == (int(((plan == 1) | (plan == 2)).sum()), 200, int((plan == 3).sum()))
    assert 1400 < L.n_update < 1800 and 150 < L.n_delete < 250  # 8 % / 1 % of 20k in expectation
    od, counts = O.classify2(L.base.key, L.base.oid, L.target.key, L.target.oid)
    upd = od[(od[:, 0] != 0xFFFFFFFF) & (od[:, 1] != 0xFFFFFFFF)]
    assert upd.shape[0] == L.n_update
    assert (counts["inserts"], counts["deletes"]) == (L.n_insert, L.n_delete)
    d, off = L.base_blobs
    lens = np.diff(off)
    assert np.count_nonzero(lens) == L.n_update  # blobs only where the diff reads them
    assert 200 < lens[lens > 0].mean() < 500
    i = int(np.nonzero(lens)[0][0])
    legend, vals = msgpack.unpackb(bytes(d[off[i]:off[i + 1]]), raw=False, ext_hook=lambda c, x: (c, x))
    assert legend == list(L.legends)[0] and len(vals) == 4
    assert vals[0][0] == ord("G") and vals[0][1][:4] == b"GP\x00\x03" and len(vals[1]) == 20
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    masks, status = O.fielddiff(*L.base_blobs, *L.target_blobs, upd, maps)
    assert not status.any()
    geom_bit = 1 << 1  # union keys follow the schema order: id, geom, date_adjusted, ...
    m = masks[:, 0]
    assert np.all((m == geom_bit) | ((m & geom_bit) == 0) & (m != 0))
    assert 0.4 < np.mean(m == geom_bit) < 0.6


def test_polygons_layer_shards_concatenate():
    """bucket-range shards (bench.py --gpus N) are exactly the whole layer's entries, in order: each
    a contiguous run of the tree walk"""
    n = 30_000
    whole = synth.polygons_layer(n, seed=9)
    parts = [synth.polygons_layer(n, seed=9, shard=(r, 4)) for r in range(4)]
    for side in ("base", "target"):
        assert np.array_equal(np.concatenate([getattr(p, side).key for p in parts]), getattr(whole, side).key)
        assert np.array_equal(np.concatenate([getattr(p, side).oid for p in parts]), getattr(whole, side).oid)
    assert sum(p.n_update for p in parts) == whole.n_update
    assert sum(p.n_insert for p in parts) == whole.n_insert and sum(p.n_delete for p in parts) == whole.n_delete
    # shard edges fall between whole leaf trees: no bucket in two shards
    buckets = [set((p.base.key >> np.uint64(40)).tolist()) | set((p.target.key >> np.uint64(40)).tolist()) for p in parts]
    assert all(not (buckets[i] & buckets[j]) for i in range(4) for j in range(i + 1, 4))
    assert abs(parts[0].base.n - parts[3].base.n) < n // 40


def test_int_pk_paths_match_reference_encoder():
    """vectorised IntPathEncoder paths == the reference encoding restated per pk
    (tests/test_structure.py:851-925 KAT: 1181 -> A/A/A/S/kc0EnQ==)"""
    import base64

    import msgpack

    pks = np.array([0, 1, 63, 64, 127, 128, 255, 256, 1181, 65535, 65536, 2**24, 2**30 - 1, 2**32 - 1], np.int64)
    arena, off = synth.int_pk_paths(pks)
    alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
    for i, pk in enumerate(pks.tolist()):
        b = (pk // 64) % (1 << 24)
        tree = "/".join(alpha[(b >> (18 - 6 * k)) & 63] for k in range(4))
        want = tree + "/" + base64.urlsafe_b64encode(msgpack.packb([pk])).decode()
        assert arena[off[i]:off[i + 1]].tobytes().decode() == want
    assert arena[off[8]:off[9]].tobytes() == b"A/A/A/S/kc0EnQ=="


def test_walk_order_is_git_path_order():
    """A side's leaves as `git ls-tree -r` / kd_walk list them (bytewise path order) have ascending
    KD_KEY_INT keys: the synthetic layers, generated in walk order, are key-ordered as they stand."""
    rng = np.random.default_rng(3)
    pks = np.unique(np.concatenate([np.arange(0, 400), np.arange(65_000, 66_000), np.arange(2**24 - 70, 2**24 + 70),
                                    rng.integers(0, 2**30, 30_000)]))
    rng.shuffle(pks)
    arena, off = synth.int_pk_paths(pks)
    paths = [arena[int(off[i]):int(off[i + 1])].tobytes() for i in range(pks.shape[0])]
    walk = np.array(sorted(range(pks.shape[0]), key=lambda i: paths[i]))
    keys = synth._int_keys(pks)[walk]
    assert np.all(keys[1:] > keys[:-1])
    L = synth.polygons_layer(10_000, seed=2)
    for side in (L.base, L.target):
        p = __import__("kart_amd.packing", fromlist=["x"]).int_keys_to_pks(side.key)
        a, o = synth.int_pk_paths(p)
        ps = [a[int(o[i]):int(o[i + 1])].tobytes() for i in range(p.shape[0])]
        assert ps == sorted(ps)
