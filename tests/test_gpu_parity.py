"""HIP path (libkartdiff on an MI355X) vs the reference's golden outputs and the CPU oracle.

Every comparison is bit-exact: delta sets, update lists, changed-field masks, conflict sets,
encoded envelopes and match flags are integer / byte results.
"""
import json
import os

import numpy as np
import pytest

from checks import check_diff_case, check_merge_case
from fixtures import DIFF_FIXTURES, GOLDEN, MERGE_FIXTURES, load
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _g_classify(engine):
    def f(A, B):
        r = engine.diff2(A, B)
        return r.delta, r.upd, r.type_counts()

    return f


@pytest.mark.parametrize("name", DIFF_FIXTURES)
def test_gpu_diff2_golden(engine, name):
    fx = load(name)
    for case in fx.cases("diff2"):
        check_diff_case(fx, case, _g_classify(engine), engine.fielddiff)


@pytest.mark.parametrize("name", MERGE_FIXTURES)
def test_gpu_merge3_golden(engine, name):
    fx = load(name)
    (case,) = fx.cases("merge3")

    def m(A, O_, T):
        r = engine.merge3(A, O_, T)
        return r.conflict, r.mdelta, r.n_clean

    check_merge_case(fx, case, m)


def test_gpu_spatial_points_golden(engine):
    from test_oracle_golden import _arena, _geoms_of_side

    fx = load("repo_points")
    sp = fx.meta["spatial"]
    geoms, names = _geoms_of_side(fx, sp["side"])
    data, off = _arena(geoms)
    match, enc, ok, ncand = engine.envelopes(data, off, sp["filter_env"], 20)
    assert sorted(n for n, m in zip(names, match) if m == 1) == sorted(sp["matching_names"])
    assert ncand == 13
    om, oe, ook, _ = O.envelope_batch(data, off, sp["filter_env"], 20)
    assert np.array_equal(match, om) and np.array_equal(ok, ook) and np.array_equal(enc, oe)


# ------------------------------------------------------------------------------------------
# size-scaled parity vs the oracle on seeded synthetic layers
@pytest.mark.parametrize("n,seed", [(0, 1), (1, 2), (5000, 3), (300_000, 4), (2_000_000, 5)])
def test_gpu_diff2_synthetic_vs_oracle(engine, n, seed):
    from kart_amd import synth

    L = synth.points_layer(n, seed=seed)
    r = engine.diff2(L.base, L.target)
    od, counts = O.classify2(L.base.key, L.base.oid, L.target.key, L.target.oid)
    assert np.array_equal(r.delta, od)
    assert (r.n_insert, r.n_update, r.n_delete) == (counts["inserts"], counts["updates"], counts["deletes"])
    assert (r.n_insert, r.n_update, r.n_delete) == (L.n_insert, L.n_update, L.n_delete)
    if r.upd.shape[0]:
        from kart_amd.schema import FieldMaps

        maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
        gm, gs = engine.fielddiff(*L.base_blobs, *L.target_blobs, r.upd, maps)
        om, os_ = O.fielddiff(*L.base_blobs, *L.target_blobs, r.upd, maps)
        assert np.array_equal(gm, om) and np.array_equal(gs, os_)
        assert not gs.any()


def _edge_sides(rng, nA, nB, overlap, change):
    """random strictly-ascending key sets with controlled overlap / OID changes"""
    universe = np.unique(rng.integers(0, 2**63, size=int((nA + nB) * 1.5) + 10, dtype=np.uint64))
    rng.shuffle(universe)
    common = universe[: int(min(nA, nB) * overlap)]
    onlyA = universe[len(common): len(common) + nA - len(common)]
    onlyB = universe[len(common) + len(onlyA): len(common) + len(onlyA) + nB - len(common)]
    kA = np.sort(np.concatenate([common, onlyA]))
    kB = np.sort(np.concatenate([common, onlyB]))
    oA = rng.integers(0, 256, size=(kA.size, 20), dtype=np.uint8)
    oB = np.zeros((kB.size, 20), np.uint8)
    # same OID for common keys unless changed
    posA = {int(k): i for i, k in enumerate(kA)}
    oB[:] = rng.integers(0, 256, size=oB.shape, dtype=np.uint8)
    for j, k in enumerate(kB):
        i = posA.get(int(k))
        if i is not None and rng.random() >= change:
            oB[j] = oA[i]
    return kA, oA, kB, oB


@pytest.mark.parametrize("nA,nB,overlap,change", [(10, 0, 0, 0), (0, 10, 0, 0), (3000, 3000, 1.0, 0.0),
                                                  (3000, 3000, 1.0, 1.0), (5000, 200, 0.5, 0.3),
                                                  (200, 5000, 0.5, 0.3), (40000, 40000, 0.0, 0.0),
                                                  (60000, 50000, 0.9, 0.05)])
def test_gpu_diff2_edges_vs_oracle(engine, nA, nB, overlap, change):
    """merge-path tile seams: long one-sided runs, all-equal, all-changed, disjoint sets"""
    from kart_amd import packing

    rng = np.random.default_rng(nA * 7 + nB)
    kA, oA, kB, oB = _edge_sides(rng, nA, nB, overlap, change)
    A = packing.PackedSide(kA, oA, 0, np.arange(kA.size))
    B = packing.PackedSide(kB, oB, 0, np.arange(kB.size))
    r = engine.diff2(A, B)
    od, counts = O.classify2(kA, oA, kB, oB)
    assert np.array_equal(r.delta, od)
    assert r.n_update == counts["updates"]


def test_gpu_diff2_rejects_unsorted(engine):
    from kart_amd import _native as N
    from kart_amd import packing

    k = np.array([5, 3, 9], np.uint64)
    A = packing.PackedSide(k, np.zeros((3, 20), np.uint8), 0, np.arange(3))
    B = packing.PackedSide(np.array([1, 2], np.uint64), np.zeros((2, 20), np.uint8), 0, np.arange(2))
    with pytest.raises(N.Unsupported):
        engine.diff2(A, B)


@pytest.mark.parametrize("n", [1000, 200_000])
def test_gpu_merge3_synthetic_vs_oracle(engine, n):
    from kart_amd import packing

    rng = np.random.default_rng(n)
    kA = np.unique(rng.integers(0, 2**62, size=n, dtype=np.uint64))
    oA = rng.integers(0, 256, size=(kA.size, 20), dtype=np.uint8)

    def edit(seed):
        r = np.random.default_rng(seed)
        keep = r.random(kA.size) > 0.005
        k = kA[keep]
        o = oA[keep].copy()
        ch = r.random(k.size) < 0.05
        o[ch] = r.integers(0, 256, size=(int(ch.sum()), 20), dtype=np.uint8)
        ins = r.integers(0, 2**62, size=kA.size // 200, dtype=np.uint64)
        k2 = np.concatenate([k, ins])
        o2 = np.concatenate([o, r.integers(0, 256, size=(ins.size, 20), dtype=np.uint8)])
        k2, idx = np.unique(k2, return_index=True)
        return k2, np.ascontiguousarray(o2[idx])

    kO, oO = edit(1)
    kT, oT = edit(2)
    # overlapping edits: same keys changed identically on both sides (clean) and differently (conflict)
    common = np.intersect1d(kO, kT)
    pick = rng.choice(common, size=min(50, common.size), replace=False)
    iO, iT = np.searchsorted(kO, pick), np.searchsorted(kT, pick)
    same = rng.integers(0, 256, size=(pick.size, 20), dtype=np.uint8)
    oO[iO] = same
    oT[iT[: pick.size // 2]] = same[: pick.size // 2]
    sides = [packing.PackedSide(k, o, 0, np.arange(k.size)) for k, o in ((kA, oA), (kO, oO), (kT, oT))]
    r = engine.merge3(*sides)
    oc, om, oclean = O.classify3(kA, oA, kO, oO, kT, oT)
    key = lambda rows: sorted(map(tuple, rows.tolist()))
    assert key(r.conflict) == key(oc)
    assert key(r.mdelta) == key(om)
    assert r.n_clean == oclean


def _gpkg_blobs(rng, n):
    """mixed GPKG geometries: XY/XYZ envelopes (LE/BE), points without envelope, empties,
    NaN envelopes, antimeridian/wide envelopes, null geometries, one malformed blob"""
    import struct

    out = []
    for i in range(n):
        r = rng.random()
        if r < 0.02:
            out.append(b"")
            continue
        if r < 0.35:
            le = rng.random() < 0.9
            bo = "<" if le else ">"
            x, y = rng.uniform(-200, 200), rng.uniform(-95, 95)
            if rng.random() < 0.02:
                x = y = float("nan")
            flags = 1 if le else 0
            if rng.random() < 0.02:
                flags |= 0x10
            out.append(b"GP\x00" + bytes([flags]) + struct.pack(bo + "i", 4326) + struct.pack(bo + "bI", 1 if le else 0, 1)
                       + struct.pack(bo + "dd", x, y))
            continue
        le = rng.random() < 0.85
        bo = "<" if le else ">"
        et = 1 if rng.random() < 0.8 else 2
        minx = rng.uniform(-180, 180)
        w = 10 ** rng.uniform(-7, 2.6)
        miny = rng.uniform(-90, 90)
        h = 10 ** rng.uniform(-7, 1.5)
        env = [minx, minx + w, miny, miny + h] + ([0.0, 1.0] if et == 2 else [])
        if rng.random() < 0.01:
            env[1] = float("nan")
        flags = (1 if le else 0) | (et << 1)
        if rng.random() < 0.01:
            flags |= 0x10
        body = struct.pack(bo + "bI", 1 if le else 0, 6) + b"\x00" * 16
        out.append(b"GP\x00" + bytes([flags]) + struct.pack(bo + "i", 4326) + struct.pack(bo + "d" * len(env), *env) + body)
    out.append(b"GX\x00\x01")  # malformed
    return out


@pytest.mark.parametrize("bits", [20, 16, 32, 8])
def test_gpu_envelopes_vs_oracle(engine, bits):
    from test_oracle_golden import _arena

    rng = np.random.default_rng(bits)
    geoms = _gpkg_blobs(rng, 20000)
    data, off = _arena(geoms)
    for filt in [(175.8, 175.9, -37.1, -36.9), (-10.0, 10.0, -5.0, 5.0), (-180.0, 180.0, -90.0, 90.0), (0.0, 0.0, 0.0, 0.0)]:
        gm, ge, gk, gc = engine.envelopes(data, off, filt, bits)
        om, oe, ok, oc = O.envelope_batch(data, off, filt, bits)
        assert np.array_equal(gm, om)
        assert np.array_equal(gk, ok)
        assert np.array_equal(ge, oe)
        assert gc == oc


def test_gpu_env_overlap_vs_oracle(engine):
    with open(os.path.join(GOLDEN, "envelopes.json")) as f:
        E = json.load(f)
    enc = np.array([list(bytes.fromhex(h)) for h, _ in E["decode"]], np.uint8)
    for q in E["queries"]:
        g = engine.env_overlap(enc, 20, q)
        o = O.envelope_overlap(enc, 20, q)
        assert np.array_equal(g, o)


@pytest.mark.parametrize("ordered,n,layer", [
    (o, n, layer) for o in (True, False)
    for n, layer in [(1000, "points"), (3_000_000, "points"), (1000, "polygons"), (2_000_000, "polygons")]] + [
    (True, 10_000_000, "points"),       # C2 at its stated size (configs[1])
    (True, 100_000_000, "polygons"),    # C3 at its stated size (configs[2], the bench's default workload)
])
def test_gpu_device_pipeline_vs_oracle(engine, n, layer, ordered):
    """the device-resident classify2 -> fielddiff pipeline bench.py times (both compaction modes),
    on the C2 points layer and the C3 polygon layer (~370-B blobs: head + tail windows and the
    cooperative payload compares); buffers from the library's own allocator"""
    from kart_amd import synth
    from kart_amd.device import DiffPipeline
    from kart_amd.schema import FieldMaps

    L = synth.points_layer(n, seed=11) if layer == "points" else synth.polygons_layer(n, seed=12)
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    pipe = DiffPipeline(engine, L.base, L.target, L.base_blobs, L.target_blobs, maps, ordered=ordered)
    for _ in range(3):  # repeated steps reuse the workspaces and counters
        pipe.step()
    engine.sync()
    counts, delta, upd, masks, status = pipe.results()
    od, oc = O.classify2(L.base.key, L.base.oid, L.target.key, L.target.oid)
    if ordered:
        assert np.array_equal(delta, od)
    else:
        key = lambda a: sorted(map(tuple, a.tolist()))
        assert key(delta) == key(od)
    assert (counts["inserts"], counts["updates"], counts["deletes"]) == (oc["inserts"], oc["updates"], oc["deletes"])
    om, ost = O.fielddiff(*L.base_blobs, *L.target_blobs, upd, maps)
    assert np.array_equal(masks, om) and np.array_equal(status, ost)


@pytest.mark.parametrize("n,seed", [(1000, 1), (2_000_000, 2)])
def test_gpu_envelopes_c5_layer_vs_oracle(engine, n, seed):
    """the C5 bench layer (points, multipolygons, straddles, >=180-degree widths, empties, filter-edge
    envelopes) at scale: flags, EnvelopeEncoder bytes and candidate counts bit-exact"""
    from kart_amd import synth

    data, off, _ = synth.geometry_layer(n, seed=seed)
    gm, ge, gk, gc = engine.envelopes(data, off, synth.C5_FILTER, 20)
    om, oe, ok, oc = O.envelope_batch(data, off, synth.C5_FILTER, 20)
    assert np.array_equal(gm, om) and np.array_equal(gk, ok) and np.array_equal(ge, oe) and gc == oc
    assert 0 < gc < n


@pytest.mark.parametrize("n", [1000, 400_000])
def test_gpu_merge3_device_c4_layer_vs_oracle(engine, n):
    """the C4 bench layer (string PKs, MsgpackHashPathEncoder paths, mod/mod, mod/del, del/mod and
    add/add edits) through the device-resident kd_merge3_device pipeline bench.py times, and the host
    kd_merge3: conflicts and merge deltas bit-exact with the oracle, conflicts = the generator's plan"""
    from kart_amd import synth
    from kart_amd.device import MergePipeline

    M = synth.table3_layers(n, seed=n)
    pipe = MergePipeline(engine, M.ancestor, M.ours, M.theirs)
    for _ in range(2):  # repeated steps reuse the workspaces and counters
        pipe.step()
    engine.sync()
    n_clean, conf, md = pipe.results()
    oc, om, ocl = O.classify3(M.ancestor.key, M.ancestor.oid, M.ours.key, M.ours.oid, M.theirs.key, M.theirs.oid)
    key = lambda rows: sorted(map(tuple, np.asarray(rows).tolist()))
    assert key(conf) == key(oc) and key(md) == key(om) and n_clean == ocl
    assert conf.shape[0] == M.n_conflict
    r = engine.merge3(M.ancestor, M.ours, M.theirs)
    assert key(r.conflict) == key(oc) and key(r.mdelta) == key(om)


@pytest.mark.gpu
@pytest.mark.parametrize("nA,nO,nT,mode", [(0, 0, 0, "x"), (0, 500, 700, "add"), (3000, 0, 0, "del"),
                                          (3000, 3000, 0, "x"), (3000, 0, 3000, "x"), (5000, 5000, 5000, "same"),
                                          (4000, 4100, 3900, "rand"), (70_000, 70_000, 70_000, "all")])
def test_gpu_merge3_edges_vs_oracle(engine, nA, nO, nT, mode):
    """one-sided and empty merges, all paths identical, every path edited on both sides, random
    overlaps: conflicts / merge deltas bit-exact with the oracle and in key (path) order"""
    from kart_amd import packing

    rng = np.random.default_rng(nA * 7 + nO * 3 + nT)
    pool = np.unique(rng.integers(0, 2**63, size=max(nA, nO, nT) * 2 + 8, dtype=np.uint64))
    oid_of = rng.integers(0, 256, size=(pool.size, 20), dtype=np.uint8)

    def side(n, salt):
        if mode == "same" or mode == "all":
            idx = np.arange(min(n, pool.size))
        else:
            idx = np.sort(rng.choice(pool.size, size=n, replace=False))
        o = oid_of[idx].copy()
        if mode == "all" and salt:
            o[:, 0] ^= salt  # every path edited, differently on ours and theirs -> all conflicts
        elif mode == "rand" and salt:
            ch = rng.random(idx.size) < 0.3
            o[ch] = rng.integers(0, 256, size=(int(ch.sum()), 20), dtype=np.uint8)
        return pool[idx].copy(), o

    kA, oA = side(nA, 0)
    kO, oO = side(nO, 1)
    kT, oT = side(nT, 2)
    sides = [packing.PackedSide(k, o, 0, np.arange(k.size)) for k, o in ((kA, oA), (kO, oO), (kT, oT))]
    r = engine.merge3(*sides)
    oc, om, oclean = O.classify3(kA, oA, kO, oO, kT, oT)
    assert np.array_equal(np.asarray(r.conflict).reshape(-1, 3), np.asarray(oc).reshape(-1, 3))
    assert np.array_equal(np.asarray(r.mdelta).reshape(-1, 2), np.asarray(om).reshape(-1, 2))
    assert r.n_clean == oclean
    if mode == "all":
        assert len(r.conflict) == nA


@pytest.mark.gpu
@pytest.mark.parametrize("which", [0, 1, 2])
def test_gpu_merge3_rejects_unsorted(engine, which):
    from kart_amd import _native as N
    from kart_amd import packing

    ks = [np.array([1, 4, 9, 12], np.uint64) for _ in range(3)]
    ks[which] = np.array([1, 9, 4, 12], np.uint64)
    sides = [packing.PackedSide(k, np.zeros((4, 20), np.uint8), 0, np.arange(4)) for k in ks]
    with pytest.raises(N.Unsupported):
        engine.merge3(*sides)
    # the error flag is consumed: the next, valid merge succeeds
    ok = [packing.PackedSide(np.array([1, 4, 9, 12], np.uint64), np.zeros((4, 20), np.uint8), 0, np.arange(4))
          for _ in range(3)]
    assert engine.merge3(*ok).n_clean == 4


def _hash_sides(rng, n, lens):
    """hash-key sides sharing keys and filenames: names of the given lengths (random bytes, so every
    byte offset mod 4 occurs), three sides = ancestor / ours / theirs with ~10% per-side edits"""
    from kart_amd import packing
    from kart_amd import _native as N

    keys = np.unique(rng.integers(0, 2**63, size=n, dtype=np.uint64))
    ln = rng.choice(lens, size=keys.size)
    names = [rng.integers(0, 256, size=int(k), dtype=np.uint8).tobytes() for k in ln]
    oids = rng.integers(0, 256, size=(keys.size, 20), dtype=np.uint8)

    def side(sel, oid, nm):
        idx = np.flatnonzero(sel)
        arena = b"".join(nm[i] for i in idx)
        off = np.zeros(idx.size + 1, np.uint64)
        off[1:] = np.cumsum([len(nm[i]) for i in idx])
        return packing.PackedSide(keys[idx].copy(), np.ascontiguousarray(oid[idx]), N.KD_KEY_HASH,
                                  np.arange(idx.size), np.frombuffer(arena, np.uint8).copy(), off)

    return keys, names, oids, side


@pytest.mark.parametrize("lens", [[24], [1, 2, 3, 5, 7, 13, 29, 30, 31, 33, 64, 100]])
def test_gpu_hash_names_verified(engine, lens):
    """KD_KEY_HASH: matched keys with equal filenames classify normally (the batched 32-B window and
    the long-name loop both); one differing byte in one matched filename (first, middle or last
    byte, or a length change) is a key collision -> Unsupported, for diff2 and for merge3 (ancestor
    vs ours and ancestor vs theirs-without-ours)"""
    from kart_amd import _native as N

    rng = np.random.default_rng(len(lens))
    keys, names, oids, side = _hash_sides(rng, 3000, lens)
    m = keys.size
    selA = rng.random(m) > 0.1
    selO = rng.random(m) > 0.1
    selT = rng.random(m) > 0.1
    oO = oids.copy(); oO[rng.random(m) < 0.1, 0] ^= 1
    oT = oids.copy(); oT[rng.random(m) < 0.1, 1] ^= 1
    A, O_, T = side(selA, oids, names), side(selO, oO, names), side(selT, oT, names)
    r = engine.diff2(A, O_)
    od, _ = O.classify2(A.key, A.oid, O_.key, O_.oid)
    assert np.array_equal(r.delta, od)
    r3 = engine.merge3(A, O_, T)
    oc, om, ocl = O.classify3(A.key, A.oid, O_.key, O_.oid, T.key, T.oid)
    assert np.array_equal(np.asarray(r3.conflict).reshape(-1, 3), oc.reshape(-1, 3))
    assert np.array_equal(np.asarray(r3.mdelta).reshape(-1, 2), om.reshape(-1, 2)) and r3.n_clean == ocl

    both = np.flatnonzero(selA & selO & selT)
    for pick, where in ((both[5], 0), (both[len(both) // 2], -1), (both[-3], "len")):
        bad = list(names)
        b = bytearray(bad[pick])
        if where == "len":
            b += b"x"
        else:
            b[where] ^= 0x20
        bad[pick] = bytes(b)
        with pytest.raises(N.Unsupported):
            engine.diff2(A, side(selO, oO, bad))
        with pytest.raises(N.Unsupported):
            engine.merge3(A, side(selO, oO, bad), T)
    # ancestor and theirs matched, ours absent: the ancestor/theirs filenames are checked directly
    only_at = np.flatnonzero(selA & ~selO & selT)
    bad = list(names)
    b = bytearray(bad[only_at[0]]); b[-1] ^= 1; bad[only_at[0]] = bytes(b)
    with pytest.raises(N.Unsupported):
        engine.merge3(A, O_, side(selT, oT, bad))


# ---------------------------------------------------------------------------------------------
# GPU packing: kd_sort_side (LDS-ranked LSD radix sort of the join keys + OID permute)
def _sort_dev(engine, keys, oids):
    from kart_amd import packing

    n = keys.shape[0]
    dk, do, dord = packing.sort_on_device(engine, keys, oids)
    return dk.download(np.uint64, n), do.download(np.uint8, 20 * n).reshape(n, 20), dord.download(np.uint32, n)


@pytest.mark.parametrize("n,kind", [(1, "rand"), (2, "rand"), (4095, "rand"), (4097, "rand"), (100_000, "rand"),
                                    (3_000_000, "rand"), (1_000_000, "int30"), (300_000, "hi_bits"),
                                    (50_000, "one_bit")])
def test_gpu_sort_side_vs_argsort(engine, n, kind):
    """the device sort equals a stable host argsort: keys, order and the OIDs that travel with them
    (random 64-bit keys = 8 passes; int keys of pks < 2**30 = 4 passes; keys varying only in the top
    byte or in one bit)"""
    rng = np.random.default_rng(n)
    if kind == "rand":
        keys = np.unique(rng.integers(0, 2**64 - 1, size=n + n // 8, dtype=np.uint64))[:n]
        rng.shuffle(keys)
    elif kind == "int30":
        from kart_amd import synth

        keys = synth._int_keys(rng.permutation(n).astype(np.int64) * 3)
    elif kind == "hi_bits":
        keys = (np.arange(n, dtype=np.uint64) << np.uint64(40)) | np.uint64(0xABCDE)
        rng.shuffle(keys)
    else:
        keys = np.array([5, 5 | (1 << 63)] * (n // 2), np.uint64)[:n]
        keys = np.unique(keys)
    n = keys.shape[0]
    oids = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
    k, o, order = _sort_dev(engine, keys, oids)
    ref = np.argsort(keys, kind="stable")
    assert np.array_equal(order, ref.astype(np.uint32))
    assert np.array_equal(k, keys[ref]) and np.array_equal(o, oids[ref])


def test_gpu_sort_side_duplicates_rejected(engine):
    from kart_amd import packing

    keys = np.array([9, 3, 7, 3], np.uint64)
    with pytest.raises(packing.PackError):
        packing.sort_on_device(engine, keys, np.zeros((4, 20), np.uint8))


@pytest.mark.parametrize("n", [1000, 2_000_000])
def test_gpu_pack_side_equals_host_pack(engine, n):
    """pack_side(engine=...) (native parse + GPU sort, device-resident result) == the host packer,
    and a diff of two GPU-packed sides == the oracle's"""
    from kart_amd import packing, synth

    L = synth.polygons_layer(n, seed=3)
    sides = []
    for S in (L.base, L.target):
        pks = (S.key >> np.uint64(40)).astype(np.int64) * 64 + (S.key & np.uint64(63)).astype(np.int64)
        perm = np.random.default_rng(n).permutation(S.n)  # leaves in another (walk) order
        arena, off = synth.int_pk_paths(pks[perm])
        host = packing.pack_side(arena, S.oid[perm], packing.INT_PK_ENCODING, rel_off=off)
        dev = packing.pack_side(arena, S.oid[perm], packing.INT_PK_ENCODING, rel_off=off, engine=engine)
        assert np.array_equal(dev.key, host.key) and np.array_equal(dev.oid, host.oid)
        assert np.array_equal(dev.order, host.order) and np.array_equal(dev.key, S.key)
        sides.append(dev)
    r = engine.diff2(*sides)
    od, _ = O.classify2(L.base.key, L.base.oid, L.target.key, L.target.oid)
    assert np.array_equal(r.delta, od)
