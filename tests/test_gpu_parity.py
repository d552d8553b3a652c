"""HIP path (libkartdiff on an MI355X) vs the reference's golden outputs and the CPU oracle.

Every comparison is bit-exact: delta sets, update lists, changed-field masks, conflict sets,
encoded envelopes and match flags are integer / byte results.
"""
import ctypes
import json
import os

import numpy as np
import pytest

from checks import check_diff_case, check_merge_case
from fixtures import DIFF_FIXTURES, GOLDEN, MERGE_FIXTURES, load
from oracle import oracle as O

from kart_amd import _native as N

pytestmark = pytest.mark.gpu


def _g_classify(engine):
    def f(A, B):
        r = engine.diff2(A, B)
        return r.delta, r.upd, r.type_counts()

    return f


@pytest.mark.parametrize("kern", ["win", "walk"])
@pytest.mark.parametrize("name", DIFF_FIXTURES)
def test_gpu_fielddiff_kernels_golden(engine, request, name, kern):
    """every golden diff case (schema changes, legend changes, the reference's own repositories)
    through the windowed and the walked field-diff kernels, whatever size picks by default"""
    _fd_kernel(engine, request, kern)
    fx = load(name)
    for case in fx.cases("diff2"):
        check_diff_case(fx, case, _g_classify(engine), engine.fielddiff)


@pytest.mark.parametrize("kern", ["win", "walk"])
@pytest.mark.parametrize("layer", ["points", "polygons", "polygons_same"])
def test_gpu_fielddiff_kernels_pairs(engine, request, layer, kern):
    """pair-indexed arenas (every entry's blob, the bench's sparse form) through both kernels"""
    from kart_amd import synth
    from kart_amd.schema import FieldMaps

    _fd_kernel(engine, request, kern)
    L = (synth.points_layer(300_000, seed=21) if layer == "points" else
         synth.polygons_layer(600_000, seed=22, same_len=0.6 if layer == "polygons_same" else 0.0))
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    r = engine.diff2(L.base, L.target)
    gm, gs = engine.fielddiff(*L.base_blobs, *L.target_blobs, r.upd, maps)
    om, ost = O.fielddiff(*L.base_blobs, *L.target_blobs, r.upd, maps)
    assert np.array_equal(gm, om) and np.array_equal(gs, ost)


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


@pytest.mark.parametrize("ordered,n,layer,walk", [
    (o, n, layer, False) for o in (True, False)
    for n, layer in [(1000, "points"), (3_000_000, "points"), (1000, "polygons"), (2_000_000, "polygons")]] + [
    (True, 1000, "points", "late"), (True, 3_000_000, "points", "late"), (False, 2_000_000, "polygons", "late"),
    (True, 1000, "points", "gather"), (True, 2_000_000, "polygons", "gather"),
    (True, 10_000_000, "points", False),    # C2 at its stated size (configs[1])
    (True, 100_000_000, "polygons", False),  # C3 at its stated size (configs[2], the bench's default
                                             # workload): walk-order sides, no sort, pk-order sorts included
    (True, 20_000_000, "polygons", "late"),  # the fallback side sorts at 20M
    # rows shuffled inside each leaf tree (a walk mixing pk wraps): the per-leaf-tree sort
    (True, 1000, "points", "leaf"), (True, 3_000_000, "points", "leaf"), (False, 2_000_000, "polygons", "leaf"),
    (True, 20_000_000, "polygons", "leaf"),
    # C3v: 60 % of the geometry edits keep their length, so their payloads are compared byte by byte
    (True, 2_000_000, "polygons_same", False), (False, 2_000_000, "polygons_same", False),
    (True, 100_000_000, "polygons_same", False),
])
def test_gpu_device_pipeline_vs_oracle(engine, n, layer, ordered, walk):
    """the device-resident classify2 -> fielddiff -> pk-order pipeline bench.py times (both compaction
    modes), on the C2 points layer and the C3 polygon layer (~370-B blobs: head + tail windows and the
    cooperative payload compares); buffers from the library's own allocator.  The sides come in git
    tree order, which is key order: no sort.  walk = "late" / "gather": the fallback for sides whose
    walk order is not key order — the rows are scrambled and every step sorts them on the GPU first
    (kd_sort_side_into): the sorted keys (and OIDs) must equal the generator's key-ordered sides and the
    order must invert the scramble, bit for bit"""
    from kart_amd import synth
    from kart_amd.device import DiffPipeline
    from kart_amd.schema import FieldMaps

    L = (synth.points_layer(n, seed=11) if layer == "points" else
         synth.polygons_layer(n, seed=12, same_len=0.6 if layer == "polygons_same" else 0.0))
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    rng = np.random.default_rng(n)
    if walk == "leaf":  # shuffled inside each leaf tree (the key's top 24 bits), in order between them
        perms = tuple(np.lexsort((rng.random(S.n), S.key >> np.uint64(40))) for S in (L.base, L.target))
    else:
        perms = (rng.permutation(L.base.n), rng.permutation(L.target.n)) if walk else None
    pipe = DiffPipeline(engine, L.base, L.target, L.base_blobs, L.target_blobs, maps, ordered=ordered, unsorted=perms,
                        late=walk in ("late", "leaf"))
    if walk:
        assert pipe.segmented == (walk == "leaf")
    if walk:  # scramble the sorted buffers first: the sort (and, gathering, its OID permute) must rewrite them
        for S in (pipe.A, pipe.B):
            N.check(engine.L.kd_memset(engine.ctx, S.key.ptr, 0xA5, S.key.nbytes), "kd_memset")
            N.check(engine.L.kd_memset(engine.ctx, S.oid.ptr, 0x5A, S.oid.nbytes), "kd_memset")
    for _ in range(3):  # repeated steps reuse the workspaces and counters
        pipe.step()
    engine.sync()
    if walk:
        for S, side, perm, order in zip((pipe.A, pipe.B), (L.base, L.target), perms, pipe.orders()):
            assert np.array_equal(S.key.download(np.uint64, side.n), side.key)
            if walk == "gather":
                assert np.array_equal(S.oid.download(np.uint8, 20 * side.n).reshape(side.n, 20), side.oid)
            assert np.array_equal(perm[order], np.arange(side.n))  # walk_keys[order] ascending
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
    if pipe.pk_order and ordered:
        check_pk_order(pipe, L.base.key, L.target.key, delta, upd)


@pytest.mark.parametrize("n,layer", [(1000, "points"), (300_000, "points"), (2_000_000, "polygons"),
                                     (2_000_000, "polygons_same"), (100_000_000, "polygons")])
def test_gpu_device_pipeline_update_arenas(engine, n, layer):
    """the pipeline bench.py times by default: the field diff from update-order arenas (the drop-in's
    form, no pairs) after the join — the polygon layers' blobs already lie in update order (only
    per-update offsets are uploaded), the points layer's are gathered"""
    from kart_amd import synth
    from kart_amd.device import DiffPipeline
    from kart_amd.schema import FieldMaps

    L = (synth.points_layer(n, seed=13) if layer == "points" else
         synth.polygons_layer(n, seed=14, same_len=0.6 if layer == "polygons_same" else 0.0))
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    pipe = DiffPipeline(engine, L.base, L.target, L.base_blobs, L.target_blobs, maps)
    pipe.step()
    engine.sync()
    _, _, upd, _, _ = pipe.results()
    pipe.use_update_arenas(upd)
    for _ in range(2):
        pipe.step()
    engine.sync()
    counts, delta, upd2, masks, status = pipe.results()
    assert np.array_equal(upd2, upd)
    om, ost = O.fielddiff(*L.base_blobs, *L.target_blobs, upd, maps)
    assert np.array_equal(masks, om) and np.array_equal(status, ost)


def check_pk_order(pipe, kA, kB, delta, upd):
    """kd_delta_pk_order's outputs: the pks of the delta (and update) records ascending, and the
    record index of each — a stable argsort of the records' pks (DeltaDiff.sorted_items order)"""
    from kart_amd import walkkey

    d_pk, d_perm, u_pk, u_perm = pipe.pk_results()
    for rec, pk_out, perm_out in ((delta, d_pk, d_perm), (upd, u_pk, u_perm)):
        a, b = rec[:, 0], rec[:, 1]
        keys = np.where(a != 0xFFFFFFFF, kA[np.minimum(a, max(kA.size - 1, 0))] if kA.size else 0,
                        kB[np.minimum(b, max(kB.size - 1, 0))] if kB.size else 0)
        pks = walkkey.int_keys_to_pks(keys.astype(np.uint64))
        want = np.argsort(pks, kind="stable")
        assert np.array_equal(perm_out, want.astype(np.uint32))
        assert np.array_equal(pk_out, pks[want])


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


@pytest.mark.parametrize("n", [1000, 400_000, pytest.param(50_000_000, marks=pytest.mark.timeout(900))])
def test_gpu_merge3_device_c4_layer_vs_oracle(engine, n):
    """the C4 bench layer (string PKs, MsgpackHashPathEncoder paths, mod/mod, mod/del, del/mod and
    add/add edits) through the device-resident kd_merge3_device pipeline bench.py times, and the host
    kd_merge3: conflicts and merge deltas bit-exact with the oracle, conflicts = the generator's plan.
    50M rows = C4 at its stated size (BASELINE configs[3])"""
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


@pytest.mark.parametrize("lens", [[24], [1, 2, 3, 5, 7, 13, 29, 30, 31, 33, 64, 100], [200]])
def test_gpu_hash_names_verified(engine, lens):
    """KD_KEY_HASH: matched keys with equal filenames classify normally (the join's LDS-staged tile
    names; with 200-byte names a tile's names overflow that buffer and take the global compare: the
    batched 32-B window and the long-name loop); one differing byte in one matched filename (first, middle or last
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


@pytest.mark.parametrize("n,kind", [(1, "rand"), (2, "rand"), (3, "one_bit"), (8191, "rand"), (8192, "int30"),
                                    (8193, "int30"), (4095, "rand"), (4097, "rand"), (1_000_003, "rand"),
                                    (2_000_000, "walk"), (500_000, "runs5"), (300_000, "hi_bits"), (77, "equal")])
def test_gpu_sort_side_into_vs_argsort(engine, n, kind):
    """the out-of-place device sort (the pipeline's form) equals a stable host argsort: keys, order
    and OIDs; the inputs stay untouched.  Tile edges (8192 keys per 32-bit tile, 4096 per 64-bit
    tile), random 64-bit keys (8 passes over the 64-bit compact key), int keys (compact 32-bit key),
    walk-order C3 keys, a varying-bit mask of 5 runs (merged into 4), and all-equal keys (no pass;
    flagged as duplicates)"""
    from kart_amd import synth
    from kart_amd.device import DevBuf

    rng = np.random.default_rng(n)
    if kind == "rand":
        keys = np.unique(rng.integers(0, 2**64 - 1, size=n + n // 8 + 8, dtype=np.uint64))[:n]
        rng.shuffle(keys)
    elif kind == "int30":
        keys = synth._int_keys(rng.permutation(n).astype(np.int64) * 5)
    elif kind == "walk":  # a walk of pks mixing wraps in their leaf trees: not key order
        p = np.arange(n, dtype=np.int64)
        keys = synth._int_keys(np.where(p % 3 == 0, p + (1 << 30), p))
        rng.shuffle(keys)
    elif kind == "runs5":
        spread = np.uint64(0)
        for b in (0, 1, 9, 10, 20, 33, 34, 35, 50, 63):
            spread |= np.uint64(1) << np.uint64(b)
        vals = rng.permutation(1 << 10)[: min(n, 1 << 10)].astype(np.uint64)
        keys = np.zeros(vals.shape[0], np.uint64)
        bits = [b for b in range(64) if (int(spread) >> b) & 1]
        for j, b in enumerate(bits):
            keys |= ((vals >> np.uint64(j)) & np.uint64(1)) << np.uint64(b)
        keys |= np.uint64(0x0000_0100_0004_0000)  # constant bits between the runs
    elif kind == "hi_bits":
        keys = (np.arange(n, dtype=np.uint64) << np.uint64(40)) | np.uint64(0xABCDE)
        rng.shuffle(keys)
    elif kind == "one_bit":
        keys = np.array([5 | (1 << 63), 5, 7][:n], np.uint64)
    else:
        keys = np.full(n, 12345, np.uint64)
    n = keys.shape[0]
    oids = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
    dk, do = DevBuf.from_numpy(engine, keys), DevBuf.from_numpy(engine, oids.reshape(-1))
    ko, oo, order, dup = DevBuf(engine, 8 * n), DevBuf(engine, 20 * n), DevBuf(engine, 4 * n), DevBuf(engine, 4)
    info = None
    if kind in ("int30", "walk", "runs5") and n > 0:  # the host scan sizes the passes: no read-back
        from kart_amd import packing
        info = packing.keys_scan(keys, 0 if kind != "runs5" else 1)
    N.check(engine.L.kd_sort_side_into(engine.ctx, dk.ptr, do.ptr, ko.ptr, oo.ptr, order.ptr, n, dup.ptr,
                                       ctypes.byref(info) if info is not None else None), "kd_sort_side_into")
    ref = np.argsort(keys, kind="stable")
    assert np.array_equal(order.download(np.uint32, n), ref.astype(np.uint32))
    assert np.array_equal(ko.download(np.uint64, n), keys[ref])
    assert np.array_equal(oo.download(np.uint8, 20 * n).reshape(n, 20), oids[ref])
    assert np.array_equal(dk.download(np.uint64, n), keys) and np.array_equal(do.download(np.uint8, 20 * n), oids.reshape(-1))
    assert int(dup.download(np.uint32, 1)[0]) == (1 if kind == "equal" and n > 1 else 0)


def test_gpu_sort_side_into_rejects_aliasing(engine):
    from kart_amd.device import DevBuf

    dk, do, order = DevBuf(engine, 80), DevBuf(engine, 200), DevBuf(engine, 40)
    assert engine.L.kd_sort_side_into(engine.ctx, dk.ptr, do.ptr, dk.ptr, do.ptr, order.ptr, 10, None, None) == N.KD_EINVAL


def test_gpu_sort_side_duplicates_rejected(engine):
    from kart_amd import packing

    keys = np.array([9, 3, 7, 3], np.uint64)
    with pytest.raises(packing.PackError):
        packing.sort_on_device(engine, keys, np.zeros((4, 20), np.uint8))


@pytest.mark.parametrize("n", [1000, 2_000_000])
def test_gpu_pack_side_equals_host_pack(engine, n):
    """pack_side(engine=...) (native parse + GPU key sort, OIDs late-materialised) == the host
    packer, and a diff of two GPU-packed sides (through their orders) == the oracle's"""
    from kart_amd import packing, synth

    L = synth.polygons_layer(n, seed=3)
    sides = []
    for S in (L.base, L.target):
        pks = packing.int_keys_to_pks(S.key)
        walk = packing.pack_side(*synth.int_pk_paths(pks)[:1], S.oid, packing.INT_PK_ENCODING,
                                 rel_off=synth.int_pk_paths(pks)[1], engine=engine)
        assert walk.timing["sort_on"] == "none" and np.array_equal(walk.key, S.key)  # walk order: no sort
        perm = np.random.default_rng(n).permutation(S.n)  # leaves in another order: sorted on the GPU
        arena, off = synth.int_pk_paths(pks[perm])
        host = packing.pack_side(arena, S.oid[perm], packing.INT_PK_ENCODING, rel_off=off)
        dev = packing.pack_side(arena, S.oid[perm], packing.INT_PK_ENCODING, rel_off=off, engine=engine)
        # late materialisation: keys sorted on the GPU, OIDs left in walk order behind the order
        assert dev.walk_rows and np.array_equal(dev.oid, S.oid[perm])
        m = dev.materialised()
        assert np.array_equal(m.key, host.key) and np.array_equal(m.oid, host.oid)
        assert np.array_equal(dev.order, host.order) and np.array_equal(dev.key, S.key)
        sides.append(dev)
    r = engine.diff2(*sides)
    od, _ = O.classify2(L.base.key, L.base.oid, L.target.key, L.target.oid)
    assert np.array_equal(r.delta, od)


@pytest.mark.parametrize("kind,n", [("int", 1), ("int", 5000), ("int", 2_000_000), ("hash", 300_000), ("hash", 3)])
def test_gpu_diff2_perm_equals_sorted(engine, kind, n):
    """kd_diff2_device_perm (sorted keys, OIDs + filename offsets left in a scrambled row order, read
    through the sort order) gives exactly kd_diff2_device's result on the key-ordered sides — and
    the oracle's; KD_KEY_HASH filenames are verified through the same rows"""
    from kart_amd import synth
    from kart_amd.device import DevBuf, DevSide

    if kind == "int":
        L = synth.points_layer(n, seed=21)
        A, B = L.base, L.target
    else:
        M = synth.table3_layers(n, seed=22)
        A, B = M.ours, M.theirs
    rng = np.random.default_rng(n)
    sides, orders, keep = [], [], []
    for S in (A, B):
        P = rng.permutation(S.n)  # walk row r holds sorted entry P[r]
        inv = np.argsort(P).astype(np.uint32)  # sorted entry i lives at row inv[i]
        dk = DevBuf.from_numpy(engine, S.key if S.n else np.zeros(1, np.uint64))
        do = DevBuf.from_numpy(engine, S.oid[P].reshape(-1) if S.n else np.zeros(20, np.uint8))
        orders.append(DevBuf.from_numpy(engine, inv if S.n else np.zeros(1, np.uint32)))
        s = N.KdSide()
        s.n, s.key, s.oid, s.mem, s.key_mode = S.n, dk.ptr, do.ptr, N.KD_MEM_DEVICE, S.key_mode
        s.name = s.name_off = None
        if S.key_mode == N.KD_KEY_HASH:
            lens = (S.name_off[1:] - S.name_off[:-1]).astype(np.int64)[P]
            off = np.zeros(S.n + 1, np.uint64)
            off[1:] = np.cumsum(lens)
            names = np.concatenate([S.name[int(S.name_off[p]):int(S.name_off[p + 1])] for p in P]) if S.n else \
                np.zeros(1, np.uint8)
            dn, dno = DevBuf.from_numpy(engine, names), DevBuf.from_numpy(engine, off)
            s.name, s.name_off = dn.ptr, dno.ptr
            keep += [dn, dno]
        sides.append(s)
        keep += [dk, do]
    DA, DB = DevSide(engine, A), DevSide(engine, B)
    sa, sb = DA.kd_side(), DB.kd_side()
    cap = A.n + B.n + 1
    outs = []
    for perm in (True, False):
        delta, upd, counts = DevBuf(engine, 8 * cap), DevBuf(engine, 8 * cap), DevBuf(engine, 64)
        counts.zero()
        if perm:
            rc = engine.L.kd_diff2_device_perm(engine.ctx, ctypes.byref(sides[0]), ctypes.byref(sides[1]),
                                               orders[0].ptr, orders[1].ptr, 0, delta.ptr, upd.ptr, counts.ptr,
                                               counts.ptr + 32)
        else:
            rc = engine.L.kd_diff2_device(engine.ctx, ctypes.byref(sa), ctypes.byref(sb), 0, delta.ptr, upd.ptr,
                                          counts.ptr, counts.ptr + 32)
        N.check(rc, "diff2")
        c = counts.download(np.uint64, 8)
        assert c[4] == 0
        outs.append((c[:4].tolist(), delta.download(np.uint32, 2 * int(c[3])), upd.download(np.uint32, 2 * int(c[1]))))
    assert outs[0][0] == outs[1][0]
    assert np.array_equal(outs[0][1], outs[1][1]) and np.array_equal(outs[0][2], outs[1][2])
    od, _ = O.classify2(A.key, A.oid, B.key, B.oid)
    assert np.array_equal(outs[0][1].reshape(-1, 2), od)


def _gather_arena(data, off, idx):
    """the blobs ``idx`` of an arena, back to back (contiguous in idx order)"""
    idx = np.asarray(idx, np.int64)
    lo, hi = off[idx].astype(np.int64), off[idx + 1].astype(np.int64)
    lens = hi - lo
    out_off = np.zeros(idx.size + 1, np.uint64)
    np.cumsum(lens, out=out_off[1:])
    pos = np.repeat(lo - out_off[:-1].astype(np.int64), lens) + np.arange(int(lens.sum()), dtype=np.int64)
    return np.ascontiguousarray(data[pos]), out_off


def _grow_geometry(blob, extra, rng):
    """the feature blob with its geometry payload lengthened by ``extra`` bytes (field diff compares
    geometry payloads as bytes)"""
    import msgpack

    from kart_amd.dataset import Geometry, msg_unpack

    leg, vals = msg_unpack(blob)
    vals = [Geometry(bytes(v) + rng.integers(0, 256, extra, dtype=np.uint8).tobytes()) if isinstance(v, Geometry)
            else v for v in vals]
    return msgpack.packb([leg, vals], use_bin_type=True, strict_types=True,
                         default=lambda g: msgpack.ExtType(ord("G"), bytes(g)))


# kd_fielddiff's kernels by option: (fd_stream, fd_walk)
FD_KERNELS = {"win": (0, 0), "stream": (1, 0), "walk": (0, 1)}


def _fd_kernel(engine, request, kern):
    stream, walk = FD_KERNELS[kern]
    engine.set_option("fd_stream", stream)
    engine.set_option("fd_walk", walk)

    def restore():
        engine.set_option("fd_stream", -1)
        engine.set_option("fd_walk", -1)

    request.addfinalizer(restore)


@pytest.mark.parametrize("kern", ["win", "stream", "walk"])
@pytest.mark.parametrize("case", ["c3", "c3v", "huge", "ragged", "points", "one"])
def test_gpu_fielddiff_contiguous_vs_oracle(engine, request, kern, case):
    """kd_fielddiff on update arenas laid back to back (no pairs: the drop-in's form), through the
    streamed kernel (whole tile spans into LDS), the windowed one and the walked one (k_fdwalk, every
    read straight from HBM): C3 / C3v polygons, a tile whose span overflows the LDS buffer (blobs of
    20-60 KB: the walk queues their payloads), update counts that end inside a tile, point features.
    The last blob of every arena ends at the arena's end: the walk's guarded loads"""
    from kart_amd import synth
    from kart_amd.schema import FieldMaps

    _fd_kernel(engine, request, kern)
    rng = np.random.default_rng(7)
    if case == "points":
        L = synth.points_layer(300_000, seed=3)
    else:
        L = synth.polygons_layer(400_000 if case in ("c3", "c3v", "huge") else 30_011, seed=5,
                                 same_len=0.6 if case in ("c3v", "huge") else 0.0)
    r = engine.diff2(L.base, L.target)
    upd = r.upd
    if case == "one":
        upd = upd[:1]
    od, oo = _gather_arena(*L.base_blobs, upd[:, 0])
    nd, no = _gather_arena(*L.target_blobs, upd[:, 1])
    if case == "huge":  # rows 40..79 and 2000..2004: geometries of 20-60 KB on both sides
        rows = list(range(40, 80)) + list(range(2000, 2005))
        ob = [od[int(oo[i]):int(oo[i + 1])].tobytes() for i in range(upd.shape[0])]
        nb = [nd[int(no[i]):int(no[i + 1])].tobytes() for i in range(upd.shape[0])]
        for i in rows:
            extra = int(rng.integers(20_000, 60_000))
            ob[i] = _grow_geometry(ob[i], extra, np.random.default_rng(i))
            nb[i] = _grow_geometry(nb[i], extra, np.random.default_rng(i if i % 2 else i + 1))
        from kart_amd.packing import _arena

        (od, oo), (nd, no) = _arena(ob), _arena(nb)
    maps = FieldMaps(L.schema, L.legends, L.schema, L.legends)
    gm, gs = engine.fielddiff(od, oo, nd, no, None, maps)
    om, ost = O.fielddiff(od, oo, nd, no, None, maps)
    assert np.array_equal(gm, om) and np.array_equal(gs, ost)
    assert not gs.any()
