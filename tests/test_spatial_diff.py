"""The spatially filtered diff (BaseDiffWriter.filtered_ds_feature_deltas, kart/base_diff_writer.py:
279-329; SpatialFilter.matches, kart/spatial_filter/__init__.py:534-605).

Golden: the reference's `points-edit` filter — 13 features of points HEAD^ match, 2 of the 5
edits in HEAD (tests/test_spatial_filter.py:666-704).  The CPU tests pin the oracle's restatement
to it; the GPU tests run kd_geom_filter against the oracle (codes, kept deltas, index envelopes) on
the fixtures, the synthetic polygon layer and crafted feature blobs, and run the drop-in
``filtered_ds_feature_deltas`` on the golden."""
import msgpack
import numpy as np
import pytest

from fixtures import load
from kart_amd import dataset as D
from kart_amd import spatial as S
from kart_amd.schema import Legend
from oracle import oracle as O
from test_dropin import version
from test_gpu_parity import _gpkg_blobs
from test_oracle_golden import _arena

NONE = O.NONE
POINTS_EDIT = (175.8, 175.9, -37.1, -36.9)  # bbox_as_wkt_polygon(175.8, 175.9, -36.9, -37.1)


def _cols(fx, key):
    """{legend hex: geometry value index} of a fixture side"""
    gcol = fx.schema(key).geometry_columns[0].id
    return {h: (list(lg.non_pk_columns).index(gcol) if gcol in lg.non_pk_columns else -1)
            for h, lg in fx.legends.items()}


def _side_arena(fx, key):
    idx = fx.a[f"{key}_blob"]
    return _arena([fx.blob(int(b)) for b in idx])


def test_oracle_points_edit_golden():
    """oracle restatement: 13 of HEAD^'s inserts and 2 of HEAD's 5 updates pass `points-edit`"""
    fx = load("repo_points")
    assert fx.meta["spatial"]["filter_env"] == list(POINTS_EDIT)
    cols = _cols(fx, "head1")
    hd, ho = _side_arena(fx, "head1")
    n = int(ho.shape[0]) - 1
    pairs = np.stack([np.full(n, NONE, np.uint32), np.arange(n, dtype=np.uint32)], axis=1)
    codes, keep, _, _ = O.geom_filter(hd, ho, hd, ho, pairs, cols, cols, POINTS_EDIT, True)
    assert len(keep) == 13 and set(codes[keep, 1].tolist()) == {O.GF_MATCH}
    names = fx.names("head1")
    assert sorted(names[i] for i in keep) == sorted(fx.meta["spatial"]["matching_names"])
    # HEAD^ -> HEAD: the 5 updates (classify2 on the fixture sides)
    A, B = fx.packed("head1"), fx.packed("head")
    delta, _ = O.classify2(A.key, A.oid, B.key, B.oid)
    od, oo = _side_arena(fx, "head1")
    nd, no = _side_arena(fx, "head")
    # arenas are in fixture (path) order; the delta indices are sorted-entry indices
    pairs = np.stack([np.where(delta[:, 0] == NONE, NONE, A.order[np.minimum(delta[:, 0], A.n - 1)]),
                      np.where(delta[:, 1] == NONE, NONE, B.order[np.minimum(delta[:, 1], B.n - 1)])],
                     axis=1).astype(np.uint32)
    codes, keep, _, _ = O.geom_filter(od, oo, nd, no, pairs, cols, _cols(fx, "head"), POINTS_EDIT, True)
    assert len(delta) == 5 and len(keep) == 2


def test_host_spatial_filter_semantics():
    """SpatialFilter.matches on the host: None -> MATCHING, bbox miss -> NON_MATCHING, points inside a
    rectangle or a ring are exact, empties never match"""
    import struct

    pt = lambda x, y: b"GP\x00\x01" + struct.pack("<i", 4326) + struct.pack("<bIdd", 1, 1, x, y)
    sf = S.SpatialFilter.from_rectangle(0, 10, 0, 10, "geom")
    assert sf.matches({"geom": None}) is S.MatchResult.MATCHING
    assert sf.matches(None) is S.MatchResult.NONEXISTENT
    assert sf.matches({"geom": pt(5, 5)}) is S.MatchResult.MATCHING
    assert sf.matches({"geom": pt(10, 5)}) is S.MatchResult.NON_MATCHING  # bbox_intersects_fast: zero width at the edge
    assert sf.matches({"geom": pt(11, 5)}) is S.MatchResult.NON_MATCHING
    empty = b"GP\x00\x11" + struct.pack("<i", 4326) + struct.pack("<bII", 1, 3, 0)
    assert sf.matches({"geom": empty}) is S.MatchResult.NON_MATCHING
    tri = S.SpatialFilter.from_ring([(0, 0), (10, 0), (0, 10), (0, 0)], "geom")
    assert not tri.rectangle
    assert tri.matches({"geom": pt(2, 2)}) is S.MatchResult.MATCHING
    assert tri.matches({"geom": pt(8, 8)}) is S.MatchResult.NON_MATCHING  # in the bbox, outside the triangle
    assert S.SpatialFilter.MATCH_ALL.matches({"geom": pt(99, 99)}) is S.MatchResult.MATCHING
    assert S.SpatialFilter.from_ring([(0, 0), (4, 0), (4, 2), (0, 2), (0, 0)]).rectangle


# ---------------------------------------------------------------------------------------------
# GPU
def _crafted(rng, n):
    """feature blobs around the fast path's assumptions: geometry first/later, null, nested values,
    16+ values (array16), ext8/16/32 geometries, unknown legends, short blobs"""
    geoms = _gpkg_blobs(rng, n)
    legends = {
        "first": Legend(["pk"], ["g", "a", "b"]),
        "later": Legend(["pk"], ["a", "b", "g"]),
        "wide": Legend(["pk"], ["g"] + ["x%d" % i for i in range(18)]),
        "nogeom": Legend(["pk"], ["a", "b"]),
    }
    hexes = {k: lg.hexhash() for k, lg in legends.items()}
    cols = {hexes["first"]: 0, hexes["later"]: 2, hexes["wide"]: 0, hexes["nogeom"]: -1}
    blobs = []
    big = b"GP\x00\x03" + b"\x00" * 4 + np.array([170.0, 176.0, -40.0, -35.0]).tobytes() + \
        b"\x01\x02\x00\x00\x00" + np.uint32(5000).tobytes() + rng.random(10000).tobytes()
    for i, g in enumerate(geoms):
        r = rng.random()
        gv = msgpack.ExtType(ord("G"), g) if g else None
        if i % 997 == 5:
            gv = msgpack.ExtType(ord("G"), big)  # ext32 (> 64 KiB)
        if i % 991 == 7:
            gv = msgpack.ExtType(ord("G"), g + b"\x00" * 300)  # ext16
        if r < 0.55:
            vals = [gv, int(rng.integers(1 << 40)), "s" * int(rng.integers(0, 40))]
            h = hexes["first"]
        elif r < 0.75:
            vals = [float(rng.random()), "t" * int(rng.integers(0, 300)), gv]
            h = hexes["later"]
        elif r < 0.85:
            vals = [gv] + [int(x) for x in rng.integers(0, 1000, 18)]
            h = hexes["wide"]
        elif r < 0.90:
            vals = [1, 2]
            h = hexes["nogeom"]
        elif r < 0.93:
            vals = [[1, 2], "x", gv]  # nested value before the geometry
            h = hexes["later"]
        elif r < 0.96:
            vals = [gv, 1, 2]
            h = "f" * 40  # unknown legend
        else:
            vals = [None, 3, "z"]  # short blob, null geometry
            h = hexes["first"]
        blobs.append(msgpack.packb([h, vals], use_bin_type=True))
    return blobs, cols


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [0, 20])
def test_gpu_geom_filter_vs_oracle_crafted(engine, bits):
    rng = np.random.default_rng(11)
    ob, cols = _crafted(rng, 6000)
    nb, _ = _crafted(np.random.default_rng(12), 6000)
    od, oo = _arena(ob)
    nd, no = _arena(nb)
    n = 7000
    pairs = np.stack([rng.integers(0, len(ob), n), rng.integers(0, len(nb), n)], axis=1).astype(np.uint32)
    pairs[rng.random(n) < 0.2, 0] = NONE
    pairs[rng.random(n) < 0.2, 1] = NONE
    gc = S.GeomCols.__new__(S.GeomCols)
    hx = np.frombuffer(b"".join(h.encode() for h in sorted(cols)), np.uint8).copy()
    gi = np.array([cols[h] for h in sorted(cols)], np.int16)
    gc.old_hex = gc.new_hex = hx
    gc.old_gidx = gc.new_gidx = gi
    gc.old_map = gc.new_map = cols
    for filt, rect in [((170.0, 178.0, -45.0, -30.0), True), ((-10.0, 10.0, -5.0, 5.0), False),
                       ((-180.0, 180.0, -90.0, 90.0), True)]:
        codes, keep, enc, ok = S.geom_filter(engine, (od, oo), (nd, no), pairs, gc, filt, rect, bits)
        oc, okeep, oenc, ook = O.geom_filter(od, oo, nd, no, pairs, cols, cols, filt, rect, bits or 20)
        assert np.array_equal(codes, oc), np.argwhere(codes != oc)[:5]
        assert np.array_equal(keep, okeep)
        if bits:
            assert np.array_equal(ok, ook)
            assert np.array_equal(enc[ok == 1], oenc[ook == 1])
        # the heads form: kd_geom_heads on the host, 48 bytes per blob to the GPU
        hs = [S.geom_heads(d, o, gc.old_hex, gc.old_gidx, len(cols)) for d, o in ((od, oo), (nd, no))]
        hc, hk, he, hok = S.geom_filter_heads(engine, hs[0], hs[1], pairs, filt, rect, bits, arenas=((od, oo), (nd, no)))
        assert np.array_equal(hc, oc) and np.array_equal(hk, okeep)
        if bits:
            assert np.array_equal(hok, ook) and np.array_equal(he[hok == 1], oenc[ook == 1])
        # without the arenas a geometry that needs more than its head (XYZ envelope, NaN envelope)
        # comes back FALLBACK, every other side as before
        hc2, _, _, _ = S.geom_filter_heads(engine, hs[0], hs[1], pairs, filt, rect, bits)
        diff = hc2 != oc
        assert diff.any() and (hc2[diff] == 3).all()
    assert {0, 1, 2, 3, 4} <= set(np.unique(oc).tolist())


@pytest.mark.gpu
def test_gpu_index_envelopes_heads_equal_arena_path(engine):
    """the spatial indexer's batch (spatial_index._index_envelopes: heads to the GPU, the rows a
    head cannot decide re-run whole through kd_geom_filter) equals the blob-arena kernel row for
    row on the crafted blobs (XYZ / NaN envelopes, ext16/32, unknown legends, nested values)"""
    from kart_amd.spatial_index import WORLD, _index_envelopes

    blobs, cols = _crafted(np.random.default_rng(21), 8000)
    d, o = _arena(blobs)
    gc = S.GeomCols.__new__(S.GeomCols)
    gc.old_hex = gc.new_hex = np.frombuffer(b"".join(h.encode() for h in sorted(cols)), np.uint8).copy()
    gc.old_gidx = gc.new_gidx = np.array([cols[h] for h in sorted(cols)], np.int16)
    gc.old_map = gc.new_map = cols
    rows = np.random.default_rng(22).permutation(len(blobs))[:7000]
    pairs = np.full((rows.size, 2), NONE, np.uint32)
    pairs[:, 1] = rows
    codes, enc, ok = _index_envelopes(engine, d, o, pairs, gc, 20)
    ac, _, ae, aok = S.geom_filter(engine, (np.zeros(0, np.uint8), np.zeros(1, np.uint64)), (d, o), pairs, gc, WORLD,
                                   False, 20)
    assert np.array_equal(codes, ac) and np.array_equal(ok, aok) and np.array_equal(enc[ok == 1], ae[aok == 1])
    assert ok.sum() > 5000 and (codes[:, 1] == 3).any()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2000, 300_000])
def test_gpu_geom_filter_polygon_layer(engine, n):
    """the synthetic polygon layer (C3/C5 shape): classify2 deltas, then the filter over them"""
    from kart_amd import synth

    L = synth.polygons_layer(n, seed=5, delta_blobs=True)
    r = engine.diff2(L.base, L.target)
    hexes = sorted(L.legends)
    cols = {h: 0 for h in hexes}
    gc = S.GeomCols.__new__(S.GeomCols)
    gc.old_hex = gc.new_hex = np.frombuffer(b"".join(h.encode() for h in hexes), np.uint8).copy()
    gc.old_gidx = gc.new_gidx = np.zeros(len(hexes), np.int16)
    gc.old_map = gc.new_map = cols
    (od, oo), (nd, no) = L.base_blobs, L.target_blobs
    filt = synth.C5_FILTER
    codes, keep, enc, ok = S.geom_filter(engine, (od, oo), (nd, no), r.delta, gc, filt, False, 20)
    oc, okeep, oenc, ook = O.geom_filter(od, oo, nd, no, r.delta, cols, cols, filt, False, 20)
    assert np.array_equal(codes, oc)
    assert np.array_equal(keep, okeep) and 0 < len(keep) < len(r.delta)
    assert np.array_equal(ok, ook) and np.array_equal(enc[ok == 1], oenc[ook == 1])
    hs = [S.geom_heads(d, o, gc.old_hex, gc.old_gidx, len(hexes)) for d, o in ((od, oo), (nd, no))]
    hc, hk, he, hok = S.geom_filter_heads(engine, hs[0], hs[1], r.delta, filt, False, 20)  # XY envelopes: no arena
    assert np.array_equal(hc, oc) and np.array_equal(hk, okeep)
    assert np.array_equal(hok, ook) and np.array_equal(he[hok == 1], oenc[ook == 1])


@pytest.mark.gpu
def test_gpu_filtered_diff_points_edit_golden(engine):
    """the drop-in: `kart show HEAD^` / `kart show HEAD` on points with the points-edit filter
    yield 13 and 2 features (tests/test_spatial_filter.py:666-704)"""
    fx = load("repo_points")
    head1, head = version(fx, "head1"), version(fx, "head")
    sf = S.SpatialFilter.from_rectangle(*POINTS_EDIT)
    ds = D.get_dataset_diff(engine, None, head1)
    got = list(S.filtered_ds_feature_deltas(engine, ds, None, head1, sf))
    assert len(got) == 13
    assert sorted(k for k, _ in got) == sorted(head1.decode_path_to_1pk(n) for n in fx.meta["spatial"]["matching_names"])
    ds = D.get_dataset_diff(engine, head1, head)
    got = list(S.filtered_ds_feature_deltas(engine, ds, head1, head, sf))
    assert len(got) == 2 and all(d.type == "update" for _, d in got)
    assert [k for k, _ in got] == sorted(k for k, _ in got)
    # match-all and a filter missing everything
    assert len(list(S.filtered_ds_feature_deltas(engine, ds, head1, head, S.SpatialFilter.MATCH_ALL))) == 5
    far = S.SpatialFilter.from_rectangle(0, 1, 0, 1)
    assert list(S.filtered_ds_feature_deltas(engine, ds, head1, head, far)) == []


@pytest.mark.gpu
@pytest.mark.parametrize("n,heads", [(200_000, False), (200_000, True), (5_000_000, False), (5_000_000, True),
                                     pytest.param(100_000_000, True, marks=pytest.mark.timeout(900))])
def test_gpu_filter_pipeline_device_resident(engine, n, heads):
    """FilterPipeline: classify2's device delta list straight into kd_geom_filter (device count),
    equal to the oracle over the same deltas (the C restatement, kdo_geom_filter).  100M features =
    C5 at its stated size (BASELINE configs[4]): ~10M deltas, both sides' codes, the kept list and
    the new side's index envelopes bit-exact"""
    import types

    from kart_amd import synth
    from kart_amd.device import FilterPipeline

    L = synth.polygons_layer(n, seed=9, delta_blobs=True)
    ver = types.SimpleNamespace(schema=L.schema, legends=L.legends)
    pipe = FilterPipeline(engine, L.base, L.target, L.base_blobs, L.target_blobs, S.GeomCols(ver, ver, "geom", "geom"),
                          synth.C5_FILTER, False, 20, heads=heads)
    pipe.step()
    pipe.step()  # a second step over the same buffers gives the same answer
    counts, delta, codes, keep, enc, ok = pipe.results()
    assert (counts["inserts"], counts["updates"], counts["deletes"]) == (L.n_insert, L.n_update, L.n_delete)
    cols = {h: 0 for h in L.legends}
    (od, oo), (nd, no) = L.base_blobs, L.target_blobs
    oc, okeep, oenc, ook = O.geom_filter(od, oo, nd, no, delta, cols, cols, synth.C5_FILTER, False, 20)
    assert np.array_equal(codes, oc) and np.array_equal(keep, okeep) and counts["kept"] == len(okeep)
    assert np.array_equal(ok, ook) and np.array_equal(enc[ok == 1], oenc[ook == 1])


@pytest.mark.gpu
@pytest.mark.parametrize("n,gather", [(200_000, False), (200_000, True), (3_000_000, False), (3_000_000, True),
                                      pytest.param(100_000_000, False, marks=pytest.mark.timeout(900))])
def test_gpu_filter_pipeline_c5_mix_delta_order(engine, n, gather):
    """C5 as SURVEY §8(d) defines it (synth.c5_layer: 30 % points, EMPTY points, polygons straddling
    +180, >= 180 degrees wide, starting on the filter's edge, XYZ envelopes the heads cannot decide):
    classify2, then the filter from the deltas' heads in delta order with the blob fallback through
    the step's delta pairs (kd_geom_filter_deltas: heads laid out in delta order by the host as the
    blob reader leaves them, KD_GF_DELTA_HEADS; or ``gather``: per-entry heads gathered into delta
    order on the device) — codes, kept list and index envelopes bit-exact with the oracle"""
    import types

    from kart_amd import synth
    from kart_amd.device import FilterPipeline

    L = synth.c5_layer(n, seed=13)
    ver = types.SimpleNamespace(schema=L.schema, legends=L.legends)
    gc = S.GeomCols(ver, ver, "geom", "geom")
    pipe = FilterPipeline(engine, L.base, L.target, L.base_blobs, L.target_blobs, gc, synth.C5_FILTER, False, 20,
                          heads=True, delta_order=True, gather=gather)
    pipe.step()
    pipe.step()
    counts, delta, codes, keep, enc, ok = pipe.results()
    assert (counts["inserts"], counts["updates"], counts["deletes"]) == (L.n_insert, L.n_update, L.n_delete)
    cols = {h: 0 for h in L.legends}  # the geometry is the first non-pk value
    (od, oo), (nd, no) = L.base_blobs, L.target_blobs
    oc, okeep, oenc, ook = O.geom_filter(od, oo, nd, no, delta, cols, cols, synth.C5_FILTER, False, 20)
    assert np.array_equal(codes, oc) and np.array_equal(keep, okeep) and counts["kept"] == len(okeep)
    assert np.array_equal(ok, ook) and np.array_equal(enc[ok == 1], oenc[ook == 1])
    # the mix reaches every branch: candidates, points, and heads that needed their blob
    heads = pipe.heads_host
    st = [h["goff_status"] >> 24 for h in heads]
    assert 0 < len(keep) and (oc == 1).any()
    flags = np.concatenate([h["gpkg"][:, 3][s == 0] for h, s in zip(heads, st)])
    assert (flags == 0x01).any() and (flags == 0x11).any() and (flags == 0x05).any()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [40, 130, 1000, 3_000_000])  # (1 and 13 deltas: one partial chunk)
def test_gpu_filter_head_layouts_agree(engine, n):
    """k_gf_dense over delta-order heads (prebuilt: KD_GF_DELTA_HEADS; or gathered on the device) and
    the pair-indexed k_gf_heads over per-entry heads give the oracle's codes, kept list and index
    envelopes"""
    import types

    from kart_amd import synth
    from kart_amd.device import FilterPipeline

    L = synth.c5_layer(n, seed=21)
    ver = types.SimpleNamespace(schema=L.schema, legends=L.legends)
    gc = S.GeomCols(ver, ver, "geom", "geom")
    cols = {h: 0 for h in L.legends}
    (od, oo), (nd, no) = L.base_blobs, L.target_blobs
    ref = None
    for mode in ({"delta_order": True}, {"delta_order": True, "gather": True}, {"delta_order": False}):
        pipe = FilterPipeline(engine, L.base, L.target, L.base_blobs, L.target_blobs, gc, synth.C5_FILTER, False, 20,
                              heads=True, **mode)
        pipe.step()
        counts, delta, codes, keep, enc, ok = pipe.results()
        if ref is None:
            ref = O.geom_filter(od, oo, nd, no, delta, cols, cols, synth.C5_FILTER, False, 20)
        oc, okeep, oenc, ook = ref
        assert np.array_equal(codes, oc) and np.array_equal(keep, okeep) and counts["kept"] == len(okeep), mode
        assert np.array_equal(ok, ook) and np.array_equal(enc[ok == 1], oenc[ook == 1]), mode
        del pipe


@pytest.mark.parametrize("bits", [20, 16])
def test_oracle_geom_filter_c_equals_python(bits):
    """the C restatement of the filtered diff's per-side decision (kdo_geom_filter, what the
    full-size C5 check uses) equals the Python one (msgpack.unpackb + the envelope functions) on
    crafted blobs: nested values, ext8/16/32 geometries, unknown legends, null and empty geometries,
    truncated and trailing-byte blobs"""
    rng = np.random.default_rng(bits)
    ob, cols = _crafted(rng, 3000)
    nb, _ = _crafted(np.random.default_rng(bits + 1), 3000)
    h = sorted(cols)[0]
    extra = [msgpack.packb([h, [msgpack.ExtType(ord("G"), b""), 1, 2]], use_bin_type=True),  # empty ext 'G'
             msgpack.packb([h, [msgpack.ExtType(ord("G"), b"XX123456"), 1, 2]], use_bin_type=True),  # not GPKG
             msgpack.packb([h, [msgpack.ExtType(5, b"abc"), 1, 2]], use_bin_type=True),  # another ext
             msgpack.packb([h, [1.5, 1, 2]], use_bin_type=True), msgpack.packb([h, []], use_bin_type=True),
             msgpack.packb([h], use_bin_type=True), msgpack.packb([h, [None], 3], use_bin_type=True),
             msgpack.packb({"a": 1, "b": 2}, use_bin_type=True), b"\x92", b"",
             msgpack.packb([h, [{"k": [1, {"x": None}]}, 1, 2]], use_bin_type=True) + b"\x00"]
    ob = ob + extra
    nb = nb + extra
    od, oo = _arena(ob)
    nd, no = _arena(nb)
    n = 6000
    pairs = np.stack([rng.integers(0, len(ob), n), rng.integers(0, len(nb), n)], axis=1).astype(np.uint32)
    pairs[-2 * len(extra):-len(extra), 0] = np.arange(len(ob) - len(extra), len(ob))
    pairs[-len(extra):, 1] = np.arange(len(nb) - len(extra), len(nb))
    pairs[rng.random(n) < 0.2, 0] = NONE
    pairs[rng.random(n) < 0.2, 1] = NONE
    for filt, rect in [((170.0, 178.0, -45.0, -30.0), True), ((-10.0, 10.0, -5.0, 5.0), False),
                       ((-180.0, 180.0, -90.0, 90.0), True)]:
        c = O.geom_filter(od, oo, nd, no, pairs, cols, cols, filt, rect, bits)
        p = O.geom_filter_py(od, oo, nd, no, pairs, cols, cols, filt, rect, bits)
        for x, y in zip(c, p):
            assert np.array_equal(x, y)
    assert {0, 1, 2, 3, 4} <= set(np.unique(c[0]).tolist())


def test_geom_heads_equal_oracle_feature_geometry():
    """kd_geom_heads (host, the blob reader's pass) against the oracle's feature_geometry
    (msgpack.unpackb + the legend's geometry position): status, GPKG length and its first 40 bytes,
    on the crafted blobs (nested values, ext8/16/32, unknown legends, null geometries) and malformed
    ones (trailing bytes, empty, wrong top-level shape, non-'G' ext, empty ext 'G')"""
    from kart_amd import _native as N

    rng = np.random.default_rng(3)
    blobs, cols = _crafted(rng, 4000)
    h = sorted(cols)[0]
    blobs += [msgpack.packb([h, [msgpack.ExtType(ord("G"), b""), 1, 2]], use_bin_type=True),
              msgpack.packb([h, [msgpack.ExtType(ord("G"), b"XX123456"), 1, 2]], use_bin_type=True),
              msgpack.packb([h, [msgpack.ExtType(5, b"abc"), 1, 2]], use_bin_type=True),
              msgpack.packb([h, [1.5, 1, 2]], use_bin_type=True), msgpack.packb([h, []], use_bin_type=True),
              msgpack.packb([h], use_bin_type=True), msgpack.packb([h, [None], 3], use_bin_type=True),
              msgpack.packb({"a": 1, "b": 2}, use_bin_type=True), b"\x92", b"",
              msgpack.packb([h, [{"k": [1, {"x": None}]}, 1, 2]], use_bin_type=True) + b"\x00"]
    data, off = _arena(blobs)
    hexes = sorted(cols)
    hx = np.frombuffer(b"".join(x.encode() for x in hexes), np.uint8).copy()
    gi = np.array([cols[x] for x in hexes], np.int16)
    heads = S.geom_heads(data, off, hx, gi, len(hexes), threads=3)
    seen = set()
    for i, b in enumerate(blobs):
        st, g = O.feature_geometry(b, cols)
        hs = int(heads["goff_status"][i]) >> 24
        if st:
            assert hs == N.KD_GH_FALLBACK, i
        elif g is None:
            assert hs == N.KD_GH_NULL, i
        else:
            assert hs == N.KD_GH_GEOM and int(heads["glen"][i]) == len(g), i
            assert heads["gpkg"][i].tobytes()[:min(40, len(g))] == g[:40]
            goff = int(heads["goff_status"][i]) & 0xFFFFFF
            assert bytes(blobs[i][goff:goff + len(g)]) == g
        seen.add(hs)
    assert seen == {N.KD_GH_GEOM, N.KD_GH_NULL, N.KD_GH_FALLBACK}
