"""Pin the CPU oracle (oracle/kd_oracle.c) against the reference's own outputs (tests/golden/).

CPU only.  These tests also exercise the product's host packing (kd_pack_* in libkartdiff, CPU
code) and the legend -> union-key maps (kart_amd.schema) on every golden case.
"""
import json
import os
import struct

import numpy as np
import pytest

from checks import check_diff_case, check_merge_case
from fixtures import DIFF_FIXTURES, GOLDEN, MERGE_FIXTURES, load
from oracle import oracle as O


def _o_classify(A, B):
    delta, counts = O.classify2(A.key, A.oid, B.key, B.oid)
    upd = delta[(delta[:, 0] != O.NONE) & (delta[:, 1] != O.NONE)]
    return delta, upd, counts


@pytest.mark.parametrize("name", DIFF_FIXTURES)
def test_oracle_diff2_golden(name):
    fx = load(name)
    n_upd = 0
    for case in fx.cases("diff2"):
        n_upd += check_diff_case(fx, case, _o_classify, O.fielddiff)
    if name in ("repo_points", "conflicts_polygons", "synth_int", "synth_int_same"):
        assert n_upd > 0


def _o_merge(A, O_, T):
    return O.classify3(A.key, A.oid, O_.key, O_.oid, T.key, T.oid)


@pytest.mark.parametrize("name", MERGE_FIXTURES)
def test_oracle_merge3_golden(name):
    fx = load(name)
    (case,) = fx.cases("merge3")
    check_merge_case(fx, case, _o_merge)


def test_pinned_reference_numbers():
    """The numbers the reference's own tests pin, re-checked on the fixtures."""
    pts = load("repo_points")
    (fwd,) = [c for c in pts.cases("diff2") if c["base"] == "head1" and c["target"] == "head"]
    assert sorted(int(d["old_pk"]["int"]) for d in fwd["deltas"]) == [1095, 1166, 1168, 1181, 1182]  # test_diff.py:1061
    assert sum(len(d["changed"]) for d in fwd["deltas"]) == 13
    assert len(pts.meta["spatial"]["matching_names"]) == 13  # test_spatial_filter.py:682
    poly = load("conflicts_polygons")
    (m,) = poly.cases("merge3")
    assert len(m["conflicts"]) == 4 and m["n_entries"] == 237  # test_conflicts.py:27-28


def test_oracle_paths_golden():
    """IntPathEncoder / MsgpackHashPathEncoder vectors (dataset3_paths.py) vs the oracle keys
    and the product packer (kd_pack_*)."""
    from kart_amd import packing

    with open(os.path.join(GOLDEN, "paths.json")) as f:
        P = json.load(f)
    uniq = dict((p, pk) for pk, p in P["int"])
    rel = list(uniq)
    side = packing.pack_side(rel, np.zeros((len(rel), 20), np.uint8), packing.INT_PK_ENCODING)
    pks = packing.int_keys_to_pks(side.key)
    want = sorted(int(pk) for pk in uniq.values())
    assert sorted(pks.tolist()) == want
    alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
    for pk_s, path in P["int"]:
        pk = int(pk_s)
        key = np.zeros(1, np.uint64)
        assert O.C().kdo_int_walk_key(pk, key.ctypes.data) == 0
        assert int(key[0]) == packing.pk_to_int_key(pk)
        # the key's bucket bits are the IntPathEncoder tree path, each character as its ASCII rank
        tree = path.rsplit("/", 1)[0].replace("/", "")
        rank = 0
        for ch in tree:
            rank = rank * 64 + sorted(alpha).index(ch)
        assert int(key[0]) >> 40 == rank
    # these vectors mix 2**30 wraps in one leaf tree (0, 2**30, -2**30 all live in A/A/A/A): their
    # git order is not key order, and the packer says so
    paths = sorted(uniq, key=str.encode)
    side = packing.pack_side(paths, np.zeros((len(paths), 20), np.uint8), packing.INT_PK_ENCODING)
    assert side.info.ascending == 0 and side.timing["sort_on"] == "host"
    # hashed paths: packer == oracle, bucket bits == tree chars
    for enc, vecs, levels, hexm in ((packing.GENERAL_ENCODING, P["hash"], 4, 0),):
        rel = [p for _, p in vecs]
        side = packing.pack_side(rel, np.zeros((len(rel), 20), np.uint8), enc)
        for k, i in enumerate(side.order):
            b = rel[i].encode()
            key = np.zeros(1, np.uint64)
            assert O.C().kdo_hash_path_key(b, len(b), levels, hexm, key.ctypes.data) == 0
            assert int(key[0]) == int(side.key[k])
    leg = [p for pk, p in P["legacy"] if pk.startswith("s:")]
    side = packing.pack_side(leg, np.zeros((len(leg), 20), np.uint8), packing.LEGACY_ENCODING)
    assert side.n == len(leg)


@pytest.mark.parametrize("name", [n for n in DIFF_FIXTURES if not n.startswith("synth")])
def test_reference_repo_sides_need_no_sort(name):
    """Every int-PK side of the reference's own repositories, in the order `git ls-tree -r` listed it
    (the fixtures keep that order), packs to strictly ascending keys: no sort before the join."""
    fx = load(name)
    for key in fx.meta["sides"]:
        side = fx.packed(key)
        if side.key_mode == 0 and side.n:
            assert side.timing["sort_on"] == "none", (name, key)


def test_walk_key_oracle_vs_packer_random():
    """The packer's table-driven keys (kd_walkkey.h / walkkey.py) equal the oracle's brute-force
    restatement (every block's 64 filenames compared) on pks across every msgpack width and sign,
    and the key inverts to the pk."""
    from kart_amd import packing, walkkey

    rng = np.random.default_rng(7)
    edges = [0, 63, 64, 127, 128, 255, 256, 65535, 65536, 2**32 - 1, 2**32, 2**63 - 1, -1, -32, -33, -64, -65,
             -128, -129, -32768, -32769, -2**31, -2**31 - 1, -2**63, 2**30 - 1, 2**30, -2**30, -2**30 - 1]
    pks = np.concatenate([np.array(edges, np.int64), np.arange(-300, 300, dtype=np.int64),
                          rng.integers(-2**63, 2**63 - 1, 3000, dtype=np.int64),
                          rng.integers(-2**33, 2**33, 3000, dtype=np.int64)])
    key = np.zeros(1, np.uint64)
    got = walkkey.int_keys(pks)
    for pk, k in zip(pks.tolist(), got.tolist()):
        assert O.C().kdo_int_walk_key(pk, key.ctypes.data) == 0
        assert int(key[0]) == k, pk
    assert np.array_equal(packing.int_keys_to_pks(got), pks)
    assert np.array_equal(walkkey.int_keys_to_pks(got), pks)


def test_walk_key_order_is_git_path_order():
    """Sorting IntPathEncoder paths bytewise (git's tree order) == sorting their keys, for pk ranges
    whose leaf trees hold one 2**30 wrap (negative, small, msgpack width edges, the wrap's end)."""
    from kart_amd import walkkey

    alpha = walkkey.B64.decode()

    def path(p):
        b = (p // 64) % (1 << 24)
        return ("/".join(alpha[(b >> (18 - 6 * k)) & 63] for k in range(4)) + "/" + walkkey.filename(p)).encode()

    for lo, hi in [(-5000, 5000), (60000, 70000), (2**32 - 3000, 2**32 + 3000), (2**30 - 5000, 2**30),
                   (-2**30, -2**30 + 5000), (-40000, -30000)]:
        ps = np.arange(lo, hi, dtype=np.int64)
        if lo < 0 < hi:  # negative and non-negative pks share no bucket here (|pk| < 2**29)
            pass
        by_path = sorted(ps.tolist(), key=path)
        by_key = ps[np.argsort(walkkey.int_keys(ps))].tolist()
        assert by_path == by_key, (lo, hi)
    # a leaf tree mixing wraps (pk and pk + 2**30 share a bucket): the keys still invert, but the
    # walk order can differ from key order — kd_keys_scan reports it and the side gets sorted
    ps = np.array([5, 5 + 2**30, 6, 6 + 2**30], np.int64)
    walk = sorted(ps.tolist(), key=path)
    keys = walkkey.int_keys(np.array(walk, np.int64))
    from kart_amd import packing
    info = packing.keys_scan(keys, 0)
    assert info.ascending == int(bool(np.all(keys[1:] > keys[:-1])))


def _hexf(x):
    return float.fromhex(x)


def test_oracle_envelope_encoder_golden():
    with open(os.path.join(GOLDEN, "envelopes.json")) as f:
        E = json.load(f)
    L = O.C()
    out = np.zeros(16, np.uint8)
    for env, hx in E["encode"]:
        e = np.array(env, np.float64)
        assert L.kdo_envelope_encode(e.ctypes.data, 20, out.ctypes.data) == 0
        assert out[:10].tobytes().hex() == hx, (env, hx)
    dec = np.zeros(4, np.float64)
    for bits, env, hx, decoded in E["bits"]:
        e = np.array(env, np.float64)
        assert L.kdo_envelope_encode(e.ctypes.data, bits, out.ctypes.data) == 0
        assert out[:bits // 2].tobytes().hex() == hx
        b = np.frombuffer(bytes.fromhex(hx), np.uint8).copy()
        L.kdo_envelope_decode(b.ctypes.data, bits, dec.ctypes.data)
        assert [float(x).hex() for x in dec] == decoded
    for hx, decoded in E["decode"]:
        b = np.frombuffer(bytes.fromhex(hx), np.uint8).copy()
        L.kdo_envelope_decode(b.ctypes.data, 20, dec.ctypes.data)
        assert [float(x).hex() for x in dec] == decoded


def test_oracle_geometry_golden():
    with open(os.path.join(GOLDEN, "envelopes.json")) as f:
        E = json.load(f)
    L = O.C()
    for a, b, want in E["bbox"]:
        aa, bb = np.array(a, np.float64), np.array(b, np.float64)
        assert L.kdo_bbox_intersects(aa.ctypes.data, bb.ctypes.data) == int(want)
    for x, y in E["wrap_lon"]:
        assert L.kdo_wrap_lon(_hexf(x)).hex() == y
    env = np.zeros(4, np.float64)
    for src, want in E["identity_env"]:
        s = np.array([_hexf(v) for v in src], np.float64)  # (minx, miny, maxx, maxy)
        gp = np.array([s[0], s[2], s[1], s[3]], np.float64)  # -> (minx, maxx, miny, maxy)
        rc = L.kdo_index_envelope(gp.ctypes.data, env.ctypes.data)
        if want is None:
            assert rc == 0
        else:
            assert rc == 1 and [float(v).hex() for v in env] == want, (src, want, env)
    for ghex, want in E["gpkg_env"]:
        g = np.frombuffer(bytes.fromhex(ghex), np.uint8).copy()
        rc = L.kdo_gpkg_envelope(g.ctypes.data, g.size, env.ctypes.data)
        if want is None:
            assert rc in (0, 2)
        else:
            assert rc == 1 and [float(v).hex() for v in env] == want


def test_oracle_spatial_points_golden():
    """13 of points HEAD^'s features pass the 'points-edit' bbox (test_spatial_filter.py:682)."""
    fx = load("repo_points")
    sp = fx.meta["spatial"]
    geoms, names = _geoms_of_side(fx, sp["side"])
    data, off = _arena(geoms)
    match, enc, ok, npass = O.envelope_batch(data, off, sp["filter_env"], 20)
    got = sorted(n for n, m in zip(names, match) if m == 1)
    assert got == sorted(sp["matching_names"])
    assert npass == 13


def _geoms_of_side(fx, key):
    """geometry column value of every feature on a side (msgpack ext 'G' payload)."""
    import msgpack

    out, names = [], fx.names(key)
    schema = fx.schema(key)
    gcol = schema.geometry_columns[0].id
    for i, bi in enumerate(fx.a[f"{key}_blob"]):
        lh, vals = msgpack.unpackb(fx.blob(int(bi)), raw=False, ext_hook=lambda c, d: d)
        leg = fx.legends[lh]
        g = vals[leg.non_pk_columns.index(gcol)] if gcol in leg.non_pk_columns else None
        out.append(g or b"")
    return out, names


def _arena(bs):
    off = np.zeros(len(bs) + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs])
    return np.frombuffer(b"".join(bs), np.uint8).copy(), off


def test_oracle_fielddiff_vs_python_semantics():
    """C oracle field compare == Python's own == on msgpack-decoded values, seeded edge values."""
    fx = load("synth_int_same")
    (case,) = [c for c in fx.cases("diff2") if c["base"] == "base"]
    A, B = fx.packed("base"), fx.packed("target")
    delta, counts = O.classify2(A.key, A.oid, B.key, B.oid)
    upd = delta[(delta[:, 0] != O.NONE) & (delta[:, 1] != O.NONE)]
    maps = __import__("checks").field_maps(fx, "base", "target")
    od, oo = fx.arena("base")
    nd, no = fx.arena("target")
    masks, status = O.fielddiff(od, oo, nd, no, upd, maps)
    sa, sb = fx.schema("base"), fx.schema("target")
    for u, (a, b) in enumerate(upd.tolist()):
        ob = od[int(oo[a]):int(oo[a + 1])].tobytes()
        nb = nd[int(no[b]):int(no[b + 1])].tobytes()
        import msgpack
        lo = fx.legends[msgpack.unpackb(ob, raw=False, ext_hook=lambda c, d: d)[0]]
        ln = fx.legends[msgpack.unpackb(nb, raw=False, ext_hook=lambda c, d: d)[0]]
        pk = int(__import__("kart_amd.packing", fromlist=["x"]).int_keys_to_pks(A.key[a:a + 1])[0])
        old = O.py_feature(ob, [pk], lo, sa)
        new = O.py_feature(nb, [pk], ln, sb)
        assert maps.changed_names(masks[u]) == O.py_changed_fields(old, new)


def _seg_max_ref(keys):
    b = keys >> np.uint64(40)
    if keys.size == 0:
        return 0
    if np.any(b[1:] < b[:-1]):
        return -1
    edges = np.flatnonzero(np.diff(b)) + 1
    runs = np.diff(np.concatenate([[0], edges, [keys.size]]))
    return int(runs.max())


def test_keys_scan_seg_max():
    """kd_keys_scan's seg_max (the longest run of keys in one leaf tree, -1 when the tree bits descend)
    equals a numpy restatement — threaded parts included (runs crossing the part boundaries)"""
    from kart_amd import packing

    rng = np.random.default_rng(1)
    for n in (0, 1, 5, 1000, 70_000, 300_000):
        for kind in ("asc", "runs", "onebucket", "desc"):
            if kind == "asc":
                k = np.sort(rng.integers(0, 2**63, n, dtype=np.uint64))
            elif kind == "runs":  # buckets ascending, each bucket's entries scrambled (a walk mixing wraps)
                b = np.sort(rng.integers(0, 1 << 12, n, dtype=np.uint64))
                k = (b << np.uint64(40)) | rng.integers(0, 1 << 40, n, dtype=np.uint64)
            elif kind == "onebucket":
                k = (np.uint64(7) << np.uint64(40)) | rng.permutation(n).astype(np.uint64)
            else:
                k = rng.integers(0, 2**63, n, dtype=np.uint64)
            info = packing.keys_scan(k, 0 if kind != "onebucket" else 1)
            assert info.seg_max == _seg_max_ref(k), (n, kind)
