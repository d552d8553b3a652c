"""Seeded synthetic layers, generated directly as packed side arrays + msgpack feature blobs.

Shapes follow SURVEY.md §8(d): the reference's own feature encoding (kart/dataset3.py:185-215,
kart/serialise_util.py:34-41) — blob = msgpack [legend_hexhash, [non-pk values]] with geometries as
ext 'G' GeoPackage binaries — and its int-PK path layout (kart/dataset3_paths.py:292-299), so the
engine sees exactly what a Kart repo's trees would hand it.  Blob OIDs are synthetic (a seeded
64-bit mix of (pk, version)): equal content <=> equal OID, which is all classification relies on.
No git repository is involved.

Every side comes out in git tree order — the order the tree walk lists the leaves, which for
int pks is ascending KD_KEY_INT key order (kart_amd/walkkey.py): no side needs a sort.

Generation is vectorised numpy, fast enough for the 10M-point C2 layer in seconds.
"""
from dataclasses import dataclass

import os

import numpy as np

from . import packing, walkkey
from .schema import Legend, Schema

SEED = 0x4B415254

POINT_SCHEMA = [
    {"id": "c-fid", "name": "fid", "dataType": "integer", "primaryKeyIndex": 0, "size": 64},
    {"id": "c-geom", "name": "geom", "dataType": "geometry", "geometryType": "POINT", "geometryCRS": "EPSG:4326"},
    {"id": "c-t50", "name": "t50_fid", "dataType": "integer", "size": 32},
    {"id": "c-na", "name": "name_ascii", "dataType": "text", "length": 75},
    {"id": "c-mac", "name": "macronated", "dataType": "text", "length": 1},
    {"id": "c-name", "name": "name", "dataType": "text", "length": 75},
]

POLYGON_SCHEMA = [
    {"id": "p-fid", "name": "id", "dataType": "integer", "primaryKeyIndex": 0, "size": 64},
    {"id": "p-geom", "name": "geom", "dataType": "geometry", "geometryType": "MULTIPOLYGON", "geometryCRS": "EPSG:4326"},
    {"id": "p-date", "name": "date_adjusted", "dataType": "timestamp"},
    {"id": "p-sid", "name": "survey_reference", "dataType": "text", "length": 50},
    {"id": "p-adj", "name": "adjusted_nodes", "dataType": "integer", "size": 32},
]


def splitmix64(x):
    x = (np.asarray(x, np.uint64) + np.uint64(0x9E3779B97F4A7C15))
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def synth_oids(pk, version):
    """[n, 20] uint8 OIDs: a seeded mix of (pk, version) — distinct for distinct content."""
    pk = np.asarray(pk, np.int64).view(np.uint64)
    v = np.asarray(version, np.uint64)
    h0 = splitmix64(pk * np.uint64(0x100000001B3) ^ (v << np.uint64(56)) ^ np.uint64(SEED))
    h1 = splitmix64(h0 ^ np.uint64(0xA5A5A5A5))
    h2 = splitmix64(h1 ^ np.uint64(0x5A5A5A5A))
    w = np.stack([h0, h1, h2], 1).view(np.uint8).reshape(-1, 24)
    return np.ascontiguousarray(w[:, :20])


@dataclass
class Layer:
    """One synthetic commit pair (base, target) of one dataset."""

    base: packing.PackedSide
    target: packing.PackedSide
    base_blobs: tuple  # (data uint8, off uint64[n+1]) in base sorted order
    target_blobs: tuple
    schema: Schema
    legends: dict
    n_insert: int
    n_update: int
    n_delete: int

    @property
    def n_pairs(self):
        return self.base.n + self.n_insert


def _put_u(arena, pos, val, width):
    """big-endian unsigned ints (val [n]) at arena[pos + 0..width)"""
    v = np.asarray(val, np.uint64)
    for k in range(width):
        arena[pos + k] = ((v >> np.uint64(8 * (width - 1 - k))) & np.uint64(0xFF)).astype(np.uint8)


def _put_const(arena, pos, bs):
    for k, b in enumerate(bs):
        arena[pos + k] = b


def _put_bytes2d(arena, pos, mat):
    """mat [n, w] uint8 -> arena[pos_i + j]"""
    n, w = mat.shape
    if n == 0 or w == 0:
        return
    idx = pos[:, None] + np.arange(w, dtype=np.int64)[None, :]
    arena[idx.ravel()] = mat.ravel()


def point_blobs(pk, version, legend_hex, rng_seed=SEED):
    """Points-layer feature blobs (the shape of tests/data/points: ~85-151 B).

    values = [geom POINT (ext 'G', 29-byte GPKG), t50_fid int32, name_ascii str|None,
              macronated 'N'|'Y', name str|None]; content is a function of (pk, version)."""
    pk = np.asarray(pk, np.int64)
    n = pk.shape[0]
    h = splitmix64(pk.view(np.uint64) ^ (np.asarray(version, np.uint64) << np.uint64(48)) ^ np.uint64(rng_seed))
    h2 = splitmix64(h)
    x = 166.0 + (h & np.uint64(0xFFFFFF)).astype(np.float64) / float(1 << 24) * 12.0
    y = -47.0 + ((h >> np.uint64(24)) & np.uint64(0xFFFFFF)).astype(np.float64) / float(1 << 24) * 13.0
    t50 = (h2 & np.uint64(0x7FFFFFFF)).astype(np.uint64)
    kind = ((h2 >> np.uint64(40)) % np.uint64(4)).astype(np.int64)  # 0 nil, 1..3 name lengths 8/16/24
    lens = np.array([0, 8, 16, 24], np.int64)[kind]
    mac = np.where(((h2 >> np.uint64(50)) & np.uint64(1)) == 1, ord("Y"), ord("N")).astype(np.uint8)
    # layout: 92 d9 28 <40> 95 | c7 1d 47 <29 gpkg> | ce <4> | str | a1 <1> | str
    fixed = 3 + 40 + 1 + 32 + 5 + 2
    strlen = np.where(kind == 0, 1, 1 + lens)
    blen = fixed + 2 * strlen
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(blen)
    if n == 0:
        return np.zeros(0, np.uint8), off
    W = int(blen.max())
    mat = np.zeros((n, W), np.uint8)  # one padded row per blob, compacted at the end
    mat[:, 0:44] = np.frombuffer(b"\x92\xd9\x28" + legend_hex.encode() + b"\x95", np.uint8)
    mat[:, 44:60] = np.frombuffer(b"\xc7\x1d\x47GP\x00\x01\xe6\x10\x00\x00\x01\x01\x00\x00\x00", np.uint8)
    mat[:, 60:76] = np.stack([x, y], 1).astype("<f8").view(np.uint8).reshape(n, 16)
    mat[:, 76] = 0xCE
    mat[:, 77:81] = t50.astype(">u4").view(np.uint8).reshape(n, 4)
    pool = (splitmix64(np.arange(4096 * 24, dtype=np.uint64) ^ np.uint64(rng_seed)) % np.uint64(26)).astype(np.uint8)
    pool = pool.reshape(4096, 24) + np.uint8(ord("a"))
    chars = pool[((h2 >> np.uint64(8)) & np.uint64(4095)).astype(np.int64)]
    for k in range(4):
        sel = np.nonzero(kind == k)[0]
        if sel.size == 0:
            continue
        L = int((0, 8, 16, 24)[k])
        c = 81
        for field in range(2):  # name_ascii, (macronated), name
            if k == 0:
                mat[sel, c] = 0xC0
            else:
                mat[sel, c] = 0xA0 | L
                mat[sel, c + 1:c + 1 + L] = chars[sel, :L]
            c += 1 + L
            if field == 0:
                mat[sel, c] = 0xA1
                mat[sel, c + 1] = mac[sel]
                c += 2
    arena = mat[np.arange(W)[None, :] < blen[:, None]]
    return arena, off


def points_layer(n, frac_update=0.01, frac_delete=0.01, frac_insert=0.01, seed=SEED, pk0=0):
    """C2: n int-PK points (pks pk0..pk0+n-1); seeded 1% updates / deletes / inserts.  Both sides
    in git tree (= key) order."""
    rng = np.random.default_rng(seed)
    schema = Schema.from_column_dicts(POINT_SCHEMA)
    legend = Legend(["c-fid"], [c["id"] for c in POINT_SCHEMA[1:]])
    lh = legend.hexhash()
    n_upd, n_del, n_ins = int(n * frac_update), int(n * frac_delete), int(n * frac_insert)
    perm = rng.permutation(n)  # edits picked by pk (index = pk - pk0)
    tgt_ver = np.zeros(n + n_ins, np.uint64)
    tgt_ver[perm[:n_upd]] = 1
    tgt_ver[n:] = 2
    keep = np.ones(n + n_ins, bool)
    keep[perm[n_upd:n_upd + n_del]] = False
    allp = walkkey.walk_order_range(pk0, pk0 + n + n_ins)  # every pk of either side, walk order
    j = allp - pk0
    pks = allp[j < n]
    t_pk = allp[keep[j]]
    t_ver = tgt_ver[t_pk - pk0]
    base_ver = np.zeros(n, np.uint64)
    base = packing.PackedSide(key=walkkey.int_keys(pks), oid=synth_oids(pks, base_ver), key_mode=0,
                              order=np.arange(n, dtype=np.int64), encoding=packing.INT_PK_ENCODING)
    target = packing.PackedSide(key=walkkey.int_keys(t_pk), oid=synth_oids(t_pk, t_ver), key_mode=0,
                                order=np.arange(t_pk.shape[0], dtype=np.int64), encoding=packing.INT_PK_ENCODING)
    bb = point_blobs(pks, base_ver, lh)
    tb = point_blobs(t_pk, t_ver, lh)
    return Layer(base, target, bb, tb, schema, {lh: legend}, n_ins, n_upd, n_del)


def polygon_blobs(pk, gver, aver, legend_hex, rng_seed=SEED, same_len=0.0):
    """Polygons-layer feature blobs (the shape of tests/data/polygons: 245-582 B).

    values = [geom MULTIPOLYGON (ext 'G': 8-B GPKG header, XY envelope, one ring of 5-24 points),
              date_adjusted str (20-char timestamp), survey_reference str|None, adjusted_nodes int32].
    The geometry is a function of (pk, gver), the attributes of (pk, aver), so a geometry edit and an
    attribute edit change different fields.  Canonical (smallest-width) msgpack headers throughout.
    ``same_len``: the fraction of features (by a hash of the pk) whose ring size depends on the pk
    only, so a geometry edit moves vertices and keeps the blob's length (0: every edit redraws it)."""
    pk = np.asarray(pk, np.int64)
    n = pk.shape[0]
    u = pk.view(np.uint64)
    hg = splitmix64(u ^ (np.asarray(gver, np.uint64) << np.uint64(48)) ^ np.uint64(rng_seed ^ 0x6706))
    ha = splitmix64(u ^ (np.asarray(aver, np.uint64) << np.uint64(48)) ^ np.uint64(rng_seed ^ 0xA77A))
    ha2 = splitmix64(ha)
    hsize = hg
    if same_len > 0:
        hp = splitmix64(u ^ np.uint64(rng_seed ^ 0x5E1E))
        hsize = np.where(hp % np.uint64(1000) < np.uint64(int(round(same_len * 1000))), hp, hg)
    npts = (5 + (hsize >> np.uint64(58)) % np.uint64(20)).astype(np.int64)  # 5..24 ring points
    glen = 8 + 32 + 22 + 16 * npts  # GPKG header + envelope + MULTIPOLYGON/POLYGON/ring headers + xy
    ehdr = np.where(glen <= 255, 3, 4)  # c7 len 47 | c8 len16 47
    has_ref = ((ha2 >> np.uint64(7)) & np.uint64(3)) != 0
    rlen = (8 + (ha2 >> np.uint64(20)) % np.uint64(9)).astype(np.int64)  # 8..16 chars
    reflen = np.where(has_ref, 1 + rlen, 1)
    blen = 3 + 40 + 1 + ehdr + glen + 21 + reflen + 5
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(blen, out=off[1:])
    if n == 0:
        return np.zeros(0, np.uint8), off
    W = int(blen.max()) + 16  # slack: a group's 16 reference chars are written before its length cut
    mat = np.zeros((n, W), np.uint8)
    lon = -180.0 + (hg & np.uint64(0xFFFFFF)).astype(np.float64) / float(1 << 24) * 359.0
    lat = -85.0 + ((hg >> np.uint64(24)) & np.uint64(0xFFFFFF)).astype(np.float64) / float(1 << 24) * 169.0
    w = 1e-4 * (1 + ((hg >> np.uint64(48)) & np.uint64(0x3FF)).astype(np.float64))
    # date_adjusted: "20YY-MM-DDThh:mm:ssZ" from the attribute hash
    yy = 2000 + (ha % np.uint64(25)).astype(np.int64)
    mo = 1 + ((ha >> np.uint64(8)) % np.uint64(12)).astype(np.int64)
    dd = 1 + ((ha >> np.uint64(16)) % np.uint64(28)).astype(np.int64)
    hh = ((ha >> np.uint64(24)) % np.uint64(24)).astype(np.int64)
    mi = ((ha >> np.uint64(32)) % np.uint64(60)).astype(np.int64)
    ss = ((ha >> np.uint64(40)) % np.uint64(60)).astype(np.int64)
    dig = lambda v, w_: [(v // 10 ** (w_ - 1 - j)) % 10 + 48 for j in range(w_)]
    date = np.stack(dig(yy, 4) + [np.full(n, 45)] + dig(mo, 2) + [np.full(n, 45)] + dig(dd, 2) + [np.full(n, 84)] +
                    dig(hh, 2) + [np.full(n, 58)] + dig(mi, 2) + [np.full(n, 58)] + dig(ss, 2) + [np.full(n, 90)],
                    1).astype(np.uint8)
    chars = (splitmix64(ha2[:, None] ^ np.arange(16, dtype=np.uint64)[None, :]) % np.uint64(26)).astype(np.uint8) + 65
    nodes = ((ha2 >> np.uint64(32)) & np.uint64(0xFFFFF)).astype(">u4").view(np.uint8).reshape(n, 4)
    legend_row = np.frombuffer(b"\x92\xd9\x28" + legend_hex.encode() + b"\x94", np.uint8)
    wkb = np.frombuffer(b"GP\x00\x03" + np.array([4326], "<i4").tobytes(), np.uint8)
    wkb2 = np.frombuffer(b"\x01\x06\x00\x00\x00\x01\x00\x00\x00\x01\x03\x00\x00\x00\x01\x00\x00\x00", np.uint8)
    # fixed layout per ring size: slice writes per group, the variable tail (survey_reference,
    # adjusted_nodes) by a 5-column gather
    for npv in np.unique(npts):
        sel = np.nonzero(npts == npv)[0]
        m = sel.size
        gl = 62 + 16 * int(npv)
        eh = 3 if gl <= 255 else 4
        g0 = 44 + eh
        sub = np.zeros((m, W), np.uint8)
        sub[:, 0:44] = legend_row
        sub[:, 44] = 0xC7 if eh == 3 else 0xC8
        if eh == 3:
            sub[:, 45] = gl
        else:
            sub[:, 45], sub[:, 46] = gl >> 8, gl & 0xFF
        sub[:, g0 - 1] = 0x47
        sub[:, g0:g0 + 8] = wkb
        lo, la, ww = lon[sel], lat[sel], w[sel]
        sub[:, g0 + 8:g0 + 40] = np.stack([lo, lo + ww, la, la + ww], 1).astype("<f8").view(np.uint8).reshape(m, 32)
        sub[:, g0 + 40:g0 + 58] = wkb2
        sub[:, g0 + 58:g0 + 62] = np.array([npv], "<u4").view(np.uint8)
        k = np.arange(2 * int(npv), dtype=np.float64)[None, :]
        xy = np.where(k % 2 == 0, lo[:, None] + ww[:, None] * ((k * 0.37) % 1.0),
                      la[:, None] + ww[:, None] * ((k * 0.61) % 1.0))
        sub[:, g0 + 62:g0 + gl] = xy.astype("<f8").view(np.uint8).reshape(m, 16 * int(npv))
        c = g0 + gl
        sub[:, c] = 0xB4
        sub[:, c + 1:c + 21] = date[sel]
        c += 21
        hr, rl = has_ref[sel], rlen[sel]
        sub[:, c] = np.where(hr, 0xA0 | rl, 0xC0).astype(np.uint8)
        sub[:, c + 1:c + 17] = chars[sel]
        ci = c + np.where(hr, 1 + rl, 1)  # adjusted_nodes: ce <u32 BE>
        cols = ci[:, None] + np.arange(5)[None, :]
        vals = np.concatenate([np.full((m, 1), 0xCE, np.uint8), nodes[sel]], 1)
        np.put_along_axis(sub, cols, vals, axis=1)
        mat[sel] = sub
    arena = mat[np.arange(W)[None, :] < blen[:, None]]
    return arena, off


def _sparse_arena(n, sel, data, off_sel):
    """arena holding blobs only for entries `sel` (ascending); every other entry is zero-length"""
    lens = np.zeros(n, np.uint64)
    lens[sel] = off_sel[1:] - off_sel[:-1]
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    return data, off


C3_SEED = 0x43334C59  # edit selection of the C3 layer (a hash of the pk: any pk range is generable alone)


def c3_plan(pk, n, seed=C3_SEED):
    """Edit class of base pks (0 unchanged, 1 geometry update, 2 attribute update, 3 delete): a seeded
    hash of the pk, 4 % / 4 % / 1 % in expectation (10 % edits with the 1 % inserts)."""
    h = splitmix64(np.asarray(pk, np.int64).view(np.uint64) ^ np.uint64(seed)) % np.uint64(10000)
    return np.where(h < 400, 1, np.where(h < 800, 2, np.where(h < 900, 3, 0))).astype(np.uint8)


def polygons_layer(n, seed=SEED, shard=None, batch=1 << 20, delta_blobs=False, same_len=0.0):
    """C3: n int-PK MULTIPOLYGON features (pks 0..n-1) and n // 100 inserts (pks n..), 10 % edits =
    4 % geometry updates + 4 % attribute updates + 1 % deletes + 1 % inserts, edits
    picked by a hash of the pk (c3_plan).  Both sides in git tree (= key) order.

    ``shard=(rank, world)``: generate only that bucket-range shard of the same layer — a contiguous
    run of the tree walk (shard_rank_range), as bench.py --gpus N splits it.
    Feature blobs are materialised for the updated features only (both versions): the diff reads no
    other blob — classification needs only keys and OIDs — so every other entry has a zero-length
    blob in the arena.  ``delta_blobs``: also the deleted features' base blobs and the inserted
    features' target blobs (what a spatially filtered diff reads: C5).  ``same_len``: the fraction of
    features whose geometry edits keep the blob length (vertex moves; polygon_blobs)."""
    schema = Schema.from_column_dicts(POLYGON_SCHEMA)
    legend = Legend(["p-fid"], [c["id"] for c in POLYGON_SCHEMA[1:]])
    lh = legend.hexhash()
    n_ins = n // 100
    n_pks = n + n_ins
    r_lo, r_hi = shard_rank_range(*shard, n_pks) if shard else (0, 1 << 24)
    allp = walkkey.walk_order_pks(n_pks, r_lo, r_hi)  # every pk of either side in the shard, walk order
    is_b = allp < n
    plan = np.zeros(allp.shape[0], np.uint8)
    plan[is_b] = c3_plan(allp[is_b], n)
    in_t = ~is_b | (plan != 3)
    bpos = np.cumsum(is_b) - 1  # base / target index of each walk position
    tpos = np.cumsum(in_t) - 1
    pks, t_pk = allp[is_b], allp[in_t]
    gver = (plan == 1).astype(np.uint64)
    aver = (plan == 2).astype(np.uint64)
    ver_t = np.where(is_b, gver | (aver << np.uint64(1)), np.uint64(4))[in_t]
    base = packing.PackedSide(key=walkkey.int_keys(pks), oid=synth_oids(pks, np.zeros(pks.shape[0], np.uint64)),
                              key_mode=0, order=np.arange(pks.shape[0], dtype=np.int64), encoding=packing.INT_PK_ENCODING)
    target = packing.PackedSide(key=walkkey.int_keys(t_pk), oid=synth_oids(t_pk, ver_t), key_mode=0,
                                order=np.arange(t_pk.shape[0], dtype=np.int64), encoding=packing.INT_PK_ENCODING)
    upd = (plan == 1) | (plan == 2)

    def blobs(idx_pk, gv, av):
        parts, offs = [], [np.zeros(1, np.uint64)]
        for s in range(0, idx_pk.shape[0], batch):
            d, o = polygon_blobs(idx_pk[s:s + batch], gv[s:s + batch], av[s:s + batch], lh, seed, same_len)
            parts.append(d)
            offs.append(o[1:] + offs[-1][-1])
        return (np.concatenate(parts) if parts else np.zeros(0, np.uint8)), np.concatenate(offs)

    bw = np.nonzero(upd | (plan == 3) if delta_blobs else upd)[0]  # walk positions with a base blob
    tw = np.nonzero(upd | ~is_b if delta_blobs else upd)[0]  # ... with a target blob
    bd, bo = blobs(allp[bw], np.zeros(bw.size, np.uint64), np.zeros(bw.size, np.uint64))
    td, to = blobs(allp[tw], gver[tw], aver[tw])
    bb = _sparse_arena(pks.shape[0], bpos[bw], bd, bo)
    tb = _sparse_arena(t_pk.shape[0], tpos[tw], td, to)
    return Layer(base, target, bb, tb, schema, {lh: legend}, int(np.count_nonzero(~is_b)), int(np.count_nonzero(upd)),
                 int(np.count_nonzero(plan == 3)))


def shard_rank_range(rank, world, n_pks):
    """[lo, hi) of rank's bucket-range shard of a layer with int pks 0..n_pks-1, in rank-mapped bucket
    space (the key's top 24 bits): a contiguous run of the tree walk holding about n_pks / world pks
    in whole leaf trees.  Shards in rank order tile the walk."""
    if n_pks > (1 << 30):
        raise ValueError("synthetic layer exceeds one bucket wrap (2**30 pks)")
    nb = (n_pks + 63) // 64
    rk = np.sort(walkkey.rank_digits(np.arange(nb, dtype=np.uint64)))
    a, b = nb * rank // world, nb * (rank + 1) // world
    lo = 0 if rank == 0 else int(rk[a])
    hi = (1 << 24) if rank == world - 1 else int(rk[b])
    return lo, hi


_B64 = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_", np.uint8)


def int_pk_paths(pk):
    """IntPathEncoder relative paths (kart/dataset3_paths.py:292-299) of non-negative int pks below
    2**32, vectorised: 'c/c/c/c/' + urlsafe_b64(msgpack([pk])) -> (uint8 arena, uint64 off[n+1])."""
    pk = np.asarray(pk, np.int64)
    n = pk.shape[0]
    if n and (pk.min() < 0 or pk.max() >= (1 << 32)):
        raise ValueError("int_pk_paths: pks in [0, 2**32)")
    # msgpack([pk]): 0x91 + positive fixint / uint8 / uint16 / uint32
    w = np.where(pk < 128, 0, np.where(pk < 256, 1, np.where(pk < 65536, 2, 4)))
    mlen = 2 + w
    mp = np.zeros((n, 6), np.uint8)
    mp[:, 0] = 0x91
    mp[:, 1] = np.where(w == 0, pk, np.where(w == 1, 0xCC, np.where(w == 2, 0xCD, 0xCE))).astype(np.uint8)
    for k in range(4):  # big-endian payload bytes at 2 .. 2+w
        shift = 8 * (w - 1 - k)
        byte = (pk >> np.maximum(shift, 0)) & 0xFF
        mp[:, 2 + k] = np.where(k < w, byte, 0).astype(np.uint8)
    # base64 of mlen bytes: 4 chars per 3-byte group, '=' padded
    blen = 4 * ((mlen + 2) // 3)
    g = mp.reshape(n, 2, 3).astype(np.uint32)
    v = g[:, :, 0] << 16 | g[:, :, 1] << 8 | g[:, :, 2]
    ch = _B64[np.stack([(v >> 18) & 63, (v >> 12) & 63, (v >> 6) & 63, v & 63], 2).reshape(n, 8)]
    pad = blen - (4 * mlen + 2) // 3  # '=' count: (3 - mlen % 3) % 3
    pos = np.arange(8)[None, :]
    ch = np.where(pos >= (blen - pad)[:, None], ord("="), ch).astype(np.uint8)
    bucket = (pk // 64) % (1 << 24)
    tree = np.stack([_B64[(bucket >> (18 - 6 * k)) & 63] for k in range(4)], 1)
    rows = np.zeros((n, 16), np.uint8)
    rows[:, 0:8:2] = tree
    rows[:, 1:8:2] = ord("/")
    rows[:, 8:] = ch
    plen = 8 + blen
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(plen, out=off[1:])
    arena = rows[np.arange(16)[None, :] < plen[:, None]]
    return arena, off


def walk_perm(keys):
    """perm such that keys[perm] is ascending: for a side in walk order this is the identity, except
    where a leaf tree mixes pk wraps (the fallback sort's case); tests use it on shuffled sides"""
    return np.argsort(np.asarray(keys, np.uint64), kind="stable")


def _int_keys(pk):
    """vectorised KD_KEY_INT (kart_amd/walkkey.py; same keys as kd_pack_int_keys)"""
    return walkkey.int_keys(pk)


# ---------------------------------------------------------------------------------------------
# C5: GPKG geometry blobs of a spatially filtered layer
C5_FILTER = (170.0, 180.0, -50.0, -30.0)  # (min-x, max-x, min-y, max-y) of the spatial filter


def geometry_layer(n, seed=SEED, frac_point=0.3):
    """n GPKG geometry blobs, EPSG:4326, as one arena (uint8 data, uint64 off[n+1]).

    30 % points (8-B header + 21-B WKB, no stored envelope), 70 % MULTIPOLYGONs (8-B header + 32-B
    XY envelope + WKB body, 245-582 B in total: polygon bodies are zero-filled — only the header,
    envelope and WKB type are ever read on this path).  lon U[-180, 180), lat U[-85, 85]; polygon
    widths log-U[1e-6, 10] degrees; 1 % straddle +180; 0.1 % >= 180 degrees wide (no index
    envelope); 0.1 % EMPTY points; 1 % of polygons start exactly on the filter's east edge."""
    rng = np.random.default_rng(seed)
    is_pt = rng.random(n) < frac_point
    npt, npoly = int(is_pt.sum()), int(n - is_pt.sum())
    size = np.where(is_pt, 29, rng.integers(245, 583, size=n)).astype(np.uint64)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(size, out=off[1:])
    data = np.zeros(int(off[-1]), np.uint8)
    start = off[:-1]
    lon = rng.uniform(-180.0, 180.0, n)
    lat = rng.uniform(-85.0, 85.0, n)

    # points: GP 00 flags srs | 01 01000000 x y
    pi = np.nonzero(is_pt)[0]
    rec = np.zeros((npt, 29), np.uint8)
    rec[:, 0], rec[:, 1], rec[:, 2] = ord("G"), ord("P"), 0
    empty = rng.random(npt) < 0.001
    rec[:, 3] = np.where(empty, 0x11, 0x01)
    rec[:, 4:8] = np.array([4326], "<i4").view(np.uint8)
    rec[:, 8] = 1
    rec[:, 9:13] = np.array([1], "<u4").view(np.uint8)
    xy = np.stack([lon[pi], lat[pi]], 1)
    xy[empty] = np.nan
    rec[:, 13:29] = xy.astype("<f8").view(np.uint8).reshape(npt, 16)
    data[(start[pi, None] + np.arange(29, dtype=np.uint64)[None, :]).ravel()] = rec.ravel()

    # polygons: GP 00 03 srs | minx maxx miny maxy | 01 06000000 01000000 ...
    qi = np.nonzero(~is_pt)[0]
    w = 10.0 ** rng.uniform(-6, 1, npoly)
    h = 10.0 ** rng.uniform(-6, 1, npoly)
    minx, miny = lon[qi], lat[qi]
    u = rng.random(npoly)
    straddle = u < 0.01
    minx = np.where(straddle, 180.0 - w / 2, minx)
    wide = (u >= 0.01) & (u < 0.011)
    w = np.where(wide, 180.0 + 10.0 * rng.random(npoly), w)
    edge = (u >= 0.011) & (u < 0.021)
    minx = np.where(edge, C5_FILTER[1], minx)
    env = np.stack([minx, minx + w, miny, np.minimum(miny + h, 90.0)], 1)
    rec = np.zeros((npoly, 49), np.uint8)
    rec[:, 0], rec[:, 1], rec[:, 2], rec[:, 3] = ord("G"), ord("P"), 0, 0x03
    rec[:, 4:8] = np.array([4326], "<i4").view(np.uint8)
    rec[:, 8:40] = env.astype("<f8").view(np.uint8).reshape(npoly, 32)
    rec[:, 40] = 1
    rec[:, 41:45] = np.array([6], "<u4").view(np.uint8)
    rec[:, 45:49] = np.array([1], "<u4").view(np.uint8)
    data[(start[qi, None] + np.arange(49, dtype=np.uint64)[None, :]).ravel()] = rec.ravel()
    return data, off, is_pt


# ---------------------------------------------------------------------------------------------
# C5 as SURVEY §8(d) defines it: the filtered diff of a 100M-feature layer of mixed geometries
MIXED_SCHEMA = [
    {"id": "g-fid", "name": "id", "dataType": "integer", "primaryKeyIndex": 0, "size": 64},
    {"id": "g-geom", "name": "geom", "dataType": "geometry", "geometryType": "GEOMETRY", "geometryCRS": "EPSG:4326"},
    {"id": "g-date", "name": "date_adjusted", "dataType": "timestamp"},
    {"id": "g-sid", "name": "survey_reference", "dataType": "text", "length": 50},
    {"id": "g-adj", "name": "adjusted_nodes", "dataType": "integer", "size": 32},
]


def _concat_segments(segs, n):
    """rows of variable-length byte segments -> (arena, off[n+1]): segs = [(mat [n, W], len [n]), ...]"""
    lens = np.zeros(n, np.int64)
    for _, ln in segs:
        lens += ln
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    arena = np.zeros(int(off[-1]), np.uint8)
    pos = off[:-1].astype(np.int64).copy()
    for mat, ln in segs:
        W = mat.shape[1]
        if W:
            cols = np.arange(W, dtype=np.int64)[None, :]
            m = cols < ln[:, None]
            arena[(pos[:, None] + cols)[m]] = mat[m]
        pos += ln
    return arena, off


def mixed_blobs(pk, gver, aver, legend_hex, rng_seed=SEED):
    """C5 feature blobs: values = [geom, date_adjusted, survey_reference, adjusted_nodes]; the
    geometry (a function of (pk, gver)) is, by a hash of the pk, a point (30 %: 8-B GPKG header + 21-B
    WKB, no stored envelope; 0.1 % of them EMPTY) or a MULTIPOLYGON (8-B header + XY envelope + a
    5..24-point ring; 0.2 % carry an XYZ envelope, which the geometry heads cannot decide: the filter's
    blob fallback).  lon U[-180, 180), lat U[-85, 85]; polygon widths and heights log-U[1e-6, 10]
    degrees; 1 % straddle +180, 0.1 % are >= 180 degrees wide, 1 % start exactly on the filter's east
    edge."""
    pk = np.asarray(pk, np.int64)
    n = pk.shape[0]
    u = pk.view(np.uint64)
    hk = splitmix64(u ^ np.uint64(rng_seed ^ 0xC5C5))  # per feature, fixed across versions
    hg = splitmix64(u ^ (np.asarray(gver, np.uint64) << np.uint64(48)) ^ np.uint64(rng_seed ^ 0x6706))
    hg2 = splitmix64(hg)
    ha = splitmix64(u ^ (np.asarray(aver, np.uint64) << np.uint64(48)) ^ np.uint64(rng_seed ^ 0xA77A))
    ha2 = splitmix64(ha)
    is_pt = (hk % np.uint64(1000)) < np.uint64(300)
    f = lambda h, sh: ((h >> np.uint64(sh)) & np.uint64(0xFFFFFF)).astype(np.float64) / float(1 << 24)
    lon = -180.0 + f(hg, 0) * 360.0
    lat = -85.0 + f(hg, 24) * 170.0
    w = 10.0 ** (-6.0 + 7.0 * f(hg2, 0))
    hh = 10.0 ** (-6.0 + 7.0 * f(hg2, 24))
    cls = (hg2 >> np.uint64(48)) % np.uint64(10000)
    straddle, wide = cls < 100, (cls >= 100) & (cls < 110)
    edge, xyz = (cls >= 110) & (cls < 210), (cls >= 210) & (cls < 230)
    empty = is_pt & ((hk >> np.uint64(20)) % np.uint64(1000) == 0)
    minx = np.where(straddle, 180.0 - w / 2, np.where(edge, C5_FILTER[1], lon))
    w = np.where(wide, 180.0 + 10.0 * f(hg2, 8), w)
    env = np.stack([minx, minx + w, lat, np.minimum(lat + hh, 90.0)], 1)
    npts = (5 + (hg >> np.uint64(58)) % np.uint64(20)).astype(np.int64)
    # geometry value: GPKG header [+ envelope] + WKB
    elen = np.where(is_pt, 0, np.where(xyz, 48, 32))
    glen = np.where(is_pt, 29, 8 + elen + 22 + 16 * npts)
    G = np.zeros((n, 8 + 48 + 22), np.uint8)  # header + envelope + WKB head (the ring's xy follow)
    G[:, 0], G[:, 1] = ord("G"), ord("P")
    G[:, 3] = np.where(is_pt, np.where(empty, 0x11, 0x01), np.where(xyz, 0x05, 0x03))
    G[:, 4:8] = np.array([4326], "<i4").view(np.uint8)
    pxy = np.stack([lon, lat], 1)
    pxy[empty] = np.nan
    ptw = np.concatenate([np.frombuffer(b"\x01\x01\x00\x00\x00", np.uint8)[None, :].repeat(n, 0),
                          pxy.astype("<f8").view(np.uint8).reshape(n, 16)], 1)
    envb = env.astype("<f8").view(np.uint8).reshape(n, 32)
    zb = np.stack([np.zeros(n), np.ones(n)], 1).astype("<f8").view(np.uint8).reshape(n, 16)
    G[:, 8:40] = np.where(is_pt[:, None], 0, envb)
    G[:, 40:56] = np.where(xyz[:, None], zb, 0)
    wk = np.zeros((n, 22), np.uint8)
    wk[:, :18] = np.frombuffer(b"\x01\x06\x00\x00\x00\x01\x00\x00\x00\x01\x03\x00\x00\x00\x01\x00\x00\x00", np.uint8)
    wk[:, 18:22] = npts.astype("<u4").view(np.uint8).reshape(n, 4)
    # points: the WKB right after the 8-B header; polygons: after the envelope
    head = np.zeros((n, 78), np.uint8)
    head[:, :8] = G[:, :8]
    head[:, 8:29] = np.where(is_pt[:, None], ptw, 0)
    pe = (8 + elen)
    cols = np.arange(78)[None, :]
    for k in range(48):  # polygon envelope bytes
        sel = ~is_pt & (k < elen)
        head[sel, 8 + k] = G[sel, 8 + k]
    for k in range(22):
        sel = ~is_pt
        head[np.nonzero(sel)[0], (pe[sel] + k)] = wk[sel, k]
    hlen = np.where(is_pt, 29, pe + 22)
    maxp = int(npts.max()) if n else 0
    kk = np.arange(2 * maxp, dtype=np.float64)[None, :]
    ring = np.where(kk % 2 == 0, env[:, 0:1] + (env[:, 1:2] - env[:, 0:1]) * ((kk * 0.37) % 1.0),
                    env[:, 2:3] + (env[:, 3:4] - env[:, 2:3]) * ((kk * 0.61) % 1.0))
    ringb = ring.astype("<f8").view(np.uint8).reshape(n, 16 * maxp)
    rlen = np.where(is_pt, 0, 16 * npts)
    ext = np.zeros((n, 4), np.uint8)
    small = glen <= 255
    ext[:, 0] = np.where(small, 0xC7, 0xC8)
    ext[:, 1] = np.where(small, glen, glen >> 8).astype(np.uint8)
    ext[:, 2] = np.where(small, 0x47, glen & 0xFF).astype(np.uint8)
    ext[:, 3] = 0x47
    extlen = np.where(small, 3, 4)
    # attributes (as polygon_blobs): date string, survey reference str|nil, adjusted_nodes u32
    yy = 2000 + (ha % np.uint64(25)).astype(np.int64)
    mo = 1 + ((ha >> np.uint64(8)) % np.uint64(12)).astype(np.int64)
    dd = 1 + ((ha >> np.uint64(16)) % np.uint64(28)).astype(np.int64)
    dig = lambda v, w_: [(v // 10 ** (w_ - 1 - j)) % 10 + 48 for j in range(w_)]
    date = np.stack([np.full(n, 0xB4)] + dig(yy, 4) + [np.full(n, 45)] + dig(mo, 2) + [np.full(n, 45)] + dig(dd, 2) +
                    [np.full(n, ord(c)) for c in "T12:00:00Z"], 1).astype(np.uint8)
    has_ref = ((ha2 >> np.uint64(7)) & np.uint64(3)) != 0
    rl = (8 + (ha2 >> np.uint64(20)) % np.uint64(9)).astype(np.int64)
    ref = np.zeros((n, 17), np.uint8)
    ref[:, 0] = np.where(has_ref, 0xA0 | rl, 0xC0)
    ref[:, 1:] = (splitmix64(ha2[:, None] ^ np.arange(16, dtype=np.uint64)[None, :]) % np.uint64(26)).astype(np.uint8) + 65
    reflen = np.where(has_ref, 1 + rl, 1)
    nodes = np.concatenate([np.full((n, 1), 0xCE, np.uint8),
                            ((ha2 >> np.uint64(32)) & np.uint64(0xFFFFF)).astype(">u4").view(np.uint8).reshape(n, 4)], 1)
    lead = np.frombuffer(b"\x92\xd9\x28" + legend_hex.encode() + b"\x94", np.uint8)[None, :].repeat(n, 0)
    return _concat_segments([(lead, np.full(n, 44)), (ext, extlen), (head, hlen), (ringb, rlen),
                             (date, np.full(n, 21)), (ref, reflen), (nodes, np.full(n, 5))], n)


def c5_layer(n, seed=SEED, shard=None, batch=1 << 20):
    """C5: n int-PK features of mixed geometries (mixed_blobs) and n // 100 inserts, the C3 edit plan
    (4 % geometry + 4 % attribute updates, 1 % deletes, 1 % inserts); both sides in git tree (= key)
    order; blobs materialised for every delta's old and new version (what the filtered diff reads)."""
    schema = Schema.from_column_dicts(MIXED_SCHEMA)
    legend = Legend(["g-fid"], [c["id"] for c in MIXED_SCHEMA[1:]])
    lh = legend.hexhash()
    n_ins = n // 100
    n_pks = n + n_ins
    r_lo, r_hi = shard_rank_range(*shard, n_pks) if shard else (0, 1 << 24)
    allp = walkkey.walk_order_pks(n_pks, r_lo, r_hi)
    is_b = allp < n
    plan = np.zeros(allp.shape[0], np.uint8)
    plan[is_b] = c3_plan(allp[is_b], n)
    in_t = ~is_b | (plan != 3)
    bpos, tpos = np.cumsum(is_b) - 1, np.cumsum(in_t) - 1
    pks, t_pk = allp[is_b], allp[in_t]
    gver = (plan == 1).astype(np.uint64)
    aver = (plan == 2).astype(np.uint64)
    ver_t = np.where(is_b, gver | (aver << np.uint64(1)), np.uint64(4))[in_t]
    base = packing.PackedSide(key=walkkey.int_keys(pks), oid=synth_oids(pks, np.zeros(pks.shape[0], np.uint64)),
                              key_mode=0, order=np.arange(pks.shape[0], dtype=np.int64), encoding=packing.INT_PK_ENCODING)
    target = packing.PackedSide(key=walkkey.int_keys(t_pk), oid=synth_oids(t_pk, ver_t), key_mode=0,
                                order=np.arange(t_pk.shape[0], dtype=np.int64), encoding=packing.INT_PK_ENCODING)
    upd = (plan == 1) | (plan == 2)

    def blobs(idx_pk, gv, av):
        parts, offs = [], [np.zeros(1, np.uint64)]
        for s in range(0, idx_pk.shape[0], batch):
            d, o = mixed_blobs(idx_pk[s:s + batch], gv[s:s + batch], av[s:s + batch], lh, seed)
            parts.append(d)
            offs.append(o[1:] + offs[-1][-1])
        return (np.concatenate(parts) if parts else np.zeros(0, np.uint8)), np.concatenate(offs)

    bw = np.nonzero(upd | (plan == 3))[0]
    tw = np.nonzero(upd | ~is_b)[0]
    bd, bo = blobs(allp[bw], np.zeros(bw.size, np.uint64), np.zeros(bw.size, np.uint64))
    td, to = blobs(allp[tw], gver[tw], aver[tw])
    bb = _sparse_arena(pks.shape[0], bpos[bw], bd, bo)
    tb = _sparse_arena(t_pk.shape[0], tpos[tw], td, to)
    return Layer(base, target, bb, tb, schema, {lh: legend}, int(np.count_nonzero(~is_b)), int(np.count_nonzero(upd)),
                 int(np.count_nonzero(plan == 3)))


# ---------------------------------------------------------------------------------------------
# C4: string-PK attribute table, three-way merge (ancestor / ours / theirs)
# ---------------------------------------------------------------------------------------------
@dataclass
class Merge3Layer:
    ancestor: packing.PackedSide
    ours: packing.PackedSide
    theirs: packing.PackedSide
    n_conflict: int  # libgit2 rule over the generator's plan (o == t -> o; a == o -> t; a == t -> o)
    plan: dict = None  # the edit mix as generated (counts per kind)


PK_W = 36  # text pks up to 24 characters, 3 of them up to 4 B: 33 bytes (36 with slack)
PATH_W = 8 + 52  # 'c/c/c/c/' + the longest filename (4 * ceil((3 + PK_W) / 3))
_SYNTH = None


def _synth_lib():
    """libkdsynth.so (kart_amd/csrc/kd_synth.cpp): host-only generator helpers, not the product ABI"""
    global _SYNTH
    if _SYNTH is None:
        import ctypes

        L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkdsynth.so"))
        P, U, I, D = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_double
        L.kds_text_pks.argtypes = [P, U, U, I, I, D, P, I, P, I]
        L.kds_text_pk_paths.argtypes = [P, P, U, I, P, I, P, I]
        L.kds_walk_order.argtypes = [P, U, I, P, I]
        L.kds_gather_paths.argtypes = [P, I, P, P, U, P, P, I]
        L.kds_gather_paths.restype = None
        _SYNTH = L
    return _SYNTH


def _threads():
    return max(1, min(16, os.cpu_count() or 1))


def _p(a):
    return a.ctypes.data_as(__import__("ctypes").c_void_p)


def text_pks(ids, seed=SEED, lmin=12, lmax=24, p_mb=0.05):
    """The C4 table's text pks: 12–24 characters, 5 % of the rows holding 1–3
    multibyte UTF-8 characters (2-, 3- and 4-byte).  Characters 0–4 are a bijective base-62
    scramble of the row id (pks are distinct), the rest seeded filler (kds_text_pks).
    -> (UTF-8 bytes [n, PK_W] zero-padded, byte lengths [n])"""
    ids = np.ascontiguousarray(ids, np.int64)
    n = ids.size
    out = np.empty((n, PK_W), np.uint8)
    nb = np.empty(n, np.int64)
    if _synth_lib().kds_text_pks(_p(ids), n, seed & (2**64 - 1), lmin, lmax, p_mb, _p(out), PK_W, _p(nb), _threads()):
        raise ValueError("bad text-pk shape")
    return out, nb


def text_pk_paths(pkb, nb):
    """MsgpackHashPathEncoder paths (kart/dataset3_paths.py:202-215) of text pks given as UTF-8
    bytes: packed = msgpack([pk]) (fixstr up to 31 B, else str8; serialise_util.py:34-41), tree =
    the first 24 bits of sha256(packed) as 4 base64 chars (b64hash, serialise_util.py:82-85), one
    per level, filename = urlsafe_b64(packed) with '=' padding (:64-66); kds_text_pk_paths.
    -> (paths [n, PATH_W] zero-padded, path lengths [n])"""
    pkb = np.ascontiguousarray(pkb, np.uint8)
    nb = np.ascontiguousarray(nb, np.int64)
    n = pkb.shape[0]
    paths = np.empty((n, PATH_W), np.uint8)
    plen = np.empty(n, np.int64)
    if _synth_lib().kds_text_pk_paths(_p(pkb), _p(nb), n, pkb.shape[1], _p(paths), PATH_W, _p(plen), _threads()):
        raise ValueError("a text pk's path does not fit")
    return paths, plen


def _hash_keys(paths, plen):
    """KD_KEY_HASH join keys of padded paths (kd_pack_hash_keys over the packed arena)"""
    from . import _native as N

    n = paths.shape[0]
    arena, off = _arena(paths, plen, np.arange(n, dtype=np.int64))
    keys = np.empty(n, np.uint64)
    status = np.empty(n, np.uint8)
    bad = N.lib().kd_pack_hash_keys(N.ptr(arena), N.ptr(off), n, 4, 0, N.ptr(keys), N.ptr(status))
    if bad:
        raise packing.PackError(f"{bad} synthetic paths not packable")
    return keys


def _arena(paths, plen, rows):
    """the name arena (rows' paths back to back) + offsets [len(rows)+1] (kds_gather_paths)"""
    rows = np.ascontiguousarray(rows, np.int64)
    m = rows.shape[0]
    off = np.zeros(m + 1, np.uint64)
    np.cumsum(plen[rows], out=off[1:])
    arena = np.empty(int(off[-1]), np.uint8)
    _synth_lib().kds_gather_paths(_p(paths), paths.shape[1], _p(plen), _p(rows), m, _p(off), _p(arena), _threads())
    return arena, off


def _walk_order(paths):
    """git tree order of the padded paths 'c/c/c/c/<filename>': the four one-character tree
    levels, then the filename bytes, a shorter name that is a prefix of another first
    (kds_walk_order: counting sort on the trees, memcmp inside each leaf tree)"""
    n = paths.shape[0]
    order = np.empty(n, np.int64)
    if _synth_lib().kds_walk_order(_p(np.ascontiguousarray(paths)), n, paths.shape[1], _p(order), _threads()):
        raise packing.PackError("two synthetic paths are equal")
    return order


def _side(keys, paths, plen, oid_of, rows_mask, order):
    """PackedSide of the rows of ``rows_mask``, in ``order`` (walk order or key order)"""
    from . import _native as N

    rows = order[rows_mask[order]]
    s = packing.PackedSide(key=np.ascontiguousarray(keys[rows]), oid=np.ascontiguousarray(oid_of(rows)),
                           key_mode=N.KD_KEY_HASH, order=rows.astype(np.int64), encoding=packing.GENERAL_ENCODING)
    s.name, s.name_off = _arena(paths, plen, rows)
    return s


def table3_layers(n, seed=SEED, p_mod=0.05, p_del=0.005, p_ins=0.005, p_conflict=0.005, p_same=0.005,
                  p_addadd=0.0005, walk=False, pks=None):
    """C4 as SURVEY §8(d) states it: an ancestor of n text-pk rows (12–24 characters, 5 % with
    multibyte UTF-8; MsgpackHashPathEncoder paths, kart/dataset3_paths.py:202-215) and two
    descendants edited from independent seeds — each side updates 5 %, deletes 0.5 % and inserts
    0.5 % new rows — plus 0.5 % of the rows edited differently on both sides (conflicts), 0.5 %
    edited identically on both (clean), and 0.05 % new pks added on both sides (add/add, half with
    the same content).  ``walk``: the sides in git tree order (as the tree walk lists them) instead
    of key order.  ``pks``: override the ancestor's pks (list of str), e.g. the reference's KATs."""
    rng = np.random.default_rng(seed)
    n_ins, n_aa = int(n * p_ins), int(n * p_addadd)
    total = n + 2 * n_ins + n_aa
    gid = np.arange(total, dtype=np.int64)
    pkb, nb = text_pks(gid, seed)
    if pks is not None:
        for i, p in enumerate(pks):
            e = p.encode()
            if len(e) > PK_W:
                raise ValueError("pk too long for the generator")
            pkb[i] = 0
            pkb[i, :len(e)], nb[i] = np.frombuffer(e, np.uint8), len(e)
    paths, plen = text_pk_paths(pkb, nb)
    keys = _hash_keys(paths, plen)
    sk = np.sort(keys)
    if total > 1 and not np.all(sk[1:] > sk[:-1]):
        raise packing.PackError("synthetic key collision")
    del sk
    order = _walk_order(paths) if walk else np.argsort(keys)

    # the edit plan over ancestor rows: per side 0 keep, 1 modify, 2 delete (independent draws)
    act = []
    for _ in range(2):
        u = rng.random(n)
        act.append(np.where(u < p_mod, 1, np.where(u < p_mod + p_del, 2, 0)).astype(np.int8))
    u = rng.random(n)
    planted = u < p_conflict  # modified differently on both sides
    same = (u >= p_conflict) & (u < p_conflict + p_same)  # modified identically on both sides
    for k in range(2):
        act[k][planted | same] = 1
    ver = np.zeros((2, total), np.uint64)  # content version per side; 0 = the ancestor's
    ver[0, :n] = np.where(act[0] == 1, 1, 0)
    ver[1, :n] = np.where(act[1] == 1, 2, 0)
    ver[:, :n][:, same] = 3
    ins_o = np.arange(n, n + n_ins)
    ins_t = np.arange(n + n_ins, n + 2 * n_ins)
    aa = np.arange(n + 2 * n_ins, total)
    aa_same = rng.random(n_aa) < 0.5
    ver[0, ins_o], ver[1, ins_t] = 1, 2
    ver[0, aa] = np.where(aa_same, 3, 1)
    ver[1, aa] = np.where(aa_same, 3, 2)

    mem_a = gid < n
    mem_o = np.zeros(total, bool)
    mem_o[:n] = act[0] != 2
    mem_o[ins_o] = mem_o[aa] = True
    mem_t = np.zeros(total, bool)
    mem_t[:n] = act[1] != 2
    mem_t[ins_t] = mem_t[aa] = True
    anc = _side(keys, paths, plen, lambda r: synth_oids(r, 0), mem_a, order)
    ours = _side(keys, paths, plen, lambda r: synth_oids(r, ver[0, r]), mem_o, order)
    theirs = _side(keys, paths, plen, lambda r: synth_oids(r, ver[1, r]), mem_t, order)
    a0, a1 = act
    conflict_rows = ((a0 == 1) & (a1 == 1) & ~same) | ((a0 == 1) & (a1 == 2)) | ((a0 == 2) & (a1 == 1))
    n_conflict = int(conflict_rows.sum()) + int((~aa_same).sum())
    plan = {"rows": n, "pk_chars": "12-24", "pk_multibyte_rows": int(np.count_nonzero((pkb[:n] >= 0x80).any(axis=1))),
            "ours_updates": int(np.count_nonzero(a0 == 1)), "ours_deletes": int(np.count_nonzero(a0 == 2)),
            "theirs_updates": int(np.count_nonzero(a1 == 1)), "theirs_deletes": int(np.count_nonzero(a1 == 2)),
            "inserts_each": n_ins, "add_add": n_aa, "planted_conflicts": int(planted.sum()),
            "identical_edits": int(same.sum()), "conflicts": n_conflict}
    lens = plen[:n]
    plan["path_bytes_min_mean_max"] = [int(lens.min()) if n else 0, round(float(lens.mean()), 2) if n else 0,
                                       int(lens.max()) if n else 0]
    return Merge3Layer(anc, ours, theirs, n_conflict, plan)
