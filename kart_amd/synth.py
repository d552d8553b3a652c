"""Seeded synthetic layers, generated directly as packed side arrays + msgpack feature blobs.

Shapes follow SURVEY.md §8(d): the reference's own feature encoding (kart/dataset3.py:185-215,
kart/serialise_util.py:34-41) — blob = msgpack [legend_hexhash, [non-pk values]] with geometries as
ext 'G' GeoPackage binaries — and its int-PK path layout (kart/dataset3_paths.py:292-299), so the
engine sees exactly what a Kart repo's trees would hand it.  Blob OIDs are synthetic (a seeded
64-bit mix of (pk, version)): equal content <=> equal OID, which is all classification relies on.
No git repository is involved.

Generation is vectorised numpy, fast enough for the 10M-point C2 layer in seconds.
"""
from dataclasses import dataclass

import numpy as np

from . import packing
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
    """C2: n int-PK points (pks pk0..pk0+n-1); seeded 1% updates / deletes / inserts."""
    rng = np.random.default_rng(seed)
    schema = Schema.from_column_dicts(POINT_SCHEMA)
    legend = Legend(["c-fid"], [c["id"] for c in POINT_SCHEMA[1:]])
    lh = legend.hexhash()
    pks = np.arange(pk0, pk0 + n, dtype=np.int64)
    n_upd, n_del, n_ins = int(n * frac_update), int(n * frac_delete), int(n * frac_insert)
    perm = rng.permutation(n)
    upd_i = np.sort(perm[:n_upd])
    del_i = np.sort(perm[n_upd:n_upd + n_del])
    base_ver = np.zeros(n, np.uint64)
    tgt_ver = base_ver.copy()
    tgt_ver[upd_i] = 1
    keep = np.ones(n, bool)
    keep[del_i] = False
    ins_pk = np.arange(pk0 + n, pk0 + n + n_ins, dtype=np.int64)
    t_pk = np.concatenate([pks[keep], ins_pk])
    t_ver = np.concatenate([tgt_ver[keep], np.full(n_ins, 2, np.uint64)])
    keys_b = _int_keys(pks)
    keys_t = _int_keys(t_pk)
    base = packing.PackedSide(key=keys_b, oid=synth_oids(pks, base_ver), key_mode=0,
                              order=np.arange(n, dtype=np.int64), encoding=packing.INT_PK_ENCODING)
    target = packing.PackedSide(key=keys_t, oid=synth_oids(t_pk, t_ver), key_mode=0,
                                order=np.arange(t_pk.shape[0], dtype=np.int64), encoding=packing.INT_PK_ENCODING)
    bb = point_blobs(pks, base_ver, lh)
    tb = point_blobs(t_pk, t_ver, lh)
    return Layer(base, target, bb, tb, schema, {lh: legend}, n_ins, n_upd, n_del)


def _int_keys(pk):
    """vectorised KD_KEY_INT (same formula as kd_pack_int_keys / packing.pk_to_int_key)"""
    pk = np.asarray(pk, np.int64)
    q = pk >> 6
    r = (pk - (q << 6)).astype(np.uint64)
    bucket = (q & ((1 << 24) - 1)).astype(np.uint64)
    k = ((pk >> 30) + (1 << 33)).astype(np.uint64)
    return np.ascontiguousarray((bucket << np.uint64(40)) | (k << np.uint64(6)) | r)


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
