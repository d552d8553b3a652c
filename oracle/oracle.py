"""Python face of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg import this module,
and only as the checker / baseline.  The product package (kart_amd) never imports it.

* ``C``: ctypes binding of ``oracle/libkdoracle.so`` (kd_oracle.c, plain sequential C).
* ``py_changed_fields``: the strongest available restatement of the field compare — decode with
  the same msgpack library + ext hook the reference uses (kart/serialise_util.py:26-48) and compare
  with Python's own ``==`` (kart/text_diff_writer.py:135-145).  Pure Python: small cases only.
"""
import base64
import ctypes
import os
import subprocess

import msgpack
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libkdoracle.so")

_u8 = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def C():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.kdo_classify2.restype = ctypes.c_int64
        L.kdo_classify2.argtypes = [ctypes.c_uint64, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp]
        L.kdo_classify3.restype = ctypes.c_int64
        L.kdo_classify3.argtypes = [ctypes.c_uint64, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint64, _vp, _vp,
                                    _vp, _vp, _vp, _vp, _vp, _vp]
        L.kdo_fielddiff.restype = ctypes.c_int
        L.kdo_fielddiff.argtypes = [ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, _vp, _vp, ctypes.c_int, _vp, _vp, _vp, _vp, _vp]
        L.kdo_envelope_batch.restype = ctypes.c_int64
        L.kdo_envelope_batch.argtypes = [ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_int, _vp, _vp, _vp]
        L.kdo_envelope_encode.restype = ctypes.c_int
        L.kdo_envelope_encode.argtypes = [_vp, ctypes.c_int, _vp]
        L.kdo_envelope_decode.restype = None
        L.kdo_envelope_decode.argtypes = [_vp, ctypes.c_int, _vp]
        L.kdo_envelope_overlap.restype = ctypes.c_int
        L.kdo_envelope_overlap.argtypes = [_vp, ctypes.c_int, _vp]
        L.kdo_sf_filter_batch.restype = None
        L.kdo_sf_filter_batch.argtypes = [ctypes.c_uint64, _vp, _vp, ctypes.c_int, ctypes.c_uint64, _vp, _vp, _vp, _vp]
        L.kdo_geom_filter.restype = ctypes.c_int64
        L.kdo_geom_filter.argtypes = [ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, ctypes.c_int, _vp, _vp, ctypes.c_int,
                                      _vp, _vp, _vp, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp]
        L.kdo_bbox_intersects.restype = ctypes.c_int
        L.kdo_bbox_intersects.argtypes = [_vp, _vp]
        L.kdo_wrap_lon.restype = ctypes.c_double
        L.kdo_wrap_lon.argtypes = [ctypes.c_double]
        L.kdo_index_envelope.restype = ctypes.c_int
        L.kdo_index_envelope.argtypes = [_vp, _vp]
        L.kdo_gpkg_envelope.restype = ctypes.c_int
        L.kdo_gpkg_envelope.argtypes = [_vp, ctypes.c_uint64, _vp]
        L.kdo_point_envelope.restype = ctypes.c_int
        L.kdo_point_envelope.argtypes = [_vp, ctypes.c_uint64, _vp]
        L.kdo_int_pk_key.restype = ctypes.c_int
        L.kdo_int_pk_key.argtypes = [ctypes.c_int64, ctypes.c_uint64, _vp]
        L.kdo_int_walk_key.restype = ctypes.c_int
        L.kdo_int_walk_key.argtypes = [ctypes.c_int64, _vp]
        L.kdo_decode_int_filename.restype = ctypes.c_int
        L.kdo_decode_int_filename.argtypes = [_vp, ctypes.c_int, _vp, _vp]
        L.kdo_hash_path_key.restype = ctypes.c_int
        L.kdo_hash_path_key.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp]
        L.kdo_hex_wkb_batch.restype = None
        L.kdo_hex_wkb_batch.argtypes = [ctypes.c_uint64, _vp, _vp, _vp, _vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


NONE = 0xFFFFFFFF


def classify2(keyA, oidA, keyB, oidB):
    """-> (delta uint32 [n,2], counts {inserts, updates, deletes})"""
    nA, nB = keyA.shape[0], keyB.shape[0]
    cap = nA + nB + 1
    oa = np.empty(cap, np.uint32)
    ob = np.empty(cap, np.uint32)
    counts = np.zeros(3, np.uint64)
    z8 = np.zeros(1, np.uint64)
    zo = np.zeros(20, np.uint8)
    nd = C().kdo_classify2(nA, _p(keyA) if nA else _p(z8), _p(oidA) if nA else _p(zo), nB, _p(keyB) if nB else _p(z8),
                           _p(oidB) if nB else _p(zo), _p(oa), _p(ob), _p(counts))
    if nd < 0:
        raise ValueError("oracle classify2: keys not strictly ascending")
    return np.stack([oa[:nd], ob[:nd]], 1), {"inserts": int(counts[0]), "updates": int(counts[1]),
                                              "deletes": int(counts[2])}


def classify3(kA, oA, kO, oO, kT, oT):
    """-> (conflicts uint32 [n,3], mdeltas uint32 [m,2], n_clean)"""
    cap = kA.shape[0] + kO.shape[0] + kT.shape[0] + 1
    ca, co, ct, mo, mt = (np.empty(cap, np.uint32) for _ in range(5))
    counts = np.zeros(3, np.uint64)
    z8, zo = np.zeros(1, np.uint64), np.zeros(20, np.uint8)
    args = []
    for k, o in ((kA, oA), (kO, oO), (kT, oT)):
        args += [k.shape[0], _p(k) if k.shape[0] else _p(z8), _p(o) if k.shape[0] else _p(zo)]
    rc = C().kdo_classify3(*args, _p(ca), _p(co), _p(ct), _p(mo), _p(mt), _p(counts))
    if rc < 0:
        raise ValueError("oracle classify3: keys not strictly ascending")
    nc, nm = int(counts[1]), int(counts[2])
    return np.stack([ca[:nc], co[:nc], ct[:nc]], 1), np.stack([mo[:nm], mt[:nm]], 1), int(counts[0])


def fielddiff(old_data, old_off, new_data, new_off, pairs, maps):
    """C restatement; maps = kart_amd.schema.FieldMaps (its arrays are plain data)."""
    n = pairs.shape[0] if pairs is not None else old_off.shape[0] - 1
    oi = np.ascontiguousarray(pairs[:, 0], np.uint32) if pairs is not None else None
    ni = np.ascontiguousarray(pairs[:, 1], np.uint32) if pairs is not None else None
    masks = np.zeros((max(n, 1), maps.words), np.uint64)
    status = np.zeros(max(n, 1), np.uint8)
    od = old_data if old_data.size else np.zeros(1, np.uint8)
    nd = new_data if new_data.size else np.zeros(1, np.uint8)
    C().kdo_fielddiff(n, _p(od), _p(old_off), _p(oi), _p(nd), _p(new_off), _p(ni), maps.n_keys, maps.words,
                      max(1, len(maps.old_hashes)), _p(maps.leg_old_hex), _p(maps.map_old),
                      max(1, len(maps.new_hashes)), _p(maps.leg_new_hex), _p(maps.map_new), _p(maps.cmp_mask),
                      _p(masks), _p(status))
    return masks[:n], status[:n]


def envelope_batch(data, off, filt_env, bits=20):
    n = off.shape[0] - 1
    nb = bits // 2
    match = np.zeros(max(n, 1), np.uint8)
    enc = np.zeros((max(n, 1), nb), np.uint8)
    ok = np.zeros(max(n, 1), np.uint8)
    fe = np.asarray(filt_env, np.float64)
    d = data if data.size else np.zeros(1, np.uint8)
    npass = C().kdo_envelope_batch(n, _p(d), _p(off), _p(fe), bits, _p(match), _p(enc), _p(ok))
    return match[:n], enc[:n], ok[:n], int(npass)


def envelope_decode(enc, bits=20):
    """EnvelopeEncoder.decode (kart/spatial_filter/index.py:532-548): encoded bytes -> (w, s, e, n)"""
    e = np.ascontiguousarray(np.frombuffer(bytes(enc), np.uint8))
    out = np.zeros(4)
    C().kdo_envelope_decode(_p(e), bits, _p(out))
    return tuple(float(x) for x in out)


def sf_filter_batch(idx_oid, idx_env, bits, oid, is_feature, q):
    """sf_filter_blob over a batch (vendor/spatial-filter/spatial_filter.cpp:212-260); the index
    rows in any order (sorted here by blob id)"""
    idx_oid = np.ascontiguousarray(idx_oid, np.uint8).reshape(-1, 20)
    idx_env = np.ascontiguousarray(idx_env, np.uint8).reshape(idx_oid.shape[0], -1)
    srt = np.argsort(idx_oid.view("S20").reshape(-1), kind="stable")
    io, ie = np.ascontiguousarray(idx_oid[srt]), np.ascontiguousarray(idx_env[srt])
    oid = np.ascontiguousarray(oid, np.uint8).reshape(-1, 20)
    m = oid.shape[0]
    out = np.zeros(max(m, 1), np.uint8)
    feat = None if is_feature is None else np.ascontiguousarray(is_feature, np.uint8)
    pad = np.zeros(20, np.uint8)
    C().kdo_sf_filter_batch(io.shape[0], _p(io if io.size else pad), _p(ie if ie.size else pad), bits, m,
                            _p(oid if m else pad), _p(feat) if feat is not None else None,
                            _p(np.asarray(q, np.float64)), _p(out))
    return out[:m]


def envelope_overlap(enc, bits, q):
    qa = np.asarray(q, np.float64)
    out = np.zeros(enc.shape[0], np.uint8)
    for i in range(enc.shape[0]):
        r = C().kdo_envelope_overlap(_p(np.ascontiguousarray(enc[i])), bits, _p(qa))
        out[i] = 2 if r < 0 else r
    return out


# ------------------------------------------------------------------------------------------
# spatially filtered diff restated (kart/base_diff_writer.py:279-329 + SpatialFilter.matches,
# kart/spatial_filter/__init__.py:534-605), envelope part only: per side 0 NON_MATCHING,
# 1 CANDIDATE (exact Intersects outstanding), 2 MATCHING, 3 FALLBACK (OGR / malformed), 4 NONEXISTENT
GF_NON, GF_CAND, GF_MATCH, GF_FALLBACK, GF_NONE = range(5)


class _GeomExt(bytes):
    pass


def _gf_hook(code, data):
    return _GeomExt(data) if code == ord("G") else msgpack.ExtType(code, data)


def sf_envelope_code(g, filt_env, rect):
    """SpatialFilter.matches for a GPKG geometry (bytes or None), without the exact test"""
    if g is None:
        return GF_MATCH  # geometry None: MATCHING (:549-551)
    gb = np.frombuffer(bytes(g), np.uint8) if len(g) else np.zeros(1, np.uint8)
    env = np.zeros(4)
    r = C().kdo_gpkg_envelope(_p(gb), len(g), _p(env))
    if r < 0:
        return GF_FALLBACK  # the reference raises (ValueError / NotImplementedError)
    if r == 0 and g[3] & 0x10:
        return GF_NON  # empty: envelope (0,0,0,0) from OGR, then Intersects(empty) is False
    if r != 1:  # no stored envelope (or NaN): OGR's envelope — a point's is (x, x, y, y)
        pc = C().kdo_point_envelope(_p(gb), len(g), _p(env))
        if pc == 0:
            return GF_NON  # empty point
        if pc < 0:
            return GF_FALLBACK  # needs OGR
    fe = np.asarray(filt_env, np.float64)
    x = C().kdo_bbox_intersects(_p(fe), _p(env))
    if x < 0:
        return GF_FALLBACK
    if x == 0:
        return GF_NON
    if rect and fe[0] <= env[0] and env[1] <= fe[1] and fe[2] <= env[2] and env[3] <= fe[3]:
        return GF_MATCH  # inside a rectangular filter: Intersects is certain
    return GF_CAND


def feature_geometry(blob, gidx_by_legend):
    """(status, GPKG bytes | None) of a feature blob: status 0 ok, 3 fallback (unknown legend,
    malformed, geometry value not an ext 'G')"""
    try:
        legend, values = msgpack.unpackb(bytes(blob), raw=False, ext_hook=_gf_hook)
    except Exception:
        return GF_FALLBACK, None
    if legend not in gidx_by_legend:
        return GF_FALLBACK, None
    gi = gidx_by_legend[legend]
    if gi < 0:
        return 0, None
    if gi >= len(values):
        return GF_FALLBACK, None
    v = values[gi]
    if v is None:
        return 0, None
    if not isinstance(v, _GeomExt):
        return GF_FALLBACK, None
    return 0, bytes(v)


def _cols_arrays(cols):
    hexes = sorted(cols)
    hx = np.frombuffer(b"".join(h.encode() for h in hexes), np.uint8).copy() if hexes else np.zeros(40, np.uint8)
    gi = np.array([cols[h] for h in hexes] or [-1], np.int16)
    return len(hexes), hx, gi


def geom_filter(old_data, old_off, new_data, new_off, pairs, old_cols, new_cols, filt_env, rect, bits=20):
    """codes [n, 2], kept delta indices, new-side index envelopes (enc [n, bits/2], enc_ok [n]).
    old_cols/new_cols: {legend hex: geometry value index | -1}.  The C restatement
    (kdo_geom_filter) of geom_filter_py below, fast enough for C5's 10M deltas."""
    pairs = np.ascontiguousarray(pairs, np.uint32).reshape(-1, 2)
    n = pairs.shape[0]
    nlo, hxo, gio = _cols_arrays(old_cols)
    nln, hxn, gin = _cols_arrays(new_cols)
    codes = np.zeros((max(n, 1), 2), np.uint8)
    enc = np.zeros((max(n, 1), bits // 2), np.uint8)
    ok = np.zeros(max(n, 1), np.uint8)
    pad = np.zeros(16, np.uint8)
    od = old_data if old_data.size else pad
    nd = new_data if new_data.size else pad
    C().kdo_geom_filter(n, _p(od), _p(np.ascontiguousarray(old_off, np.uint64)), _p(nd),
                        _p(np.ascontiguousarray(new_off, np.uint64)), _p(pairs if n else np.zeros(2, np.uint32)),
                        nlo, _p(hxo), _p(gio), nln, _p(hxn), _p(gin), _p(np.asarray(filt_env, np.float64)),
                        1 if rect else 0, bits, _p(codes), _p(enc), _p(ok))
    codes, enc, ok = codes[:n], enc[:n], ok[:n]
    keep = np.nonzero(((codes >= 1) & (codes <= 3)).any(axis=1))[0].astype(np.uint32)
    return codes, keep, enc, ok


def geom_filter_py(old_data, old_off, new_data, new_off, pairs, old_cols, new_cols, filt_env, rect, bits=20):
    """the Python restatement (msgpack.unpackb with the ext hook, per delta): the reference for
    kdo_geom_filter on small inputs"""
    n = pairs.shape[0]
    codes = np.zeros((n, 2), np.uint8)
    geoms_new = []
    for d in range(n):
        for s, (data, off, cols) in enumerate(((old_data, old_off, old_cols), (new_data, new_off, new_cols))):
            bi = int(pairs[d, s])
            g = None
            if bi == NONE:
                codes[d, s] = GF_NONE
            else:
                st, g = feature_geometry(data[int(off[bi]):int(off[bi + 1])].tobytes(), cols)
                codes[d, s] = st if st else sf_envelope_code(g, filt_env, rect)
            if s == 1:
                geoms_new.append(g if codes[d, 1] not in (GF_NONE, GF_FALLBACK) else None)
    keep = np.nonzero(((codes >= 1) & (codes <= 3)).any(axis=1))[0].astype(np.uint32)
    gb = [g or b"" for g in geoms_new]
    goff = np.zeros(n + 1, np.uint64)
    if n:
        goff[1:] = np.cumsum([len(g) for g in gb])
    gdata = np.frombuffer(b"".join(gb), np.uint8) if n else np.zeros(0, np.uint8)
    _, enc, ok, _ = envelope_batch(gdata, goff, filt_env, bits)
    return codes, keep, enc, ok


# ------------------------------------------------------------------------------------------
# pure-Python restatement of the field compare (Python's own == on msgpack-decoded values)
class _Geometry(bytes):
    pass


def _ext_hook(code, data):
    if code == ord("G"):
        if not data:
            return None
        if not data.startswith(b"GP"):
            raise ValueError("Invalid StandardGeoPackageBinary geometry")
        return _Geometry(data)
    return msgpack.ExtType(code, data)


def py_feature(blob, pk_values, legend, schema):
    """Dataset3.get_feature restated: msg_unpack + Legend + Schema projection."""
    legend_hash, non_pk = msgpack.unpackb(blob, raw=False, ext_hook=_ext_hook)
    raw = legend.value_tuples_to_raw_dict(pk_values, non_pk)
    return schema.feature_from_raw_dict(raw)


_NULL = object()


def py_changed_fields(old, new):
    keys = list(old.keys()) + [k for k in new.keys() if k not in old]
    return [k for k in keys if not k.startswith("__") and old.get(k, _NULL) != new.get(k, _NULL)]


def decode_pk_from_filename(name):
    """Dataset3.decode_path_to_1pk restated (kart/dataset3.py:250-259)."""
    pks = msgpack.unpackb(base64.urlsafe_b64decode(name), raw=False)
    if len(pks) != 1:
        raise ValueError(f"Expected a single pk_value, got {pks}")
    return pks[0]


# ------------------------------------------------------------------------------------------
# writer formatting restated (kart/geometry.py:227-252,346-375; kart/feature_output.py:54-55)
_ENV_SIZES = {0: 0, 1: 32, 2: 48, 3: 48, 4: 64}


def hex_wkb(gpkg):
    """gpkg_geom_to_hex_wkb restated: None -> None; 'fallback' where the reference uses OGR
    (big-endian WKB) or raises (invalid GPKG / empty WKB)."""
    if gpkg is None or len(gpkg) == 0:
        return None
    if len(gpkg) < 8 or gpkg[0:2] != b"GP" or gpkg[2] != 0 or gpkg[3] & 0x20:
        return "fallback"
    size = _ENV_SIZES.get((gpkg[3] & 0b1110) >> 1)
    if size is None:
        return "fallback"
    wkb = gpkg[8 + size:]
    if len(wkb) == 0 or wkb[0] == 0:
        return "fallback"
    return wkb.hex().upper()


def hex_wkb_batch(data, off):
    """kdo_hex_wkb_batch: (hex buffer [2 * off[-1]] with blob i's WKB hex at 2 * (off[i] + start),
    status [n]: 0 ok, 1 null, 3 fallback).  ``off`` may start past 0 (a shard of an arena)."""
    n = off.shape[0] - 1
    base = int(off[0]) if n >= 0 else 0
    loc = np.ascontiguousarray(off - np.uint64(base), np.uint64)
    seg = np.ascontiguousarray(data[base:int(off[-1])]) if n > 0 else np.zeros(1, np.uint8)
    hexb = np.zeros(max(1, 2 * int(loc[-1])), np.uint8)
    status = np.zeros(max(1, n), np.uint8)
    C().kdo_hex_wkb_batch(n, _p(seg if seg.size else np.zeros(1, np.uint8)), _p(loc), _p(hexb), _p(status))
    return hexb[:2 * int(loc[-1])], status[:n]
