"""Writer formatting on the GPU: hex WKB of geometries and hex of bytes values.

Mirrors the reference's per-value formatting, batched:
  * ``hex_wkb_batch``     <- ``gpkg_geom_to_hex_wkb`` / ``Geometry.to_hex_wkb``
                             (kart/geometry.py:346-375, :142-143); ``hex_wkb_arena`` gives the same
                             hex as one buffer + bounds for writers that stream bytes
  * ``bytes_hex_batch``   <- ``bytes.hex(v)`` as ``feature_as_json`` applies it (kart/feature_output.py:54-55)
  * ``features_as_json``  <- ``feature_as_json(row, pk_value)`` with no geometry transform
                             (kart/feature_output.py:34-56), for a list of rows at once.
  * ``feature_as_text`` / ``feature_field_as_text`` <- the text writer's field lines
                             (kart/feature_output.py:9-31): geometries as "<TYPE>(...)" or
                             "<TYPE> EMPTY" from the GPKG header + WKB type word
                             (Geometry.geometry_type_name, kart/geometry.py:189-198), other bytes as
                             "BLOB(...)", None as "␀"; ``geometry_type_names`` does the type names of a
                             whole geometry arena at once (numpy over the headers).

Every hex string is produced by ``kd_hex_encode`` (kd_output.hip).  Geometries the kernel flags
as needing the CPU path (big-endian WKB, which the reference re-encodes through OGR, or invalid
GPKG, for which the reference raises) are returned in ``fallback`` for the caller's own path;
nothing here computes a hex string on the CPU.
"""
import struct

import numpy as np

from . import _native as N

# GeometryType (kart/geometry.py:40-47)
GEOMETRY_TYPES = {1: "POINT", 2: "LINESTRING", 3: "POLYGON", 4: "MULTIPOINT", 5: "MULTILINESTRING",
                  6: "MULTIPOLYGON", 7: "GEOMETRYCOLLECTION"}
_WKB25D = 0x80000000  # OGR's wkb25DBitInternalUse
_ENV_SIZES = {0: 0, 1: 32, 2: 48, 3: 48, 4: 64}  # GPKG_ENVELOPE_SIZES (kart/geometry.py:24-30)


def _ogr_flatten_z_m(t):
    """OGR_GT_Flatten / OGR_GT_HasZ / OGR_GT_HasM of a WKB geometry type word: ISO 1000 / 2000 /
    3000 offsets and the old 2.5D bit"""
    z = bool(t & _WKB25D)
    t &= ~_WKB25D & 0xFFFFFFFF
    m = False
    if 1000 <= t < 2000:
        t, z = t - 1000, True
    elif 2000 <= t < 3000:
        t, m = t - 2000, True
    elif 3000 <= t < 4000:
        t, z, m = t - 3000, True, True
    return t, z, m


def geometry_type_name(gpkg):
    """Geometry.geometry_type_name (kart/geometry.py:179-198) of a GPKG geometry: envelope size from
    the flags byte (ValueError for an invalid envelope indicator), the WKB's endianness byte (read
    signed: nonzero = little-endian) and type word, GeometryType of the flattened type (ValueError
    outside 1..7), " Z" / " M" / " ZM" suffixes"""
    g = bytes(gpkg)
    flags = g[3]
    et = (flags & 0x0E) >> 1
    if et not in _ENV_SIZES:
        raise ValueError("Invalid envelope contents indicator")
    wkb = 8 + _ENV_SIZES[et]
    (is_le,) = struct.unpack_from("b", g, offset=wkb)
    (typ,) = struct.unpack_from("<I" if is_le else ">I", g, offset=wkb + 1)
    flat, z, m = _ogr_flatten_z_m(typ)
    if flat not in GEOMETRY_TYPES:
        raise ValueError(f"{flat} is not a valid GeometryType")
    suffix = "Z" * z + "M" * m
    return f"{GEOMETRY_TYPES[flat]} {suffix}" if suffix else GEOMETRY_TYPES[flat]


def feature_field_as_text(row, key, prefix, geometry_type=None):
    """feature_field_as_text (kart/feature_output.py:18-31)"""
    if geometry_type is None:
        from .dataset import Geometry as geometry_type
    val = row[key]
    if isinstance(val, geometry_type):
        typ = geometry_type_name(val)
        val = f"{typ} EMPTY" if val[3] & 0x10 else f"{typ}(...)"
    elif isinstance(val, bytes):
        val = "BLOB(...)"
    val = "\u2400" if val is None else val
    return f"{prefix}{key:>40} = {val}"


def feature_as_text(row, prefix="", geometry_type=None):
    """feature_as_text (kart/feature_output.py:9-15): one line per field, "__" keys skipped"""
    return "\n".join(feature_field_as_text(row, k, prefix, geometry_type) for k in row.keys() if not k.startswith("__"))


def geometry_type_names(data, off):
    """The text writer's geometry label of every geometry of an arena (GPKG bytes; length 0 =
    None), vectorised over the headers: object array of "<TYPE>(...)" / "<TYPE> EMPTY" / None (a
    null geometry), plus the indices whose header the reference would reject (short, invalid
    envelope indicator, unknown type: geometry_type_name raises) for the caller's own path."""
    data = np.ascontiguousarray(data, np.uint8)
    off = np.ascontiguousarray(off, np.uint64).astype(np.int64)
    n = off.shape[0] - 1
    start, ln = off[:-1], off[1:] - off[:-1]
    out = np.empty(n, object)
    bad = np.zeros(n, bool)
    flags = np.where(ln >= 4, data[np.minimum(start + 3, max(data.size - 1, 0))] if data.size else 0, 0).astype(np.int64)
    et = (flags & 0x0E) >> 1
    esz = np.select([et == 0, et == 1, (et == 2) | (et == 3), et == 4], [0, 32, 48, 64], -1)
    wkb = 8 + esz
    ok = (ln > 0) & (esz >= 0) & (ln >= wkb + 5)
    bad |= (ln > 0) & ~ok
    idx = np.nonzero(ok)[0]
    p = start[idx] + wkb[idx]
    le = data[p].astype(np.int8) != 0
    b = [data[p + 1 + k].astype(np.uint64) for k in range(4)]
    t_le = b[0] | b[1] << np.uint64(8) | b[2] << np.uint64(16) | b[3] << np.uint64(24)
    t_be = b[3] | b[2] << np.uint64(8) | b[1] << np.uint64(16) | b[0] << np.uint64(24)
    typ = np.where(le, t_le, t_be).astype(np.int64)
    z = (typ & _WKB25D) != 0
    t = typ & ~np.int64(_WKB25D) & 0xFFFFFFFF
    iso = t // 1000
    z |= (iso == 1) | (iso == 3)
    m = (iso == 2) | (iso == 3)
    flat = np.where((iso >= 1) & (iso <= 3), t - 1000 * iso, t)
    valid = (flat >= 1) & (flat <= 7)
    bad[idx[~valid]] = True
    empty = (flags[idx] & 0x10) != 0
    labels = {}
    for j, i in enumerate(idx.tolist()):
        if not valid[j]:
            continue
        key = (int(flat[j]), bool(z[j]), bool(m[j]), bool(empty[j]))
        lab = labels.get(key)
        if lab is None:
            suffix = "Z" * key[1] + "M" * key[2]
            name = f"{GEOMETRY_TYPES[key[0]]} {suffix}" if suffix else GEOMETRY_TYPES[key[0]]
            lab = labels[key] = f"{name} EMPTY" if key[3] else f"{name}(...)"
        out[i] = lab
    return out, np.nonzero(bad)[0]


try:
    from . import _kd_pystr as _pystr  # built with libkartdiff (kart_amd/csrc/Makefile)
except ImportError:  # pragma: no cover - the helper is optional host code
    _pystr = None


def _arena(values):
    lens = np.fromiter((len(v) for v in values), np.uint64, len(values))
    off = np.zeros(len(values) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    data = np.frombuffer(b"".join(values), np.uint8) if values else np.zeros(0, np.uint8)
    return data, off


def _slices(hexbuf, lo, hi):
    """the hex strings [lo[i], hi[i]) of one output buffer, one str per value: built in C straight
    from the buffer (kart_amd/_kd_pystr: PyUnicode_New + memcpy per value); without that helper,
    one decode of the buffer and a slice per value"""
    buf = np.ascontiguousarray(hexbuf, np.uint8)
    lo = np.ascontiguousarray(lo, np.int64)
    hi = np.ascontiguousarray(hi, np.int64)
    if _pystr is not None:
        return _pystr.ascii_slices(buf, lo, hi)
    text = str(memoryview(buf), "ascii")
    return list(map(text.__getitem__, map(slice, lo.tolist(), hi.tolist())))


def hex_wkb_arena(engine, geoms=None, arena=None):
    """The hex WKB of many geometries without building a str per value — for a writer that
    streams bytes: (hex uint8 buffer, lo int64[n], hi int64[n], status uint8[n]); geometry i's
    uppercase hex WKB is buffer[lo[i]:hi[i]] (empty unless status[i] == 0: 1 None / empty bytes,
    3 the reference's OGR path or error).  ``arena=(data, off)``: geometries already in one buffer
    (e.g. a blob read's arena sliced to the geometry values) — nothing is joined on the host."""
    if arena is None:
        data, off = _arena([b"" if g is None else g for g in geoms])
    else:
        data, off = arena
    hexbuf, start, status = engine.hex_encode(data, off, N.KD_HEX_GPKG_WKB)
    n = int(np.asarray(off).shape[0]) - 1
    off = np.asarray(off, np.uint64)
    lo = 2 * (off[:n].astype(np.int64) + start.astype(np.int64))
    hi = np.where(status == 0, 2 * off[1:].astype(np.int64), lo)
    return hexbuf, lo, hi, status


def hex_wkb_batch(engine, geoms):
    """geoms: sequence of GPKG geometry bytes or None.  Returns (hex_list, fallback_indices):
    hex_list[i] is the uppercase hex WKB (str), None for a None/empty-bytes geometry, or None with
    i in fallback_indices when the reference would go through OGR or raise."""
    hexbuf, lo, hi, status = hex_wkb_arena(engine, geoms)
    ok = status == 0
    out = _slices(hexbuf, lo, hi)
    bad = np.nonzero(~ok)[0]
    for i in bad.tolist():
        out[i] = None
    return out, np.nonzero(status == 3)[0].tolist()


def bytes_hex_batch(engine, values):
    """bytes.hex(v) for each bytes value (lowercase)."""
    vals = [bytes(v) for v in values]
    data, off = _arena(vals)
    hexbuf, _, _ = engine.hex_encode(data, off, N.KD_HEX_BYTES)
    o = 2 * off.astype(np.int64)
    return _slices(hexbuf, o[:-1], o[1:])


def features_as_json(engine, rows, geometry_type=None):
    """feature_as_json for many rows (dicts): geometries (instances of ``geometry_type``, by default
    kart_amd.dataset.Geometry — what this package's get_feature returns; Kart passes its own
    ``Geometry``) -> hex WKB, other ``bytes`` values -> bytes.hex, everything else (bytearray
    included, as kart/feature_output.py:54 tests isinstance(v, bytes)) unchanged.
    Raises NotImplementedError naming the first geometry that needs the CPU (OGR) path."""
    if geometry_type is None:
        from .dataset import Geometry as geometry_type
    geo_at, geoms, byt_at, byts = [], [], [], []
    for r, row in enumerate(rows):
        for k, v in row.items():
            if isinstance(v, geometry_type):
                geo_at.append((r, k)); geoms.append(v)
            elif isinstance(v, bytes):
                byt_at.append((r, k)); byts.append(v)
    out = [dict(row) for row in rows]
    if geoms:
        hexes, fb = hex_wkb_batch(engine, geoms)
        if fb:
            r, k = geo_at[fb[0]]
            raise NotImplementedError(f"geometry {k!r} of row {r} needs the OGR path (big-endian or invalid WKB)")
        for (r, k), h in zip(geo_at, hexes):
            out[r][k] = h
    if byts:
        for (r, k), h in zip(byt_at, bytes_hex_batch(engine, byts)):
            out[r][k] = h
    return out
