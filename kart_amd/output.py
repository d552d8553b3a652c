"""Writer formatting on the GPU: hex WKB of geometries and hex of bytes values.

Mirrors the reference's per-value formatting, batched:
  * ``hex_wkb_batch``     <- ``gpkg_geom_to_hex_wkb`` / ``Geometry.to_hex_wkb``
                             (kart/geometry.py:346-375, :142-143); ``hex_wkb_arena`` gives the same
                             hex as one buffer + bounds for writers that stream bytes
  * ``bytes_hex_batch``   <- ``bytes.hex(v)`` as ``feature_as_json`` applies it (kart/feature_output.py:54-55)
  * ``features_as_json``  <- ``feature_as_json(row, pk_value)`` with no geometry transform
                             (kart/feature_output.py:34-56), for a list of rows at once.

Every hex string is produced by ``kd_hex_encode`` (kd_output.hip).  Geometries the kernel flags
as needing the CPU path (big-endian WKB, which the reference re-encodes through OGR, or invalid
GPKG, for which the reference raises) are returned in ``fallback`` for the caller's own path;
nothing here computes a hex string on the CPU.
"""
import numpy as np

from . import _native as N


def _arena(values):
    lens = np.fromiter((len(v) for v in values), np.uint64, len(values))
    off = np.zeros(len(values) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    data = np.frombuffer(b"".join(values), np.uint8) if values else np.zeros(0, np.uint8)
    return data, off


def _slices(hexbuf, lo, hi):
    """the hex strings [lo[i], hi[i]) of one output buffer: decoded to one str once, then sliced
    with bounds computed in numpy (no per-value int() / bytes slice / decode)"""
    text = hexbuf.tobytes().decode("ascii")
    return [text[a:b] for a, b in zip(lo.tolist(), hi.tolist())]


def hex_wkb_arena(engine, geoms):
    """The hex WKB of many geometries without building a str per value — for a writer that
    streams bytes: (hex uint8 buffer, lo int64[n], hi int64[n], status uint8[n]); geometry i's
    uppercase hex WKB is buffer[lo[i]:hi[i]] (empty unless status[i] == 0: 1 None / empty bytes,
    3 the reference's OGR path or error)."""
    vals = [b"" if g is None else g for g in geoms]
    data, off = _arena(vals)
    hexbuf, start, status = engine.hex_encode(data, off, N.KD_HEX_GPKG_WKB)
    n = len(vals)
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
