"""The spatial filter and the spatially filtered diff behind Kart's diff writers.

* ``SpatialFilter`` <- kart/spatial_filter/__init__.py:435-605 (``matches``,
  ``matches_delta_value``, ``MATCH_ALL``, the per-dataset form ``transform_for_schema_and_crs``
  :657-683 for an identity CRS).  The envelope quick-check is the reference's own
  (``bbox_intersects_fast`` :709-734); the exact test — OGR's prepared ``Intersects`` — is the
  caller's ``intersects`` callable.  Without one it is decided where the envelope makes it certain
  (a point, or an envelope inside a rectangular filter) and otherwise the feature counts as
  matching (a superset; counted in ``stats["unverified"]``), as the reference does when its test
  cannot run (:586-590).
* ``filtered_ds_feature_deltas`` <- BaseDiffWriter.filtered_ds_feature_deltas
  (kart/base_diff_writer.py:279-329): every delta's old and new geometry is found in its feature
  blob and envelope-tested on the GPU in one batch (``kd_geom_filter``), the deltas that may match
  come back compacted in key order, and only those are resolved on the host.
"""
import ctypes
import struct
from enum import Enum, auto

import numpy as np

from . import _native as N

# placeholder a native call gets for an empty host array: a module-level array, alive for every call
_PAD = np.zeros(16, np.uint8)
from . import packing
from .deltas import WORKING_COPY_EDIT

CODE_NON, CODE_CAND, CODE_MATCH, CODE_FALLBACK, CODE_NONE = range(5)


class MatchResult(Enum):
    """kart/spatial_filter/__init__.py:413-432"""

    NONEXISTENT = auto()
    PROMISED = auto()
    NON_MATCHING = auto()
    MATCHING = auto()

    def __bool__(self):
        return self is self.MATCHING


def _range_overlaps(a, b):
    (a1, a2), (b1, b2) = a, b
    if a1 > a2 or b1 > b2:
        raise ValueError("I was passed a range that didn't make sense: (%r, %r), (%r, %r)" % (a1, a2, b1, b2))
    if b1 < a1:
        return b2 > a1
    if a1 < b1:
        return a2 > b1
    return b2 != b1 and a2 != a1


def bbox_intersects_fast(a, b):
    """(min-x, max-x, min-y, max-y) boxes overlap (kart/spatial_filter/__init__.py:709-734)"""
    return _range_overlaps((a[0], a[1]), (b[0], b[1])) and _range_overlaps((a[2], a[3]), (b[2], b[3]))


_ENV_SIZES = {0: 0, 1: 32, 2: 48, 3: 48, 4: 64}


def gpkg_envelope_2d(g):
    """(envelope (minx, maxx, miny, maxy) | None, empty?) of GPKG bytes: the stored envelope, else a
    point's (x, x, y, y) — what geom_envelope + OGR's GetEnvelope give without OGR
    (kart/geometry.py:638-700).  Raises NotImplementedError where OGR would be needed."""
    g = bytes(g)
    if len(g) < 8 or g[:2] != b"GP" or g[2] != 0:
        raise ValueError("Expected GeoPackage Binary Geometry")
    flags = g[3]
    if flags & 0x20:
        raise NotImplementedError("ExtendedGeoPackageBinary")
    if flags & 0x10:
        return None, True
    et = (flags >> 1) & 7
    if et not in _ENV_SIZES:
        raise ValueError("Invalid envelope contents indicator")
    end = "<" if flags & 1 else ">"
    if et:
        env = struct.unpack_from(end + "dddd", g, 8)
        if not any(c != c for c in env):
            return env, False
    off = 8 + _ENV_SIZES[et]
    if len(g) >= off + 21:
        wend = "<" if g[off] == 1 else ">"
        typ = struct.unpack_from(wend + "I", g, off + 1)[0] & 0x0FFFFFFF
        if typ >= 1000:
            typ %= 1000
        if typ == 1:
            x, y = struct.unpack_from(wend + "dd", g, off + 5)
            if x != x and y != y:
                return None, True  # empty point
            return (x, x, y, y), False
    raise NotImplementedError("envelope needs OGR")


class SpatialFilter:
    """A spatial filter in a dataset's CRS: ``filter_env`` (min-x, max-x, min-y, max-y) of the filter
    geometry, the dataset's geometry column, and the exact test ``intersects(gpkg_bytes) -> bool``
    (the prepared filter geometry's Intersects; optional)."""

    def __init__(self, filter_env=None, geom_column_name=None, intersects=None, rectangle=False, match_all=False):
        self.match_all = match_all
        self.filter_env = None if match_all else tuple(float(x) for x in filter_env)
        self.geom_column_name = geom_column_name
        self.intersects = intersects
        self.rectangle = bool(rectangle)
        self.stats = {"unverified": 0}

    @classmethod
    def from_rectangle(cls, min_x, max_x, min_y, max_y, geom_column_name=None):
        """an axis-aligned rectangle filter (e.g. bbox_as_wkt_polygon): Intersects is decided by the
        envelopes alone for points and for envelopes inside it"""
        return cls((min_x, max_x, min_y, max_y), geom_column_name, rectangle=True)

    @classmethod
    def from_ring(cls, ring, geom_column_name=None, intersects=None):
        """a polygon filter from its exterior ring [(x, y), ...]; a point's Intersects is tested
        exactly (point in polygon, boundary included), other geometries need ``intersects``"""
        xs, ys = [p[0] for p in ring], [p[1] for p in ring]
        env = (min(xs), max(xs), min(ys), max(ys))
        corners = {(env[0], env[2]), (env[1], env[2]), (env[1], env[3]), (env[0], env[3])}
        rect = len(set(ring)) == 4 and set(ring) == corners
        return cls(env, geom_column_name, intersects=intersects or _ring_point_test(ring), rectangle=rect)

    def for_schema(self, schema):
        """transform_for_schema_and_crs (identity CRS): the dataset's first geometry column; a schema
        without one (or no schema) matches everything"""
        if self.match_all or schema is None:
            return SpatialFilter.MATCH_ALL
        cols = [c for c in schema.columns if c.data_type == "geometry"]
        if not cols:
            return SpatialFilter.MATCH_ALL
        out = SpatialFilter(self.filter_env, cols[0].name, self.intersects, self.rectangle)
        out.stats = self.stats
        return out

    # ---- the reference's per-feature interface (host) -------------------------------------------
    def matches(self, feature):
        """SpatialFilter.matches (kart/spatial_filter/__init__.py:534-590)"""
        if feature is None:
            return MatchResult.NONEXISTENT
        if self.match_all:
            return MatchResult.MATCHING
        g = feature[self.geom_column_name]
        if g is None:
            return MatchResult.MATCHING
        return self.matches_geometry(g)

    def matches_geometry(self, g):
        try:
            env, empty = gpkg_envelope_2d(g)
        except NotImplementedError:
            env, empty = None, False
        if empty:
            return MatchResult.NON_MATCHING  # Intersects(empty) is False
        if env is not None and not bbox_intersects_fast(self.filter_env, env):
            return MatchResult.NON_MATCHING
        return self._exact(g, env)

    def _exact(self, g, env):
        if env is not None and self.rectangle and self._inside(env):
            return MatchResult.MATCHING
        if self.intersects is not None:
            r = self.intersects(bytes(g))
            if r is not None:
                return MatchResult.MATCHING if r else MatchResult.NON_MATCHING
        self.stats["unverified"] += 1
        return MatchResult.MATCHING

    def _inside(self, env):
        f = self.filter_env
        return f[0] <= env[0] and env[1] <= f[1] and f[2] <= env[2] and env[3] <= f[3]

    def matches_delta_value(self, kv):
        """kart/spatial_filter/__init__.py:592-605: None -> NONEXISTENT, a promised blob -> PROMISED"""
        if kv is None:
            return MatchResult.NONEXISTENT
        try:
            return self.matches(kv.get_lazy_value())
        except KeyError as e:
            if not self.match_all and getattr(e, "subcode", None) == -3003:  # EOBJECTPROMISED
                return MatchResult.PROMISED
            raise


SpatialFilter.MATCH_ALL = SpatialFilter(match_all=True)


def _ring_point_test(ring):
    """intersects() for point geometries against a polygon ring (boundary counts as inside);
    None (undecided) for other geometries"""
    pts = [(float(x), float(y)) for x, y in ring]

    def test(g):
        try:
            env, empty = gpkg_envelope_2d(g)
        except NotImplementedError:
            return None
        if empty or env is None or env[0] != env[1] or env[2] != env[3]:
            return None
        x, y = env[0], env[2]
        inside = False
        for (x1, y1), (x2, y2) in zip(pts, pts[1:] + pts[:1]):
            if min(x1, x2) <= x <= max(x1, x2) and min(y1, y2) <= y <= max(y1, y2) and \
                    (x2 - x1) * (y - y1) == (y2 - y1) * (x - x1):
                return True  # on an edge
            if (y1 > y) != (y2 > y) and x < (x2 - x1) * (y - y1) / (y2 - y1) + x1:
                inside = not inside
        return inside

    return test


class GeomCols:
    """kd_geom_cols for one (old, new) pair of dataset versions: per legend, the value index of the
    geometry column the filter reads (-1: the legend has no such column -> value None)."""

    def __init__(self, old_version, new_version, old_name, new_name):
        self.old_hex, self.old_gidx, self.old_map = self._side(old_version, old_name)
        self.new_hex, self.new_gidx, self.new_map = self._side(new_version, new_name)

    @staticmethod
    def _side(version, name):
        if version is None:
            return np.zeros(40, np.uint8), np.zeros(1, np.int16), {}
        hashes = sorted(version.legends)
        col = next((c for c in version.schema.columns if c.name == name), None) if name else None
        gidx, m = [], {}
        for h in hashes:
            nonpk = list(version.legends[h].non_pk_columns)
            gi = nonpk.index(col.id) if col is not None and col.id in nonpk else -1
            gidx.append(gi)
            m[h] = gi
        hexarr = np.frombuffer(b"".join(h.encode("ascii") for h in hashes), np.uint8).copy() if hashes \
            else np.zeros(40, np.uint8)
        return hexarr, np.asarray(gidx or [0], np.int16), m

    def kd_cols(self):
        c = N.KdGeomCols()
        c.n_leg_old = len(self.old_map)
        c.n_leg_new = len(self.new_map)
        c.leg_old_hex = N.ptr(self.old_hex)
        c.gidx_old = N.ptr(self.old_gidx)
        c.leg_new_hex = N.ptr(self.new_hex)
        c.gidx_new = N.ptr(self.new_gidx)
        return c


def geom_filter(engine, old_arena, new_arena, pairs, cols, filt_env, rectangle=False, bits=0):
    """kd_geom_filter over host arenas: (codes uint8 [n, 2], keep uint32 [k], enc, enc_ok)."""
    (od, oo), (nd, no) = old_arena, new_arena
    pairs = np.ascontiguousarray(pairs, np.uint32).reshape(-1, 2)
    n = pairs.shape[0]
    blobs = []
    for d, o in ((od, oo), (nd, no)):
        b = N.KdBlobs()
        b.n = int(o.shape[0]) - 1
        b.data = N.ptr(d) if d.size else N.ptr(_PAD)
        b.off = N.ptr(o)
        b.mem = N.KD_MEM_HOST
        blobs.append(b)
    match = np.zeros((max(n, 1), 2), np.uint8)
    keep = np.zeros(max(n, 1), np.uint32)
    nk = ctypes.c_uint64()
    nb = bits // 2
    enc = np.zeros((max(n, 1), max(nb, 1)), np.uint8) if bits else None
    ok = np.zeros(max(n, 1), np.uint8) if bits else None
    fe = (ctypes.c_double * 4)(*[float(x) for x in filt_env])
    kc = cols.kd_cols()
    N.check(engine.L.kd_geom_filter(engine.ctx, ctypes.byref(blobs[0]), ctypes.byref(blobs[1]), N.ptr(pairs), n, None,
                                    N.KD_MEM_HOST, ctypes.byref(kc), fe, N.KD_GF_RECT if rectangle else 0, int(bits),
                                    N.ptr(match), N.ptr(keep), ctypes.byref(nk), N.ptr(enc), N.ptr(ok), N.KD_MEM_HOST),
            "kd_geom_filter")
    k = int(nk.value)
    return match[:n], keep[:k], (enc[:n] if bits else None), (ok[:n] if bits else None)


# kd_geom_head: the first 40 bytes of a blob's geometry value, its length, (status << 24) | offset
GEOM_HEAD = np.dtype([("gpkg", np.uint8, 40), ("glen", "<u4"), ("goff_status", "<u4")])


def geom_heads(data, off, hexarr, gidx, n_leg, threads=0):
    """kd_geom_heads over a host arena of feature blobs: one 48-byte head per blob (status
    KD_GH_GEOM / KD_GH_NULL / KD_GH_FALLBACK in the top byte of goff_status)"""
    data = np.ascontiguousarray(data, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    n = int(off.shape[0]) - 1
    out = np.zeros(max(n, 1), GEOM_HEAD)
    N.check(N.lib().kd_geom_heads(N.ptr(data) if data.size else N.ptr(_PAD), N.ptr(off), n, int(n_leg), N.ptr(hexarr),
                                  N.ptr(gidx), int(threads), out.ctypes.data), "kd_geom_heads")
    return out[:n]


def geom_filter_heads(engine, old_heads, new_heads, pairs, filt_env, rectangle=False, bits=0, arenas=None,
                      delta_heads=False):
    """kd_geom_filter_heads over host heads: (codes uint8 [n, 2], keep uint32 [k], enc, enc_ok).
    ``arenas`` ((od, oo), (nd, no)) for the geometries whose decode needs more than their head;
    without them such sides come back 3 (FALLBACK: the host decides).  ``delta_heads``: the heads are
    in delta order (row d = delta d's, ceil(n / 64) * 64 rows per side: KD_GF_DELTA_HEADS, the dense
    kernel); else the pairs index them."""
    pairs = np.ascontiguousarray(pairs, np.uint32).reshape(-1, 2)
    n = pairs.shape[0]
    hs = [np.ascontiguousarray(h, GEOM_HEAD) for h in (old_heads, new_heads)]
    blobs = [None, None]
    if arenas is not None:
        for s, (d, o) in enumerate(arenas):
            b = N.KdBlobs()
            b.n = int(o.shape[0]) - 1
            b.data = N.ptr(d) if d.size else N.ptr(_PAD)
            b.off = N.ptr(o)
            b.mem = N.KD_MEM_HOST
            blobs[s] = b
    match = np.zeros((max(n, 1), 2), np.uint8)
    keep = np.zeros(max(n, 1), np.uint32)
    nk = ctypes.c_uint64()
    nb = bits // 2
    enc = np.zeros((max(n, 1), max(nb, 1)), np.uint8) if bits else None
    ok = np.zeros(max(n, 1), np.uint8) if bits else None
    fe = (ctypes.c_double * 4)(*[float(x) for x in filt_env])
    N.check(engine.L.kd_geom_filter_heads(
        engine.ctx, hs[0].ctypes.data if hs[0].size else None, hs[0].shape[0], hs[1].ctypes.data if hs[1].size else None,
        hs[1].shape[0], N.KD_MEM_HOST, ctypes.byref(blobs[0]) if blobs[0] else None,
        ctypes.byref(blobs[1]) if blobs[1] else None, N.ptr(pairs), n, None, N.KD_MEM_HOST, fe,
        (N.KD_GF_RECT if rectangle else 0) | (N.KD_GF_DELTA_HEADS if delta_heads else 0), int(bits), N.ptr(match), N.ptr(keep), ctypes.byref(nk), N.ptr(enc), N.ptr(ok),
        N.KD_MEM_HOST), "kd_geom_filter_heads")
    k = int(nk.value)
    return match[:n], keep[:k], (enc[:n] if bits else None), (ok[:n] if bits else None)


def _blob_of(kv):
    """the LazyBlob behind a delta half's lazy value (Delta.old / .new), or None"""
    if kv is None:
        return None
    v = kv.value if hasattr(kv, "value") else None
    args = getattr(v, "args", None)
    return args[0] if args else None


def filtered_ds_feature_deltas(engine, ds_diff, old_version, new_version, spatial_filter):
    """BaseDiffWriter.filtered_ds_feature_deltas (kart/base_diff_writer.py:279-329): yields
    (key, delta) of ds_diff["feature"].sorted_items() whose old or new value matches the filter
    (working-copy edits always).  old_version / new_version: the DatasetVersions the deltas came
    from (their schemas place the geometry column)."""
    if "feature" not in ds_diff:
        return
    items = ds_diff["feature"].sorted_items()
    if spatial_filter.match_all:
        yield from items
        return
    old_sf = spatial_filter.for_schema(old_version.schema if old_version is not None else None)
    new_sf = spatial_filter.for_schema(new_version.schema if new_version is not None else None)
    if old_sf.match_all and new_sf.match_all:
        yield from items
        return
    n = len(items)
    if n == 0:
        return
    # the old / new blobs of every delta, batch-read per dataset version

    promised = np.zeros((n, 2), bool)
    sides = []
    pairs = np.full((n, 2), N.KD_NONE, np.uint32)
    for s, attr in enumerate(("old", "new")):
        blobs, rows = [], []
        for i, (_, d) in enumerate(items):
            b = _blob_of(getattr(d, attr))
            if b is not None:
                blobs.append(b)
                rows.append(i)
        data, off, ok = _safe_arena(blobs)
        for j, i in enumerate(rows):
            if ok[j]:
                pairs[i, s] = j
            else:
                promised[i, s] = True
        sides.append((data, off))
    cols = GeomCols(old_version, new_version, old_sf.geom_column_name, new_sf.geom_column_name)
    env = (old_sf if not old_sf.match_all else new_sf).filter_env
    rect = (old_sf if not old_sf.match_all else new_sf).rectangle
    # the blob reader's host pass: 48-byte geometry heads, the only bytes that go to the GPU (a
    # geometry whose decode needs more comes back FALLBACK and is decided below on the host)
    heads = [geom_heads(sides[0][0], sides[0][1], cols.old_hex, cols.old_gidx, len(cols.old_map)),
             geom_heads(sides[1][0], sides[1][1], cols.new_hex, cols.new_gidx, len(cols.new_map))]
    # laid out in delta order (row i = delta i's head; an absent side's row is never read): the dense
    # kernel reads its heads without a pair -> head dependency
    slots = (n + 63) // 64 * 64
    dense = []
    for s, h in enumerate(heads):
        d = np.zeros(slots, GEOM_HEAD)
        pres = np.nonzero(pairs[:, s] != N.KD_NONE)[0]
        d[pres] = h[pairs[pres, s].astype(np.int64)]
        dense.append(d)
    codes, keep, _, _ = geom_filter_heads(engine, dense[0], dense[1], pairs, env, rect, delta_heads=True)
    kept = np.zeros(n, bool)
    kept[keep] = True
    for i, (key, d) in enumerate(items):
        wc = bool(getattr(d, "flags", 0) & WORKING_COPY_EDIT)
        if not (kept[i] or wc or promised[i].any()):
            continue
        res = []
        for s, (sf, attr) in enumerate(((old_sf, "old"), (new_sf, "new"))):
            kv = getattr(d, attr)
            if promised[i, s]:
                res.append(sf.matches_delta_value(kv))  # PROMISED, or the reference's KeyError
            elif sf.match_all:
                res.append(MatchResult.MATCHING if kv is not None else MatchResult.NONEXISTENT)
            else:
                res.append(_resolve(sf, int(codes[i, s]), kv))
        if wc or res[0] or res[1]:
            yield key, d


def _resolve(sf, code, kv):
    if code == CODE_NONE:
        return MatchResult.NONEXISTENT
    if code == CODE_NON:
        return MatchResult.NON_MATCHING
    if code == CODE_MATCH:
        return MatchResult.MATCHING
    if code == CODE_CAND:
        g = kv.get_lazy_value()[sf.geom_column_name]
        return sf._exact(g, None)
    return sf.matches(kv.get_lazy_value())  # FALLBACK: the host path decides


def _safe_arena(blobs):
    """(data, off, ok[]) of LazyBlobs; a blob missing from the repository gets ok False (its
    KeyError is raised — or turned into PROMISED — when that side is resolved on the host)"""
    from .dataset import prefetch_blobs

    ok = prefetch_blobs(blobs)
    raw = []
    for k, b in enumerate(blobs):
        if ok[k]:
            try:
                raw.append(bytes(b.data))
            except KeyError:
                ok[k] = False
                raw.append(b"")
        else:
            raw.append(b"")
    data, off = packing._arena(raw)
    return data, off, ok
