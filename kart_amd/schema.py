"""Schema / Legend host mirror and the legend -> union-key maps that kd_fielddiff consumes.

Reference: Legend (kart/schema.py:19-102), Schema.feature_from_raw_dict (:288-293),
Legend.value_tuples_to_raw_dict (:66-79), BaseDiffWriter._all_feature_keys
(kart/base_diff_writer.py:181-187) and the text writer's field loop
(kart/text_diff_writer.py:135-145).

For an update delta the reference builds ``old = {c.name: raw_old.get(c.id) for c in old_schema}``
and ``new`` likewise, then marks key ``k`` (old keys in order, then new-only keys; ``__``-prefixed
keys skipped) changed iff ``old.get(k, _NULL) != new.get(k, _NULL)``.  Per side and per legend
this reduces to one source code per union key:

    >= 0  index into the blob's non-pk value array
    -1    key not in this side's schema            (-> _NULL)
    -2    column id not in this blob's legend      (-> None)
    -3    primary-key column                       (-> pk from the path, equal on both sides)
"""
import hashlib
from dataclasses import dataclass
from typing import Dict, List, Tuple

import msgpack
import numpy as np

from . import _native as N

SRC_NULL, SRC_NONE, SRC_PK = -1, -2, -3


@dataclass(frozen=True)
class Column:
    id: str
    name: str
    data_type: str
    pk_index: object = None


class Schema:
    def __init__(self, columns: List[Column]):
        self.columns = list(columns)

    @classmethod
    def from_column_dicts(cls, dicts):
        return cls([Column(d["id"], d["name"], d.get("dataType"), d.get("primaryKeyIndex")) for d in dicts])

    @property
    def pk_columns(self):
        return sorted([c for c in self.columns if c.pk_index is not None], key=lambda c: c.pk_index)

    @property
    def geometry_columns(self):
        return [c for c in self.columns if c.data_type == "geometry"]

    def names(self):
        return [c.name for c in self.columns]

    def feature_from_raw_dict(self, raw):
        return {c.name: raw.get(c.id, None) for c in self.columns}


class Legend:
    def __init__(self, pk_columns, non_pk_columns):
        self.pk_columns = tuple(pk_columns)
        self.non_pk_columns = tuple(non_pk_columns)

    @classmethod
    def loads(cls, data):
        pk, non_pk = msgpack.unpackb(data, raw=False)
        return cls(pk, non_pk)

    def dumps(self):
        return msgpack.packb([list(self.pk_columns), list(self.non_pk_columns)], use_bin_type=True)

    def hexhash(self):
        return hashlib.sha256(self.dumps()).hexdigest()[:40]

    def value_tuples_to_raw_dict(self, pk_values, non_pk_values):
        assert len(pk_values) == len(self.pk_columns)
        assert len(non_pk_values) == len(self.non_pk_columns)
        raw = dict(zip(self.pk_columns, pk_values))
        raw.update(zip(self.non_pk_columns, non_pk_values))
        return raw


def union_keys(old_schema, new_schema):
    """Field order of BaseDiffWriter._all_feature_keys: old keys, then new-only keys."""
    old = old_schema.names() if old_schema is not None else []
    new = new_schema.names() if new_schema is not None else []
    seen = set(old)
    return old + [k for k in new if k not in seen]


def side_maps(schema: Schema, legends: Dict[str, Legend], keys: List[str]) -> Tuple[List[str], np.ndarray]:
    """Per legend (sorted by hash), the source code of every union key for this side."""
    hashes = sorted(legends)
    by_name = {c.name: c for c in schema.columns} if schema is not None else {}
    m = np.full((max(len(hashes), 1), len(keys)), SRC_NULL, np.int16)
    for li, h in enumerate(hashes):
        lg = legends[h]
        pos = {cid: i for i, cid in enumerate(lg.non_pk_columns)}
        pks = set(lg.pk_columns)
        for k, name in enumerate(keys):
            c = by_name.get(name)
            if c is None:
                m[li, k] = SRC_NULL
            elif c.id in pks:
                m[li, k] = SRC_PK
            elif c.id in pos:
                m[li, k] = pos[c.id]
            else:
                m[li, k] = SRC_NONE
    return hashes, m


class FieldMaps:
    """Everything kd_fielddiff needs for one (old dataset version, new dataset version) pair."""

    def __init__(self, old_schema, old_legends, new_schema, new_legends):
        self.keys = union_keys(old_schema, new_schema)
        self.n_keys = len(self.keys)
        self.words = max(1, (self.n_keys + 63) // 64)
        self.old_hashes, self.map_old = side_maps(old_schema, old_legends, self.keys)
        self.new_hashes, self.map_new = side_maps(new_schema, new_legends, self.keys)
        self.leg_old_hex = self._hex(self.old_hashes)
        self.leg_new_hex = self._hex(self.new_hashes)
        self.cmp_mask = np.zeros(self.words, np.uint64)
        for k, name in enumerate(self.keys):
            if not name.startswith("__"):
                self.cmp_mask[k >> 6] |= np.uint64(1 << (k & 63))

    @staticmethod
    def _hex(hashes):
        if not hashes:
            return np.zeros(40, np.uint8)
        b = b"".join(h.encode("ascii") for h in hashes)
        assert len(b) == 40 * len(hashes), "legend hashes must be 40 hex chars"
        return np.frombuffer(b, np.uint8).copy()

    def kd_maps(self):
        s = N.KdLegendMaps()
        s.n_keys = self.n_keys
        s.words = self.words
        s.n_leg_old = max(1, len(self.old_hashes))
        s.n_leg_new = max(1, len(self.new_hashes))
        s.leg_old_hex = N.ptr(self.leg_old_hex)
        s.map_old = N.ptr(self.map_old)
        s.leg_new_hex = N.ptr(self.leg_new_hex)
        s.map_new = N.ptr(self.map_new)
        s.cmp_mask = N.ptr(self.cmp_mask)
        return s

    def changed_names(self, mask_row):
        """mask words of one update -> changed key names in union-key order"""
        out = []
        for k, name in enumerate(self.keys):
            if (int(mask_row[k >> 6]) >> (k & 63)) & 1:
                out.append(name)
        return out

    def changed_names_rows(self, masks):
        """changed_names of every row of ``masks`` [n, words], one fresh list per row; each
        distinct mask (a layer's updates share a handful) is decoded once"""
        masks = np.ascontiguousarray(masks, np.uint64).reshape(-1, self.words)
        if masks.shape[0] == 0:
            return []
        # one key per row (the words' bytes as one void scalar): np.unique(axis=0) sorts row
        # objects, ten times slower
        rows = masks.reshape(-1) if self.words == 1 else masks.view(np.dtype((np.void, 8 * self.words))).reshape(-1)
        uniq, inv = np.unique(rows, return_inverse=True)
        uniq = np.ascontiguousarray(uniq).view(np.uint64).reshape(-1, self.words)
        names = [list(self.changed_names(row)) for row in uniq]
        return list(map(list.copy, map(names.__getitem__, inv.reshape(-1).tolist())))
