"""Loading the committed golden fixtures (tests/golden/*.npz + *.json) into engine inputs.

The fixtures were generated from the reference itself by tests/golden/gen_golden.py; nothing here
reads /root/reference, so these run on the GPU box too.
"""
import functools
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from kart_amd import packing  # noqa: E402
from kart_amd.schema import Legend, Schema  # noqa: E402

DIFF_FIXTURES = ["repo_points", "repo_polygons", "repo_table", "repo_string_pks", "conflicts_points",
                 "conflicts_polygons", "conflicts_table", "synth_int", "synth_int_same", "synth_str", "meta_edits"]
MERGE_FIXTURES = ["conflicts_points", "conflicts_polygons", "conflicts_table"]


class Fixture:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.a = {k: z[k] for k in z.files}
        with open(os.path.join(GOLDEN, name + ".json")) as f:
            self.meta = json.load(f)
        self.blob_data = self.a["blob_data"]
        self.blob_off = self.a["blob_off"].astype(np.uint64)
        self.legends = {h: Legend(v[0], v[1]) for h, v in self.meta["legends"].items()}
        self._packed = {}

    def n(self, key):
        return self.meta["sides"][key]["n"]

    def names(self, key):
        d, o = self.a[f"{key}_names"], self.a[f"{key}_name_off"]
        return [d[o[i]:o[i + 1]].tobytes().decode() for i in range(len(o) - 1)]

    def oids(self, key):
        return self.a[f"{key}_oid"].reshape(-1, 20)

    def blob(self, i):
        return self.blob_data[int(self.blob_off[i]):int(self.blob_off[i + 1])].tobytes()

    def encoding(self, key):
        ps = self.meta["sides"][key]["path_structure"]
        if ps is None:  # empty side: use the other side's encoding
            for k, s in self.meta["sides"].items():
                if s["path_structure"] is not None:
                    ps = s["path_structure"]
                    break
        return packing.PathEncoding.from_dict(ps)

    def schema(self, key):
        sj = self.meta["sides"][key]["schema"]
        return Schema.from_column_dicts(sj) if sj is not None else None

    def packed(self, key):
        if key not in self._packed:
            enc = self.encoding(key)
            if self.n(key) == 0:
                self._packed[key] = packing.empty_side(enc)
            else:
                d = self.a[f"{key}_names"]
                o = self.a[f"{key}_name_off"].astype(np.uint64)
                self._packed[key] = packing.pack_side(d, self.oids(key), enc, rel_off=o)
        return self._packed[key]

    def meta_files(self, key):
        """{path relative to the meta tree: bytes} of a side (legends apart), as the repo holds them"""
        return {k: bytes.fromhex(v) for k, v in self.meta["sides"][key].get("meta_files", {}).items()}

    def attachments(self, key):
        return {k: bytes.fromhex(v) for k, v in self.meta["sides"][key].get("attachments", {}).items()}

    def sorted_names(self, key):
        names = self.names(key)
        return [names[i] for i in self.packed(key).order]

    def arena(self, key, sorted_order=True):
        """blob arena of a side's entries (in sorted-key order by default)"""
        idx = self.a[f"{key}_blob"]
        if sorted_order:
            idx = idx[self.packed(key).order]
        lens = (self.blob_off[idx + 1] - self.blob_off[idx]).astype(np.uint64)
        off = np.zeros(len(idx) + 1, np.uint64)
        off[1:] = np.cumsum(lens)
        data = np.concatenate([self.blob_data[int(self.blob_off[i]):int(self.blob_off[i + 1])] for i in idx]) \
            if len(idx) else np.zeros(0, np.uint8)
        return np.ascontiguousarray(data, np.uint8), off

    def cases(self, kind):
        return [c for c in self.meta["cases"] if c["kind"] == kind]


@functools.lru_cache(maxsize=None)
def load(name):
    return Fixture(name)


def pk_of(v):
    """golden json_safe pk -> python value"""
    if v is None:
        return None
    if "int" in v:
        return int(v["int"])
    if "str" in v:
        return v["str"]
    raise ValueError(v)
