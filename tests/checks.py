"""Shared golden-vector checks, parameterised by the implementation under test
(HIP engine in -m gpu tests, the C oracle in CPU tests)."""
import os

import numpy as np

from fixtures import load, pk_of
from kart_amd import packing
from kart_amd.schema import FieldMaps

NONE = 0xFFFFFFFF


def _pk(fx, key, k):
    side = fx.packed(key)
    if side.key_mode == 0:  # KD_KEY_INT: pk straight from the key
        return int(packing.int_keys_to_pks(side.key[k:k + 1])[0])
    from oracle.oracle import decode_pk_from_filename
    name = fx.sorted_names(key)[k]
    return decode_pk_from_filename(os.path.basename(name))


def delta_set(fx, base, target, delta):
    out = set()
    for a, b in delta.tolist():
        old = _pk(fx, base, a) if a != NONE else None
        new = _pk(fx, target, b) if b != NONE else None
        t = "insert" if a == NONE else "delete" if b == NONE else "update"
        out.add((t, old, new))
    return out


def golden_set(case):
    return {(d["type"], pk_of(d["old_pk"]), pk_of(d["new_pk"])) for d in case["deltas"]}


def field_maps(fx, base, target):
    return FieldMaps(fx.schema(base), fx.legends, fx.schema(target), fx.legends)


def check_diff_case(fx, case, classify, fielddiff):
    """classify(PackedSide, PackedSide) -> (delta [n,2], upd [m,2], counts dict)
    fielddiff(old_data, old_off, new_data, new_off, pairs, maps) -> (masks, status)"""
    base, target = case["base"], case["target"]
    A, B = fx.packed(base), fx.packed(target)
    delta, upd, counts = classify(A, B)
    got = delta_set(fx, base, target, delta)
    want = golden_set(case)
    assert got == want, (fx.name, base, target, sorted(got ^ want, key=str)[:10])
    want_counts = {k: v for k, v in case["counts"].items() if v}
    assert {k: v for k, v in counts.items() if v} == want_counts
    # key order of the delta list: base/target keys ascending
    keys = [A.key[a] if a != NONE else B.key[b] for a, b in delta.tolist()]
    assert all(int(x) < int(y) for x, y in zip(keys, keys[1:]))
    if upd.shape[0] == 0:
        return 0
    maps = field_maps(fx, base, target)
    od, oo = fx.arena(base)
    nd, no = fx.arena(target)
    masks, status = fielddiff(od, oo, nd, no, upd, maps)
    assert not status.any(), (fx.name, np.unique(status))
    golden_changed = {}
    for d in case["deltas"]:
        if d["type"] == "update":
            golden_changed[pk_of(d["old_pk"])] = d["changed"]
    for u, (a, b) in enumerate(upd.tolist()):
        pk = _pk(fx, base, a)
        assert maps.changed_names(masks[u]) == golden_changed[pk], (fx.name, pk)
    return upd.shape[0]


def check_merge_case(fx, case, merge3):
    """merge3(PackedSide x3) -> (conflicts [n,3], mdelta [m,2], n_clean)"""
    keys = case["sides"]
    sides = [fx.packed(k) for k in keys]
    conf, md, n_clean = merge3(*sides)
    names = [fx.sorted_names(k) for k in keys]
    oids = [fx.packed(k).oid for k in keys]
    ds = fx.meta["ds_path"] + "/.table-dataset/feature/"
    got = set()
    for row in conf.tolist():
        path = next(names[s][i] for s, i in enumerate(row) if i != NONE)
        got.add((ds + path,) + tuple(oids[s][i].tobytes().hex() if i != NONE else None for s, i in enumerate(row)))
    want = {(c["path"], c["ancestor"], c["ours"], c["theirs"]) for c in case["conflicts"]
            if c["path"].startswith(ds)}
    assert got == want, (fx.name, got ^ want)
    # merged entries (feature paths) = ours + mdeltas applied, minus conflicts
    ours = {names[1][i]: oids[1][i].tobytes().hex() for i in range(len(names[1]))}
    for o, t in md.tolist():
        if o != NONE:
            del ours[names[1][o]]
        if t != NONE:
            ours[names[2][t]] = oids[2][t].tobytes().hex()
    conflict_paths = {p[len(ds):] for p, *_ in want}
    merged = {p: v for p, v in ours.items() if p not in conflict_paths}
    want_entries = {p[len(ds):]: v for p, v in case["entries_sha"] if p.startswith(ds) and p[len(ds):] not in conflict_paths}
    assert merged == want_entries
    assert n_clean == len(want_entries)
