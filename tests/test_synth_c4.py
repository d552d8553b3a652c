"""The C4 bench generator (kart_amd/synth.py table3_layers): MsgpackHashPathEncoder paths and the
planned conflict count, checked on the CPU against the oracle and a direct restatement of the path
encoder (kart/dataset3_paths.py:202-215; serialise_util.py:64-66, 82-85)."""
import base64
import hashlib

import numpy as np

from kart_amd import synth
from oracle import oracle as O


def _ref_path(pk):
    packed = b"\x91" + bytes([0xA0 | len(pk)]) + pk.encode()
    h = base64.urlsafe_b64encode(hashlib.sha256(packed).digest()[:20]).decode()
    return "/".join(h[:4]) + "/" + base64.urlsafe_b64encode(packed).decode()


def test_hash_paths_match_reference_encoder():
    ids = np.array([0, 1, 7, 123456, 999_999_999])
    p = synth._hash_paths(ids)
    for i, row in zip(ids, p):
        assert bytes(row).decode() == _ref_path("R%09d" % i)


def test_planned_conflicts_match_oracle():
    M = synth.table3_layers(60_000, seed=3)
    oc, om, ocl = O.classify3(M.ancestor.key, M.ancestor.oid, M.ours.key, M.ours.oid, M.theirs.key, M.theirs.oid)
    assert len(oc) == M.n_conflict > 0
    assert len(om) > 0
    # every side strictly ascending, names are the sorted entries' paths
    for s in (M.ancestor, M.ours, M.theirs):
        assert np.all(s.key[1:] > s.key[:-1])
        assert s.name.size == 24 * s.n
