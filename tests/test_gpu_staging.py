"""Host-form entry points across the library's transfer paths (kd_ctx.hip): inputs below 64 KB and
from 32 MB up go through the runtime's pageable copies, those in between through the two pinned
4-MB chunks (stage_h2d, several chunks per buffer); results come back through k_to_host into the
mapped pinned chunks (stage_d2h) or, from 32 MB up, pageable.  Every size class, interleaved in
one context (workspaces grow, the chunk ring keeps turning), must equal the oracle bit for bit."""
import numpy as np
import pytest

from kart_amd import packing
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _sides(n, seed):
    """two int-key sides of about n entries: half the keys shared, a tenth of those re-versioned"""
    rng = np.random.default_rng(seed)
    kA = np.arange(0, 2 * n, 2, dtype=np.uint64)
    kB = np.arange(n, 3 * n, 2, dtype=np.uint64) if n > 1 else kA.copy()
    oA = rng.integers(0, 256, size=(kA.size, 20), dtype=np.uint8)
    oB = rng.integers(0, 256, size=(kB.size, 20), dtype=np.uint8)
    # shared keys keep A's OID unless re-versioned
    ia = np.searchsorted(kA, kB)
    shared = (ia < kA.size) & (kA[np.minimum(ia, kA.size - 1)] == kB)
    keep = shared & (rng.random(kB.size) >= 0.1)
    oB[keep] = oA[ia[keep]]
    A = packing.PackedSide(kA, oA, 0, np.arange(kA.size))
    B = packing.PackedSide(kB, oB, 0, np.arange(kB.size))
    return A, B


@pytest.mark.parametrize("sizes", [(1, 3000, 700_000, 2_200_000, 5000, 4_500_000, 700_001)])
def test_gpu_diff2_host_transfer_sizes(engine, sizes):
    for i, n in enumerate(sizes):
        A, B = _sides(n, seed=100 + i)
        r = engine.diff2(A, B)
        od, oc = O.classify2(A.key, A.oid, B.key, B.oid)
        assert np.array_equal(r.delta, od), n
        assert (r.n_insert, r.n_update, r.n_delete) == (oc["inserts"], oc["updates"], oc["deletes"]), n
        # the update list is the delta list's matched rows
        m = (od[:, 0] != 0xFFFFFFFF) & (od[:, 1] != 0xFFFFFFFF)
        assert np.array_equal(r.upd, od[m]), n


def test_gpu_merge3_host_transfer_sizes(engine):
    for n in (2000, 900_000):
        rng = np.random.default_rng(n)
        k = np.arange(n, dtype=np.uint64) * 3
        oK = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
        oO, oT = oK.copy(), oK.copy()
        chg_o, chg_t = rng.random(n) < 0.2, rng.random(n) < 0.2
        oO[chg_o] ^= 1
        oT[chg_t] ^= 2
        sides = [packing.PackedSide(k, o, 0, np.arange(n)) for o in (oK, oO, oT)]
        r = engine.merge3(*sides)
        oc, om, ocl = O.classify3(k, oK, k, oO, k, oT)
        assert np.array_equal(r.conflict.reshape(-1, 3), np.asarray(oc).reshape(-1, 3)), n
        assert np.array_equal(r.mdelta.reshape(-1, 2), np.asarray(om).reshape(-1, 2)), n
        assert r.n_clean == ocl and r.conflict.shape[0] == int((chg_o & chg_t).sum()), n
