import sys, numpy as np
sys.path.insert(0, '.')
from kart_amd import packing
from kart_amd.engine import Engine
from kart_amd import _native as N
e = Engine(0)
rng = np.random.default_rng(1)
for n in [100, 511, 512, 513, 1000, 1500, 3000]:
    for kind in ["rand", "small"]:
        k = np.unique(rng.integers(0, 2**63, size=n + 10, dtype=np.uint64))[:n] if kind == "rand" else np.arange(n, dtype=np.uint64) * 7 + 5
        o = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
        A = packing.PackedSide(k, o, 0, np.arange(n)); B = packing.PackedSide(k.copy(), o.copy(), 0, np.arange(n))
        try:
            r = e.diff2(A, B)
            print(n, kind, "ok", r.n_insert, r.n_update, r.n_delete)
        except N.Unsupported as ex:
            print(n, kind, "ERR", ex)
