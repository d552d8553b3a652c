"""The C ABI library builds/loads and exports exactly what include/kartdiff.h declares (CPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

from kart_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "kartdiff.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(kd_[a-z0-9_]+)\s*\(", src))


def test_header_matches_binding():
    assert _declared() == set(N.SIGNATURES)


def test_library_exports_every_symbol():
    L = N.lib()
    for name in _declared():
        assert hasattr(L, name), name
    assert L.kd_abi_version() == 1


def test_no_gpu_init_fails_cleanly():
    """Without a GPU, kd_init must fail with an error code (never crash, never fall back)."""
    ctx = ctypes.c_void_p()
    rc = N.lib().kd_init(0, ctypes.byref(ctx))
    if rc == N.KD_OK:
        N.lib().kd_fini(ctx)
        pytest.skip("GPU present")
    assert rc in (N.KD_EINVAL, N.KD_EHIP)
    assert N.lib().kd_last_error()


def test_library_loads_without_torch():
    """the product path needs no GPU framework: a fresh interpreter loads the library and the
    package without importing torch"""
    import subprocess
    import sys

    code = ("import sys; sys.path.insert(0, %r); from kart_amd import _native, engine, device, shard, dataset; "
            "_native.lib(); assert 'torch' not in sys.modules, 'torch imported'" % ROOT)
    subprocess.run([sys.executable, "-c", code], check=True)


def test_engine_requires_native(monkeypatch):
    """The product path raises loudly when the HIP library is absent."""
    monkeypatch.setattr(N, "_lib", None)
    monkeypatch.setattr(N, "LIB_PATH", "/nonexistent/libkartdiff.so")
    from kart_amd.engine import Engine

    with pytest.raises(N.NativeUnavailable):
        Engine(0)


def test_pack_int_keys_roundtrip():
    from kart_amd import packing

    rng = np.random.default_rng(0)
    pks = np.concatenate([rng.integers(-(2**63), 2**63 - 1, 5000, dtype=np.int64),
                          np.array([0, 1, -1, -64, 63, 64, 2**30, -(2**30), 2**63 - 1, -(2**63)], np.int64)])
    pks = np.unique(pks)
    import base64

    import msgpack

    names = ["A/A/A/A/" + base64.urlsafe_b64encode(msgpack.packb([int(p)])).decode() for p in pks]
    side = packing.pack_side(names, np.zeros((len(names), 20), np.uint8), packing.INT_PK_ENCODING)
    back = packing.int_keys_to_pks(side.key)
    assert np.array_equal(np.sort(back), np.sort(pks))
    assert np.array_equal(side.key, np.sort(side.key))
    # key order == pk order inside [-(2**30), 2**30) ... and the same bucket-major order the
    # vectorised synthetic generator uses
    from kart_amd.synth import _int_keys

    assert np.array_equal(np.sort(_int_keys(pks)), side.key)


def test_pack_rejects_bad_paths():
    from kart_amd import packing

    with pytest.raises(packing.PackError):
        packing.pack_side(["A/A/A/A/kQ0=", "A/A/A/A/!!"], np.zeros((2, 20), np.uint8), packing.INT_PK_ENCODING)
    with pytest.raises(packing.PackError):  # uint64 pk >= 2**63 is outside the key range
        import base64

        import msgpack

        n = base64.urlsafe_b64encode(msgpack.packb([2**64 - 1])).decode()
        packing.pack_side(["A/A/A/A/" + n], np.zeros((1, 20), np.uint8), packing.INT_PK_ENCODING)
