"""Which diff structures the engine returns.

Inside Kart the engine must hand back Kart's own ``kart.diff_structs`` objects (``Delta``,
``DeltaDiff``, ``DatasetDiff``, ...; kart/diff_structs.py:12-480) so the text / JSON / HTML / quiet
writers, ``status`` and ``merge`` consume them unchanged.  ``use_structs(kart.diff_structs)`` points
the engine at them (INTEGRATION.md does this at import); when Kart itself is importable that
module is picked up automatically.  Without Kart (this repository's tests, the GPU box) the
behavioural mirror ``kart_amd.deltas`` is used.
"""
import types

_NAMES = ("KeyValue", "Delta", "DeltaDiff", "DatasetDiff", "RepoDiff")
_structs = None


def use_structs(module):
    """Return ``module``'s diff structures from now on (a module or object with the five classes)."""
    global _structs
    missing = [n for n in _NAMES if not hasattr(module, n)]
    if missing:
        raise TypeError(f"{module!r} lacks {missing}")
    _structs = types.SimpleNamespace(**{n: getattr(module, n) for n in _NAMES}, source=getattr(module, "__name__", repr(module)))
    return _structs


def structs():
    """The active diff structures (kart.diff_structs when Kart is importable, else kart_amd.deltas)."""
    if _structs is None:
        try:
            import kart.diff_structs as ds  # inside a Kart installation
        except Exception:
            from . import deltas as ds
        use_structs(ds)
    return _structs


def reset():
    """forget the choice (tests)"""
    global _structs
    _structs = None
