"""Delta / DeltaDiff / DatasetDiff / RepoDiff: the boundary contract's output types.

Behavioural mirror of kart/diff_structs.py (KeyValue :12-40, Delta :47-188 incl. the
concatenation algebra :142-180, DeltaDiff :375-458, DatasetDiff/RepoDiff :461-480), so the engine
can hand back objects the diff writers already understand.  Inside Kart the engine returns
``kart.diff_structs`` itself (``kart_amd.adaptor.use_structs``, picked automatically when Kart is
importable); this module is what it uses when Kart is not (this repo's tests, the GPU box).
"""
from collections import UserDict
from numbers import Number

WORKING_COPY_EDIT = 0x1


class Conflict(Exception):
    pass


class KeyValue:
    """(key, value) where value may be a zero-arg callable evaluated at most once."""

    __slots__ = ("key", "value", "_cache")

    def __init__(self, key, value):
        self.key = key
        self.value = value

    @classmethod
    def of(cls, obj):
        if type(obj) is tuple and len(obj) == 2:
            return cls(obj[0], obj[1])
        if obj is None or isinstance(obj, KeyValue):
            return obj
        if isinstance(obj, tuple):
            return cls(*obj)
        raise ValueError(f"Expected (key, value) tuple - got {type(obj)}")

    def get_lazy_value(self):
        if not callable(self.value):
            return self.value
        try:
            return self._cache
        except AttributeError:
            self._cache = self.value()
            return self._cache

    def __eq__(self, other):
        return isinstance(other, KeyValue) and (self.key, self.value) == (other.key, other.value)

    def __repr__(self):
        return f"KeyValue(key={self.key!r}, value={self.value!r})"


class Delta:
    """old -> new change of one object; either side may be None (insert / delete).  The fields are
    slots (filled directly by the native delta builder, kart_amd/csrc/kd_pystr.c); ``__dict__`` keeps
    other attributes settable as on the reference's class."""

    __slots__ = ("old", "new", "type", "flags", "changed_fields", "__dict__")

    def __init__(self, old, new):
        self.old = old = KeyValue.of(old)
        self.new = new = KeyValue.of(new)
        if old is None:
            if new is None:
                raise ValueError("Empty Delta")
            self.type = "insert"
        else:
            self.type = "delete" if new is None else "update"
        self.flags = 0

    insert = staticmethod(lambda new: Delta(None, new))
    update = staticmethod(lambda old, new: Delta(old, new))
    delete = staticmethod(lambda old: Delta(old, None))

    @staticmethod
    def maybe_update(old, new):
        return None if old.get_lazy_value() == new.get_lazy_value() else Delta(old, new)

    def __invert__(self):
        return Delta(self.new, self.old)

    @property
    def old_key(self):
        return None if self.old is None else self.old.key

    @property
    def new_key(self):
        return None if self.new is None else self.new.key

    @property
    def old_value(self):
        return None if self.old is None else self.old.get_lazy_value()

    @property
    def new_value(self):
        return None if self.new is None else self.new.get_lazy_value()

    @property
    def key(self):
        k = self.old_key
        return k if k is not None else self.new_key

    # (self.type, other.type) -> result constructor; None = both sides cancel; Conflict raises
    def __add__(self, other):
        kind = (self.type, other.type)
        if kind in (("insert", "insert"), ("update", "insert"), ("delete", "delete"), ("delete", "update")):
            raise Conflict()
        if kind == ("insert", "update"):
            result = Delta.insert(other.new)
        elif kind == ("insert", "delete"):
            result = None
        elif kind == ("update", "update") or kind == ("delete", "insert"):
            result = Delta.maybe_update(self.old, other.new)
        else:  # ("update", "delete")
            result = Delta.delete(self.old)
        if result is not None:
            result.flags = self.flags | other.flags
        return result

    def __eq__(self, other):
        return isinstance(other, Delta) and (self.old, self.new) == (other.old, other.new)

    def to_plus_minus_dict(self):
        d = {}
        if self.old:
            d["-"] = self.old_value
        if self.new:
            d["+"] = self.new_value
        return d

    def __repr__(self):
        return f"Delta(old={self.old!r}, new={self.new!r})"


class _TypedDict(UserDict):
    child_type = None

    def __setitem__(self, key, value):
        if type(value) is not self.child_type:
            raise TypeError(f"{type(self).__name__} accepts {self.child_type.__name__}, got {type(value).__name__}")
        super().__setitem__(key, value)

    def copy(self):
        return type(self)(self)

    def empty_copy(self):
        return type(self)()

    def __eq__(self, other):
        return type(self) is type(other) and self.data == other.data

    def prune(self, recurse=True):
        if not issubclass(self.child_type, _TypedDict):
            return
        for key in list(self.keys()):
            child = self[key]
            if recurse:
                child.prune()
            if not child:
                del self[key]

    @classmethod
    def concatenated(cls, *diffs, overwrite_original=False):
        result = None
        for d in diffs:
            if d is None:
                continue
            if result is None:
                result = d
            elif overwrite_original:
                result += d
            else:
                result = result + d
        return cls() if result is None else result

    def __invert__(self):
        out = self.empty_copy()
        for k, v in self.items():
            out[k] = ~v
        return out

    def _combine(self, other, out):
        if type(self) is not type(other):
            raise TypeError(f"Diff type mismatch: {type(self)} != {type(other)}")
        for key in other.keys():
            rhs = other[key]
            lhs = out.get(key)
            if lhs is None:
                out[key] = rhs
                continue
            both = lhs + rhs
            if both:
                out[key] = both
            else:
                out.pop(key, None)
        return out

    def __add__(self, other):
        return self._combine(other, self.copy())

    def __iadd__(self, other):
        return self._combine(other, self)

    def type_counts(self):
        return {k: v.type_counts() for k, v in self.items()}

    def __json__(self):
        return dict(self.items())


class DeltaDiff(_TypedDict):
    """{key: Delta}, every delta stored at its own key."""

    child_type = Delta

    def __init__(self, initial=()):
        super().__init__()
        if isinstance(initial, (dict, UserDict)):
            for k, v in initial.items():
                self[k] = v
        else:
            data = self.data
            for delta in initial:  # add_delta, inlined for bulk construction
                if type(delta) is not Delta:
                    self.add_delta(delta)  # raises the type error
                old = delta.old
                data[old.key if old is not None else delta.new.key] = delta

    def __setitem__(self, key, delta):
        if key != delta.key:
            raise ValueError("Delta must be added at the appropriate key")
        super().__setitem__(key, delta)

    def add_delta(self, delta):
        self[delta.key] = delta

    def __invert__(self):
        out = self.empty_copy()
        for d in self.values():
            out.add_delta(~d)
        return out

    def to_filter(self):
        keys = set()
        for d in self.values():
            if d.old is not None:
                keys.add(str(d.old.key))
            if d.new is not None:
                keys.add(str(d.new.key))
        return keys

    def type_counts(self):
        counts = {}
        for d in self.values():
            counts[d.type] = counts.get(d.type, 0) + 1
        return {f"{t}s": n for t, n in counts.items()}

    @classmethod
    def diff_dicts_as_deltas(cls, old, new, delta_flags=0):
        for k in set(old) | set(new):
            a, b = old.get(k), new.get(k)
            if a == b:
                continue
            d = Delta((k, a) if a is not None else None, (k, b) if b is not None else None)
            d.flags = delta_flags
            yield d

    @classmethod
    def diff_dicts(cls, old, new, delta_flags=0):
        return cls(cls.diff_dicts_as_deltas(old, new, delta_flags))

    def sorted_items(self):
        """None first, then numbers ascending, then strings (others by str())."""
        inf = float("inf")

        def order(item):
            k = item[0]
            if k is None:
                return (-inf, "")
            if isinstance(k, Number):
                return (k, "")
            return (inf, k if isinstance(k, str) else str(k))

        return sorted(self.items(), key=order)


class DatasetDiff(_TypedDict):
    child_type = DeltaDiff

    def __json__(self):
        out = {}
        if "meta" in self:
            out["meta"] = {k: v.to_plus_minus_dict() for k, v in self["meta"].items()}
        if "feature" in self:
            out["feature"] = (v for _, v in self["feature"].sorted_items())
        return out


class RepoDiff(_TypedDict):
    child_type = DatasetDiff
