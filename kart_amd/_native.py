"""ctypes binding of libkartdiff.so (include/kartdiff.h).

The product path has no CPU fallback of its own: if the HIP library is missing or fails to load,
every engine call raises ``NativeUnavailable`` loudly.  (The reference-style CPU path that callers
fall back to on ``KD_EUNSUPPORTED`` is the caller's, i.e. Kart's own code, not ours.)
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KART_AMD_LIB", os.path.join(HERE, "libkartdiff.so"))

KD_OK = 0
KD_EINVAL = -1
KD_EHIP = -2
KD_EUNSUPPORTED = -3
KD_ENOTFOUND = -4
KD_WALK_ALL = -1
KD_NONE = 0xFFFFFFFF
KD_MEM_HOST = 0
KD_MEM_DEVICE = 1
KD_KEY_INT = 0
KD_KEY_HASH = 1
KD_DIFF_UNORDERED = 0x1
KD_HEX_BYTES = 0
KD_HEX_GPKG_WKB = 1
KD_COPY_H2D = 1
KD_COPY_D2H = 2
KD_COPY_D2D = 3
KD_COMM_ID_BYTES = 128
KD_GH_GEOM, KD_GH_NULL, KD_GH_FALLBACK = 0, 2, 3
KD_GF_RECT = 0x1
KD_GF_DELTA_HEADS = 0x2  # the geometry heads are in delta order (slot d = delta d)

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_i16p = ctypes.POINTER(ctypes.c_int16)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_dblp = ctypes.POINTER(ctypes.c_double)


class NativeUnavailable(RuntimeError):
    pass


class KdError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libkartdiff error {code}: {msg}")
        self.code = code


class Unsupported(KdError):
    """KD_EUNSUPPORTED: this input needs the reference CPU path."""


class NotFound(KdError):
    """KD_ENOTFOUND: a git object is not in the object database."""


class KdLeaves(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("path_off", c_u64p),
        ("mode", c_u32p),
        ("oid", c_u8p),
        ("path", c_u8p),
        ("present", ctypes.c_int32),
    ]


class KdSide(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("key", ctypes.c_void_p),
        ("oid", ctypes.c_void_p),
        ("name", ctypes.c_void_p),
        ("name_off", ctypes.c_void_p),
        ("mem", ctypes.c_uint32),
        ("key_mode", ctypes.c_uint32),
    ]


class KdBlobs(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("data", ctypes.c_void_p),
        ("off", ctypes.c_void_p),
        ("mem", ctypes.c_uint32),
        ("size_hint", ctypes.c_uint32),
    ]


class KdLegendMaps(ctypes.Structure):
    _fields_ = [
        ("n_keys", ctypes.c_int32),
        ("words", ctypes.c_int32),
        ("n_leg_old", ctypes.c_int32),
        ("n_leg_new", ctypes.c_int32),
        ("leg_old_hex", ctypes.c_void_p),
        ("map_old", ctypes.c_void_p),
        ("leg_new_hex", ctypes.c_void_p),
        ("map_new", ctypes.c_void_p),
        ("cmp_mask", ctypes.c_void_p),
    ]


class KdGeomCols(ctypes.Structure):
    _fields_ = [
        ("n_leg_old", ctypes.c_int32),
        ("n_leg_new", ctypes.c_int32),
        ("leg_old_hex", ctypes.c_void_p),
        ("gidx_old", ctypes.c_void_p),
        ("leg_new_hex", ctypes.c_void_p),
        ("gidx_new", ctypes.c_void_p),
    ]


class KdKeysInfo(ctypes.Structure):
    _fields_ = [
        ("vary", ctypes.c_uint64),
        ("key0", ctypes.c_uint64),
        ("pk_min", ctypes.c_int64),
        ("pk_max", ctypes.c_int64),
        ("ascending", ctypes.c_int32),
        ("seg_max", ctypes.c_int32),  # longest run of keys sharing their top 24 (bucket) bits; -1: buckets descend
    ]


class KdDiffResult(ctypes.Structure):
    _fields_ = [
        ("n_insert", ctypes.c_uint64),
        ("n_update", ctypes.c_uint64),
        ("n_delete", ctypes.c_uint64),
        ("n_delta", ctypes.c_uint64),
        ("delta", c_u32p),
        ("upd", c_u32p),
    ]


class KdMergeResult(ctypes.Structure):
    _fields_ = [
        ("n_clean", ctypes.c_uint64),
        ("n_conflict", ctypes.c_uint64),
        ("n_mdelta", ctypes.c_uint64),
        ("conflict", c_u32p),
        ("mdelta", c_u32p),
    ]


# name -> (restype, argtypes); every symbol include/kartdiff.h declares
SIGNATURES = {
    "kd_abi_version": (ctypes.c_int, []),
    "kd_last_error": (ctypes.c_char_p, []),
    "kd_init": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "kd_fini": (ctypes.c_int, [ctypes.c_void_p]),
    "kd_set_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "kd_set_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]),
    "kd_get_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
    "kd_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "kd_reserve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]),
    "kd_free": (None, [ctypes.c_void_p]),
    "kd_diff2": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdSide), ctypes.POINTER(KdSide), ctypes.c_uint32,
         ctypes.POINTER(ctypes.POINTER(KdDiffResult))],
    ),
    "kd_diff2_device": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdSide), ctypes.POINTER(KdSide), ctypes.c_uint32,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "kd_fielddiff": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdBlobs), ctypes.POINTER(KdBlobs), ctypes.c_void_p,
         ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(KdLegendMaps),
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32],
    ),
    "kd_merge3": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdSide), ctypes.POINTER(KdSide), ctypes.POINTER(KdSide),
         ctypes.c_uint32, ctypes.POINTER(ctypes.POINTER(KdMergeResult))],
    ),
    "kd_merge3_device": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdSide), ctypes.POINTER(KdSide), ctypes.POINTER(KdSide),
         ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "kd_merge3_device_perm": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdSide), ctypes.POINTER(KdSide), ctypes.POINTER(KdSide), ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p],
    ),
    "kd_envelopes": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdBlobs), c_dblp, ctypes.c_int, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, c_u64p],
    ),
    "kd_env_overlap": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, c_dblp, ctypes.c_void_p,
         ctypes.c_uint32],
    ),
    "kd_geom_heads": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "kd_geom_filter_heads": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, c_dblp,
         ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, c_u64p, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_uint32],
    ),
    "kd_geom_filter_deltas": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(KdBlobs),
         ctypes.POINTER(KdBlobs), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, c_dblp, ctypes.c_uint32, ctypes.c_int,
         ctypes.c_void_p, ctypes.c_void_p, c_u64p, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "kd_shard_cuts": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kd_sf_index_build": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                          ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    "kd_sf_filter": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     c_dblp, ctypes.c_void_p, ctypes.c_uint32]),
    "kd_sf_index_free": (ctypes.c_int, [ctypes.c_void_p]),
    "kd_geom_filter": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdBlobs), ctypes.POINTER(KdBlobs), ctypes.c_void_p, ctypes.c_uint64,
         ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(KdGeomCols), c_dblp, ctypes.c_uint32, ctypes.c_int,
         ctypes.c_void_p, ctypes.c_void_p, c_u64p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32],
    ),
    "kd_hex_encode": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdBlobs), ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_uint32],
    ),
    "kd_sort_side": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_void_p]),
    "kd_diff2_device_perm": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p]),
    "kd_sort_side_into": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.POINTER(KdKeysInfo)]),
    "kd_keys_scan": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.POINTER(KdKeysInfo)]),
    "kd_sort_segmented_into": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "kd_delta_pk_order": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(KdSide), ctypes.POINTER(KdSide),
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "kd_diff2_device_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(KdSide), ctypes.POINTER(KdSide),
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "kd_malloc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    "kd_mfree": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "kd_host_alloc": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    "kd_host_free": (ctypes.c_int, [ctypes.c_void_p]),
    "kd_memcpy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]),
    "kd_memset": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64]),
    "kd_device_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "kd_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "kd_comm_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "kd_comm_fini": (ctypes.c_int, [ctypes.c_void_p]),
    "kd_comm_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "kd_allgather_u64": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "kd_diff2_gather": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdSide), ctypes.POINTER(KdSide), ctypes.c_uint64, ctypes.c_uint64,
         ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "kd_diff2_gather_begin": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(KdSide), ctypes.POINTER(KdSide), ctypes.c_uint64, ctypes.c_uint64,
         ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "kd_diff2_gather_end": (
        ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p],
    ),
    "kd_diff2_sharded": (
        ctypes.c_int,
        [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.POINTER(KdSide), ctypes.POINTER(KdSide), ctypes.c_int,
         ctypes.c_uint32, ctypes.POINTER(ctypes.POINTER(KdDiffResult))],
    ),
    "kd_pack_int_keys": (
        ctypes.c_int64,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "kd_pack_hash_keys": (
        ctypes.c_int64,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
         ctypes.c_void_p, ctypes.c_void_p],
    ),
    "kd_int_keys_to_pks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "kd_odb_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]),
    "kd_odb_close": (ctypes.c_int, [ctypes.c_void_p]),
    "kd_odb_set_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]),
    "kd_odb_get_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
    "kd_odb_read": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(c_u8p), c_u64p],
    ),
    "kd_odb_read_batch": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(c_u8p), ctypes.c_void_p,
         ctypes.c_void_p],
    ),
    "kd_walk": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.POINTER(ctypes.POINTER(KdLeaves))],
    ),
    "kd_prof_enable": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "kd_prof_select": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    "kd_prof_get": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_char_p, c_u64p, c_dblp],
    ),
    "kd_prof_reset": (ctypes.c_int, [ctypes.c_void_p]),
}

_lib = None


def lib():
    """Load libkartdiff.so once; raise NativeUnavailable (never silently fall back).  The library
    needs no GPU framework: it allocates, copies and communicates itself (kd_malloc, kd_memcpy,
    kd_comm_*)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(
                f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`"
            )
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc == KD_OK:
        return
    msg = lib().kd_last_error().decode(errors="replace")
    if rc == KD_EUNSUPPORTED:
        raise Unsupported(rc, f"{what}: {msg}")
    if rc == KD_ENOTFOUND:
        raise NotFound(rc, f"{what}: {msg}")
    raise KdError(rc, f"{what}: {msg}")


def ptr(a):
    """data pointer of a numpy array (or None)"""
    if a is None:
        return None
    return a.ctypes.data
