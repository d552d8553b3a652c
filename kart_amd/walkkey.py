"""The int-PK join key in numpy: ascending in git's tree order (kart_amd/csrc/kd_walkkey.h restated).

A side's leaves come from the tree walk in git path order (kart/dataset3.py:225-231): tree names
byte-compared, so the four bucket levels order by the ASCII rank of each base-64 character, and the
filenames ``b64(msgpack([pk]))`` of one leaf tree by their text (kart/dataset3_paths.py:283-299).
``key = rank24(bucket) << 40 | (pk // 2**30 + 2**33) << 6 | frank(pk)`` is a bijection with the pk
that ascends in exactly that order whenever a leaf tree holds one 2**30 wrap of pks (DESIGN.md
"join key"); the tables here are derived by sorting the filenames themselves.
"""
import base64

import msgpack
import numpy as np

B64 = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
RANK = np.array([sum(c < v for c in B64) for v in B64], np.uint64)  # digit value -> ASCII rank
IRANK = np.argsort(RANK).astype(np.uint64)
# representative block starts of the 8 filename-order classes (block_class)
CLASS_BLOCK = (128, 0, 64, 256, 320, 384, 448, -64)


def filename(pk):
    """the IntPathEncoder filename of pk (kart/dataset3_paths.py:164-165)"""
    return base64.urlsafe_b64encode(msgpack.packb([int(pk)])).decode()


def _frank_tables():
    fr = np.zeros((8, 64), np.uint64)
    for c, s in enumerate(CLASS_BLOCK):
        names = [filename(s + j) for j in range(64)]
        order = sorted(range(64), key=lambda j: names[j].encode())
        fr[c, order] = np.arange(64, dtype=np.uint64)
    return fr, np.argsort(fr, axis=1).astype(np.uint64)


FR, IFR = _frank_tables()


def block_class(s):
    """filename-order class of the blocks starting at s (multiples of 64), vectorised"""
    s = np.asarray(s, np.int64)
    c0 = ((s >= 128) & (s < 256)) | (s == -128) | ((s >= 65536) & (s < 1 << 32)) | ((s >= -(1 << 31)) & (s < -32768))
    cls = np.where(c0, 0, 3 + ((s & 0xFF) >> 6))
    cls = np.where((s >= 0) & (s < 128), 1 + (s >> 6), cls)
    return np.where(s == -64, 7, cls).astype(np.int64)


def rank_digits(x, digits=4):
    x = np.asarray(x, np.uint64)
    out = np.zeros_like(x)
    for k in range(digits):
        sh = np.uint64(6 * k)
        out |= RANK[((x >> sh) & np.uint64(63)).astype(np.int64)] << sh
    return out


def irank_digits(x, digits=4):
    x = np.asarray(x, np.uint64)
    out = np.zeros_like(x)
    for k in range(digits):
        sh = np.uint64(6 * k)
        out |= IRANK[((x >> sh) & np.uint64(63)).astype(np.int64)] << sh
    return out


def int_keys(pk):
    """KD_KEY_INT keys of int64 pks (vectorised; the native packer's kd_walkkey.h)"""
    pk = np.asarray(pk, np.int64)
    q = pk >> 6
    s = q << 6
    r = (pk - s).astype(np.int64)
    bucket = (q & ((1 << 24) - 1)).astype(np.uint64)
    wrap = ((pk >> 30) + (1 << 33)).astype(np.uint64)
    low = FR[block_class(s), r]
    return np.ascontiguousarray((rank_digits(bucket) << np.uint64(40)) | (wrap << np.uint64(6)) | low)


def int_keys_to_pks(keys):
    keys = np.asarray(keys, np.uint64)
    bucket = irank_digits(keys >> np.uint64(40))
    wrap = (keys >> np.uint64(6)) & np.uint64((1 << 34) - 1)
    s = ((((wrap - np.uint64(1 << 33)) << np.uint64(24)) + bucket) << np.uint64(6)).view(np.int64)
    return s + IFR[block_class(s), (keys & np.uint64(63)).astype(np.int64)].astype(np.int64)


def pk_to_int_key(pk):
    """one Python-int pk -> its KD_KEY_INT key; ValueError outside [-2**63, 2**63)"""
    if not -(1 << 63) <= pk < (1 << 63):
        raise ValueError(f"pk {pk} outside [-2**63, 2**63)")
    return int(int_keys(np.array([pk], np.int64))[0])


def walk_order_range(lo, hi):
    """the pks in [lo, hi) (within one wrap: 0 <= lo, hi <= 2**30) in git tree order"""
    if not 0 <= lo <= hi <= 1 << 30:
        raise ValueError("walk_order_range: [lo, hi) within [0, 2**30)")
    b0, b1 = lo // 64, (hi + 63) // 64
    buckets = np.arange(b0, b1, dtype=np.uint64)
    b = buckets[np.argsort(rank_digits(buckets), kind="stable")].astype(np.int64)
    pks = ((b[:, None] << 6) + IFR[block_class(b << 6)].astype(np.int64)).reshape(-1)
    return np.ascontiguousarray(pks[(pks >= lo) & (pks < hi)])


def walk_order_pks(n_pks, rank_lo=0, rank_hi=1 << 24):
    """the pks 0..n_pks-1 (n_pks <= 2**30) in git tree order, restricted to the leaf trees whose
    rank-mapped bucket lies in [rank_lo, rank_hi) — a bucket-range shard, which is a contiguous run
    of the walk.  Returns int64 pks; their keys ascend."""
    if n_pks > 1 << 30:
        raise ValueError("walk_order_pks: at most 2**30 pks (one wrap)")
    nb = (n_pks + 63) // 64
    buckets = np.arange(nb, dtype=np.uint64)
    rk = rank_digits(buckets)
    sel = np.nonzero((rk >= np.uint64(rank_lo)) & (rk < np.uint64(rank_hi)))[0]
    b = buckets[sel][np.argsort(rk[sel], kind="stable")].astype(np.int64)
    pks = (b[:, None] << 6) + IFR[block_class(b << 6)].astype(np.int64)
    pks = pks.reshape(-1)
    return np.ascontiguousarray(pks[pks < n_pks])
