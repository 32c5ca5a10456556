"""ctypes wrapper of the C restatement (oracle/ldoracle.c) -- TEST INFRASTRUCTURE ONLY.

Used by tests/ for parity at sizes the pure-Python oracle is too slow for, and
by bench.py's cpu_baseline leg.  See oracle/ldoracle.py for the rules and the
reference citations.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Dict, List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libldoracle.so")
_lib = None

_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.ldo_table_create.restype = _p
        L.ldo_table_create.argtypes = [_i64, _p, _p, _p, _i32]
        L.ldo_table_create_masks.restype = _p
        L.ldo_table_create_masks.argtypes = [_i64, _p, _p, _p, _p, _i32]
        L.ldo_table_destroy.argtypes = [_p]
        L.ldo_score.restype = ctypes.c_int
        L.ldo_score.argtypes = [_p, _p, _i32, _p, _p, _i64, _p, _p, _i32]
        L.ldo_hits.restype = _i64
        L.ldo_hits.argtypes = [_p, _p, _i32, _p, _p, _i64]
        L.ldo_count.restype = _p
        L.ldo_count.argtypes = [_p, _p, _p, _i64, _i32, _p, _i32]
        L.ldo_count_mt.restype = _p
        L.ldo_count_mt.argtypes = [_p, _p, _p, _i64, _i32, _p, _i32, _i32]
        L.ldo_counts_size.restype = _i64
        L.ldo_counts_size.argtypes = [_p]
        L.ldo_counts_key_bytes.restype = _i64
        L.ldo_counts_key_bytes.argtypes = [_p]
        L.ldo_counts_export.argtypes = [_p, _p, _p, _p]
        L.ldo_counts_pairs.restype = _i64
        L.ldo_counts_pairs.argtypes = [_p]
        L.ldo_counts_export_sparse.argtypes = [_p, _p, _p, _p, _p, _p]
        L.ldo_counts_destroy.argtypes = [_p]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def pack_keys(keys: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    off = np.zeros(len(keys) + 1, dtype=np.int64)
    if keys:
        off[1:] = np.cumsum([len(k) for k in keys])
    blob = np.frombuffer(b"".join(keys) + b"\0", dtype=np.uint8).copy()
    return blob, off


class Table:
    """A gram -> fp64 row map (the reference's Map[Seq[Byte], Array[Double]])."""

    def __init__(self, table: Dict[bytes, Sequence[float]], n_langs: int):
        keys = list(table.keys())
        self.L = n_langs
        blob, off = pack_keys(keys)
        rows = np.asarray([list(table[k]) for k in keys], dtype=np.float64).reshape(len(keys), n_langs)
        rows = np.ascontiguousarray(rows)
        self._h = lib().ldo_table_create(len(keys), _ptr(blob), _ptr(off), _ptr(rows), n_langs)

    @classmethod
    def from_masks(cls, key_bytes: np.ndarray, key_offsets: np.ndarray, masks: np.ndarray, vals: np.ndarray,
                   n_langs: int) -> "Table":
        """Mask form (row i = vals[i] at the set bits of masks[i], 0.0 elsewhere)
        from packed arrays: tables too large for a dict of dense rows."""
        self = cls.__new__(cls)
        self.L = n_langs
        kb = np.ascontiguousarray(key_bytes, dtype=np.uint8)
        ko = np.ascontiguousarray(key_offsets, dtype=np.int64)
        mk = np.ascontiguousarray(masks, dtype=np.uint64)
        vv = np.ascontiguousarray(vals, dtype=np.float64)
        assert mk.shape == (len(ko) - 1, (n_langs + 63) // 64) and vv.shape == (len(ko) - 1,)
        self._h = lib().ldo_table_create_masks(len(ko) - 1, _ptr(kb), _ptr(ko), _ptr(mk), _ptr(vv), n_langs)
        return self

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ldo_table_destroy(self._h)
            self._h = None

    def score(self, gram_lengths: Sequence[int], data: np.ndarray, offsets: np.ndarray,
              want_scores: bool = False, nthreads: int = 1):
        g = np.asarray(gram_lengths, dtype=np.int32)
        n = len(offsets) - 1
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        labels = np.zeros(n, dtype=np.int32)
        scores = np.zeros((n, self.L), dtype=np.float64) if want_scores else None
        rc = lib().ldo_score(self._h, _ptr(g), len(g), _ptr(data), _ptr(offsets), n, _ptr(labels),
                             _ptr(scores) if scores is not None else None, nthreads)
        if rc != 0:
            raise ValueError("ldo_score: invalid arguments")
        return labels, scores

    def hits(self, gram_lengths: Sequence[int], data: np.ndarray, offsets: np.ndarray) -> int:
        """windows (of every n in gram_lengths) whose key is in the table"""
        g = np.asarray(gram_lengths, dtype=np.int32)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        return int(lib().ldo_hits(self._h, _ptr(g), len(g), _ptr(data), _ptr(offsets), len(offsets) - 1))


def count(data: np.ndarray, offsets: np.ndarray, doc_lang: np.ndarray, n_langs: int,
          gram_lengths: Sequence[int], nthreads: int = 1) -> Tuple[List[bytes], np.ndarray]:
    """computeGrams + reduceGrams: distinct grams sorted by (len, bytes) and raw
    int64 counts [n_grams, L] (apply the JVM Int wrap separately).  nthreads > 1:
    ldo_count_mt (per-thread tables, then a hash-partitioned reduce)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    doc_lang = np.ascontiguousarray(doc_lang, dtype=np.int32)
    g = np.asarray(gram_lengths, dtype=np.int32)
    L = lib()
    if nthreads > 1:
        h = L.ldo_count_mt(_ptr(data), _ptr(offsets), _ptr(doc_lang), len(offsets) - 1, n_langs, _ptr(g), len(g),
                           nthreads)
    else:
        h = L.ldo_count(_ptr(data), _ptr(offsets), _ptr(doc_lang), len(offsets) - 1, n_langs, _ptr(g), len(g))
    try:
        n = L.ldo_counts_size(h)
        nb = L.ldo_counts_key_bytes(h)
        blob = np.zeros(max(nb, 1), dtype=np.uint8)
        off = np.zeros(n + 1, dtype=np.int64)
        cnt = np.zeros((n, n_langs), dtype=np.int64)
        L.ldo_counts_export(h, _ptr(blob), _ptr(off), _ptr(cnt))
    finally:
        L.ldo_counts_destroy(h)
    keys = [bytes(blob[off[i]:off[i + 1]]) for i in range(n)]
    return keys, cnt


def export_sparse(h):
    """The (gram, language) pairs of an ldo_counts handle in (length, bytes,
    language) order: (key_bytes, key_offsets [n+1], pair_offsets [n+1],
    pair_langs int32, pair_counts int64) -- the form of
    ldgpu_counts_export_sparse."""
    L = lib()
    n = L.ldo_counts_size(h)
    nb = L.ldo_counts_key_bytes(h)
    npairs = L.ldo_counts_pairs(h)
    kb = np.zeros(max(nb, 1), dtype=np.uint8)
    ko = np.zeros(n + 1, dtype=np.int64)
    po = np.zeros(n + 1, dtype=np.int64)
    pl = np.zeros(max(npairs, 1), dtype=np.int32)
    pc = np.zeros(max(npairs, 1), dtype=np.int64)
    L.ldo_counts_export_sparse(h, _ptr(kb), _ptr(ko), _ptr(po), _ptr(pl), _ptr(pc))
    return kb[:nb], ko, po, pl[:npairs], pc[:npairs]


def count_sparse(data: np.ndarray, offsets: np.ndarray, doc_lang: np.ndarray, n_langs: int,
                 gram_lengths: Sequence[int], nthreads: int = 1):
    """count() in sparse form (export_sparse): no dense row of L per gram."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    doc_lang = np.ascontiguousarray(doc_lang, dtype=np.int32)
    g = np.asarray(gram_lengths, dtype=np.int32)
    L = lib()
    h = L.ldo_count_mt(_ptr(data), _ptr(offsets), _ptr(doc_lang), len(offsets) - 1, n_langs, _ptr(g), len(g),
                       max(nthreads, 1))
    try:
        return export_sparse(h)
    finally:
        L.ldo_counts_destroy(h)
