"""Thin owners of libldgpu.so handles: device gram tables (SCORE) and device
count tables (FIT).  Everything here calls straight into the HIP library."""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .encoding import pack, pack_table


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _grams(gram_lengths: Sequence[int]) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(list(gram_lengths), dtype=np.int32))


class _Owner:
    lib = None

    def _check(self, rc: int) -> None:
        _lib.check(rc, self.lib)


class PinnedArray(_Owner):
    """Page-locked host memory (ldgpu_host_alloc) viewed as a numpy array:
    host-buffer scoring copies from / to it directly, with no staging copy."""

    def __init__(self, shape, dtype, device: Optional[int] = None):
        self.lib = _lib.load()
        self.ctx = _lib.context(device)
        dt = np.dtype(dtype)
        shape = (shape,) if isinstance(shape, int) else tuple(shape)
        n = int(np.prod(shape)) * dt.itemsize
        p = ctypes.c_void_p()
        self._check(self.lib.ldgpu_host_alloc(self.ctx, n, ctypes.byref(p)))
        self.p = p.value
        buf = (ctypes.c_uint8 * max(n, 1)).from_address(self.p)
        self.array = np.frombuffer(buf, dtype=np.uint8, count=n).view(dt).reshape(shape)

    def close(self):
        if getattr(self, "p", None):
            self.array = None
            self.lib.ldgpu_host_free(self.ctx, ctypes.c_void_p(self.p))
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceModel(_Owner):
    """A gram -> probability-row table resident on one GPU
    (LanguageDetectorModel's broadcast table, LanguageDetectorModel.scala:222)."""

    def __init__(self, table: Dict, n_langs: int, gram_lengths: Sequence[int], device: Optional[int] = None,
                 variant: str = "product"):
        """variant="diag": the diagnostics library (tests of alternative paths)."""
        self.lib = _lib.load(variant=variant)
        self.ctx = _lib.context(device, variant)
        self.L = int(n_langs)
        self.gram_lengths = list(gram_lengths)
        kb, ko, rows, ok = pack_table(table, self.L)
        g = _grams(gram_lengths)
        out = ctypes.c_void_p()
        self._check(self.lib.ldgpu_model_create(self.ctx, len(ko) - 1, _ptr(kb), _ptr(ko), _ptr(rows), _ptr(ok),
                                               self.L, _ptr(g), len(g), ctypes.byref(out)))
        self.h = out.value

    @classmethod
    def from_masks(cls, key_bytes: np.ndarray, key_offsets: np.ndarray, masks: np.ndarray, vals: np.ndarray,
                   n_langs: int, gram_lengths: Sequence[int], device: Optional[int] = None,
                   variant: str = "product") -> "DeviceModel":
        """A mask-form table (row i = vals[i] at the languages set in masks[i])
        as packed arrays, e.g. DeviceCounts.fit_table_masks (ldgpu_model_create_masks)."""
        self = cls.__new__(cls)
        self.lib = _lib.load(variant=variant)
        self.ctx = _lib.context(device, variant)
        self.L = int(n_langs)
        self.gram_lengths = list(gram_lengths)
        kb = np.ascontiguousarray(key_bytes, dtype=np.uint8)
        ko = np.ascontiguousarray(key_offsets, dtype=np.int64)
        mk = np.ascontiguousarray(masks, dtype=np.uint64)
        vv = np.ascontiguousarray(vals, dtype=np.float64)
        assert mk.shape == (len(ko) - 1, (self.L + 63) // 64) and vv.shape == (len(ko) - 1,)
        g = _grams(gram_lengths)
        out = ctypes.c_void_p()
        self._check(self.lib.ldgpu_model_create_masks(self.ctx, len(ko) - 1, _ptr(kb), _ptr(ko), _ptr(mk), _ptr(vv),
                                                     self.L, _ptr(g), len(g), ctypes.byref(out)))
        self.h = out.value
        return self

    def close(self):
        if getattr(self, "h", None):
            self.lib.ldgpu_model_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> Dict[str, int]:
        mode = ctypes.c_int32()
        vals = [ctypes.c_int64() for _ in range(4)]
        self._check(self.lib.ldgpu_model_info(self.h, ctypes.byref(mode), *[ctypes.byref(v) for v in vals]))
        flags = ctypes.c_int32()
        self._check(self.lib.ldgpu_model_layout(self.h, ctypes.byref(flags)))
        return {"mode": mode.value, "n_keys": vals[0].value, "table_slots": vals[1].value,
                "filter_bits": vals[2].value, "device_bytes": vals[3].value,
                "layout": sorted(k for k, b in _lib.LAYOUT_FLAGS.items() if flags.value & b)}

    def score(self, data: np.ndarray, offsets: np.ndarray, want_scores: bool = False,
              out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        """Host buffers -> (labels int32[n], scores fp64[n, L] or None);
        `out` (e.g. a PinnedArray's array) receives the labels."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        n = len(offsets) - 1
        if out is not None:
            labels = out
            assert labels.dtype == np.int32 and labels.shape == (max(n, 0),) and labels.flags.c_contiguous
        else:
            labels = np.zeros(max(n, 0), dtype=np.int32)
        scores = np.zeros((max(n, 0), self.L), dtype=np.float64) if want_scores else None
        self._check(self.lib.ldgpu_score(self.h, _ptr(data), _ptr(offsets), n, _ptr(labels), _ptr(scores)))
        return labels, scores

    def stream(self) -> int:
        """The context's hipStream_t."""
        return self.lib.ldgpu_ctx_stream(self.ctx) or 0

    def score_device(self, d_bytes: int, n_bytes: int, d_offsets: int, n_docs: int, d_labels: int,
                     d_scores: int = 0, stream: Optional[int] = None) -> None:
        """Device pointers (e.g. torch tensors' data_ptr()) -> labels in place,
        async on `stream` (a hipStream_t; 0 = the null stream, None = the
        context's stream)."""
        st = self.stream() if stream is None else stream
        self._check(self.lib.ldgpu_score_device(self.h, ctypes.c_void_p(d_bytes), n_bytes, ctypes.c_void_p(d_offsets),
                                               n_docs, ctypes.c_void_p(d_labels),
                                               ctypes.c_void_p(d_scores) if d_scores else None,
                                               ctypes.c_void_p(st) if st else None))


class DeviceCounts(_Owner):
    """A (gram, language) -> count table on one GPU (computeGrams + reduceGrams)."""

    def __init__(self, n_langs: int, gram_lengths: Sequence[int], capacity_hint: int = 0,
                 device: Optional[int] = None, variant: str = "product"):
        """variant="diag": the diagnostics library (tests of alternative paths)."""
        self.lib = _lib.load(variant=variant)
        self.ctx = _lib.context(device, variant)
        self.device = device
        self.variant = variant
        self.L = int(n_langs)
        self.gram_lengths = list(gram_lengths)
        g = _grams(gram_lengths)
        out = ctypes.c_void_p()
        self._check(self.lib.ldgpu_counts_create(self.ctx, self.L, _ptr(g), len(g), int(capacity_hint),
                                                ctypes.byref(out)))
        self.h = out.value

    def close(self):
        if getattr(self, "h", None):
            self.lib.ldgpu_counts_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def count(self, data: np.ndarray, offsets: np.ndarray, doc_lang: np.ndarray) -> None:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        doc_lang = np.ascontiguousarray(doc_lang, dtype=np.int32)
        self._check(self.lib.ldgpu_count(self.h, _ptr(data), _ptr(offsets), _ptr(doc_lang), len(offsets) - 1))

    def count_device(self, d_bytes: int, n_bytes: int, d_offsets: int, d_doc_lang: int, n_docs: int,
                     stream: Optional[int] = None) -> None:
        st = (self.lib.ldgpu_ctx_stream(self.ctx) or 0) if stream is None else stream
        self._check(self.lib.ldgpu_count_device(self.h, ctypes.c_void_p(d_bytes), n_bytes, ctypes.c_void_p(d_offsets),
                                               ctypes.c_void_p(d_doc_lang), n_docs,
                                               ctypes.c_void_p(st) if st else None))

    def size(self) -> int:
        n = ctypes.c_int64()
        self._check(self.lib.ldgpu_counts_size(self.h, ctypes.byref(n), None))
        return n.value

    def stats(self) -> Dict[str, int]:
        """Distinct grams, distinct (gram, language) pairs, total count."""
        v = [ctypes.c_int64() for _ in range(3)]
        self._check(self.lib.ldgpu_counts_stats(self.h, *[ctypes.byref(x) for x in v]))
        return {"grams": v[0].value, "pairs": v[1].value, "total": v[2].value}

    def export_arrays(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(key_bytes uint8, key_offsets int64 [n+1], counts int64 [n, L]),
        sorted by (length, bytes): export() without per-key Python objects."""
        n = ctypes.c_int64()
        nb = ctypes.c_int64()
        self._check(self.lib.ldgpu_counts_size(self.h, ctypes.byref(n), ctypes.byref(nb)))
        kb = np.zeros(max(nb.value, 1), dtype=np.uint8)
        ko = np.zeros(n.value + 1, dtype=np.int64)
        cnt = np.zeros((n.value, self.L), dtype=np.int64)
        self._check(self.lib.ldgpu_counts_export(self.h, _ptr(kb), _ptr(ko), _ptr(cnt)))
        return kb[:int(ko[-1])], ko, cnt

    def export(self) -> Tuple[List[bytes], np.ndarray]:
        """Distinct grams sorted by (length, bytes) and int64 counts [n, L]."""
        n = ctypes.c_int64()
        nb = ctypes.c_int64()
        self._check(self.lib.ldgpu_counts_size(self.h, ctypes.byref(n), ctypes.byref(nb)))
        kb = np.zeros(max(nb.value, 1), dtype=np.uint8)
        ko = np.zeros(n.value + 1, dtype=np.int64)
        cnt = np.zeros((n.value, self.L), dtype=np.int64)
        self._check(self.lib.ldgpu_counts_export(self.h, _ptr(kb), _ptr(ko), _ptr(cnt)))
        b = kb.tobytes()
        return [b[ko[i]:ko[i + 1]] for i in range(n.value)], cnt

    def export_sparse(self, first: int = 0, n: Optional[int] = None):
        """Grams [first, first + n) in (length, bytes) order with their nonzero
        (language, count) pairs: (key_bytes uint8, key_offsets int64 [n+1],
        pair_offsets int64 [n+1], pair_langs int32, pair_counts int64)."""
        if n is None:
            n = self.size() - first
        nb = ctypes.c_int64()
        npairs = ctypes.c_int64()
        self._check(self.lib.ldgpu_counts_sparse_size(self.h, first, n, ctypes.byref(nb), ctypes.byref(npairs)))
        kb = np.zeros(max(nb.value, 1), dtype=np.uint8)
        ko = np.zeros(n + 1, dtype=np.int64)
        po = np.zeros(n + 1, dtype=np.int64)
        pl = np.zeros(max(npairs.value, 1), dtype=np.int32)
        pc = np.zeros(max(npairs.value, 1), dtype=np.int64)
        self._check(self.lib.ldgpu_counts_export_sparse(self.h, first, n, _ptr(kb), _ptr(ko), _ptr(po), _ptr(pl),
                                                       _ptr(pc)))
        return kb[:nb.value], ko, po, pl[:npairs.value], pc[:npairs.value]

    def add_sparse(self, key_bytes: np.ndarray, key_offsets: np.ndarray, pair_offsets: np.ndarray,
                   pair_langs: np.ndarray, pair_counts: np.ndarray) -> None:
        kb = np.ascontiguousarray(key_bytes, dtype=np.uint8)
        ko = np.ascontiguousarray(key_offsets, dtype=np.int64)
        po = np.ascontiguousarray(pair_offsets, dtype=np.int64)
        pl = np.ascontiguousarray(pair_langs, dtype=np.int32)
        pc = np.ascontiguousarray(pair_counts, dtype=np.int64)
        self._check(self.lib.ldgpu_counts_add_sparse(self.h, len(ko) - 1, _ptr(kb if len(kb) else np.zeros(1, np.uint8)),
                                                    _ptr(ko), _ptr(po), _ptr(pl), _ptr(pc)))

    def add(self, keys: Sequence[bytes], counts: np.ndarray) -> None:
        counts = np.ascontiguousarray(counts, dtype=np.int64).reshape(len(keys), self.L)
        kb, ko = pack(list(keys))
        self._check(self.lib.ldgpu_counts_add(self.h, len(keys), _ptr(kb), _ptr(ko), _ptr(counts)))

    def export_device(self, stream: Optional[int] = None):
        """(keys int64 [n] packed u64, counts int64 [n, L]) as torch tensors on
        this context's GPU, unordered (ldgpu_counts_export_device)."""
        import torch
        n = self.size()
        dev = torch.device("cuda", _lib.default_device() if self.device is None else self.device)
        keys = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        counts = torch.empty((max(n, 1), self.L), dtype=torch.int64, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream if stream is None else stream
        got = ctypes.c_int64()
        self._check(self.lib.ldgpu_counts_export_device(self.h, max(n, 1), ctypes.c_void_p(keys.data_ptr()),
                                                       ctypes.c_void_p(counts.data_ptr()), ctypes.byref(got),
                                                       ctypes.c_void_p(st) if st else None))
        return keys[:got.value], counts[:got.value]

    def add_device(self, keys, counts, stream: Optional[int] = None) -> None:
        """Add device tensors (packed u64 keys as int64 [n], int64 counts [n, L])."""
        import torch
        keys = keys.contiguous()
        counts = counts.contiguous()
        st = torch.cuda.current_stream(keys.device).cuda_stream if stream is None else stream
        self._check(self.lib.ldgpu_counts_add_device(self.h, int(keys.numel()), ctypes.c_void_p(keys.data_ptr()),
                                                    ctypes.c_void_p(counts.data_ptr()),
                                                    ctypes.c_void_p(st) if st else None))

    def fit_table(self, profile_size: int) -> Dict[bytes, List[float]]:
        """computeProbabilities + filterTopGrams -> {gram: row}."""
        n = ctypes.c_int64()
        nb = ctypes.c_int64()
        self._check(self.lib.ldgpu_fit_table_size(self.h, int(profile_size), ctypes.byref(n), ctypes.byref(nb)))
        kb = np.zeros(max(nb.value, 1), dtype=np.uint8)
        ko = np.zeros(n.value + 1, dtype=np.int64)
        rows = np.zeros((n.value, self.L), dtype=np.float64)
        self._check(self.lib.ldgpu_fit_table_export(self.h, _ptr(kb), _ptr(ko), _ptr(rows)))
        b = kb.tobytes()
        return {b[ko[i]:ko[i + 1]]: rows[i].tolist() for i in range(n.value)}

    def cached_table_masks(self):
        """The table of the last fit_table / fit_table_masks call, exported
        again (ldgpu_fit_table_info + ldgpu_fit_table_export_masks): the same
        arrays as fit_table_masks returned, without a rebuild."""
        n = ctypes.c_int64()
        nb = ctypes.c_int64()
        self._check(self.lib.ldgpu_fit_table_info(self.h, ctypes.byref(n), ctypes.byref(nb)))
        S = (self.L + 63) // 64
        kb = np.zeros(max(nb.value, 1), dtype=np.uint8)
        ko = np.zeros(n.value + 1, dtype=np.int64)
        masks = np.zeros((max(n.value, 1), S), dtype=np.uint64)
        vals = np.zeros(max(n.value, 1), dtype=np.float64)
        self._check(self.lib.ldgpu_fit_table_export_masks(self.h, _ptr(kb), _ptr(ko), _ptr(masks), _ptr(vals)))
        return kb, ko, masks[:n.value], vals[:n.value]

    def fit_table_masks(self, profile_size: int):
        """The fit table in mask form, as packed arrays: (key_bytes uint8,
        key_offsets int64 [n+1], masks uint64 [n, S], vals fp64 [n]) -- what
        DeviceModel.from_masks takes; no per-row Python objects, so tables of
        10M rows x 200 languages stay cheap."""
        n = ctypes.c_int64()
        nb = ctypes.c_int64()
        self._check(self.lib.ldgpu_fit_table_size(self.h, int(profile_size), ctypes.byref(n), ctypes.byref(nb)))
        S = (self.L + 63) // 64
        kb = np.zeros(max(nb.value, 1), dtype=np.uint8)
        ko = np.zeros(n.value + 1, dtype=np.int64)
        masks = np.zeros((max(n.value, 1), S), dtype=np.uint64)
        vals = np.zeros(max(n.value, 1), dtype=np.float64)
        self._check(self.lib.ldgpu_fit_table_export_masks(self.h, _ptr(kb), _ptr(ko), _ptr(masks), _ptr(vals)))
        return kb, ko, masks[:n.value], vals[:n.value]



def case_tables() -> Tuple[np.ndarray, np.ndarray]:
    """The host language's 1:1 lower-case mapping of UTF-16 units (str.lower of
    one character; Java: Character.toLowerCase) and the `special` bitmap of the
    units whose String.toLowerCase is not that mapping or needs context
    (include/ldgpu.h PREPROCESS): U+0130 (-> "i" + U+0307), capital sigma
    (Final_Sigma), and the high surrogates of supplementary planes holding
    cased letters."""
    global _CASE_TABLES
    if _CASE_TABLES is None:
        lower = np.arange(65536, dtype=np.uint16)
        special = np.zeros(65536, dtype=bool)
        for c in range(65536):
            if 0xD800 <= c <= 0xDFFF:
                continue
            low = chr(c).lower()
            if len(low) == 1 and ord(low) < 0x10000:
                lower[c] = ord(low)
            else:
                special[c] = True
        special[0x3A3] = True
        for c in range(0x10000, 0x110000):
            if chr(c).lower() != chr(c):
                special[0xD800 + ((c - 0x10000) >> 10)] = True
        _CASE_TABLES = (lower, np.packbits(special, bitorder="little"))
    return _CASE_TABLES


_CASE_TABLES = None


def locale_class(lang_tag) -> int:
    """Locale.forLanguageTag(tag).getLanguage() -> the device's locale class."""
    from .preprocessing import _language_of
    lang = _language_of(lang_tag)
    return _lib.LOCALE_TR_AZ if lang in ("tr", "az") else (_lib.LOCALE_LT if lang == "lt" else _lib.LOCALE_ROOT)


class DeviceCaseMap(_Owner):
    """The preprocessors on the GPU (ldgpu_preprocess; include/ldgpu.h
    PREPROCESS): lower-casing and the symbol / space cleanup over UTF-16 units."""

    def __init__(self, device: Optional[int] = None, variant: str = "product"):
        self.lib = _lib.load(variant=variant)
        self.ctx = _lib.context(device, variant=variant)
        lower, special = case_tables()
        h = ctypes.c_void_p()
        self._check(self.lib.ldgpu_casemap_create(self.ctx, _ptr(lower), _ptr(special), ctypes.byref(h)))
        self.h = h.value

    @staticmethod
    def pack_units(texts: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
        """Java strings: UTF-16 code units (u16) and offsets in units."""
        enc = [t.encode("utf-16-le", "surrogatepass") for t in texts]
        lens = np.fromiter((len(e) // 2 for e in enc), dtype=np.int64, count=len(enc))
        off = np.zeros(len(enc) + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        units = np.frombuffer(b"".join(enc) + b"\0\0", dtype=np.uint16)
        return np.ascontiguousarray(units), off

    def run(self, units: np.ndarray, offsets: np.ndarray, locale: Optional[np.ndarray], flags: int
            ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(output units or bytes, output offsets, host flags) of ldgpu_preprocess."""
        n = len(offsets) - 1
        units = np.ascontiguousarray(units, dtype=np.uint16)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        if locale is not None:
            locale = np.ascontiguousarray(locale, dtype=np.uint8)
        cap = max(int(offsets[-1] - offsets[0]) if n else 0, 1)
        out = np.zeros(cap + 4, dtype=np.uint8 if flags & _lib.PRE_LOW_BYTES else np.uint16)
        out_off = np.zeros(n + 1, dtype=np.int64)
        host = np.zeros(max(n, 1), dtype=np.uint8)
        self._check(self.lib.ldgpu_preprocess(self.h, _ptr(units), _ptr(offsets), n, _ptr(locale), flags,
                                              _ptr(out), _ptr(out_off), _ptr(host)))
        return out, out_off, host[:n]

    def close(self):
        if getattr(self, "h", None):
            self.lib.ldgpu_casemap_destroy(ctypes.c_void_p(self.h))
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
