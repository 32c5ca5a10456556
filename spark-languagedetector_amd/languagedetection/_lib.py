"""ctypes binding of libldgpu.so (include/ldgpu.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU
is visible, the calls below raise.  ``torch`` (when importable) is imported
before the library is loaded so that both share torch's HIP runtime (its
libamdhip64.so carries the same SONAME, so the loader reuses it).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import List, Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libldgpu.so")
# LDGPU_LIB: another build of the library for A/B timing (tools only)
_LIB_OVERRIDE = os.environ.get("LDGPU_LIB")
# diagnostics build (make -C spark-languagedetector_amd diag): the only one that
# reads the LDGPU_* path / ablation switches from the environment; tests load
# it explicitly (variant="diag") to cover the alternative kernel paths
DIAG_LIB_PATH = os.environ.get("LDGPU_DIAG_LIB") or os.path.join(PKG_ROOT, "lib", "libldgpu_diag.so")  # (override: A/B tools only)

LDGPU_OK = 0
LDGPU_EINVAL = 1
LDGPU_EROWLEN = 2
LDGPU_ENOMEM = 3
LDGPU_EDEVICE = 4
LDGPU_EUNSUPPORTED = 5
LDGPU_ENODEV = 6
MAX_GRAM = 2147483647  # SCORE tables: any gram length (beyond 15: the general-key table)
MAX_FIT_GRAM = 16777215  # FIT counting (grams of 8..15 bytes: two words; longer: the general-key table)
MAX_LANGS = 4096
# ldgpu_model_layout flags
LAYOUT_FLAGS = {"lds_bloom": 0x01, "keyed_bloom": 0x02, "keyed_bloom_lines": 0x04, "buckets": 0x08,
                "wide_keys": 0x10, "direct": 0x20, "packs": 0x40, "lang_blocks": 0x80,
                "general_keys": 0x100, "keyed_bloom_chunks": 0x200, "classes": 0x400}

_p = ctypes.c_void_p
_pp = ctypes.POINTER(ctypes.c_void_p)
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_pi32 = ctypes.POINTER(ctypes.c_int32)
_pi64 = ctypes.POINTER(ctypes.c_int64)

# (name, restype, argtypes) -- exactly the entry points of include/ldgpu.h
SIGNATURES = [
    ("ldgpu_version", ctypes.c_char_p, []),
    ("ldgpu_build_id", ctypes.c_char_p, []),
    ("ldgpu_last_error", ctypes.c_char_p, []),
    ("ldgpu_device_count", ctypes.c_int, [_pi32]),
    ("ldgpu_ctx_create", ctypes.c_int, [_i32, _pp]),
    ("ldgpu_ctx_destroy", ctypes.c_int, [_p]),
    ("ldgpu_ctx_synchronize", ctypes.c_int, [_p]),
    ("ldgpu_ctx_stream", _p, [_p]),
    ("ldgpu_host_alloc", ctypes.c_int, [_p, _i64, _pp]),
    ("ldgpu_host_free", ctypes.c_int, [_p, _p]),
    ("ldgpu_model_create", ctypes.c_int, [_p, _i64, _p, _p, _p, _p, _i32, _p, _i32, _pp]),
    ("ldgpu_model_create_masks", ctypes.c_int, [_p, _i64, _p, _p, _p, _p, _i32, _p, _i32, _pp]),
    ("ldgpu_model_destroy", ctypes.c_int, [_p]),
    ("ldgpu_model_info", ctypes.c_int, [_p, _pi32, _pi64, _pi64, _pi64, _pi64]),
    ("ldgpu_model_layout", ctypes.c_int, [_p, _pi32]),
    ("ldgpu_model_langs", ctypes.c_int, [_p, _pi32]),
    ("ldgpu_score", ctypes.c_int, [_p, _p, _p, _i64, _p, _p]),
    ("ldgpu_score_device", ctypes.c_int, [_p, _p, _i64, _p, _i64, _p, _p, _p]),
    ("ldgpu_counts_create", ctypes.c_int, [_p, _i32, _p, _i32, _i64, _pp]),
    ("ldgpu_counts_destroy", ctypes.c_int, [_p]),
    ("ldgpu_counts_langs", ctypes.c_int, [_p, _pi32]),
    ("ldgpu_count", ctypes.c_int, [_p, _p, _p, _p, _i64]),
    ("ldgpu_count_device", ctypes.c_int, [_p, _p, _i64, _p, _p, _i64, _p]),
    ("ldgpu_counts_size", ctypes.c_int, [_p, _pi64, _pi64]),
    ("ldgpu_counts_stats", ctypes.c_int, [_p, _pi64, _pi64, _pi64]),
    ("ldgpu_counts_export", ctypes.c_int, [_p, _p, _p, _p]),
    ("ldgpu_counts_add", ctypes.c_int, [_p, _i64, _p, _p, _p]),
    ("ldgpu_counts_sparse_size", ctypes.c_int, [_p, _i64, _i64, _pi64, _pi64]),
    ("ldgpu_counts_export_sparse", ctypes.c_int, [_p, _i64, _i64, _p, _p, _p, _p, _p]),
    ("ldgpu_counts_add_sparse", ctypes.c_int, [_p, _i64, _p, _p, _p, _p, _p]),
    ("ldgpu_counts_export_device", ctypes.c_int, [_p, _i64, _p, _p, _pi64, _p]),
    ("ldgpu_counts_add_device", ctypes.c_int, [_p, _i64, _p, _p, _p]),
    ("ldgpu_comm_unique_id", ctypes.c_int, [_p]),
    ("ldgpu_comm_create_rccl", ctypes.c_int, [_p, _p, _i32, _i32, _pp]),
    ("ldgpu_comm_create_host", ctypes.c_int, [_p, _i32, _i32, _p, _pp]),
    ("ldgpu_comm_destroy", ctypes.c_int, [_p]),
    ("ldgpu_counts_merge", ctypes.c_int, [_p, _p]),
    ("ldgpu_fit_table_size", ctypes.c_int, [_p, _i32, _pi64, _pi64]),
    ("ldgpu_fit_table_info", ctypes.c_int, [_p, _pi64, _pi64]),
    ("ldgpu_fit_table_export", ctypes.c_int, [_p, _p, _p, _p]),
    ("ldgpu_fit_table_export_masks", ctypes.c_int, [_p, _p, _p, _p, _p]),
    ("ldgpu_casemap_create", ctypes.c_int, [_p, _p, _p, _pp]),
    ("ldgpu_casemap_destroy", ctypes.c_int, [_p]),
    ("ldgpu_preprocess_device", ctypes.c_int, [_p, _p, _p, _i64, _p, _i32, _p, _p, _p, _p]),
    ("ldgpu_preprocess", ctypes.c_int, [_p, _p, _p, _i64, _p, _i32, _p, _p, _p]),
]

# include/ldgpu.h PREPROCESS
PRE_LOWER, PRE_CLEAN, PRE_LOW_BYTES = 1, 2, 4
LOCALE_ROOT, LOCALE_TR_AZ, LOCALE_LT = 0, 1, 2

_libs = {}
_lock = threading.RLock()


COMM_ID_BYTES = 128

# ldgpu_host_coll (include/ldgpu.h): collectives over host memory supplied by
# the caller (the FIT merge's host transport)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, _pi64, ctypes.c_void_p, _pi64)


class HostColl(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("allgather", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN)]


class LdgpuError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def load(path: Optional[str] = None, variant: str = "product"):
    """Load libldgpu.so (or, variant="diag", libldgpu_diag.so); raises if it
    has not been built."""
    with _lock:
        if path is None and variant in _libs:
            return _libs[variant]
        if path is None and variant == "product" and _LIB_OVERRIDE:
            lib = load(_LIB_OVERRIDE)
            _libs[variant] = lib
            return lib
        p = path or (DIAG_LIB_PATH if variant == "diag" else LIB_PATH)
        if not os.path.exists(p):
            raise ImportError(
                f"{os.path.basename(p)} not found at {p}: build it with `make -C spark-languagedetector_amd"
                f"{' diag' if variant == 'diag' else ''}` (or __graft_entry__.build()); there is no CPU fallback")
        try:
            import torch  # noqa: F401  -- share torch's HIP runtime (same SONAME)
        except Exception:
            pass
        lib = ctypes.CDLL(p)
        for name, res, args in SIGNATURES:
            if path is not None and not hasattr(lib, name):
                continue  # an explicitly named older build (A/B timing): only its own entry points
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _libs[variant] = lib
        return lib


def exported_symbols() -> List[str]:
    return [s[0] for s in SIGNATURES]


def check(rc: int, lib=None) -> None:
    if rc == LDGPU_OK:
        return
    msg = (lib or load()).ldgpu_last_error().decode("utf-8", "replace")
    if rc in (LDGPU_EINVAL, LDGPU_EROWLEN):
        raise ValueError(msg)
    if rc == LDGPU_ENOMEM:
        raise MemoryError(msg)
    if rc == LDGPU_EUNSUPPORTED:
        raise NotImplementedError(msg)
    raise LdgpuError(rc, msg)


# ------------------------------------------------------------------ contexts
_ctx = {}


def default_device() -> int:
    return int(os.environ.get("LDGPU_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def context(device: Optional[int] = None, variant: str = "product") -> int:
    """A process-wide context per device (one executor per GPU) and library."""
    d = default_device() if device is None else int(device)
    with _lock:
        h = _ctx.get((variant, d))
    if h is not None:
        return h
    lib = load(variant=variant)
    out = ctypes.c_void_p()
    check(lib.ldgpu_ctx_create(d, ctypes.byref(out)), lib)
    with _lock:
        _ctx.setdefault((variant, d), out.value)
        return _ctx[(variant, d)]


def device_count() -> int:
    n = ctypes.c_int32(0)
    check(load().ldgpu_device_count(ctypes.byref(n)))
    return n.value


# the sources the library is built from, in the Makefile's PROV order
_PROV = ["csrc/ldgpu_api.hip", "csrc/ldgpu_score.hip", "csrc/ldgpu_fit.hip", "csrc/ldgpu_general.hip",
         "csrc/ldgpu_long.hip", "csrc/ldgpu_replay.hip", "csrc/ldgpu_pre.hip", "csrc/ldgpu_common.h",
         "csrc/ldgpu_internal.h", "csrc/ldgpu_fit.h", "../include/ldgpu.h"]


def tree_source_hash() -> str:
    """sha256 (16 hex digits) of the library's sources in this tree."""
    import hashlib
    h = hashlib.sha256()
    for f in _PROV:
        with open(os.path.join(PKG_ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def provenance(variant: str = "product") -> dict:
    """The loaded library's build id against this tree's sources.  The id is
    the sources' hash, plus "+<flags hash>" for a library built with other
    compile flags than the product's (diagnostics, sanitizer and tuning
    builds; spark-languagedetector_amd/Makefile): `match` holds when the
    sources are this tree's and -- for the product variant -- the flags are
    the product's."""
    lib = load(variant=variant)
    built = lib.ldgpu_build_id().decode()
    src, _, flags = built.partition("+")
    tree = tree_source_hash()
    return {"library_source_hash": src, "build_flags_tag": flags or None, "tree_source_hash": tree,
            "match": src == tree and (variant != "product" or not flags)}

