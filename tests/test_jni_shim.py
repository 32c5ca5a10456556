"""The JNI shim's buffer checks (jni/ldgpu_jni.c): every direct buffer must
cover what the C ABI reads or writes, sized from the library's own handles
(language counts, cached table sizes), in overflow-checked 64-bit
arithmetic; a short buffer fails with LDGPU_EINVAL before the library touches
it.  There is no JDK here, so the shim is compiled against a test-only
stand-in jni.h (tests/jni_harness/) and driven through ctypes with fake
direct buffers whose capacity can be smaller than their memory."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from languagedetection import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
FN = "Java_org_apache_spark_ml_feature_languagedetection_LdgpuNative_00024_"
EINVAL = _lib.LDGPU_EINVAL


@pytest.fixture(scope="module")
def jh(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("jh") / "libjh.so")
    libdir = os.path.join(ROOT, "spark-languagedetector_amd", "lib")
    subprocess.run(["gcc", "-O1", "-shared", "-fPIC", "-Wall", "-Wextra", "-Werror", "-I",
                    os.path.join(HERE, "jni_harness"), "-o", out, os.path.join(HERE, "jni_harness", "harness.c"),
                    os.path.join(ROOT, "jni", "ldgpu_jni.c"), "-L", libdir, "-lldgpu", f"-Wl,-rpath,{libdir}"],
                   check=True)
    _lib.load()  # the same libldgpu.so instance as the harness's (one loaded copy)
    L = ctypes.CDLL(out)
    L.jh_env.restype = ctypes.c_void_p
    L.jh_buf.restype = ctypes.c_void_p
    L.jh_buf.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    L.jh_arr.restype = ctypes.c_void_p
    L.jh_arr.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.jh_free.argtypes = [ctypes.c_void_p]
    getattr(L, FN + "lastError").restype = ctypes.c_char_p
    getattr(L, FN + "lastError").argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return L


class Shim:
    """Calls a shim entry point with fake buffers: numpy arrays become direct
    buffers (capacity = their size unless given), None stays null."""

    def __init__(self, L):
        self.L = L
        self.env = L.jh_env()
        self.keep = []

    def buf(self, a, cap=None):
        if a is None:
            return None
        self.keep.append(a)
        return self.L.jh_buf(a.ctypes.data, a.nbytes if cap is None else cap)

    def arr(self, a):
        self.keep.append(a)
        return self.L.jh_arr(a.ctypes.data, len(a))

    def call(self, name, *args):
        f = getattr(self.L, FN + name)
        f.restype = ctypes.c_int
        conv = []
        for a in args:
            conv.append(ctypes.c_int64(a) if isinstance(a, int) else ctypes.c_void_p(a))
        return f(ctypes.c_void_p(self.env), None, *conv)

    def err(self):
        return getattr(self.L, FN + "lastError")(self.env, None).decode()


def docs(n, length=16):
    data = np.frombuffer(b"ab" * (n * length // 2 + 1), dtype=np.uint8)[:n * length].copy()
    off = np.arange(n + 1, dtype=np.int64) * length
    return data, off


def test_score_rejects_short_and_bad_buffers(jh):
    s = Shim(jh)
    data, off = docs(10)
    lab = np.zeros(10, np.int32)
    # offsets one entry short
    assert s.call("score", 0, s.buf(data), s.buf(off, 8 * 10), 10, s.buf(lab), None, 3) == EINVAL
    assert "offsets holds 80 bytes" in s.err()
    # bytes shorter than offsets[n]
    assert s.call("score", 0, s.buf(data, len(data) - 1), s.buf(off), 10, s.buf(lab), None, 3) == EINVAL
    assert "bytes holds" in s.err()
    # labels short
    assert s.call("score", 0, s.buf(data), s.buf(off), 10, s.buf(lab, 39), None, 3) == EINVAL
    assert "labels" in s.err()
    # a negative first offset, a last offset before the first
    bad = off.copy()
    bad[0] = -4
    assert s.call("score", 0, s.buf(data), s.buf(bad), 10, s.buf(lab), None, 3) == EINVAL
    bad = off.copy()
    bad[0], bad[-1] = 100, 50
    assert s.call("score", 0, s.buf(data), s.buf(bad), 10, s.buf(lab), None, 3) == EINVAL
    # a scores buffer is sized by the model's language count: no model, no size
    sc = np.zeros((10, 3))
    assert s.call("score", 0, s.buf(data), s.buf(off), 10, s.buf(lab), s.buf(sc), 3) == EINVAL
    # a document count whose byte sizes overflow int64
    assert s.call("count", 0, s.buf(data), s.buf(off), (1 << 62), s.buf(lab)) == EINVAL
    assert "overflowing" in s.err() or "holds" in s.err()


def test_count_add_and_table_exports_need_handles(jh):
    s = Shim(jh)
    kb = np.frombuffer(b"abcabc", dtype=np.uint8).copy()
    ko = np.array([0, 3, 6], np.int64)
    po = np.array([5, 2, 3], np.int64)  # last pair offset before the first
    pl = np.zeros(4, np.int32)
    pc = np.ones(4, np.int64)
    assert s.call("countsAddSparse", 0, 2, s.buf(kb), s.buf(ko), s.buf(po), s.buf(pl), s.buf(pc)) == EINVAL
    # rows sized by the table's language count: a null table has none
    rows = np.zeros((2, 4), np.int64)
    assert s.call("countsAdd", 0, 2, s.buf(kb), s.buf(ko), s.buf(rows), 4) == EINVAL
    # the cached table's sizes come from the library, not from the caller
    assert s.call("fitTableExport", 0, s.buf(kb), s.buf(ko), s.buf(rows), 2, 6, 4) == EINVAL


def test_preprocess_buffers_are_checked(jh):
    """casemapCreate needs the whole case map (65536 units + 8192 bitmap
    bytes); preprocess needs units up to offsets[n], an output buffer for the
    worst case (every unit kept: units, or bytes with LOW_BYTES), n + 1 output
    offsets and n host flags -- all checked before the library is reached."""
    s = Shim(jh)
    lower = np.arange(65536, dtype=np.uint16)
    special = np.zeros(8192, np.uint8)
    h = np.zeros(1, np.int64)
    assert s.call("casemapCreate", 0, s.buf(lower, 2 * 65536 - 2), s.buf(special), s.arr(h)) == EINVAL
    assert "lower holds" in s.err()
    assert s.call("casemapCreate", 0, s.buf(lower), s.buf(special, 8191), s.arr(h)) == EINVAL
    assert "special" in s.err()
    units = np.frombuffer("Hello World, Straße".encode("utf-16-le"), np.uint16).copy()
    off = np.array([0, 5, 11, len(units)], np.int64)
    n = 3
    out = np.zeros(len(units), np.uint16)
    oo = np.zeros(n + 1, np.int64)
    host = np.zeros(n, np.uint8)
    args = lambda u, o, ob, oob, hb, flags=_lib.PRE_LOWER: (
        "preprocess", 0, u, o, n, None, flags, ob, oob, hb)
    assert s.call(*args(s.buf(units, 2 * len(units) - 1), s.buf(off), s.buf(out), s.buf(oo), s.buf(host))) == EINVAL
    assert "units holds" in s.err()
    assert s.call(*args(s.buf(units), s.buf(off), s.buf(out, 2 * len(units) - 2), s.buf(oo), s.buf(host))) == EINVAL
    assert "out holds" in s.err()
    # bytes output: half the buffer is enough, less is not
    assert s.call(*args(s.buf(units), s.buf(off), s.buf(out, len(units) - 1), s.buf(oo), s.buf(host),
                        _lib.PRE_LOWER | _lib.PRE_LOW_BYTES)) == EINVAL
    assert s.call(*args(s.buf(units), s.buf(off), s.buf(out), s.buf(oo, 8 * n), s.buf(host))) == EINVAL
    assert "outOffsets" in s.err()
    assert s.call(*args(s.buf(units), s.buf(off), s.buf(out), s.buf(oo), s.buf(host, n - 1))) == EINVAL
    assert "host" in s.err()
    loc = np.zeros(n - 1, np.uint8)
    assert s.call("preprocess", 0, s.buf(units), s.buf(off), n, s.buf(loc), _lib.PRE_LOWER, s.buf(out), s.buf(oo),
                  s.buf(host)) == EINVAL
    assert "locale" in s.err()
    # right-sized buffers reach the library, which refuses the null map
    assert s.call(*args(s.buf(units), s.buf(off), s.buf(out), s.buf(oo), s.buf(host))) == EINVAL
    assert "casemap" in s.err()


@pytest.mark.gpu
def test_shim_on_device_handles(jh):
    """Real handles: the scores buffer and count rows are sized by the
    handle's language count and the fit table export by the library's cached
    table; a caller whose n_langs / n_rows / key bytes differ from the
    handle's is refused (its rows would take another stride), right-sized
    calls work."""
    from languagedetection.runtime import DeviceCounts, DeviceModel
    s = Shim(jh)
    L = 5
    table = {b"ab": [1.0, 0.0, 0.0, 0.0, 0.0], b"ba": [0.0, 0.5, 0.0, 0.0, 0.0]}
    m = DeviceModel(table, L, [2])
    data, off = docs(8)
    lab = np.zeros(8, np.int32)
    sc = np.zeros((8, L))
    # a scores buffer for 4 of the model's 5 languages: refused
    assert s.call("score", m.h, s.buf(data), s.buf(off), 8, s.buf(lab), s.buf(sc, 8 * 8 * 4), L) == EINVAL
    assert "scores" in s.err()
    # a big enough buffer but another language count: refused, not scrambled
    assert s.call("score", m.h, s.buf(data), s.buf(off), 8, s.buf(lab), s.buf(sc), 4) == EINVAL
    assert "nLangs" in s.err()
    assert s.call("score", m.h, s.buf(data), s.buf(off), 8, s.buf(lab), s.buf(sc), L) == 0
    expect, escore = m.score(data, off, want_scores=True)
    assert np.array_equal(lab, expect) and np.array_equal(sc, escore)

    c = DeviceCounts(L, [1, 2])
    c.count(data, off, np.zeros(8, np.int32))
    n, nb = c.size(), 2 + 4 * 2   # grams a, b, ab, ba
    assert n == 4
    kb = np.zeros(nb, np.uint8)
    ko = np.zeros(n + 1, np.int64)
    cnt = np.zeros((n, L), np.int64)
    assert s.call("countsExport", c.h, s.buf(kb), s.buf(ko), s.buf(cnt, 8 * n * 3), 3) == EINVAL
    assert s.call("countsExport", c.h, s.buf(kb), s.buf(ko), s.buf(cnt), 3) == EINVAL
    assert "nLangs" in s.err()
    assert s.call("countsExport", c.h, s.buf(kb), s.buf(ko), s.buf(cnt), L) == 0
    k2, c2 = c.export()
    assert np.array_equal(cnt, c2)
    out = np.zeros(2, np.int64)
    assert s.call("fitTableSize", c.h, 10, s.arr(out)) == 0
    rows_n, key_b = int(out[0]), int(out[1])
    tk = np.zeros(max(key_b, 1), np.uint8)
    tko = np.zeros(rows_n + 1, np.int64)
    rows = np.zeros((rows_n, L))
    # the caller's row count, key bytes and language count must be the table's
    assert s.call("fitTableExport", c.h, s.buf(tk), s.buf(tko), s.buf(rows, 8 * rows_n * 2), rows_n, key_b,
                  L) == EINVAL
    assert s.call("fitTableExport", c.h, s.buf(tk), s.buf(tko), s.buf(rows), 1, key_b, L) == EINVAL
    assert "nRows" in s.err()
    assert s.call("fitTableExport", c.h, s.buf(tk), s.buf(tko), s.buf(rows), rows_n, key_b, 2) == EINVAL
    assert s.call("fitTableExport", c.h, s.buf(tk), s.buf(tko), s.buf(rows), rows_n, key_b, L) == 0
    assert {bytes(tk[tko[i]:tko[i + 1]]): list(rows[i]) for i in range(rows_n)} == c.fit_table(10)
    m.close()
    c.close()


@pytest.mark.gpu
def test_shim_preprocess_on_the_device(jh):
    """A case map made through the shim lower-cases and cleans exactly as
    DeviceCaseMap (the Python binding of the same ABI) does."""
    from languagedetection.runtime import DeviceCaseMap, case_tables
    s = Shim(jh)
    lower, special = case_tables()
    ctx = _lib.context(None)
    h = np.zeros(1, np.int64)
    assert s.call("casemapCreate", ctx, s.buf(lower), s.buf(special), s.arr(h)) == 0
    texts = ["Hello  World!", "ISTANBUL (İ)", "Straße #1", "ΟΔΟΣ", ""]
    loc = np.array([0, 1, 0, 0, 0], np.uint8)
    dm = DeviceCaseMap()
    units, off = dm.pack_units(texts)
    for flags in (_lib.PRE_LOWER, _lib.PRE_LOWER | _lib.PRE_CLEAN, _lib.PRE_CLEAN | _lib.PRE_LOW_BYTES):
        ob = np.zeros(len(units) + 4, np.uint8 if flags & _lib.PRE_LOW_BYTES else np.uint16)
        oo = np.zeros(len(texts) + 1, np.int64)
        host = np.zeros(len(texts), np.uint8)
        assert s.call("preprocess", int(h[0]), s.buf(units), s.buf(off), len(texts), s.buf(loc), flags, s.buf(ob),
                      s.buf(oo), s.buf(host)) == 0, s.err()
        e_out, e_oo, e_host = dm.run(units, off, loc, flags)
        assert np.array_equal(oo, e_oo) and np.array_equal(host, e_host)
        assert np.array_equal(ob[:oo[-1]], e_out[:e_oo[-1]])
    assert s.call("casemapDestroy", int(h[0])) == 0
    dm.close()
