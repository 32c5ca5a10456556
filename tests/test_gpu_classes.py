"""GPU parity of class mode: labels-only SCORE calls on a mask table whose rows
hold at most a few distinct finite values (a fit table's presence classes,
LanguageDetector.scala:98-105).  The kernel counts hits per (value, language),
labels a document from the counts when a rounding bound separates its top
language from every other, and replays the rest in reference order
(LanguageDetectorModel.scala:139-154).  Labels must equal the oracle's exactly,
ties and near ties included; scores calls keep the ordered replay.  Both the
device-buffer call and the host-buffer pipeline (ldgpu_score) take class mode,
and both stay asynchronous (the replay is sized on the device)."""
import math

import numpy as np
import pytest
import torch

import ldoracle_c as OC
from languagedetection import encoding
from languagedetection.runtime import DeviceModel

pytestmark = pytest.mark.gpu

ALPHABET = np.frombuffer(b"abcdefgh ", dtype=np.uint8)


def class_table(rng, L, n_keys, grams, values):
    """Each row: one of `values` at a random subset of the languages."""
    table = {}
    for _ in range(n_keys):
        k = bytes(rng.choice(ALPHABET, size=int(rng.choice(grams))))
        m = rng.random(L) < rng.uniform(0.02, 0.5)
        if not m.any():
            m[int(rng.integers(0, L))] = True
        v = float(values[int(rng.integers(0, len(values)))])
        table[k] = [v if b else 0.0 for b in m]
    return table


def oracle_labels(table, L, grams, data, off):
    return OC.Table(table, L).score(grams, data, off, want_scores=False, nthreads=8)[0]


def labels_device(m, data, off):
    """Labels-only scoring through ldgpu_score_device (HBM-resident buffers)."""
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(np.ascontiguousarray(off, dtype=np.int64)).to(dev)
    n = len(off) - 1
    d_lab = torch.full((n,), -7, dtype=torch.int32, device=dev)
    m.score_device(d_bytes.data_ptr(), len(data), d_off.data_ptr(), n, d_lab.data_ptr(), 0,
                   torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    return d_lab.cpu().numpy()


def docs_of(rng, n, hi):
    lens = rng.integers(0, hi, size=n)
    lens[:6] = [0, 1, 2, 3, 7, 64]
    return encoding.pack([bytes(rng.choice(ALPHABET, size=int(x))) for x in lens])


# presence-class values: log(1 + 1/k), the shape of a fit table's probabilities
PRESENCE = [math.log(1.0 + 1.0 / k) for k in (1, 2, 3, 5)]


@pytest.mark.parametrize("L,grams,n_cls", [
    (3, [1, 2, 3], 2), (20, [1, 2, 3, 4, 5], 4), (20, [1, 2, 3, 4, 5], 1), (64, [2, 3], 3),
    (65, [3, 1], 4), (130, [1, 2, 3, 4, 5, 6, 7], 2), (200, [5, 5, 2], 3), (256, [4, 2], 2),
])
def test_class_mode_labels_match_oracle(L, grams, n_cls, monkeypatch):
    """n_cls = 1: a one-value table takes count mode in the product library;
    the diagnostics library's LDGPU_NO_COUNT_MODE sends it to class mode with
    one class (exact ties decided by the counts)."""
    rng = np.random.default_rng(L * 13 + n_cls)
    values = PRESENCE[:n_cls] if n_cls > 1 else [-0.25]
    table = class_table(rng, L, 400, grams, values)
    data, off = docs_of(rng, 800, 200)
    variant = "product"
    if n_cls == 1:
        monkeypatch.setenv("LDGPU_NO_COUNT_MODE", "1")
        variant = "diag"
    m = DeviceModel(table, L, grams, variant=variant)
    assert "classes" in m.info()["layout"], m.info()
    ol = oracle_labels(table, L, grams, data, off)
    assert np.array_equal(labels_device(m, data, off), ol)
    labels, _ = m.score(data, off)  # the host pipeline (class mode too)
    assert np.array_equal(labels, ol)
    # a scores call keeps the ordered replay: same labels, scores bit-exact
    lab2, sc = m.score(data, off, want_scores=True)
    ol, os_ = OC.Table(table, L).score(grams, data, off, want_scores=True, nthreads=8)
    assert np.array_equal(lab2, ol)
    assert np.array_equal(np.ascontiguousarray(sc).view(np.uint64), np.ascontiguousarray(os_).view(np.uint64))


def test_class_mode_order_dependent_ties():
    """Two languages with the same (value, count) multiset in a different hit
    order: the folds differ in the last bit (ln2, ln1.5, ln1.5 against ln1.5,
    ln1.5, ln2), so neither the counts nor a first-maximum rule can decide --
    only the ordered replay of those documents gives the reference's label."""
    v1, v2 = math.log(2.0), math.log(1.5)
    assert (0.0 + v1 + v2) + v2 != (0.0 + v2 + v2) + v1
    table = {b"a": [v1, 0.0, 0.0], b"b": [v2, 0.0, 0.0], b"c": [0.0, v2, 0.0], b"d": [0.0, v1, 0.0],
             b"e": [0.0, 0.0, v1], b"ab": [v2, v2, 0.0]}
    rng = np.random.default_rng(5)
    docs = [b"abbccd", b"ccdabb", b"abb", b"ccd", b"dcc", b"bba", b"", b"zzz", b"e"]
    docs += [bytes(rng.choice(np.frombuffer(b"abcde", dtype=np.uint8), size=int(n)))
             for n in rng.integers(1, 12, size=3000)]
    data, off = encoding.pack(docs)
    m = DeviceModel(table, 3, [1, 2])
    assert "classes" in m.info()["layout"]
    labels = labels_device(m, data, off)
    ol = oracle_labels(table, 3, [1, 2], data, off)
    assert np.array_equal(labels, ol), np.nonzero(labels != ol)[0][:10]
    # the hand-made pair really is decided by order: labels differ between them
    assert ol[0] != ol[2] or ol[0] == ol[1]


def test_class_mode_device_api_and_all_ambiguous():
    """ldgpu_score_device (device pointers, the stream the caller names): a
    corpus where every document is an exact multi-class tie -- all of it goes
    through the replay step."""
    v1, v2 = math.log(2.0), math.log(1.5)
    table = {b"a": [v1, v1], b"b": [v2, v2]}
    docs = [b"ab" * int(n) for n in range(1, 400)] + [b"ba" * 3, b"aab", b"bba"]
    data, off = encoding.pack(docs)
    m = DeviceModel(table, 2, [1])
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_lab = torch.full((len(docs),), 7, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    m.score_device(d_bytes.data_ptr(), len(data), d_off.data_ptr(), len(docs), d_lab.data_ptr(), 0, st.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(d_lab.cpu().numpy(), oracle_labels(table, 2, [1], data, off))


def test_too_many_values_keep_the_ordered_replay():
    """More distinct values than the counters hold: no class mode, labels from
    the ordered replay, still exact."""
    rng = np.random.default_rng(9)
    table = class_table(rng, 20, 300, [1, 2, 3], [math.log(1.0 + 1.0 / k) for k in range(1, 9)])
    data, off = docs_of(rng, 500, 150)
    m = DeviceModel(table, 20, [1, 2, 3])
    assert "classes" not in m.info()["layout"]
    assert np.array_equal(labels_device(m, data, off), oracle_labels(table, 20, [1, 2, 3], data, off))


def test_class_mode_switched_off_in_diag_library(monkeypatch):
    """LDGPU_NO_CLASS_MODE (diagnostics library) forces the ordered replay on
    the same table: the two paths agree."""
    rng = np.random.default_rng(21)
    table = class_table(rng, 20, 400, [1, 2, 3, 4, 5], PRESENCE)
    data, off = docs_of(rng, 600, 200)
    a = DeviceModel(table, 20, [1, 2, 3, 4, 5])
    monkeypatch.setenv("LDGPU_NO_CLASS_MODE", "1")
    b = DeviceModel(table, 20, [1, 2, 3, 4, 5], variant="diag")
    assert "classes" in a.info()["layout"] and "classes" not in b.info()["layout"]
    assert np.array_equal(labels_device(a, data, off), labels_device(b, data, off))


@pytest.mark.parametrize("L,n_cls", [(20, 2), (63, 1), (40, 3)])
def test_class_mode_direct_tables(L, n_cls, monkeypatch):
    """Every 1-/2-byte key names one language (a fit table's unique grams),
    L <= 63: class mode counts those windows from the LDS direct tables (an
    entry = language | class << 6) and the longer keys through the split
    verify; labels equal to the oracle's."""
    rng = np.random.default_rng(L * 3 + n_cls)
    values = PRESENCE[:n_cls] if n_cls > 1 else [0.375]
    table = {}
    for _ in range(600):
        n = int(rng.choice([1, 2, 3, 4, 5]))
        k = bytes(rng.choice(ALPHABET, size=n))
        v = float(values[int(rng.integers(0, len(values)))])
        if n <= 2:
            row = [0.0] * L
            row[int(rng.integers(0, L))] = v
        else:
            m = rng.random(L) < rng.uniform(0.02, 0.4)
            if not m.any():
                m[0] = True
            row = [v if b else 0.0 for b in m]
        table[k] = row
    data, off = docs_of(rng, 3000, 300)
    variant = "product"
    if n_cls == 1:
        monkeypatch.setenv("LDGPU_NO_COUNT_MODE", "1")
        variant = "diag"
    m = DeviceModel(table, L, [1, 2, 3, 4, 5], variant=variant)
    lay = m.info()["layout"]
    assert "classes" in lay and "direct" in lay, lay
    assert np.array_equal(labels_device(m, data, off), oracle_labels(table, L, [1, 2, 3, 4, 5], data, off))
    lab2, sc = m.score(data[:int(off[500])], off[:501], want_scores=True)
    ol, os_ = OC.Table(table, L).score([1, 2, 3, 4, 5], data[:int(off[500])], off[:501], want_scores=True, nthreads=8)
    assert np.array_equal(lab2, ol)
    assert np.array_equal(np.ascontiguousarray(sc).view(np.uint64), np.ascontiguousarray(os_).view(np.uint64))


def _ulps(a, b):
    """distance of two finite doubles of one sign in units in the last place"""
    ia = np.asarray(a, dtype=np.float64).view(np.int64)
    ib = np.asarray(b, dtype=np.float64).view(np.int64)
    return np.abs(ia - ib)


@pytest.mark.parametrize("L,tiny", [(2, False), (3, True), (20, True)])
def test_class_mode_near_ties_at_many_hits(L, tiny):
    """Near ties at 100-2,000 hits per document: the top two languages' folds
    differ by 0-4 ulps.  Values 0.1 and 0.3 (and 2^-40 when `tiny`) make exact
    sums that differ by far less than an ulp (a + 3b = c + 3d hits), so the
    label is decided by the fold's roundings, i.e. by hit ORDER -- class_label's
    rounding bound (ldgpu_score.hip) must send every such document to the
    ordered replay, and a document it labels from counts must be one whose
    fold agrees.  `tiny` adds one-off hits of 2^-40, which move the exact sums
    apart by amounts around the bound itself (~1e-11 at these sizes).  Each
    1-byte key names one (language, value): letters a/b -> language 0 with
    0.1/0.3, c/d -> language 1, e/f -> 2^-40, g -> every language 0.1."""
    v1, v3, vt = 0.1, 0.3, 2.0 ** -40
    table = {b"a": [v1] + [0.0] * (L - 1), b"b": [v3] + [0.0] * (L - 1),
             b"c": [0.0, v1] + [0.0] * (L - 2), b"d": [0.0, v3] + [0.0] * (L - 2),
             b"g": [v1] * L}
    if tiny:
        table[b"e"] = [vt] + [0.0] * (L - 1)
        table[b"f"] = [0.0, vt] + [0.0] * (L - 2)
    if L > 2:  # a third language well behind
        table[b"h"] = [0.0, 0.0, v3] + [0.0] * (L - 3)
    rng = np.random.default_rng(L * 7 + tiny)
    docs = []
    for _ in range(3000):
        n = int(rng.integers(100, 2001))
        b = int(rng.integers(0, n // 4))
        a = n - 3 * b if n - 3 * b > 0 else n
        d = int(rng.integers(max(0, b - 30), b + 31))
        c = a + 3 * (b - d)
        if c < 0:
            c, d = a, b
        parts = [b"a"] * a + [b"b"] * b + [b"c"] * c + [b"d"] * d + [b"g"] * int(rng.integers(0, 40))
        if tiny:  # equal tiny counts in half of the documents, else 1-2 apart
            ne = int(rng.integers(0, 40))
            nf = max(0, ne + (int(rng.integers(-2, 3)) if rng.random() < 0.5 else 0))
            parts += [b"e"] * ne + [b"f"] * nf
        if L > 2:
            parts += [b"h"] * int(rng.integers(0, 20))
        rng.shuffle(parts)
        docs.append(b"".join(parts))
    data, off = encoding.pack(docs)
    m = DeviceModel(table, L, [1])
    assert "classes" in m.info()["layout"], m.info()
    ol, os_ = OC.Table(table, L).score([1], data, off, want_scores=True, nthreads=8)
    # the corpus really is made of near ties: most documents' top two folds
    # are within 4 ulps, and order decides many of them
    top2 = np.sort(os_, axis=1)[:, -2:]
    gap = _ulps(top2[:, 0], top2[:, 1])
    assert (gap <= 4).mean() > 0.25, np.bincount(np.minimum(gap, 10))
    assert ((gap >= 1) & (gap <= 4)).sum() >= 300
    assert np.array_equal(labels_device(m, data, off), ol)
    labels, _ = m.score(data, off)   # the host pipeline, class mode
    assert np.array_equal(labels, ol)
