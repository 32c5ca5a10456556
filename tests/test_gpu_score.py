"""GPU parity of SCORE (LanguageDetectorModel.detect, LanguageDetectorModel.scala:131-156)
through the C ABI: labels AND fp64 scores bit-identical to the oracle."""
import ctypes
import json
import math
import os

import numpy as np
import pytest

import ldoracle as O
import ldoracle_c as OC
from conftest import GOLDEN
from languagedetection import LanguageDetectorModel, _lib, encoding, synth
from languagedetection.runtime import DeviceModel

pytestmark = pytest.mark.gpu


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def dec_table(enc):
    return {bytes.fromhex(k): [float.fromhex(v) for v in row] for k, row in enc}


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def oracle_c(table, L, grams, data, off, scores=True):
    t = OC.Table(table, L)
    return t.score(grams, data, off, want_scores=scores, nthreads=8)


def check_parity(table, L, grams, data, off, variant="product"):
    m = DeviceModel(table, L, grams, variant=variant)
    labels, scores = m.score(data, off, want_scores=True)
    ol, os_ = oracle_c(table, L, grams, data, off)
    assert np.array_equal(labels, ol), np.nonzero(labels != ol)[0][:10]
    assert np.array_equal(bits(scores), bits(os_))
    return m


def test_reference_score_kat_transform():
    """LanguageDetectorModelSpecs.scala:15-44 through the Model API."""
    import pandas as pd
    k = load("reference_kats.json")["score_kat"]
    model = LanguageDetectorModel(gramProbabilities=k["table"], gramLengths=k["gram_lengths"],
                                  languages=k["languages"])
    out = model.transform(pd.DataFrame({"fulltext": k["docs"]}))
    labels = list(out["lang"])
    assert len(out) == k["expect_rows"]
    for lang, n in k["expect_count"].items():
        assert labels.count(lang) == n
    assert labels == ["de", "de", "en", "en"]
    assert list(out.columns) == ["fulltext", "lang"]


@pytest.mark.parametrize("case", load("score_cases.json"), ids=lambda c: c["name"])
def test_golden_score_cases(case):
    table = dec_table(case["table"])
    docs = [bytes.fromhex(h) for h in case["docs_hex"]]
    data, off = encoding.pack(docs)
    m = DeviceModel(table, len(case["languages"]), case["gram_lengths"])
    labels, scores = m.score(data, off, want_scores=True)
    assert labels.tolist() == case["labels"]
    assert [[v.hex() for v in row] for row in scores.tolist()] == case["scores"]


def test_detect_static_string_and_bytes():
    table = {"Die": [1.0, 0.0], "Thi": [0.0, 1.0]}
    assert LanguageDetectorModel.detect("Dies ist", table, ["de", "en"], [3]) == "de"
    assert LanguageDetectorModel.detect(b"This", table, ["de", "en"], [3]) == "en"
    assert LanguageDetectorModel.detect("", table, ["de", "en"], [3]) == "de"  # no hit -> index 0


def test_detect_sees_in_place_edits_of_the_map():
    """The reference builds its lookups from the map on every call
    (LanguageDetectorModel.scala:131-156): an edit between two calls changes
    the second call's label even though the cached device table is reused for
    unchanged maps."""
    from languagedetection import freeze_table
    table = {"Die": [1.0, 0.0], "Thi": [0.0, 1.0]}
    assert LanguageDetectorModel.detect("Dies", table, ["de", "en"], [3]) == "de"
    table["Die"][0], table["Die"][1] = 0.0, 2.0          # edit a value list in place
    assert LanguageDetectorModel.detect("Dies", table, ["de", "en"], [3]) == "en"
    table["Thi"] = [3.0, 0.0]                           # replace a non-first entry, same length
    assert LanguageDetectorModel.detect("This", table, ["de", "en"], [3]) == "de"
    del table["Thi"]
    table["Dat"] = [0.0, 1.0]                           # same length, other key
    assert LanguageDetectorModel.detect("Dat", table, ["de", "en"], [3]) == "en"
    assert LanguageDetectorModel.detect("This", table, ["de", "en"], [3]) == "de"  # no hit now
    frozen = freeze_table(table)
    assert LanguageDetectorModel.detect("Dies", frozen, ["de", "en"], [3]) == "en"
    assert LanguageDetectorModel.detect("Dat", frozen, ["de", "en"], [3]) == "en"
    with pytest.raises(TypeError):
        frozen["Dat"] = [1.0, 0.0]


def _random_table(rng, L, n_keys, grams, alphabet, mask_form, uniform=None):
    """uniform: one shared value for every row (the count-mode kernel)."""
    table = {}
    for _ in range(n_keys):
        n = int(rng.choice(grams))
        k = bytes(rng.choice(alphabet, size=n))
        if mask_form:
            m = rng.random(L) < rng.uniform(0.02, 0.6)
            if not m.any():
                m[int(rng.integers(0, L))] = True
            v = uniform if uniform is not None else math.log(1.0 + 1.0 / int(m.sum()))
            table[k] = [v if b else 0.0 for b in m]
        else:
            table[k] = rng.normal(size=L).tolist()
    return table


@pytest.mark.parametrize("L,grams,mask_form", [
    (3, [1, 2, 3], True), (20, [1, 2, 3, 4, 5], True), (64, [2, 3], True), (65, [3, 1], True),
    (130, [1, 2, 3, 4, 5, 6, 7], True), (200, [5, 5, 2], True), (256, [4], True),
    (3, [3], False), (20, [1, 2, 3, 4, 5], False), (100, [2, 7], False), (256, [1, 3], False),
])
def test_random_parity(L, grams, mask_form):
    rng = np.random.default_rng(L * 7 + len(grams) + int(mask_form))
    alphabet = np.frombuffer(b"abcdefgh ", dtype=np.uint8)
    table = _random_table(rng, L, 400, grams, alphabet, mask_form)
    lens = rng.integers(0, 300, size=600)
    lens[:8] = [0, 1, 2, 3, 6, 7, 64, 65]
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in lens]
    data, off = encoding.pack(docs)
    m = check_parity(table, L, grams, data, off)
    assert m.info()["mode"] == (0 if mask_form else 1)


@pytest.fixture(params=["count", "replay"])
def uniform_path(request, monkeypatch):
    """Uniform-value tables run the count kernel (mode 2); LDGPU_NO_COUNT_MODE
    in the diagnostics library (the product library reads no environment)
    forces the ordered-replay kernel on the same table (mode 0).
    Returns (expected mode, library variant)."""
    if request.param == "replay":
        monkeypatch.setenv("LDGPU_NO_COUNT_MODE", "1")
        return 0, "diag"
    return 2, "product"


@pytest.mark.parametrize("L,grams,v", [
    (3, [1, 2, 3], math.log(2.0)), (20, [1, 2, 3, 4, 5], math.log(2.0)), (64, [2, 3], 1.0),
    (65, [3, 1], 0.1), (130, [1, 2, 3, 4, 5, 6, 7], -0.7), (256, [4, 2], 1e-300),
])
def test_uniform_value_parity(L, grams, v, uniform_path):
    """One value in every row (all of a fit table's grams in one presence
    class): per-language counts folded through the value must equal the
    reference's ordered daxpy fold bit for bit, negative and tiny values too."""
    rng = np.random.default_rng(L * 11 + len(grams))
    alphabet = np.frombuffer(b"abcdefgh ", dtype=np.uint8)
    table = _random_table(rng, L, 400, grams, alphabet, True, uniform=v)
    lens = rng.integers(0, 300, size=600)
    lens[:8] = [0, 1, 2, 3, 6, 7, 64, 65]
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in lens]
    data, off = encoding.pack(docs)
    m = check_parity(table, L, grams, data, off, variant=uniform_path[1])
    assert m.info()["mode"] == uniform_path[0]


def test_uniform_value_counts_past_fold_table(uniform_path):
    """A language hit more than 8191 times in one document: the device
    continues the fold past the host-built table."""
    L = 3
    table = {bytes([c]): [0.3 if (c % 3) == l else 0.0 for l in range(L)] for c in range(256)}
    table[b"ab"] = [0.3, 0.3, 0.0]
    rng = np.random.default_rng(17)
    docs = [b"ab" * 9000, bytes(rng.integers(0, 256, size=30000, dtype=np.uint8)), b"", b"a"]
    data, off = encoding.pack(docs)
    m = check_parity(table, L, [1, 2, 1], data, off, variant=uniform_path[1])
    assert m.info()["mode"] == uniform_path[0]


@pytest.mark.parametrize("direct", [True, False])
@pytest.mark.parametrize("L,grams", [(20, [1, 2, 3, 4, 5]), (100, [2, 1, 2, 3]), (255, [1, 2, 7])])
def test_single_language_keys_direct_tables(L, grams, direct, monkeypatch):
    """Every row one language, one shared value (a fit table of grams unique
    to a language): 1-/2-byte keys are counted from the LDS direct tables,
    longer ones verified; LDGPU_NO_DIRECT (diagnostics library) forces them all
    through verification.  Docs of every length class: partial windows, the
    256-byte fast path, long."""
    if not direct:
        monkeypatch.setenv("LDGPU_NO_DIRECT", "1")
    rng = np.random.default_rng(L + 3 * len(grams))
    alphabet = np.frombuffer(b"abcdefghij ", dtype=np.uint8)
    v = math.log(2.0)
    table = {}
    for _ in range(600):
        n = int(rng.choice(grams))
        k = bytes(rng.choice(alphabet, size=n))
        row = [0.0] * L
        row[int(rng.integers(0, L))] = v
        table[k] = row
    lens = rng.integers(0, 400, size=800)
    lens[:10] = [0, 1, 2, 3, 6, 7, 64, 65, 256, 255]
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in lens]
    data, off = encoding.pack(docs)
    m = check_parity(table, L, grams, data, off, variant="product" if direct else "diag")
    assert m.info()["mode"] == 2


def _single_language_table(rng, L, grams, alphabet, n_keys, v):
    table = {}
    for _ in range(n_keys):
        n = int(rng.choice(grams))
        row = [0.0] * L
        row[int(rng.integers(0, L))] = v
        table[bytes(rng.choice(alphabet, size=n))] = row
    return table


@pytest.mark.parametrize("L,grams,single", [
    (20, [1, 2, 3, 4, 5], True), (100, [1, 2, 3, 4, 5], True), (100, [2, 1, 2, 3], False),
    (255, [1, 2, 7], True), (3, [3, 5], False), (130, [1, 2, 3, 4, 5, 6, 7], False),
])
def test_packed_short_documents(L, grams, single):
    """Count mode, labels only (transform): consecutive documents of
    maxg..128 bytes share one 256-position superblock (score_pack), each with
    its own counters; windows must not cross a document boundary.  Lengths
    straddle every case: shorter than maxg (partial windows, general path),
    packs of 2..4, a document that does not fit the open pack, > 128."""
    rng = np.random.default_rng(L * 5 + len(grams) + int(single))
    alphabet = np.frombuffer(b"abcdefghij ", dtype=np.uint8)
    v = math.log(2.0)
    table = (_single_language_table(rng, L, grams, alphabet, 900, v) if single
             else _random_table(rng, L, 600, grams, alphabet, True, uniform=v))
    lens = rng.integers(0, 100, size=3000)
    lens[:16] = [0, 1, 2, 7, 8, 64, 64, 64, 64, 63, 65, 128, 129, 256, 40, 40]
    lens[1000:1100] = rng.integers(max(grams), 70, size=100)
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in lens]
    data, off = encoding.pack(docs)
    m = DeviceModel(table, L, grams)
    labels, _ = m.score(data, off, want_scores=False)
    ol, _ = oracle_c(table, L, grams, data, off, scores=False)
    assert np.array_equal(labels, ol), np.nonzero(labels != ol)[0][:10]
    assert m.info()["mode"] == 2


def test_packed_path_taken(monkeypatch, capfd):
    """The diagnostics library reports whether a model packs short documents;
    LDGPU_NO_PACK turns packing off and the labels stay the same."""
    rng = np.random.default_rng(3)
    alphabet = np.frombuffer(b"abcdefghij ", dtype=np.uint8)
    L, grams = 100, [1, 2, 3, 4, 5]
    table = _single_language_table(rng, L, grams, alphabet, 900, math.log(2.0))
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in rng.integers(20, 90, size=2000)]
    data, off = encoding.pack(docs)
    monkeypatch.setenv("LDGPU_DEBUG", "1")
    packed = DeviceModel(table, L, grams, variant="diag")
    assert "pack=1" in capfd.readouterr().err
    a, _ = packed.score(data, off, want_scores=False)
    monkeypatch.setenv("LDGPU_NO_PACK", "1")
    plain = DeviceModel(table, L, grams, variant="diag")
    assert "pack=0" in capfd.readouterr().err
    b, _ = plain.score(data, off, want_scores=False)
    ol, _ = oracle_c(table, L, grams, data, off, scores=False)
    assert np.array_equal(a, ol) and np.array_equal(b, ol)


@pytest.mark.parametrize("L", [257, 300, 520])
@pytest.mark.parametrize("form", ["count", "mask", "dense"])
def test_language_blocks(L, form):
    """More than 256 languages: one launch per block of 256 languages, the
    label the first maximum across the blocks' maxima (ties keep the earlier
    block).  Uniform-value tables make cross-block ties common."""
    rng = np.random.default_rng(L + len(form))
    alphabet = np.frombuffer(b"abcdefgh ", dtype=np.uint8)
    grams = [1, 2, 3, 4]
    if form == "dense":
        table = _random_table(rng, L, 300, grams, alphabet, False)
    else:
        table = _random_table(rng, L, 300, grams, alphabet, True, uniform=math.log(2.0) if form == "count" else None)
    lens = rng.integers(0, 300, size=800)
    lens[:6] = [0, 1, 2, 40, 64, 256]
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in lens]
    data, off = encoding.pack(docs)
    m = check_parity(table, L, grams, data, off)
    labels, _ = m.score(data, off, want_scores=False)
    ol, _ = oracle_c(table, L, grams, data, off, scores=False)
    assert np.array_equal(labels, ol)


def test_language_blocks_nan_and_inf():
    """NaN / inf rows across blocks: a NaN first score keeps label 0 (block 0
    only); a NaN in a later block never wins; +inf in a later block wins."""
    L = 300
    nan, inf = float("nan"), float("inf")
    row = lambda pairs: [pairs.get(l, 0.0) for l in range(L)]
    table = {b"a": row({0: nan, 5: 1.0}), b"b": row({256: nan, 3: 2.0}), b"c": row({290: inf, 1: 5.0}),
             b"d": row({260: 7.0, 2: 7.0}), b"e": row({280: 9.0})}
    docs = [b"a", b"b", b"c", b"d", b"e", b"ab", b"bc", b"de", b"", b"zz"]
    data, off = encoding.pack(docs)
    check_parity(table, L, [1], data, off)


@pytest.mark.parametrize("grams", [[8], [1, 3, 8, 12, 15], [15, 2, 9, 9], [5, 10]])
@pytest.mark.parametrize("form", ["count", "mask", "dense"])
def test_wide_keys(grams, form):
    """Gram lengths 8..15: keys of 8..15 bytes take two words in a table of
    their own; partial windows of documents shorter than n make keys of every
    length up to n.  Labels and fp64 scores bit-identical to the oracle,
    labels-only (count argmax, packs) too."""
    rng = np.random.default_rng(sum(grams) * 7 + len(form))
    alphabet = np.frombuffer(b"abc ", dtype=np.uint8)
    L = 12
    lens_k = sorted(set(grams) | {max(1, g - 3) for g in grams})
    if form == "dense":
        table = _random_table(rng, L, 500, lens_k, alphabet, False)
    else:
        table = _random_table(rng, L, 500, lens_k, alphabet, True, uniform=math.log(2.0) if form == "count" else None)
    lens = rng.integers(0, 120, size=1500)
    lens[:10] = [0, 1, 7, 8, 9, 14, 15, 16, 255, 256]
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in lens]
    data, off = encoding.pack(docs)
    m = check_parity(table, L, grams, data, off)
    labels, _ = m.score(data, off, want_scores=False)
    ol, _ = oracle_c(table, L, grams, data, off, scores=False)
    assert np.array_equal(labels, ol)


@pytest.mark.parametrize("grams", [[16], [3, 20], [31], [1, 40, 2, 40], [17, 5, 9]])
@pytest.mark.parametrize("form", ["count", "mask", "dense"])
def test_long_keys_general_table(grams, form):
    """Gram lengths beyond 15 (the reference accepts any n,
    LanguageDetectorModel.scala:139-147): every key in the general table (hash
    + key bytes compared on the device), the reference's window order, labels
    and fp64 score bits equal to the oracle's; partial windows of documents
    shorter than n make keys of every length up to n."""
    rng = np.random.default_rng(sum(grams) * 13 + len(form))
    alphabet = np.frombuffer(b"ab ", dtype=np.uint8)
    L = 70 if form == "mask" else 9
    lens_k = sorted(set(grams) | {max(1, g - 3) for g in grams} | {1, 2})
    if form == "dense":
        table = _random_table(rng, L, 600, lens_k, alphabet, False)
    else:
        table = _random_table(rng, L, 600, lens_k, alphabet, True, uniform=math.log(2.0) if form == "count" else None)
    lens = rng.integers(0, 140, size=800)
    lens[:10] = [0, 1, 7, 8, 15, 16, 17, 31, 40, 300]
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in lens]
    data, off = encoding.pack(docs)
    m = check_parity(table, L, grams, data, off)
    lay = m.info()["layout"]
    assert "general_keys" in lay
    # a mixed table (some length <= 15) scores those lengths on the
    # LDS-filtered kernels: their layout is reported beside general_keys
    assert (len(lay) > 1) == any(g <= 15 for g in grams), lay
    labels, _ = m.score(data, off, want_scores=False)
    ol, _ = oracle_c(table, L, grams, data, off, scores=False)
    assert np.array_equal(labels, ol)


@pytest.mark.parametrize("form", ["count", "mask", "dense"])
def test_mixed_table_long_hits_and_partial_windows(form):
    """A mixed table (grams 1-5 and 16): documents that no 16-byte window
    hits keep the short lengths' result (count / class / replay kernels),
    documents with a long hit are rescored whole by the general kernel, and a
    document shorter than 16 bytes is its own partial window of n = 16 --
    which can equal a SHORT key ("abcde" below) and then counts twice."""
    L = 20
    rng = np.random.default_rng(len(form) + 7)
    alphabet = np.frombuffer(b"abcdefgh ", dtype=np.uint8)
    uniform = math.log(2.0) if form == "count" else None
    table = _random_table(rng, L, 400, [1, 2, 3, 4, 5], alphabet, form != "dense", uniform=uniform)
    long_keys = [b"abcdefgh abcdefg", b"hhhhhhhhhhhhhhhh", b"a" * 16]
    for k in long_keys:
        table[k] = (_random_table(rng, L, 1, [16], alphabet, form != "dense", uniform=uniform).popitem()[1])
    table[b"abcde"] = [uniform or 0.5] + [0.0] * (L - 1) if form != "dense" else rng.normal(size=L).tolist()
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in rng.integers(0, 300, size=1500)]
    docs += [b"abcde", b"abcd", b"xx" + long_keys[0] + b"yy", long_keys[1] * 3, b"a" * 40, b"", b"ab" * 100]
    data, off = encoding.pack(docs)
    m = check_parity(table, L, [1, 2, 3, 4, 5, 16], data, off)
    lay = m.info()["layout"]
    assert "general_keys" in lay and "lds_bloom" in lay, lay
    labels, _ = m.score(data, off, want_scores=False)
    ol, _ = oracle_c(table, L, [1, 2, 3, 4, 5, 16], data, off, scores=False)
    assert np.array_equal(labels, ol)


def test_long_keys_wrong_length_row_and_masks():
    """A 20-byte key whose row has the wrong length fails only when hit; a
    mask-form table of long keys scores as its dense rows."""
    m = LanguageDetectorModel({"abcdefghijklmnopqrst": [1.0], "xy": [0.0, 1.0]}, [2, 20], ["a", "b"])
    assert m.predict_indices(["xyxy"])[0].tolist() == [1]
    with pytest.raises(ValueError, match="requirement failed"):
        m.predict_indices(["zzabcdefghijklmnopqrstzz"])
    kb = np.frombuffer(b"0123456789abcdefgh" + b"xy", dtype=np.uint8).copy()
    ko = np.array([0, 18, 20], np.int64)
    masks = np.array([[0b10], [0b01]], np.uint64)
    vals = np.array([0.75, 0.5])
    dm = DeviceModel.from_masks(kb, ko, masks, vals, 2, [18, 2])
    docs = [b"0123456789abcdefgh", b"xyxy0123456789abcdefgh", b"zz", b""]
    data, off = encoding.pack(docs)
    labels, scores = dm.score(data, off, want_scores=True)
    table = {b"0123456789abcdefgh": [0.0, 0.75], b"xy": [0.5, 0.0]}
    ol, os_ = oracle_c(table, 2, [18, 2], data, off)
    assert np.array_equal(labels, ol) and np.array_equal(bits(scores), bits(os_))


def test_wide_keys_wrong_length_row():
    """A wide key whose row has the wrong length fails only when hit."""
    m = LanguageDetectorModel({"abcdefghij": [1.0], "xy": [0.0, 1.0]}, [2, 10], ["a", "b"])
    assert m.predict_indices(["xyxy"])[0].tolist() == [1]
    with pytest.raises(ValueError, match="requirement failed"):
        m.predict_indices(["zzabcdefghijzz"])


def test_long_documents_and_hot_keys():
    """Every 1-gram in the table: every window hits, so the per-wave candidate
    queue flushes many times per document (order must survive the flushes)."""
    rng = np.random.default_rng(5)
    L = 9
    table = {bytes([c]): rng.normal(size=L).tolist() for c in range(256)}
    table.update({bytes(rng.integers(0, 256, size=3)): rng.normal(size=L).tolist() for _ in range(500)})
    lens = [0, 1, 5000, 12345, 70000, 3]
    docs = [bytes(rng.integers(0, 256, size=n, dtype=np.uint8)) for n in lens]
    data, off = encoding.pack(docs)
    check_parity(table, L, [1, 3, 2, 1], data, off)


@pytest.mark.parametrize("form", ["mask", "dense", "uniform"])
def test_fast_path_queue_flush_mid_document(form, uniform_path):
    """Documents of max(G)..256 bytes (the single-superblock fast path) whose
    windows nearly all hit -- every 1-byte gram and most 2-/3-byte grams of a
    small alphabet are keys, gram lengths ordered with a duplicate -- so the
    per-wave candidate queue fills before the next gram length: the kernel
    verifies and replays it in order mid-document.  Labels and the bits of the
    fp64 scores equal the oracle's, on the ordered (replay) and count paths."""
    rng = np.random.default_rng({"mask": 41, "dense": 42, "uniform": 43}[form])
    L = 7
    alphabet = np.frombuffer(b"abcde", dtype=np.uint8)
    keys = [bytes([c]) for c in range(256)]
    keys += [bytes([a, b]) for a in b"abcde" for b in b"abcde"]
    keys += [bytes(rng.choice(alphabet, size=3)) for _ in range(100)]
    table = {}
    for k in keys:
        if form == "dense":
            table[k] = rng.normal(size=L).tolist()
        else:
            m = rng.random(L) < 0.4
            m[int(rng.integers(0, L))] = True
            v = 0.25 if form == "uniform" else math.log(1.0 + 1.0 / int(m.sum()))
            table[k] = [v if b else 0.0 for b in m]
    lens = rng.integers(150, 257, size=3000)
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in lens]
    data, off = encoding.pack(docs)
    m = check_parity(table, L, [1, 3, 2, 1], data, off, variant=uniform_path[1])
    if form == "dense":
        assert m.info()["mode"] == 1
    elif form == "mask":
        assert m.info()["mode"] == 0
    else:
        assert m.info()["mode"] == uniform_path[0]


def test_unaligned_offsets_and_nonzero_start():
    rng = np.random.default_rng(9)
    alphabet = np.frombuffer(b"xyz", dtype=np.uint8)
    table = _random_table(rng, 5, 50, [1, 2, 3], alphabet, True)
    raw = bytes(rng.choice(alphabet, size=1001))
    # offsets start at 3 and use odd boundaries
    off = np.array([3, 4, 9, 9, 10, 500, 777, 1001], dtype=np.int64)
    data = np.frombuffer(raw + b"\0" * 7, dtype=np.uint8)
    m = DeviceModel(table, 5, [1, 2, 3])
    labels, scores = m.score(data, off, want_scores=True)
    docs = [raw[off[i]:off[i + 1]] for i in range(len(off) - 1)]
    for i, d in enumerate(docs):
        s = O.detect_scores(d, table, 5, [1, 2, 3])
        assert scores[i].tolist() == s
        assert labels[i] == O.argmax_first(s)


def test_wrong_length_row_raises_only_when_hit():
    m = LanguageDetectorModel({"ab": [1.0, 0.0], "zz": [1.0]}, [2], ["a", "b"])
    assert m.predict_indices(["abab"])[0].tolist() == [0]
    with pytest.raises(ValueError, match="requirement failed"):
        m.predict_indices(["xzz"])


def test_duplicate_keys_last_wins():
    lib = _lib.load()
    ctx = _lib.context()
    kb, ko = encoding.pack([b"ab", b"ab"])
    rows = np.array([[1.0, 0.0], [0.0, 1.0]])
    g = np.array([2], dtype=np.int32)
    h = ctypes.c_void_p()
    _lib.check(lib.ldgpu_model_create(ctx, 2, kb.ctypes.data, ko.ctypes.data, rows.ctypes.data, None, 2,
                                      g.ctypes.data, 1, ctypes.byref(h)))
    data, off = encoding.pack([b"xab"])
    labels = np.zeros(1, dtype=np.int32)
    _lib.check(lib.ldgpu_score(h.value, data.ctypes.data, off.ctypes.data, 1, labels.ctypes.data, None))
    lib.ldgpu_model_destroy(h.value)
    assert labels.tolist() == [1]


def test_invalid_arguments():
    with pytest.raises(ValueError, match="both must be positive"):
        DeviceModel({b"a": [1.0]}, 1, [0])
    assert DeviceModel({b"a": [1.0]}, 1, [16]).info()["layout"] == ["general_keys"]  # any gram length
    m = DeviceModel({b"a": [1.0]}, 1, [1])
    with pytest.raises(ValueError, match="offsets decrease"):
        m.score(np.zeros(8, dtype=np.uint8), np.array([0, 4, 2], dtype=np.int64))


def test_device_pointer_api_with_torch():
    import torch
    ls = synth.make_languages(20, seed=1)
    data, off, _ = synth.generate(ls, 3000, 256, 256, seed=2)
    rng = np.random.default_rng(3)
    table = _random_table(rng, 20, 2000, [1, 2, 3, 4, 5], np.frombuffer(b"abcdefghijklmnopqrstuvwxyz '", np.uint8),
                          True)
    m = DeviceModel(table, 20, [1, 2, 3, 4, 5])
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(np.concatenate([data, np.zeros(8, np.uint8)])).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_lab = torch.empty(len(off) - 1, dtype=torch.int32, device=dev)
    d_sc = torch.empty((len(off) - 1, 20), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    m.score_device(d_bytes.data_ptr(), int(len(data)), d_off.data_ptr(), len(off) - 1, d_lab.data_ptr(),
                   d_sc.data_ptr(), stream)
    torch.cuda.synchronize()
    ol, os_ = oracle_c(table, 20, [1, 2, 3, 4, 5], data, off)
    assert np.array_equal(d_lab.cpu().numpy(), ol)
    assert np.array_equal(bits(d_sc.cpu().numpy()), bits(os_))


def test_host_path_chunked_pinned_and_pageable():
    """ldgpu_score pipelines chunks (64 MiB / 1M documents) over two streams:
    1.3M documents span several chunks; pageable and pinned (ldgpu_host_alloc)
    inputs and outputs give the oracle's labels and scores."""
    from languagedetection.runtime import PinnedArray
    ls = synth.make_languages(6, seed=21)
    pdata, poff, _ = synth.generate(ls, 20000, 20, 120, seed=22)
    data, off, _ = synth.tile(pdata, poff, np.zeros(20000, np.int32), 1_300_000)
    tdata, toff, tlang = synth.generate(ls, 600, 100, 400, seed=23)
    rows = list(zip([ls.names[i] for i in tlang], synth.texts(tdata, toff)))
    from languagedetection.api import LanguageDetector
    table = LanguageDetector.computeGramProbabilities(rows, [1, 2, 3], 300, ls.names)
    m = DeviceModel(table, 6, [1, 2, 3])
    ol, os_ = oracle_c(table, 6, [1, 2, 3], data, off)
    lab, sc = m.score(data, off, want_scores=True)
    assert np.array_equal(lab, ol) and np.array_equal(bits(sc), bits(os_))
    pin = PinnedArray(len(data) + 16, np.uint8)
    pin.array[:len(data)] = data
    pout = PinnedArray(len(off) - 1, np.int32)
    lab2, _ = m.score(pin.array[:len(data)], off, out=pout.array)
    assert np.array_equal(pout.array, ol)
    pin.close()
    pout.close()


def test_bench_shape_parity_sample():
    """The headline configuration's shape (L=20, grams 1-5, 256-byte docs) on a
    fit-produced table, 20k documents, against the C restatement."""
    from languagedetection.api import LanguageDetector
    ls = synth.make_languages(20)
    tdata, toff, tlang = synth.generate(ls, 2000, 200, 600, seed=synth.SEED_BASE + 100)
    rows = list(zip([ls.names[i] for i in tlang], synth.texts(tdata, toff)))
    table = LanguageDetector.computeGramProbabilities(rows, [1, 2, 3, 4, 5], 500, ls.names)
    data, off, _ = synth.generate(ls, 20000, 256, 256, seed=synth.SEED_BASE + 2)
    m = check_parity(table, 20, [1, 2, 3, 4, 5], data, off)
    assert m.info()["mode"] == 2  # every chosen gram unique to one language: count kernel


def test_config4_shape_parity_short_docs_100_langs():
    """Config 4's shape: 100 languages (two 64-lane slices), ~64-byte docs,
    grams 1-5, a fit-produced table (K=1000)."""
    from languagedetection.api import LanguageDetector
    ls = synth.make_languages(100, seed=synth.SEED_BASE + 4)
    tdata, toff, tlang = synth.generate(ls, 3000, 100, 400, seed=synth.SEED_BASE + 104)
    rows = list(zip([ls.names[i] for i in tlang], synth.texts(tdata, toff)))
    table = LanguageDetector.computeGramProbabilities(rows, [1, 2, 3, 4, 5], 1000, ls.names)
    data, off, _ = synth.generate(ls, 20000, 32, 96, seed=synth.SEED_BASE + 5)
    m = check_parity(table, 100, [1, 2, 3, 4, 5], data, off)
    assert m.info()["mode"] in (0, 2)


def test_config4_timed_kernel_labels_only_packs():
    """The kernel config 4's bench times: a GPU-fitted K=1000 table of ~100k
    rows at L=100 (every chosen gram in one presence class: count mode) whose
    keyed bloom (256 KiB) is read from L2, scored labels-only, so U[32,96]-byte
    documents go through the packs of short documents (score_pack).  The
    product library's layout flags name that path; labels equal the C
    oracle's on every document."""
    from languagedetection.runtime import DeviceCounts
    L, grams = 100, [1, 2, 3, 4, 5]
    ls = synth.make_languages(L)
    lang = np.repeat(np.arange(L, dtype=np.int32), 300)
    tdata, toff, tlang = synth.generate(ls, len(lang), 200, 2000, seed=synth.SEED_BASE + 100, doc_lang=lang)
    c = DeviceCounts(L, grams, capacity_hint=1 << 20)
    c.count(tdata, toff, tlang)
    kb, ko, masks, vals = c.fit_table_masks(1000)
    c.close()
    assert len(ko) - 1 > 64 * 1024 * 2.5 / 4  # a bloom beyond LDS
    m = DeviceModel.from_masks(kb, ko, masks, vals, L, grams)
    info = m.info()
    assert info["mode"] == 2, info
    assert "keyed_bloom_chunks" in info["layout"] and "packs" in info["layout"], info
    assert "buckets" in info["layout"], info  # 100k keys: one 64-B bucket line per verify (1.5 MiB)
    data, off, _ = synth.generate(ls, 60000, 32, 96, seed=synth.SEED_BASE + 4)
    t = OC.Table.from_masks(kb[:max(int(ko[-1]), 1)], ko, masks, vals, L)
    ol, _ = t.score(grams, data, off, want_scores=False, nthreads=8)
    lab, _ = m.score(data, off, want_scores=False)
    assert np.array_equal(lab, ol), np.nonzero(lab != ol)[0][:10]
    # the device-pointer entry point the bench calls
    import torch
    dev = torch.device("cuda", 0)
    d_bytes = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_lab = torch.empty(len(off) - 1, dtype=torch.int32, device=dev)
    m.score_device(d_bytes.data_ptr(), int(len(data)), d_off.data_ptr(), len(off) - 1, d_lab.data_ptr(), 0,
                   torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(d_lab.cpu().numpy(), ol)


def test_config5_timed_path_buckets_and_bloom_lines():
    """Config 5's exact product path: a count-mode table of more than 1.4M
    keys of >= 3 bytes at L=200, grams 1-7, so the product library puts the
    keys in 4-slot buckets AND the keyed bloom (>= 2^20 words, 4 MiB) in the
    line layout (every key of >= 4 bytes of a window position in one 64-B
    line).  Labels and fp64 scores against the C oracle, and the labels-only
    count argmax the bench times."""
    rng = np.random.default_rng(2055)
    L, grams = 200, [1, 2, 3, 4, 5, 6, 7]
    ls = synth.make_languages(L, seed=synth.SEED_BASE + 5)
    d256, o256, _ = synth.generate(ls, 5000, 256, 256, seed=synth.SEED_BASE + 506)
    dvar, ovar, _ = synth.generate(ls, 1500, 0, 400, seed=synth.SEED_BASE + 507)
    docs = [d256[o256[i]:o256[i + 1]].tobytes() for i in range(5000)]
    docs += [dvar[ovar[i]:ovar[i + 1]].tobytes() for i in range(1500)]
    data, off = encoding.pack(docs)
    keys = set()
    for n in range(1, 8):
        keys.update(_windows(data, off, n, rng, 150_000))
    while len(keys) < 1_450_000:  # misses: random keys of 3..7 bytes
        n = int(rng.integers(3, 8))
        keys.update(bytes(r) for r in rng.integers(0, 256, size=(50_000, n), dtype=np.uint8))
    keys = sorted(keys)
    kb, ko = encoding.pack(keys)
    S = (L + 63) // 64
    masks = np.zeros((len(keys), S), dtype=np.uint64)
    lang1 = rng.integers(0, L, size=len(keys))
    masks[np.arange(len(keys)), lang1 // 64] = (np.uint64(1) << (lang1 % 64).astype(np.uint64))
    multi = rng.random(len(keys)) < 0.2
    extra = rng.integers(0, L, size=len(keys))
    masks[multi, extra[multi] // 64] |= (np.uint64(1) << (extra[multi] % 64).astype(np.uint64))
    vals = np.full(len(keys), math.log(2.0))
    m = DeviceModel.from_masks(kb, ko, masks, vals, L, grams)
    info = m.info()
    assert info["mode"] == 2 and info["n_keys"] == len(keys), info
    assert "buckets" in info["layout"] and "keyed_bloom_lines" in info["layout"], info
    t = OC.Table.from_masks(kb[:max(int(ko[-1]), 1)], ko, masks, vals, L)
    ol, os_ = t.score(grams, data, off, want_scores=True, nthreads=8)
    assert (ol != 0).sum() > 1000  # hits decide the labels, not the no-hit default
    lab, sc = m.score(data, off, want_scores=True)
    assert np.array_equal(lab, ol), np.nonzero(lab != ol)[0][:10]
    assert np.array_equal(bits(sc), bits(os_))
    lab2, _ = m.score(data, off)
    assert np.array_equal(lab2, ol)


def test_failed_call_leaves_pipeline_clean(monkeypatch):
    """A host-buffer call that fails partway (an error injected after the
    first chunk, diagnostics library) drains its copies before returning; the
    next call on the same context and pipeline pool gets the oracle's labels
    and scores, with nothing of the failed call written into its buffers."""
    from languagedetection.runtime import DeviceModel as DM
    ls = synth.make_languages(5, seed=61)
    pdata, poff, _ = synth.generate(ls, 20000, 20, 120, seed=62)
    data, off, _ = synth.tile(pdata, poff, np.zeros(20000, np.int32), 2_200_000)  # 3 chunks of 1M docs
    rng = np.random.default_rng(63)
    table = _random_table(rng, 5, 300, [1, 2, 3], np.frombuffer(b"abcdefghijklmnopqrstuvwxyz ", np.uint8), True)
    m = DM(table, 5, [1, 2, 3], variant="diag")
    monkeypatch.setenv("LDGPU_FAIL_CHUNK", "2")
    with pytest.raises(_lib.LdgpuError, match="injected failure"):
        m.score(data, off, want_scores=True)
    monkeypatch.delenv("LDGPU_FAIL_CHUNK")
    small = off[:300_001]
    ol, os_ = oracle_c(table, 5, [1, 2, 3], data, small)
    lab, sc = m.score(data, small, want_scores=True)
    assert np.array_equal(lab, ol) and np.array_equal(bits(sc), bits(os_))
    lab_full, _ = m.score(data, off)
    assert np.array_equal(lab_full[:300_000], ol)


def test_config5_shape_parity_large_profile_global_filter():
    """Config 5's shape at reduced size: 200 languages (four slices), grams
    1-7, a table too large for the LDS Bloom filter (global-filter variant)."""
    rng = np.random.default_rng(55)
    L, grams = 200, [1, 2, 3, 4, 5, 6, 7]
    ls = synth.make_languages(L, seed=synth.SEED_BASE + 55)
    data, off, _ = synth.generate(ls, 3000, 256, 256, seed=synth.SEED_BASE + 56)
    raw = data.tobytes()
    # table keys: windows sampled from the documents (so hits occur) + random keys
    table = {}
    w = math.log(2.0)
    while len(table) < 120000:
        d = int(rng.integers(0, 3000))
        n = int(rng.integers(1, 8))
        p = int(rng.integers(0, 256 - n))
        key = raw[off[d] + p: off[d] + p + n]
        mask = rng.random(L) < 0.01
        mask[int(rng.integers(0, L))] = True
        k = int(mask.sum())
        table[key] = [math.log(1.0 + 1.0 / k) if b else 0.0 for b in mask]
    m = check_parity(table, L, grams, data, off)
    info = m.info()
    assert info["filter_bits"] > 64 * 1024 * 8  # bloom beyond LDS: global-filter kernel


def _windows(data, off, n, rng, count):
    """`count` random n-byte windows of the documents (table keys that hit)."""
    d = rng.integers(0, len(off) - 1, size=count)
    lens = off[d + 1] - off[d]
    ok = lens >= n
    d, lens = d[ok], lens[ok]
    p = off[d] + (rng.random(len(d)) * (lens - n + 1)).astype(np.int64)
    return [bytes(data[q:q + n]) for q in p.tolist()]


@pytest.mark.parametrize("L", [20, 100])
def test_count_mode_bucket_table_over_2pow20_keys(L):
    """Config 5's timed path: a count-mode table (every row one shared value)
    of more than 2^20 keys lives in 4-slot buckets (Bucket, ldgpu_common.h:
    bucket_place / bucket_find, secondary buckets behind overflow flags) with
    the keyed bloom in global memory.  Labels AND fp64 scores against the C
    oracle on documents of every length class."""
    rng = np.random.default_rng(1000 + L)
    ls = synth.make_languages(L, seed=synth.SEED_BASE + 500 + L)
    data, off, _ = synth.generate(ls, 6000, 0, 400, seed=synth.SEED_BASE + 501)
    keys = set()
    for n in range(1, 8):
        keys.update(_windows(data, off, n, rng, 120_000))
    while len(keys) < 1_150_000:  # misses: random keys of 3..7 bytes
        n = int(rng.integers(3, 8))
        keys.update(bytes(r) for r in rng.integers(0, 256, size=(50_000, n), dtype=np.uint8))
    keys = sorted(keys)
    kb, ko = encoding.pack(keys)
    S = (L + 63) // 64
    masks = np.zeros((len(keys), S), dtype=np.uint64)
    lang1 = rng.integers(0, L, size=len(keys))
    masks[np.arange(len(keys)), lang1 // 64] = (np.uint64(1) << (lang1 % 64).astype(np.uint64))
    multi = rng.random(len(keys)) < 0.2      # some rows name several languages (mask words read)
    extra = rng.integers(0, L, size=len(keys))
    masks[multi, extra[multi] // 64] |= (np.uint64(1) << (extra[multi] % 64).astype(np.uint64))
    vals = np.full(len(keys), math.log(2.0))
    grams = [1, 2, 3, 4, 5, 6, 7]
    m = DeviceModel.from_masks(kb, ko, masks, vals, L, grams)
    info = m.info()
    assert info["mode"] == 2 and info["n_keys"] == len(keys) > (1 << 20)
    assert info["table_slots"] < 2.5 * len(keys)          # buckets (cuckoo slots would be >= 2.5 per key)
    assert info["filter_bits"] > 64 * 1024 * 8             # keyed bloom in global memory
    t = OC.Table.from_masks(kb[:max(int(ko[-1]), 1)], ko, masks, vals, L)
    ol, os_ = t.score(grams, data, off, want_scores=True, nthreads=8)
    lab, sc = m.score(data, off, want_scores=True)
    assert np.array_equal(lab, ol), np.nonzero(lab != ol)[0][:10]
    assert np.array_equal(bits(sc), bits(os_))
    # the labels-only path (count_argmax) the bench times
    lab2, _ = m.score(data, off)
    assert np.array_equal(lab2, ol)


def test_concurrent_callers_share_one_context():
    """Spark runs several task threads per executor (Spark.scala:11 local[4]):
    4 threads call ldgpu_score on one model / context at once (ctypes drops
    the GIL) and each gets the single-thread labels and scores."""
    import threading
    from languagedetection.api import LanguageDetector
    ls = synth.make_languages(8, seed=41)
    tdata, toff, tlang = synth.generate(ls, 800, 100, 400, seed=42)
    rows = list(zip([ls.names[i] for i in tlang], synth.texts(tdata, toff)))
    table = LanguageDetector.computeGramProbabilities(rows, [1, 2, 3, 4], 300, ls.names)
    m = DeviceModel(table, 8, [1, 2, 3, 4])
    batches = [synth.generate(ls, 20000 + 5000 * i, 0, 300, seed=43 + i)[:2] for i in range(4)]
    expect = [m.score(d, o, want_scores=True) for d, o in batches]
    got = [None] * 4
    errors = []

    def run(i):
        try:
            for _ in range(3):
                got[i] = m.score(*batches[i], want_scores=True)
                assert np.array_equal(got[i][0], expect[i][0])
                assert np.array_equal(bits(got[i][1]), bits(expect[i][1]))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    ol, _ = oracle_c(table, 8, [1, 2, 3, 4], *batches[0])
    assert np.array_equal(expect[0][0], ol)


def test_product_library_ignores_env_switches(monkeypatch):
    """Diagnostics switches exist only in libldgpu_diag.so: with them set, the
    product library still takes the count path and gives the oracle's labels."""
    for k, v in (("LDGPU_ABLATE", "7"), ("LDGPU_NO_COUNT_MODE", "1"), ("LDGPU_NO_DIRECT", "1"),
                 ("LDGPU_WG_PER_CU", "1"), ("LDGPU_BLOOM_KPW", "0.05")):
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(77)
    alphabet = np.frombuffer(b"abcdefgh ", dtype=np.uint8)
    table = _random_table(rng, 20, 400, [1, 2, 3], alphabet, True, uniform=math.log(2.0))
    docs = [bytes(rng.choice(alphabet, size=int(n))) for n in rng.integers(0, 300, size=500)]
    data, off = encoding.pack(docs)
    m = check_parity(table, 20, [1, 2, 3], data, off)
    assert m.info()["mode"] == 2


@pytest.mark.parametrize("chunks,buckets", [("1", "1"), ("0", "1"), ("1", "0"), ("0", "0")])
@pytest.mark.parametrize("grams,doc_range", [
    ([1, 2, 3, 4, 5], (200, 256)),   # single documents, the fast path
    ([1, 2, 3, 4, 5], (20, 90)),     # packs of short documents
    ([3, 4, 3, 7], (0, 300)),        # partial windows, long documents, a repeated length
    ([2, 9, 12, 3], (0, 120)),       # wide keys in their chunks
])
def test_keyed_bloom_chunk_layout(chunks, buckets, grams, doc_range, monkeypatch):
    """The keyed bloom's chunk layout (count mode: every key of >= 3 bytes
    sets two bits of ONE 16-B chunk chosen by its position's first three
    bytes; config 4's 100k-key table takes it) and the word-per-key layout,
    forced through the diagnostics library (LDGPU_KB_CHUNKS), each with the
    key table in 5-slot buckets (one 64-B line per verify: the product
    layout of a keyed count-mode table beyond 2 MiB of cuckoo slots) or in
    cuckoo slots (LDGPU_BUCKETS), on a 60k-key count-mode table: labels and
    fp64 scores bit-identical to the oracle, labels-only (packs) too."""
    rng = np.random.default_rng(sum(grams) + doc_range[1] + int(chunks))
    L = 40
    ls = synth.make_languages(L, seed=93)
    data, off, _ = synth.generate(ls, 2500, doc_range[0], doc_range[1], seed=94 + len(grams))
    raw = data.tobytes()
    table = {}
    while len(table) < 60000:
        d = int(rng.integers(0, len(off) - 1))
        n = int(rng.choice(grams))
        ln = int(off[d + 1] - off[d])
        if ln < n:
            continue
        p = int(rng.integers(0, ln - n + 1))
        mask = rng.random(L) < 0.05
        mask[int(rng.integers(0, L))] = True
        table[raw[off[d] + p: off[d] + p + n]] = [math.log(2.0) if b else 0.0 for b in mask]
    monkeypatch.setenv("LDGPU_KB_CHUNKS", chunks)
    monkeypatch.setenv("LDGPU_BUCKETS", buckets)
    m = check_parity(table, L, grams, data, off, variant="diag")
    info = m.info()
    assert info["mode"] == 2 and info["filter_bits"] > 64 * 1024 * 8  # count mode, keyed (global) bloom
    assert ("keyed_bloom_chunks" in info["layout"]) == (chunks == "1"), info
    assert ("buckets" in info["layout"]) == (buckets == "1"), info
    labels, _ = m.score(data, off, want_scores=False)
    ol, _ = oracle_c(table, L, grams, data, off, scores=False)
    assert np.array_equal(labels, ol)


@pytest.mark.parametrize("form,grams,doc_range", [
    ("count", [1, 2, 3, 4, 5, 6, 7], (200, 256)),    # config-5 form: single documents
    ("count", [1, 2, 3, 4, 5], (20, 90)),             # packs of short documents
    ("mask", [2, 3, 5, 7], (0, 300)),                 # ordered replay, partial windows, long docs
    ("count", [3, 9, 12], (0, 120)),                  # wide keys in their lines
])
def test_keyed_bloom_line_layout(form, grams, doc_range, monkeypatch):
    """The keyed bloom's line layout (every key of >= 4 bytes of a window
    position in one 64-B line; the product library takes it beyond 2 MiB, as
    config 5's 16 MiB bloom): forced on a 60k-key table through the
    diagnostics library (LDGPU_KB_LINES).  Labels and fp64 scores
    bit-identical to the oracle, labels-only too; the product library's
    word-per-key layout on the same table agrees."""
    rng = np.random.default_rng(sum(grams) + doc_range[1])
    L = 40
    ls = synth.make_languages(L, seed=91)
    data, off, _ = synth.generate(ls, 2500, doc_range[0], doc_range[1], seed=92 + len(grams))
    raw = data.tobytes()
    table = {}
    while len(table) < 60000:
        d = int(rng.integers(0, len(off) - 1))
        n = int(rng.choice(grams))
        ln = int(off[d + 1] - off[d])
        if ln < n:
            continue
        p = int(rng.integers(0, ln - n + 1))
        mask = rng.random(L) < 0.05
        mask[int(rng.integers(0, L))] = True
        v = math.log(2.0) if form == "count" else math.log(1.0 + 1.0 / int(mask.sum()))
        table[raw[off[d] + p: off[d] + p + n]] = [v if b else 0.0 for b in mask]
    monkeypatch.setenv("LDGPU_KB_LINES", "1")
    m = check_parity(table, L, grams, data, off, variant="diag")
    assert m.info()["filter_bits"] > 64 * 1024 * 8  # keyed (global) bloom
    labels, _ = m.score(data, off, want_scores=False)
    ol, _ = oracle_c(table, L, grams, data, off, scores=False)
    assert np.array_equal(labels, ol)
    monkeypatch.delenv("LDGPU_KB_LINES")
    plain, _ = DeviceModel(table, L, grams).score(data, off, want_scores=False)
    assert np.array_equal(plain, ol)


def test_models_of_one_kernel_with_different_lds_sizes():
    """Two models on the same kernel instantiation (LDS bloom, count mode, one
    slice) whose dynamic LDS differs (a 64 KiB bloom against a tiny one): the
    larger model still launches after the smaller one was built, and both
    score like the oracle."""
    rng = np.random.default_rng(31)
    alphabet = np.arange(256, dtype=np.uint8)
    big = _random_table(rng, 20, 30000, [3, 4, 5], alphabet, True, uniform=0.5)
    small = _random_table(rng, 20, 50, [3, 4, 5], alphabet, True, uniform=0.5)
    data, off = encoding.pack([bytes(rng.integers(0, 256, size=int(n), dtype=np.uint8))
                               for n in rng.integers(0, 300, size=2000)])
    a = DeviceModel(big, 20, [3, 4, 5])
    la1, _ = a.score(data, off)
    b = DeviceModel(small, 20, [3, 4, 5])
    lb, _ = b.score(data, off)
    la2, _ = a.score(data, off)
    assert a.info()["mode"] == b.info()["mode"] == 2
    assert "lds_bloom" in a.info()["layout"] and "lds_bloom" in b.info()["layout"]
    assert np.array_equal(la1, la2) and np.array_equal(la1, oracle_c(big, 20, [3, 4, 5], data, off, scores=False)[0])
    assert np.array_equal(lb, oracle_c(small, 20, [3, 4, 5], data, off, scores=False)[0])
