"""CPU: the oracle against the reference's own KATs and the committed golden
vectors; the C restatement against the Python restatement."""
import json
import math
import os

import numpy as np
import pytest

import ldoracle as O
import ldoracle_c as OC

from conftest import GOLDEN


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def dec_table(enc):
    return {bytes.fromhex(k): [float.fromhex(v) for v in row] for k, row in enc}


# ------------------------------------------------------------ reference KATs
def test_reference_score_kat():
    """LanguageDetectorModelSpecs.scala:15-44."""
    k = load("reference_kats.json")["score_kat"]
    table = {g.encode("utf-8"): r for g, r in k["table"].items()}
    labels = O.transform(k["docs"], table, k["languages"], k["gram_lengths"])
    assert len(labels) == k["expect_rows"]
    for lang, n in k["expect_count"].items():
        assert labels.count(lang) == n
    assert labels == ["de", "de", "en", "en"]


def test_reference_fit_kat():
    """LanguageDetectorSpecs.scala:15-40: 10 rows of length 2."""
    k = load("reference_kats.json")["fit_kat"]
    table = O.fit([tuple(r) for r in k["rows"]], k["languages"], k["gram_lengths"], k["profile_size"])
    assert len(table) == k["expect_table_size"]
    assert all(len(r) == k["expect_row_length"] for r in table.values())
    probs = O.fit_probabilities([tuple(r) for r in k["rows"]], k["languages"], k["gram_lengths"])
    assert O.topk_contract_violations(table, probs, k["languages"], k["profile_size"]) == []


def test_reference_validation_order():
    """LanguageDetector.scala:221-238 (code order)."""
    k = load("reference_kats.json")["validation_kat"]
    with pytest.raises(O.FitValidationError) as e:
        O.fit([tuple(r) for r in k["rows"]], k["languages"], k["gram_lengths"], k["profile_size"])
    assert str(e.value) == k["code_order_raises"]
    with pytest.raises(O.FitValidationError) as e:
        O.fit([("de", "x")], ["de", "en"], [3], 5)
    assert str(e.value) == k["reference_test_expects"]


# ----------------------------------------------------------- golden vectors
@pytest.mark.parametrize("case", load("score_cases.json"), ids=lambda c: c["name"])
def test_golden_score(case):
    table = dec_table(case["table"])
    L = len(case["languages"])
    for i, dh in enumerate(case["docs_hex"]):
        d = bytes.fromhex(dh)
        s = O.detect_scores(d, table, L, case["gram_lengths"])
        assert [v.hex() for v in s] == case["scores"][i]
        assert O.argmax_first(s) == case["labels"][i]
    if "docs_text" in case:
        assert [O.score_encode(t).hex() for t in case["docs_text"]] == case["docs_hex"]


@pytest.mark.parametrize("case", load("fit_cases.json"), ids=lambda c: c["name"])
def test_golden_fit(case):
    rows = [tuple(r) for r in case["rows"]]
    reduced = O.reduce_grams(O.compute_grams(rows, case["gram_lengths"]), case["languages"])
    counts = {}
    for (lang, g), c in reduced.items():
        counts.setdefault(g.hex(), {})[lang] = c
    assert counts == case["counts"]
    probs = O.compute_probabilities(reduced, case["languages"])
    assert probs == dec_table(case["probabilities"])
    table = O.filter_top_grams(probs, case["languages"], case["profile_size"])
    assert table == dec_table(case["table"])
    assert O.topk_contract_violations(table, probs, case["languages"], case["profile_size"]) == []


# ---------------------------------------------------------------- rules
def test_sliding_partial_rule():
    assert O.sliding(b"", 3) == []
    assert O.sliding(b"ab", 3) == [b"ab"]
    assert O.sliding(b"abc", 3) == [b"abc"]
    assert O.sliding(b"abcd", 3) == [b"abc", b"bcd"]
    with pytest.raises(ValueError):
        O.sliding(b"abc", 0)


def test_encodings():
    assert O.fit_encode("ö") == b"\xc3\xb6"
    assert O.score_encode("ö") == b"\xf6"
    assert O.fit_encode("\ud800x") == b"?x"                      # lone surrogate -> '?'
    assert O.fit_encode("😀") == "😀".encode("utf-8")  # pair as 2 code points
    assert O.score_encode("😀") == b"\x3d\x00"                  # D83D DE00 low bytes
    assert O.score_encode("日") == b"\xe5"


def test_argmax_rule():
    assert O.argmax_first([0.0, 0.0]) == 0
    assert O.argmax_first([1.0, 2.0, 2.0]) == 1
    assert O.argmax_first([math.nan, 5.0]) == 0
    assert O.argmax_first([1.0, math.nan, 3.0]) == 2
    assert O.argmax_first([-0.0, 0.0]) == 0


def test_int32_wrap():
    assert O.int32_wrap(2 ** 31) == -2 ** 31
    assert O.int32_wrap(5) == 5


# --------------------------------------------- C restatement == Python one
def _rand_case(rng, L, n_keys, grams, n_docs, max_len, alphabet=b"abcde "):
    table = {}
    for _ in range(n_keys):
        n = int(rng.integers(1, max(grams) + 1))
        k = bytes(rng.choice(list(alphabet), size=n))
        table[k] = [float(x) for x in rng.normal(size=L)]
    docs = [bytes(rng.choice(list(alphabet), size=int(rng.integers(0, max_len + 1)))) for _ in range(n_docs)]
    return table, docs


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_c_oracle_matches_python_score(seed):
    rng = np.random.default_rng(seed)
    L = [3, 20, 70][seed]
    grams = [[3], [1, 2, 3], [2, 5, 2]][seed]
    table, docs = _rand_case(rng, L, 60, grams, 80, 40)
    data = np.frombuffer(b"".join(docs) + b"\0", dtype=np.uint8)
    off = np.zeros(len(docs) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(d) for d in docs])
    t = OC.Table(table, L)
    labels, scores = t.score(grams, data, off, want_scores=True, nthreads=2)
    for i, d in enumerate(docs):
        s = O.detect_scores(d, table, L, grams)
        assert scores[i].tolist() == s
        assert labels[i] == O.argmax_first(s)


def test_c_oracle_matches_python_count():
    rng = np.random.default_rng(7)
    langs = ["a", "b", "c"]
    rows = [(langs[int(rng.integers(0, 3))], bytes(rng.choice(list(b"xyz ab"), size=int(rng.integers(0, 30))))
             .decode()) for _ in range(100)]
    grams = [1, 3, 2, 3]
    reduced = O.reduce_grams(O.compute_grams(rows, grams), langs)
    data = np.frombuffer("".join(t for _, t in rows).encode() + b"\0", dtype=np.uint8)
    off = np.zeros(len(rows) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(t) for _, t in rows])
    keys, cnt = OC.count(data, off, np.array([langs.index(l) for l, _ in rows], dtype=np.int32), 3, grams)
    got = {(langs[l], k): int(cnt[i, l]) for i, k in enumerate(keys) for l in range(3) if cnt[i, l]}
    assert got == reduced
    assert keys == sorted(keys, key=O.key_order)


def test_c_oracle_mask_form_equals_dense_rows():
    """OC.Table.from_masks (ldo_table_create_masks) scores exactly as the
    dense table it stands for (used for tables too large for dense rows)."""
    import numpy as np
    rng = np.random.default_rng(8)
    L = 70
    keys = sorted({bytes(rng.integers(97, 100, size=int(rng.integers(1, 5)), dtype=np.uint8)) for _ in range(300)})
    masks = rng.integers(0, 2**63, size=(len(keys), 2), dtype=np.uint64)
    masks[:, 1] &= np.uint64((1 << 6) - 1)
    vals = rng.normal(size=len(keys))
    dense = {k: [float(vals[i]) if (int(masks[i, l // 64]) >> (l % 64)) & 1 else 0.0 for l in range(L)]
             for i, k in enumerate(keys)}
    off = np.zeros(len(keys) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(k) for k in keys])
    kb = np.frombuffer(b"".join(keys), dtype=np.uint8)
    docs = [bytes(rng.integers(97, 100, size=int(n), dtype=np.uint8)) for n in rng.integers(0, 60, size=200)]
    doff = np.zeros(len(docs) + 1, dtype=np.int64)
    doff[1:] = np.cumsum([len(d) for d in docs])
    dd = np.frombuffer(b"".join(docs) + b"\0", dtype=np.uint8)
    l1, s1 = OC.Table(dense, L).score([1, 2, 3], dd, doff, want_scores=True)
    l2, s2 = OC.Table.from_masks(kb, off, masks, vals, L).score([1, 2, 3], dd, doff, want_scores=True)
    assert np.array_equal(l1, l2) and np.array_equal(s1.view(np.uint64), s2.view(np.uint64))


def test_c_restatement_under_address_and_ub_sanitizers():
    """SURVEY §5 (race detection / sanitizers): the C restatement built with
    -fsanitize=address,undefined (make -C oracle asan) runs every entry point
    on random corpora with the rules' edge cases; any out-of-bounds access,
    leak or undefined behaviour aborts it."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle"), "asan"], check=True, timeout=240)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(root, "oracle", "build", "asan_check")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "clean" in r.stdout
