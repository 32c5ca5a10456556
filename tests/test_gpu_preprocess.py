"""GPU parity of the preprocessors: ldgpu_preprocess
(csrc/ldgpu_pre.hip) against the host restatement in preprocessing.py --
LowerCasePreprocessor.scala:44-76 (String.toLowerCase(Locale.forLanguageTag
(lang)), java_lower) and SpecialCharPreprocessor.scala:40-70's documented
intent (intended_special_char_clean).  Parity with the JVM itself is unpinned
(no JVM in this image): the host restatement is the checker."""
import numpy as np
import pandas as pd
import pytest

from languagedetection import LowerCasePreprocessor, encoding
from languagedetection.preprocessing import (_casemap, intended_special_char_clean, java_lower,
                                             preprocess_device)

pytestmark = pytest.mark.gpu

DOTTED_I = "\N{LATIN CAPITAL LETTER I WITH DOT ABOVE}"
DOT_ABOVE = "\N{COMBINING DOT ABOVE}"
SIGMA = "\N{GREEK CAPITAL LETTER SIGMA}"

# the committed cases of tests/test_preprocessing.py and more, with their labels
CASES = [
    ("Hallo WELT", "de"), ("THIS Is", "en"), ("ABC", "en"), ("ISTANBUL " + DOTTED_I + "zmir", "tr"),
    ("I" + DOT_ABOVE, "tr"), (DOTTED_I, "az"), ("ISTANBUL", "en"), (DOTTED_I, "en"),
    ("\N{LATIN CAPITAL LETTER I WITH GRAVE}", "lt"), ("I\N{COMBINING ACUTE ACCENT}", "lt"), ("IJ", "lt"),
    ("\N{GREEK CAPITAL LETTER OMICRON}" + SIGMA + " " + SIGMA, "el"), ("I", "tr-TR"), ("I", "?"),
    ("", "en"), ("a <b>  c", "en"), ("a<b>[c]  d e", "fr"), ("Ünïcödé ÀÉÎÕÜ", "fr"),
    ("\N{DESERET CAPITAL LETTER LONG I}x", "en"), ("ÇAĞRI", "tr"), ("ÇAĞRI", "en"), ("ПРИВЕТ Мир", "ru"),
    ("x" * 200 + "ÀB/C_D" * 40, "en"), ("\ud800 lone", "en"),
]


def _random_texts(rng, n):
    alphabet = list("abcXYZ ÄÖÜßÉÈ/_[]*()%^&@$#:|{}<>~`\"\\ΑΒΓσΣДЖЯiIİı\u0307\u0301") + [DOTTED_I, SIGMA]
    langs = ["en", "de", "tr", "az", "lt", "el", "ru", "tr-TR", "x"]
    texts = ["".join(rng.choice(alphabet, size=int(k))) for k in rng.integers(0, 300, size=n)]
    return texts, [langs[int(i)] for i in rng.integers(0, len(langs), size=n)]


@pytest.mark.parametrize("lower,clean", [(True, False), (False, True), (True, True)])
def test_preprocess_matches_host_restatement(lower, clean):
    rng = np.random.default_rng(int(lower) * 2 + int(clean))
    texts, langs = _random_texts(rng, 3000)
    texts += [t for t, _ in CASES]
    langs += [l for _, l in CASES]

    def host(t, l):
        t = java_lower(t, l) if lower else t
        return intended_special_char_clean(t) if clean else t

    want = [host(t, l) for t, l in zip(texts, langs)]
    assert preprocess_device(texts, langs, lower=lower, clean=clean) == want
    data, off = preprocess_device(texts, langs, lower=lower, clean=clean, score_encoding=True)
    wd, wo = encoding.pack([encoding.score_bytes(w) for w in want])
    assert np.array_equal(off, wo) and data[:int(off[-1])].tobytes() == wd[:int(wo[-1])].tobytes()


def test_device_leaves_only_context_dependent_documents_to_the_host():
    """Plain text never goes back to the host; the documented special cases
    always do (their device output is empty)."""
    m = _casemap(0)
    from languagedetection.runtime import DeviceCaseMap, locale_class
    texts = ["Hello World", "ISTANBUL", "Ünïcödé", DOTTED_I, "Ο" + SIGMA, "I" + DOT_ABOVE, "I\u0301", "ÌX",
             "\N{DESERET CAPITAL LETTER LONG I}", "ÇAĞRI"]
    langs = ["en", "tr", "fr", "en", "el", "tr", "lt", "lt", "en", "tr"]
    units, off = DeviceCaseMap.pack_units(texts)
    loc = np.array([locale_class(l) for l in langs], dtype=np.uint8)
    out, out_off, host = m.run(units, off, loc, 1)
    assert host.tolist() == [0, 0, 0, 1, 1, 1, 1, 1, 1, 0]
    assert out[out_off[1]:out_off[2]].tobytes().decode("utf-16-le") == "\N{LATIN SMALL LETTER DOTLESS I}stanbul"
    assert out_off[4] == out_off[3]   # a host document's output is empty


def test_lowercase_preprocessor_on_device():
    df = pd.DataFrame({"fulltext": [t for t, _ in CASES], "lang": [l for _, l in CASES], "id": range(len(CASES))})
    a = LowerCasePreprocessor().transform(df)
    b = LowerCasePreprocessor(device=0).transform(df)
    assert list(b.columns) == ["lang", "id", "fulltext"]
    assert list(a["fulltext"]) == list(b["fulltext"])


def test_preprocess_then_score_on_device():
    """The fused path: lower-cased, cleaned SCORE bytes straight from the
    device pass into the scoring kernel -- labels equal to host
    preprocessing + host packing."""
    from languagedetection.runtime import DeviceModel
    rng = np.random.default_rng(3)
    texts, langs = _random_texts(rng, 2000)
    table = {b"ab": [0.5, 0.0], b"x": [0.0, 0.25], b"\xe4": [0.0, 1.0], b"\xdf": [0.75, 0.0], b"i": [0.1, 0.1]}
    m = DeviceModel(table, 2, [1, 2])
    d1, o1 = preprocess_device(texts, langs, lower=True, clean=True, score_encoding=True)
    d2, o2 = encoding.pack_score([intended_special_char_clean(java_lower(t, l)) for t, l in zip(texts, langs)])
    l1, _ = m.score(d1, o1)
    l2, _ = m.score(d2, o2)
    assert np.array_equal(l1, l2)
