"""Generates the committed golden fixtures of tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

reference_kats.json -- the reference's own known-answer tests, transcribed as
                       data (inputs + expected outcomes), with file:line.
score_cases.json    -- one case per SCORE rule of SURVEY.md §8a/§8c, expected
                       labels and bit-exact scores (float.hex) from the oracle.
fit_cases.json      -- FIT counts, probability rows and the deterministic
                       top-K table for small corpora, from the oracle.
"""
from __future__ import annotations

import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import ldoracle as O  # noqa: E402

KAT_DOCS = [
    "Dies ist ein deutscher Text, das ist ja sehr schön",
    "Dies ist ein andere deutscher Text, und der ist auch sehr schön",
    "This is a text in english, and that is very nice",
    "This is another text in english and that is also nice",
]


def reference_kats():
    return {
        "score_kat": {
            "source": "LanguageDetectorModelSpecs.scala:15-44",
            "languages": ["de", "en"],
            "gram_lengths": [3],
            "table": {"Die": [1.0, 0.0], "Thi": [0.0, 1.0]},
            "docs": KAT_DOCS,
            "expect_count": {"de": 2, "en": 2},
            "expect_rows": 4,
        },
        "fit_kat": {
            "source": "LanguageDetectorSpecs.scala:15-40",
            "languages": ["de", "en"],
            "gram_lengths": [3],
            "profile_size": 5,
            "rows": [["de", KAT_DOCS[0]], ["de", KAT_DOCS[1]], ["en", KAT_DOCS[2]], ["en", KAT_DOCS[3]]],
            "expect_table_size": 10,
            "expect_row_length": 2,
        },
        "validation_kat": {
            "source": "LanguageDetectorSpecs.scala:43-66 (expects the 'No training examples' message; the code "
                      "order of LanguageDetector.scala:221-238 raises the unsupported-label message first -- "
                      "the build follows the code, SURVEY.md fact 8)",
            "languages": ["de", "en"],
            "gram_lengths": [3],
            "profile_size": 5,
            "rows": [["de", KAT_DOCS[0]], ["de", KAT_DOCS[1]], ["es", "Habla espanol"],
                     ["es", "Donde est la bibliotheka"]],
            "reference_test_expects": "No training examples found for language en. Provide examples for each "
                                      "language",
            "code_order_raises": "Input data contians es, but it is not in the list of supported languages",
        },
    }


def enc_table(table):
    return [[k.hex(), [float(v).hex() for v in row]] for k, row in table.items()]


def score_case(name, rule, table, langs, grams, docs_bytes):
    L = len(langs)
    scores = [O.detect_scores(d, table, L, grams) for d in docs_bytes]
    labels = [O.argmax_first(s) for s in scores]
    return {
        "name": name, "rule": rule, "languages": langs, "gram_lengths": grams,
        "table": enc_table(table),
        "docs_hex": [d.hex() for d in docs_bytes],
        "labels": labels,
        "scores": [[v.hex() for v in s] for s in scores],
    }


def score_cases():
    cases = []
    t3 = {b"abc": [1.0, 0.0, 0.0], b"bcd": [0.0, 2.0, 0.0], b"ab": [0.0, 0.0, 5.0], b"a": [0.25, 0.5, 0.0]}
    L3 = ["x", "y", "z"]
    # (b) short docs: len 0, 1, n-1, n, n+1 -- partial windows (fact 3)
    cases.append(score_case("short_docs", "sliding partial windows, LanguageDetectorModel.scala:143", t3, L3, [3],
                            [b"", b"a", b"ab", b"abc", b"abcd", b"b"]))
    cases.append(score_case("short_docs_multi_n", "partial windows across n", t3, L3, [1, 2, 3],
                            [b"", b"a", b"ab", b"abc", b"xabcd"]))
    # (d) all-miss -> label 0 ; (e) exact tie -> lowest index (fact 6)
    tie = {b"q": [1.0, 1.0, 0.0], b"r": [0.0, 1.0, 1.0]}
    cases.append(score_case("miss_and_tie", "breeze argmax first max, LanguageDetectorModel.scala:154", tie, L3,
                            [1], [b"zzz", b"q", b"r", b"qr", b"rr", b""]))
    # (f) duplicate n in G
    cases.append(score_case("duplicate_grams", "gramLengths order with repeats, :139", t3, L3, [3, 1, 3],
                            [b"abcabc", b"aaa", b"bcd"]))
    # (g) user table with negative / odd values (dense path), fp64 order
    odd = {b"ab": [0.1, -0.2, 1e-300], b"ba": [0.7, 0.3, -1e300], b"aa": [1.0 / 3.0, 2.0 / 3.0, 1e300],
           b"b": [-0.0, 0.0, 5e-324]}
    cases.append(score_case("dense_odd_values", "arbitrary fp64 rows, left fold :148-149", odd, L3, [2, 1],
                            [b"abab", b"aabbaa", b"ba" * 40, b"b", bytes(range(97, 99)) * 100]))
    # (c) non-ASCII: score encoding is the low byte of each UTF-16 unit (fact 2)
    na_table = {O.score_encode("ö"): [1.0, 0.0], O.fit_encode("ö")[:1]: [0.0, 1.0],
                O.score_encode("日"): [0.0, 3.0], O.score_encode("\U0001F600")[:2]: [2.0, 0.0]}
    na_docs = ["schön", "日本", "😀 smile", "\ud800 lone", "plain"]
    cases.append(score_case("non_ascii_low_byte", "text.toCharArray.map(_.toByte), :161", na_table, ["a", "b"],
                            [1, 2], [O.score_encode(t) for t in na_docs]))
    cases[-1]["docs_text"] = na_docs
    # mask-form (fit-like) table with many languages (> 64: two slices)
    L = 70
    langs = [f"l{i:02d}" for i in range(L)]
    mt = {}
    for i, g in enumerate([b"th", b"he", b"e ", b" t", b"in", b"an", b"nd", b"d "]):
        bits = [(j * 7 + i * 3) % 5 == 0 for j in range(L)]
        k = sum(bits)
        mt[g] = [math.log(1.0 + 1.0 / k) if b else 0.0 for b in bits]
    cases.append(score_case("mask_form_70_langs", "fit-produced rows, L > 64", mt, langs, [2],
                            [b"the end and then", b"in an", b"", b"dd d"]))
    return cases


def fit_case(name, rows, langs, grams, k):
    grams_out = O.compute_grams(rows, grams)
    reduced = O.reduce_grams(grams_out, langs)
    probs = O.compute_probabilities(reduced, langs)
    table = O.filter_top_grams(probs, langs, k)
    counts = {}
    for (lang, g), c in reduced.items():
        counts.setdefault(g.hex(), {})[lang] = c
    return {
        "name": name, "languages": langs, "gram_lengths": grams, "profile_size": k,
        "rows": [[l, t] for l, t in rows],
        "counts": counts,
        "probabilities": enc_table(probs),
        "table": enc_table(table),
    }


def fit_cases():
    kat = reference_kats()["fit_kat"]
    out = [fit_case("reference_fit_kat", [tuple(r) for r in kat["rows"]], kat["languages"], kat["gram_lengths"],
                    kat["profile_size"])]
    rows = [("en", "the cat"), ("en", "a"), ("de", "der hund"), ("de", ""), ("fr", "le chat ö"),
            ("fr", "ab"), ("en", "😀 x \ud800")]
    out.append(fit_case("edge_rows", rows, ["en", "de", "fr"], [1, 2, 3], 4))
    out.append(fit_case("duplicate_grams", [("a", "abab"), ("b", "baba"), ("a", "b")], ["a", "b"], [2, 2, 1], 3))
    out.append(fit_case("short_profile", [("a", "xyz"), ("b", "xy")], ["a", "b"], [3], 10))
    return out


def main():
    def dump(name, obj):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1, ensure_ascii=True)
            f.write("\n")
    dump("reference_kats.json", reference_kats())
    dump("score_cases.json", score_cases())
    dump("fit_cases.json", fit_cases())


if __name__ == "__main__":
    main()
