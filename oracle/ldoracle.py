"""CPU oracle for the spark-languagedetector hot path -- TEST INFRASTRUCTURE ONLY.

This module is a rule-by-rule restatement of the reference's FIT and SCORE
algorithms in plain Python.  It is the *checker* for the HIP path in
``libldgpu.so``: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it.  The product path never
routes through it (``languagedetection`` fails loudly without its HIP library).

Reference (read-only, Scala 2.11 / Spark 2.2, cannot run in this container --
no JVM; see DESIGN.md "Oracle pinning"):
  LanguageDetector.scala       -- computeGrams :25-46, reduceGrams :52-66,
                                  computeProbabilities :75-92,
                                  filterTopGrams :100-132, fit :210-264
  LanguageDetectorModel.scala  -- detect(Array[Byte]) :131-156,
                                  detect(String) :158-165, transform :219-240

Pinning.  The oracle is pinned by the reference's own known-answer tests
(``tests/golden/reference_kats.json``):
  * LanguageDetectorModelSpecs.scala:15-44 -- scoring KAT (labels de,de,en,en)
  * LanguageDetectorSpecs.scala:15-40      -- fit KAT (10 rows of length 2)
Rules that no reference test pins (partial windows, UTF-8 vs low-byte
encoding, argmax tie-break, no-hit default, top-K tie choice, count values)
are restated from the cited source lines; DESIGN.md lists them as
"parity unpinned by a reference test".

Third-party semantics restated here (no source in the container):
  * Scala 2.11 ``sliding(n)`` (GroupedIterator, partial=true): len 0 -> no
    window; 0 < len < n -> one window holding the whole sequence;
    otherwise len-n+1 full windows; n <= 0 -> IllegalArgumentException.
  * ``String.getBytes(UTF-8)`` (Java 8): unpaired surrogates -> b'?'.
  * ``Char.toByte``: low 8 bits of each UTF-16 code unit.
  * netlib-java F2J ``daxpy`` with a=1.0: y[i] = y[i] + x[i], exact fp64.
  * breeze 0.13 ``argmax``: first element taken, then strict ``>`` updates
    (lowest index wins ties; NaN never displaces; empty -> exception).
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Sequence, Tuple

Table = Dict[bytes, List[float]]


# ----------------------------------------------------------------------------
# Encodings (LanguageDetector.scala:37, LanguageDetectorModel.scala:161)
# ----------------------------------------------------------------------------
def java_utf16_units(text: str) -> List[int]:
    """The UTF-16 code units of a Java String equal to ``text``.

    Python strings may hold lone surrogates (surrogatepass); astral code
    points become surrogate pairs exactly as in a Java String.
    """
    b = text.encode("utf-16-le", "surrogatepass")
    return [b[i] | (b[i + 1] << 8) for i in range(0, len(b), 2)]


def fit_encode(text: str) -> bytes:
    """``text.getBytes(Charset.forName("UTF-8"))`` (LanguageDetector.scala:37).

    Java's UTF-8 encoder replaces each unpaired surrogate unit by the
    replacement byte '?' (0x3F).
    """
    units = java_utf16_units(text)
    out = bytearray()
    i = 0
    while i < len(units):
        u = units[i]
        if 0xD800 <= u <= 0xDBFF and i + 1 < len(units) and 0xDC00 <= units[i + 1] <= 0xDFFF:
            cp = 0x10000 + ((u - 0xD800) << 10) + (units[i + 1] - 0xDC00)
            out += chr(cp).encode("utf-8")
            i += 2
        elif 0xD800 <= u <= 0xDFFF:
            out += b"?"
            i += 1
        else:
            out += chr(u).encode("utf-8")
            i += 1
    return bytes(out)


def score_encode(text: str) -> bytes:
    """``text.toCharArray.map(_.toByte)`` (LanguageDetectorModel.scala:161)."""
    return bytes(u & 0xFF for u in java_utf16_units(text))


# ----------------------------------------------------------------------------
# Scala sliding (LanguageDetector.scala:39, LanguageDetectorModel.scala:143)
# ----------------------------------------------------------------------------
def sliding(seq: bytes, n: int) -> List[bytes]:
    if n <= 0:
        raise ValueError(f"requirement failed: size={n} and step=1, but both must be positive")
    ln = len(seq)
    if ln == 0:
        return []
    if ln < n:
        return [bytes(seq)]
    return [bytes(seq[i:i + n]) for i in range(ln - n + 1)]


def n_windows(ln: int, n: int) -> int:
    return 0 if ln == 0 else (1 if ln < n else ln - n + 1)


def int32_wrap(x: int) -> int:
    """JVM ``Int`` arithmetic (reduceGroups sums Ints, LanguageDetector.scala:62)."""
    return ((x + 2 ** 31) % 2 ** 32) - 2 ** 31


# ----------------------------------------------------------------------------
# FIT
# ----------------------------------------------------------------------------
def compute_grams(rows: Iterable[Tuple[str, str]], gram_lengths: Sequence[int]):
    """computeGrams (LanguageDetector.scala:25-46): per row, per n in order
    (duplicates included), count the distinct windows of the UTF-8 bytes."""
    out = []
    for lang, text in rows:
        bs = fit_encode(text)  # NPE on null text in the reference
        for n in gram_lengths:
            counts: Dict[bytes, int] = {}
            for w in sliding(bs, n):
                counts[w] = counts.get(w, 0) + 1
            for g, c in counts.items():
                out.append((lang, g, c))
    return out


def reduce_grams(grams, supported_languages: Sequence[str]) -> Dict[Tuple[str, bytes], int]:
    """reduceGrams (LanguageDetector.scala:52-66): per supported language,
    group by gram and sum the Int counts (JVM wrap-around)."""
    sup = set(supported_languages)
    acc: Dict[Tuple[str, bytes], int] = {}
    for lang, g, c in grams:
        if lang not in sup:
            continue
        acc[(lang, g)] = int32_wrap(acc.get((lang, g), 0) + c)
    return acc


def compute_probabilities(reduced: Dict[Tuple[str, bytes], int],
                          supported_languages: Sequence[str]) -> Table:
    """computeProbabilities (LanguageDetector.scala:75-92).

    Per gram: p_l = (#rows of the gram with lang l) / (#rows of the gram),
    v_l = Math.log(1.0 + p_l).  Counts are never read.
    """
    langs_of: Dict[bytes, List[str]] = {}
    for (lang, g) in reduced:
        langs_of.setdefault(g, []).append(lang)
    table: Table = {}
    for g, ls in langs_of.items():
        size = float(len(ls))
        table[g] = [math.log(1.0 + float(ls.count(l)) / size) for l in supported_languages]
    return table


def key_order(g: bytes):
    """The build's deterministic tie-break among equal values: ascending
    (length, unsigned bytes).  The reference's order among ties is Spark
    shuffle order (LanguageDetector.scala:113-119) -- a stated divergence."""
    return (len(g), g)


def filter_top_grams(probs: Table, supported_languages: Sequence[str], k: int) -> Table:
    """filterTopGrams (LanguageDetector.scala:100-132) with the deterministic
    tie-break of ``key_order``: per language i sort ALL grams by v_i
    descending, take K; union; keep the table rows of the chosen grams."""
    chosen = set()
    keys = sorted(probs, key=key_order)
    for i in range(len(supported_languages)):
        # stable sort by value desc over key-ordered input == (-v, key) order
        ranked = sorted(keys, key=lambda g: -probs[g][i])
        chosen.update(ranked[:max(k, 0)])
    return {g: probs[g] for g in chosen}


def topk_contract_violations(table: Table, probs: Table, supported_languages: Sequence[str],
                             k: int) -> List[str]:
    """The valid-outcome contract any reference run satisfies:
    rows are the probability rows; for every language i every gram with
    v_i above the K-th value is kept; every kept gram is >= the K-th value in
    some language; |table| <= L*K."""
    errs = []
    for g, row in table.items():
        if g not in probs:
            errs.append(f"gram {g!r} not in probability table")
        elif list(row) != list(probs[g]):
            errs.append(f"row of {g!r} differs")
    L = len(supported_languages)
    kth = []
    for i in range(L):
        vals = sorted((r[i] for r in probs.values()), reverse=True)
        kth.append(vals[min(k, len(vals)) - 1] if vals and k > 0 else math.inf)
        for g, r in probs.items():
            if k > 0 and r[i] > kth[i] and g not in table:
                errs.append(f"lang {i}: gram {g!r} above the K-th value missing")
    for g in table:
        if g in probs and not any(probs[g][i] >= kth[i] for i in range(L)):
            errs.append(f"gram {g!r} below the K-th value in every language")
    if len(table) > L * max(k, 0):
        errs.append("table larger than L*K")
    return errs


class FitValidationError(Exception):
    """java.lang.Exception thrown by LanguageDetector.fit validation."""


def validate_fit(rows: Sequence[Tuple[str, str]], supported_languages: Sequence[str]) -> None:
    """LanguageDetector.scala:221-238, in code order: unsupported label first
    (message typo 'contians' preserved), then per-language emptiness."""
    seen = []
    for lang, _ in rows:
        if lang not in seen:
            seen.append(lang)
    for lang in seen:
        if lang not in supported_languages:
            raise FitValidationError(
                f"Input data contians {lang}, but it is not in the list of supported languages")
    for lang in supported_languages:
        if not any(l == lang for l, _ in rows):
            raise FitValidationError(
                f"No training examples found for language {lang}. Provide examples for each language")


def fit(rows: Sequence[Tuple[str, str]], supported_languages: Sequence[str],
        gram_lengths: Sequence[int], k: int) -> Table:
    """LanguageDetector.fit (LanguageDetector.scala:210-264) -> the model table."""
    validate_fit(rows, supported_languages)
    probs = fit_probabilities(rows, supported_languages, gram_lengths)
    return filter_top_grams(probs, supported_languages, k)


def fit_probabilities(rows, supported_languages, gram_lengths) -> Table:
    reduced = reduce_grams(compute_grams(rows, gram_lengths), supported_languages)
    return compute_probabilities(reduced, supported_languages)


# ----------------------------------------------------------------------------
# SCORE
# ----------------------------------------------------------------------------
def argmax_first(values: Sequence[float]) -> int:
    """breeze argmax (LanguageDetectorModel.scala:154): first element, then
    strictly-greater updates."""
    if len(values) == 0:
        raise ValueError("No values in array")
    best, bi = values[0], 0
    for i in range(1, len(values)):
        if values[i] > best:
            best, bi = values[i], i
    return bi


def detect_scores(text: bytes, table: Table, n_langs: int,
                  gram_lengths: Sequence[int]) -> List[float]:
    """detect(Array[Byte], ...) accumulation (LanguageDetectorModel.scala:137-152):
    left fold in (n in gramLengths order, window position) order."""
    s = [0.0] * n_langs
    for n in gram_lengths:
        for w in sliding(text, n):
            row = table.get(w)
            if row is None:
                continue
            if len(row) != n_langs:  # BLAS.axpy require(x.size == y.size)
                raise ValueError("requirement failed: BLAS.axpy size mismatch")
            for l in range(n_langs):
                s[l] = s[l] + 1.0 * row[l]
    return s


def detect_index(text: bytes, table: Table, n_langs: int, gram_lengths: Sequence[int]) -> int:
    return argmax_first(detect_scores(text, table, n_langs, gram_lengths))


def detect_bytes(text: bytes, table: Table, supported_languages: Sequence[str],
                 gram_lengths: Sequence[int]) -> str:
    """LanguageDetectorModel.detect(Array[Byte], ...) (:131-156)."""
    return supported_languages[detect_index(text, table, len(supported_languages), gram_lengths)]


def detect(text: str, table: Table, supported_languages: Sequence[str],
           gram_lengths: Sequence[int]) -> str:
    """LanguageDetectorModel.detect(String, ...) (:158-165): low-byte encoding."""
    if text is None:
        raise TypeError("NullPointerException: text is null")
    return detect_bytes(score_encode(text), table, supported_languages, gram_lengths)


def transform(texts: Sequence[str], table: Table, supported_languages: Sequence[str],
              gram_lengths: Sequence[int]) -> List[str]:
    """The per-row map of LanguageDetectorModel.transform (:219-240)."""
    return [detect(t, table, supported_languages, gram_lengths) for t in texts]
