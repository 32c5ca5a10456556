"""Caller-side text preprocessors, over pandas DataFrames.

Reference (org.apache.spark.ml.feature.languagedetection.preprocessing):
  LowerCasePreprocessor    LowerCasePreprocessor.scala:19-76
  SpecialCharPreprocessor  SpecialCharPreprocessor.scala:19-70

Both are host-side Transformers a user runs before ``fit``/``transform``.
Given ``device=``, LowerCasePreprocessor lower-cases on the GPU
(ldgpu_preprocess, ``csrc/ldgpu_pre.hip``): each UTF-16 unit through the 1:1
mapping of ``str.lower``, the tr/az rules that stay 1:1 on the device, and
the documents whose lower-casing is not 1:1 or needs context (U+0130 outside
tr/az, capital sigma, the lt rules, tr/az "I" + U+0307, cased supplementary
characters) redone here by ``java_lower``.  ``preprocess_device`` also
applies the documented SpecialChar cleanup and can emit the SCORE encoding
packed for the scoring kernels.  Their behaviour is reproduced as written,
including the reference's quirks:

* ``setInputCol`` sets ``outputCol`` (LowerCase :32, SpecialChar :30): the
  transformed column is read from, and written back to, ``outputCol``
  (default "fulltext").
* The transformed column is dropped and re-appended as the LAST column
  (``transformSchema`` :38-42 / :34-38 and the row rebuild :63-71 / :59-67).
* LowerCasePreprocessor lower-cases with the row's label as the locale
  (``text.toLowerCase(Locale.forLanguageTag(lang))``, :60): Java's
  locale-sensitive rules for Turkish/Azeri (dotless i) and Lithuanian (dot
  above kept on i before accents) are restated in ``java_lower``.
* SpecialCharPreprocessor passes the symbol list of :55 to
  ``String.replaceAll`` as a REGEX.  That pattern opens a character class
  (``[``; a ``]`` right after it is a literal in java.util.regex) which its
  trailing lone backslash leaves unclosed, so ``Pattern.compile`` throws
  ``PatternSyntaxException`` for every non-null row; a null text throws
  ``NullPointerException`` first.  Reproduced as ``PatternSyntaxException``
  (the JVM's exact message index is unverified: no JVM in this image).  The
  second ``replaceAll("  *", "")`` (:56), which would delete every space, is
  never reached; ``intended_special_char_clean`` offers the documented intent
  to callers who want it.
"""
from __future__ import annotations

import re
from typing import Dict, Optional

import numpy as np

from .api import NullPointerException, _Params, _random_uid

# SpecialCharPreprocessor.scala:55 (the Scala literal ends in \" and \\: the
# characters `"` and `\`)
SPECIAL_CHAR_PATTERN = "/_[]*()%^&@$#:|{}<>~`\"\\"

_DOT_ABOVE = "\u0307"
# combining marks of canonical class 230 (Above) that Java's Lithuanian rule
# tests for (java.lang.ConditionalSpecialCasing, "More_Above")
_COMBINING_ABOVE = re.compile("[\u0300-\u0314\u033d-\u0344\u0346\u034a-\u034c\u0350-\u0352\u0357\u035b"
                              "\u0363-\u036f]")


class PatternSyntaxException(ValueError):
    """java.util.regex.PatternSyntaxException."""

    def __init__(self, desc: str, pattern: str, index: int):
        self.desc, self.pattern, self.index = desc, pattern, index
        super().__init__(f"{desc} near index {index}\n{pattern}\n{' ' * index}^")


def _language_of(tag: str) -> str:
    """Locale.forLanguageTag(tag).getLanguage(): the primary subtag in lower
    case; an ill-formed tag gives the root locale ("")."""
    if tag is None:
        raise NullPointerException("Locale.forLanguageTag(null)")
    primary = tag.split("-", 1)[0]
    if not (2 <= len(primary) <= 8 and primary.isascii() and primary.isalpha()):
        return ""
    return primary.lower()


def java_lower(text: str, lang_tag: str) -> str:
    """String.toLowerCase(Locale.forLanguageTag(lang_tag)) (LowerCasePreprocessor.scala:60).

    Outside tr/az/lt, Java's mapping is Unicode's full lower-case mapping with
    the Final_Sigma context, which ``str.lower`` implements too (U+0130 becomes
    "i" + U+0307 in both).  Locale rules of java.lang.ConditionalSpecialCasing:
      tr, az: "I" + U+0307 -> "i"; U+0130 -> "i"; "I" -> U+0131 (dotless i);
      lt:     "I", "J", U+012E followed by a mark above keep a dot above
              (U+0307 inserted); U+00CC, U+00CD, U+0128 -> "i" U+0307 + accent.
    """
    lang = _language_of(lang_tag)
    if lang in ("tr", "az"):
        text = text.replace("I" + _DOT_ABOVE, "i").replace("\u0130", "i").replace("I", "\u0131")
    elif lang == "lt":
        out = []
        for i, ch in enumerate(text):
            nxt = text[i + 1] if i + 1 < len(text) else ""
            if ch in "IJ\u012e" and nxt and _COMBINING_ABOVE.match(nxt):
                out.append(ch.lower() + _DOT_ABOVE)
            elif ch == "\u00cc":
                out.append("i" + _DOT_ABOVE + "\u0300")
            elif ch == "\u00cd":
                out.append("i" + _DOT_ABOVE + "\u0301")
            elif ch == "\u0128":
                out.append("i" + _DOT_ABOVE + "\u0303")
            else:
                out.append(ch)
        text = "".join(out)
    return text.lower()


def _move_to_end(df, col: str, values):
    """Drop ``col`` and append it, holding ``values``, as the last column
    (transformSchema + the row rebuild of both preprocessors)."""
    out = df.drop(columns=[col])
    out[col] = values
    return out


def _frame(dataset):
    import pandas as pd
    return dataset if isinstance(dataset, pd.DataFrame) else pd.DataFrame(dataset)


def _require(df, *cols: str) -> None:
    for c in cols:  # row.fieldIndex
        if c not in df.columns:
            raise ValueError(f"Field \"{c}\" does not exist.")


class LowerCasePreprocessor(_Params):
    """LowerCasePreprocessor (LowerCasePreprocessor.scala:19-76); device: lower-
    case on that GPU (preprocess_device), else on the host."""

    _defaults = {"outputCol": "fulltext", "labelCol": "lang"}

    def __init__(self, uid: Optional[str] = None, device: Optional[int] = None):
        super().__init__()
        self.uid = uid or _random_uid("LowerCasePreprocessor")
        self._device = device

    def setInputCol(self, value: str):  # sets outputCol, as in the reference (:32)
        return self._set("outputCol", value)

    def setLabelCol(self, value: str):
        return self._set("labelCol", value)

    def getOutputCol(self) -> str:
        return self.getOrDefault("outputCol")

    def getLabelCol(self) -> str:
        return self.getOrDefault("labelCol")

    def transformSchema(self, schema: Dict[str, str]) -> Dict[str, str]:
        out = {k: v for k, v in schema.items() if k != self.getOutputCol()}
        out[self.getOutputCol()] = "string"
        return out

    def transform(self, dataset):
        df = _frame(dataset)
        col, label = self.getOutputCol(), self.getLabelCol()
        _require(df, col, label)
        texts, langs = list(df[col]), list(df[label])
        for text, lang in zip(texts, langs):
            if lang is None:
                raise NullPointerException("Locale.forLanguageTag(null)")
            if text is None:
                raise NullPointerException("text is null")
        if self._device is not None:
            values = preprocess_device(texts, langs, lower=True, device=self._device)
        else:
            values = [java_lower(t, lang) for t, lang in zip(texts, langs)]
        return _move_to_end(df, col, values)


class SpecialCharPreprocessor(_Params):
    """SpecialCharPreprocessor (SpecialCharPreprocessor.scala:19-70)."""

    _defaults = {"outputCol": "fulltext"}

    def __init__(self, uid: Optional[str] = None):
        super().__init__()
        self.uid = uid or _random_uid("SpecialCharPreprocessor")

    def setInputCol(self, value: str):  # sets outputCol, as in the reference (:30)
        return self._set("outputCol", value)

    def getOutputCol(self) -> str:
        return self.getOrDefault("outputCol")

    def transformSchema(self, schema: Dict[str, str]) -> Dict[str, str]:
        out = {k: v for k, v in schema.items() if k != self.getOutputCol()}
        out[self.getOutputCol()] = "string"
        return out

    def transform(self, dataset):
        df = _frame(dataset)
        col = self.getOutputCol()
        _require(df, col)
        for text in df[col]:
            if text is None:
                raise NullPointerException("text is null")
            # String.replaceAll compiles its pattern before matching: it never compiles
            raise PatternSyntaxException("Unclosed character class", SPECIAL_CHAR_PATTERN,
                                         len(SPECIAL_CHAR_PATTERN) - 1)
        return _move_to_end(df, col, [])  # no rows: nothing is evaluated


def intended_special_char_clean(text: str) -> str:
    """What SpecialCharPreprocessor.scala:54-56 meant (doc comment :16): the
    listed symbols removed literally, then every match of "  *" (a space and
    any further spaces) removed.  Not the reference's behaviour (module doc)."""
    if text is None:
        raise NullPointerException("text is null")
    text = re.sub("[" + re.escape(SPECIAL_CHAR_PATTERN) + "]", "", text)
    return re.sub("  *", "", text)


_CASEMAPS: Dict[object, object] = {}


def _casemap(device, variant="product"):
    from .runtime import DeviceCaseMap
    key = (device, variant)
    if key not in _CASEMAPS:
        _CASEMAPS[key] = DeviceCaseMap(device, variant=variant)
    return _CASEMAPS[key]


def _host_pre(text: str, lang, lower: bool, clean: bool) -> str:
    if lower:
        text = java_lower(text, lang)
    return intended_special_char_clean(text) if clean else text


def preprocess_device(texts, langs=None, lower: bool = True, clean: bool = False, device: int = 0,
                      score_encoding: bool = False):
    """LowerCasePreprocessor's lower-casing (labels `langs` as locales) and/or
    the documented SpecialChar cleanup (``intended_special_char_clean``) on the
    GPU (ldgpu_preprocess).  Returns the texts, or with ``score_encoding`` the
    SCORE input packed as ``encoding.pack`` does (data, offsets): the low byte
    of each UTF-16 unit, what ``LanguageDetectorModel.transform`` scores.  The
    documents the device leaves to the host (not 1:1, or context-dependent)
    are done by ``java_lower`` here."""
    from . import _lib, encoding
    from .runtime import DeviceCaseMap, locale_class
    texts = list(texts)
    for t in texts:
        if t is None:
            raise NullPointerException("text is null")
    if lower:
        if langs is None:
            raise ValueError("lower-casing needs the labels (the locale of each row)")
        langs = list(langs)
        for lang in langs:
            if lang is None:
                raise NullPointerException("Locale.forLanguageTag(null)")
        locale = np.fromiter((locale_class(lang) for lang in langs), dtype=np.uint8, count=len(texts))
    else:
        langs = [None] * len(texts)
        locale = None
    flags = (_lib.PRE_LOWER if lower else 0) | (_lib.PRE_CLEAN if clean else 0) | \
        (_lib.PRE_LOW_BYTES if score_encoding else 0)
    units, off = DeviceCaseMap.pack_units(texts)
    out, out_off, host = _casemap(device).run(units, off, locale, flags)
    redo = np.nonzero(host)[0]
    if score_encoding:
        if len(redo) == 0:
            n = int(out_off[-1])
            data = np.zeros(((n + 3) // 4) * 4 + 4, dtype=np.uint8)
            data[:n] = out[:n]
            return data, out_off
        parts = [out[out_off[i]:out_off[i + 1]].tobytes() for i in range(len(texts))]
        for i in redo:
            parts[i] = encoding.score_bytes(_host_pre(texts[i], langs[i], lower, clean))
        return encoding.pack(parts)
    res = [out[out_off[i]:out_off[i + 1]].tobytes().decode("utf-16-le", "surrogatepass") for i in range(len(texts))]
    for i in redo:
        res[i] = _host_pre(texts[i], langs[i], lower, clean)
    return res
