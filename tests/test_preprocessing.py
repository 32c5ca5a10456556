"""Preprocessors: LowerCasePreprocessor.scala:19-76 and
SpecialCharPreprocessor.scala:19-70, host-only (no GPU).

Parity unpinned by any reference test (the reference has none for these
classes); expectations restate the Scala source and Java's documented
String.toLowerCase(Locale) / java.util.regex behaviour, cited per case."""
import pandas as pd
import pytest

from languagedetection import (LanguageDetectorModel, LowerCasePreprocessor, NullPointerException,
                               PatternSyntaxException, SpecialCharPreprocessor)
from languagedetection.preprocessing import SPECIAL_CHAR_PATTERN, intended_special_char_clean, java_lower

DOTTED_I = "\N{LATIN CAPITAL LETTER I WITH DOT ABOVE}"
DOTLESS_I = "\N{LATIN SMALL LETTER DOTLESS I}"
DOT_ABOVE = "\N{COMBINING DOT ABOVE}"


def test_lowercase_moves_column_last_and_lowers():
    df = pd.DataFrame({"fulltext": ["Hallo WELT", "THIS Is"], "lang": ["de", "en"], "id": [1, 2]})
    out = LowerCasePreprocessor().transform(df)
    assert list(out.columns) == ["lang", "id", "fulltext"]          # :63-71 drop + append
    assert list(out["fulltext"]) == ["hallo welt", "this is"]
    assert list(out["lang"]) == ["de", "en"] and list(out["id"]) == [1, 2]
    assert list(df.columns) == ["fulltext", "lang", "id"]          # input untouched


def test_lowercase_setinputcol_sets_outputcol():
    p = LowerCasePreprocessor().setInputCol("body").setLabelCol("language")
    assert p.getOutputCol() == "body"                               # :32
    out = p.transform(pd.DataFrame({"body": ["ABC"], "language": ["en"]}))
    assert list(out["body"]) == ["abc"]
    assert p.transformSchema({"body": "string", "language": "string"}) == {"language": "string", "body": "string"}


def test_lowercase_locale_rules():
    # Turkish / Azeri: dotless i, dotted capital I (java.lang.ConditionalSpecialCasing)
    assert java_lower("ISTANBUL " + DOTTED_I + "zmir", "tr") == DOTLESS_I + "stanbul izmir"
    assert java_lower("I" + DOT_ABOVE, "tr") == "i"
    assert java_lower(DOTTED_I, "az") == "i"
    assert java_lower("ISTANBUL", "en") == "istanbul"
    assert java_lower(DOTTED_I, "en") == "i" + DOT_ABOVE                 # U+0130 outside tr/az
    # Lithuanian: the dot above is kept before an accent
    assert java_lower("\N{LATIN CAPITAL LETTER I WITH GRAVE}", "lt") == "i" + DOT_ABOVE + "\N{COMBINING GRAVE ACCENT}"
    assert java_lower("I\N{COMBINING ACUTE ACCENT}", "lt") == "i" + DOT_ABOVE + "\N{COMBINING ACUTE ACCENT}"
    # Greek final sigma
    sigma = "\N{GREEK CAPITAL LETTER SIGMA}"
    assert java_lower("\N{GREEK CAPITAL LETTER OMICRON}" + sigma + " " + sigma, "el") == \
        "\N{GREEK SMALL LETTER OMICRON}\N{GREEK SMALL LETTER FINAL SIGMA} \N{GREEK SMALL LETTER SIGMA}"
    # region subtags and ill-formed tags
    assert java_lower("I", "tr-TR") == DOTLESS_I
    assert java_lower("I", "?") == "i"


def test_lowercase_errors():
    with pytest.raises(ValueError, match='Field "lang" does not exist'):
        LowerCasePreprocessor().transform(pd.DataFrame({"fulltext": ["a"]}))
    with pytest.raises(NullPointerException):
        LowerCasePreprocessor().transform(pd.DataFrame({"fulltext": [None], "lang": ["en"]}))
    with pytest.raises(NullPointerException):
        LowerCasePreprocessor().transform(pd.DataFrame({"fulltext": ["a"], "lang": [None]}))


def test_specialchar_pattern_never_compiles():
    # :55 hands the symbol list to replaceAll as a regex; its character class
    # is left open by the trailing lone backslash -> PatternSyntaxException
    assert SPECIAL_CHAR_PATTERN == '/_[]*()%^&@$#:|{}<>~`"\\'
    with pytest.raises(PatternSyntaxException, match="^Unclosed character class"):
        SpecialCharPreprocessor().transform(pd.DataFrame({"fulltext": ["a <b>  c"]}))
    with pytest.raises(NullPointerException):
        SpecialCharPreprocessor().transform(pd.DataFrame({"fulltext": [None]}))
    empty = SpecialCharPreprocessor().transform(pd.DataFrame({"fulltext": pd.Series([], dtype=object),
                                                              "x": pd.Series([], dtype=int)}))
    assert list(empty.columns) == ["x", "fulltext"] and len(empty) == 0
    assert SpecialCharPreprocessor().setInputCol("t").getOutputCol() == "t"


def test_specialchar_intended_clean():
    assert intended_special_char_clean("a<b>[c]  d e") == "abcde"   # "  *" removes every space


def test_pipeline_lowercase_then_model_schema():
    """The preprocessor's output feeds LanguageDetectorModel.transformSchema."""
    df = LowerCasePreprocessor().transform(pd.DataFrame({"fulltext": ["Die"], "lang": ["de"]}))
    m = LanguageDetectorModel({"die": [1.0, 0.0]}, [3], ["de", "en"]).setOutputCol("pred")
    assert m.transformSchema(m._schema_of(df)) == {"lang": "string", "fulltext": "string", "pred": "string"}


def test_language_enumeration():
    """LanguageSpecs.scala:10-13: Language.withName("de").toString == "de";
    ids are positions in isoLanguageCodes (Language.scala:13-200)."""
    from languagedetection import Language
    de = Language.withName("de")
    assert str(de) == "de"
    assert Language.isoLanguageCodes[de.id] == "de"
    assert Language.maxId == len(Language.isoLanguageCodes) == 182
    assert len(set(Language.isoLanguageCodes)) == 182
    assert Language(0).name == "ab" and str(Language(181)) == "zu"
    with pytest.raises(KeyError, match="No value found for 'xx'"):
        Language.withName("xx")


def test_case_tables_for_the_device():
    """The 1:1 lower-case table and the host-only units handed to
    ldgpu_casemap_create (include/ldgpu.h PREPROCESS)."""
    import numpy as np
    from languagedetection.runtime import case_tables, locale_class
    lower, special = case_tables()
    bits = np.unpackbits(special, bitorder="little").astype(bool)
    assert lower[ord("A")] == ord("a") and lower[ord("a")] == ord("a") and lower[0xC4] == 0xE4
    assert lower[ord("I")] == ord("i")                     # root locale; tr/az is the device's rule
    assert bits[0x130] and bits[0x3A3] and bits[0xD801] and not bits[ord("A")] and not bits[0xD800]
    assert [locale_class(t) for t in ("tr", "az-Latn", "lt", "en", "?", "TR")] == [1, 1, 2, 0, 0, 1]
