"""The reference's ``language.Language`` enumeration (Language.scala:11-200):
the ISO 639-1 codes a detector may name, each value's id = its position in
``isoLanguageCodes``.  Not on the fit / score path (the reference's fit and
transform take a plain ``Seq[String]`` of languages); kept so a caller of the
reference finds it.  ``Language.withName("de")`` is the reference's one test
(LanguageSpecs.scala:10-13)."""
from __future__ import annotations

from typing import Dict, List, Tuple

ISO_LANGUAGE_CODES: Tuple[str, ...] = (
    "ab", "aa", "af", "ak", "sq", "am", "ar", "an", "hy", "as", "av", "ae", "ay", "az", "bm", "ba",
    "eu", "be", "bn", "bh", "bi", "bs", "br", "bg", "my", "ca", "km", "ch", "ce", "ny", "zh", "cu",
    "cv", "kw", "co", "cr", "hr", "cs", "da", "dv", "nl", "dz", "en", "eo", "et", "ee", "fj", "fi",
    "fr", "ff", "gd", "gl", "lg", "ka", "de", "ki", "el", "kl", "gn", "gu", "ht", "ha", "he", "hz",
    "hi", "ho", "hu", "is", "io", "ig", "id", "ia", "ie", "iu", "ik", "ga", "it", "ja", "jv", "kn",
    "kr", "ks", "kk", "rw", "kv", "kg", "ko", "kj", "ku", "ky", "lo", "la", "lv", "lb", "li", "ln",
    "lt", "lu", "mk", "mg", "ms", "ml", "mt", "gv", "mi", "mr", "mh", "ro", "mn", "na", "nv", "nd",
    "ng", "ne", "se", "no", "nb", "nn", "ii", "oc", "oj", "or", "om", "os", "pi", "pa", "ps", "fa",
    "pl", "pt", "qu", "rm", "rn", "ru", "sm", "sg", "sa", "sc", "sr", "sn", "sd", "si", "sk", "sl",
    "so", "st", "nr", "es", "su", "sw", "ss", "sv", "tl", "ty", "tg", "ta", "tt", "te", "th", "bo",
    "ti", "to", "ts", "tn", "tr", "tk", "tw", "uk", "ur", "uz", "ve", "vi", "vo", "wa", "cy", "fy",
    "wo", "xh", "yi", "yo", "za", "zu",
)


class Value:
    """One enumeration value: ``id`` (position) and its code (``str(v)``)."""

    __slots__ = ("id", "name")

    def __init__(self, id: int, name: str):
        self.id = id
        self.name = name

    def __str__(self) -> str:
        return self.name

    def __repr__(self) -> str:
        return f"Language.{self.name}"

    def __eq__(self, other) -> bool:
        return isinstance(other, Value) and other.id == self.id

    def __hash__(self) -> int:
        return hash(self.id)


class _Enumeration:
    """scala.Enumeration's lookups: withName, apply(id), values, maxId."""

    def __init__(self, codes):
        self.isoLanguageCodes: List[str] = list(codes)
        self._values = [Value(i, c) for i, c in enumerate(codes)]
        self._by_name: Dict[str, Value] = {v.name: v for v in self._values}

    def withName(self, name: str) -> Value:
        try:
            return self._by_name[name]
        except KeyError:
            # scala.Enumeration.withName: NoSuchElementException("No value found for '...'")
            raise KeyError(f"No value found for '{name}'") from None

    def __call__(self, id: int) -> Value:
        return self._values[id]

    @property
    def values(self) -> List[Value]:
        return list(self._values)

    @property
    def maxId(self) -> int:
        return len(self._values)


Language = _Enumeration(ISO_LANGUAGE_CODES)
