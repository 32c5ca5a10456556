"""Host-side document packing (the caller-side encodings of the reference).

FIT   : ``text.getBytes(Charset.forName("UTF-8"))``  LanguageDetector.scala:37
        (Java replaces an unpaired surrogate by '?').
SCORE : ``text.toCharArray.map(_.toByte)``           LanguageDetectorModel.scala:161
        (low byte of every UTF-16 code unit).

Both produce packed ``(bytes uint8, offsets int64[n+1])`` buffers.  Pure
ASCII text -- the common case -- takes a fast path where both encodings are
the text's own bytes.
"""
from __future__ import annotations

import re
from typing import List, Sequence, Tuple

import numpy as np

_SURR = re.compile("[\ud800-\udfff]")


def _utf16_units(text: str) -> np.ndarray:
    return np.frombuffer(text.encode("utf-16-le", "surrogatepass"), dtype="<u2")


def fit_bytes(text: str) -> bytes:
    if text is None:
        raise TypeError("NullPointerException: training text is null")
    if text.isascii():
        return text.encode("ascii")
    if not _SURR.search(text):
        return text.encode("utf-8")
    # Java semantics: a surrogate pair is one code point, a lone surrogate is '?'
    units = _utf16_units(text)
    out = bytearray()
    i, n = 0, len(units)
    while i < n:
        u = int(units[i])
        if 0xD800 <= u <= 0xDBFF and i + 1 < n and 0xDC00 <= int(units[i + 1]) <= 0xDFFF:
            cp = 0x10000 + ((u - 0xD800) << 10) + (int(units[i + 1]) - 0xDC00)
            out += chr(cp).encode("utf-8")
            i += 2
        elif 0xD800 <= u <= 0xDFFF:
            out += b"?"
            i += 1
        else:
            out += chr(u).encode("utf-8")
            i += 1
    return bytes(out)


def score_bytes(text: str) -> bytes:
    if text is None:
        raise TypeError("NullPointerException: text is null")
    if text.isascii():
        return text.encode("ascii")
    return (_utf16_units(text) & 0xFF).astype(np.uint8).tobytes()


def pack(chunks: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """Pack byte strings into (data, offsets); data is padded to a multiple of
    4 bytes (+4) so device windows can read whole dwords."""
    lens = np.fromiter((len(c) for c in chunks), dtype=np.int64, count=len(chunks))
    offsets = np.zeros(len(chunks) + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    total = int(offsets[-1])
    buf = bytearray(b"".join(chunks))
    buf += b"\0" * (((total + 3) & ~3) + 4 - total)
    return np.frombuffer(bytes(buf), dtype=np.uint8), offsets


def pack_fit(texts: Sequence[str]):
    return pack([fit_bytes(t) for t in texts])


def pack_score(texts: Sequence[str]):
    return pack([score_bytes(t) for t in texts])


def gram_key(g) -> bytes:
    """A gram key as bytes: accepts bytes, str (UTF-8, as "Die".getBytes("UTF-8")
    in LanguageDetectorModelSpecs.scala:27) or a sequence of (signed) ints."""
    if isinstance(g, (bytes, bytearray, memoryview)):
        return bytes(g)
    if isinstance(g, str):
        return g.encode("utf-8")
    return bytes((int(x) & 0xFF) for x in g)


def pack_table(table, n_langs: int):
    """(key_bytes, key_offsets, rows[n][L] fp64, row_ok[n] u8) from a gram map."""
    keys: List[bytes] = []
    rows = np.zeros((len(table), n_langs), dtype=np.float64)
    ok = np.ones(len(table), dtype=np.uint8)
    for i, (g, r) in enumerate(table.items()):
        keys.append(gram_key(g))
        r = np.asarray(r, dtype=np.float64).reshape(-1)
        if r.shape[0] == n_langs:
            rows[i] = r
        else:
            ok[i] = 0
    data, offsets = pack(keys)
    return data, offsets, rows, ok
