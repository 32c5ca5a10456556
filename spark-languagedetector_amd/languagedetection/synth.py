"""Synthetic multilingual corpora (SURVEY.md §8d "Synthetic generator").

Every language is a first-order Markov chain over its own 24-30 symbol subset
of ``[a-z' ]`` plus a few capitals, with transition rows ~ Dirichlet(0.3).
Text is ASCII only, so the fit encoding (UTF-8, LanguageDetector.scala:37) and
the score encoding (low byte of UTF-16, LanguageDetectorModel.scala:161) agree.

Generation is vectorised over documents (one gather per character position),
so 1M x 256 B documents take a few seconds with numpy.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

SEED_BASE = 20261015

_ISO = ["en", "de", "fr", "es", "it", "nl", "pt", "sv", "da", "no", "fi", "pl", "cs", "sk", "hu",
        "ro", "tr", "id", "ms", "sw", "et", "lv", "lt", "sl", "hr", "sq", "is", "ga", "cy", "eu",
        "ca", "gl", "af", "zu", "xh", "so", "ha", "yo", "ig", "mt"]

_LOWER = [ord(c) for c in "abcdefghijklmnopqrstuvwxyz'"]
_UPPER = [ord(c) for c in "ABCDEFGHIJKLMNOPQRSTUVWXYZ"]
_QBITS = 12  # transition sampling resolution (4096 buckets per row)


def language_names(n: int) -> List[str]:
    if n <= len(_ISO):
        return _ISO[:n]
    return [f"l{i:03d}" for i in range(n)]


@dataclass
class LanguageSet:
    names: List[str]
    alpha: np.ndarray      # [L, S] uint8: symbol byte of state s (S = max alphabet size)
    nxt: np.ndarray        # [L, S, 4096] uint8: next state for a 12-bit uniform draw
    size: np.ndarray       # [L] alphabet size

    @property
    def n_langs(self) -> int:
        return len(self.names)


def make_languages(n_langs: int, seed: int = SEED_BASE) -> LanguageSet:
    rng = np.random.Generator(np.random.PCG64(seed))
    S = 30
    alpha = np.zeros((n_langs, S), dtype=np.uint8)
    nxt = np.zeros((n_langs, S, 1 << _QBITS), dtype=np.uint8)
    size = np.zeros(n_langs, dtype=np.int32)
    for l in range(n_langs):
        m = int(rng.integers(24, 31))
        n_upper = int(rng.integers(0, 4))
        lower = rng.choice(_LOWER, size=min(m - 1 - n_upper, len(_LOWER)), replace=False)
        upper = rng.choice(_UPPER, size=n_upper, replace=False)
        syms = np.concatenate([[ord(" ")], lower, upper]).astype(np.uint8)
        k = len(syms)
        size[l] = k
        alpha[l, :k] = syms
        P = rng.dirichlet(np.full(k, 0.3), size=k)
        cdf = np.cumsum(P, axis=1)
        cdf[:, -1] = 1.0
        u = (np.arange(1 << _QBITS) + 0.5) / (1 << _QBITS)
        for s in range(k):
            nxt[l, s] = np.minimum(np.searchsorted(cdf[s], u, side="right"), k - 1).astype(np.uint8)
    return LanguageSet(language_names(n_langs), alpha, nxt, size)


def generate(ls: LanguageSet, n_docs: int, len_lo: int, len_hi: Optional[int] = None,
             seed: int = SEED_BASE, doc_lang: Optional[np.ndarray] = None):
    """Returns (data uint8, offsets int64[n+1], doc_lang int32[n]).

    Lengths ~ U[len_lo, len_hi] (inclusive); labels uniform over languages.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    if len_hi is None:
        len_hi = len_lo
    if doc_lang is None:
        doc_lang = rng.integers(0, ls.n_langs, size=n_docs, dtype=np.int32)
    doc_lang = np.asarray(doc_lang, dtype=np.int32)
    lens = rng.integers(len_lo, len_hi + 1, size=n_docs, dtype=np.int64)
    offsets = np.zeros(n_docs + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    maxlen = int(lens.max()) if n_docs else 0
    state = rng.integers(0, 1 << 16, size=n_docs, dtype=np.int64) % ls.size[doc_lang]
    grid = np.empty((n_docs, maxlen), dtype=np.uint8)
    flat_nxt = ls.nxt.reshape(-1)
    base = doc_lang.astype(np.int64) * (ls.nxt.shape[1] << _QBITS)
    for t in range(maxlen):
        grid[:, t] = ls.alpha[doc_lang, state]
        u = rng.integers(0, 1 << _QBITS, size=n_docs, dtype=np.int64)
        state = flat_nxt[base + (state << _QBITS) + u].astype(np.int64)
    if len_lo == len_hi:
        data = grid.reshape(-1).copy()
    else:
        mask = np.arange(maxlen)[None, :] < lens[:, None]
        data = grid[mask]
    return data, offsets, doc_lang


def tile(data: np.ndarray, offsets: np.ndarray, doc_lang: np.ndarray, n_docs: int):
    """Repeat a generated pool of documents up to n_docs (bench-scale inputs)."""
    pool = len(offsets) - 1
    reps = -(-n_docs // pool)
    lens = np.diff(offsets)
    all_lens = np.tile(lens, reps)[:n_docs]
    off = np.zeros(n_docs + 1, dtype=np.int64)
    np.cumsum(all_lens, out=off[1:])
    full = np.tile(data, reps)[: int(off[-1])]
    return full, off, np.tile(doc_lang, reps)[:n_docs]


def texts(data: np.ndarray, offsets: np.ndarray) -> List[str]:
    b = data.tobytes()
    return [b[offsets[i]:offsets[i + 1]].decode("ascii") for i in range(len(offsets) - 1)]


def generate_device(ls: LanguageSet, n_docs: int, len_lo: int, len_hi: int, seed: int, device,
                    chunk_docs: int = 1 << 18):
    """The same Markov-chain text as generate(), drawn on a GPU with torch (a
    bench-scale corpus -- config 3's 6.25 GB shard per GPU -- in seconds, not
    tiled from a small pool).  Deterministic for a seed (torch's GPU Philox
    generator), not the same draws as generate().  Returns device tensors
    (bytes uint8 padded to whole dwords + 16, offsets int64 [n + 1], lang int32)."""
    import torch
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    L = ls.n_langs
    lang = torch.randint(0, L, (n_docs,), generator=g, device=dev, dtype=torch.int64)
    lens = torch.randint(len_lo, len_hi + 1, (n_docs,), generator=g, device=dev, dtype=torch.int64)
    off = torch.zeros(n_docs + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=off[1:])
    total = int(off[-1].item())
    out = torch.zeros(((total + 3) // 4) * 4 + 16, dtype=torch.uint8, device=dev)
    alpha = torch.from_numpy(ls.alpha).to(dev).reshape(-1)              # [L * S]
    nxt = torch.from_numpy(ls.nxt).to(dev).reshape(-1)                  # [L * S * 4096]
    size = torch.from_numpy(ls.size.astype(np.int64)).to(dev)
    S = ls.alpha.shape[1]
    for c0 in range(0, n_docs, chunk_docs):
        c1 = min(n_docs, c0 + chunk_docs)
        cl = lang[c0:c1]
        maxlen = int(lens[c0:c1].max().item()) if c1 > c0 else 0
        state = torch.randint(0, 1 << 16, (c1 - c0,), generator=g, device=dev, dtype=torch.int64) % size[cl]
        grid = torch.empty((c1 - c0, maxlen), dtype=torch.uint8, device=dev)
        abase = cl * S
        nbase = cl * (S << _QBITS)
        for t in range(maxlen):
            grid[:, t] = alpha[abase + state]
            u = torch.randint(0, 1 << _QBITS, (c1 - c0,), generator=g, device=dev, dtype=torch.int64)
            state = nxt[nbase + (state << _QBITS) + u].to(torch.int64)
        mask = torch.arange(maxlen, device=dev)[None, :] < lens[c0:c1, None]
        b0, b1 = int(off[c0].item()), int(off[c1].item())
        out[b0:b1] = grid[mask]
        del grid, mask
    return out, off, lang.to(torch.int32)
