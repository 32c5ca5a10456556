"""Multi-GPU execution: one process per GPU (torch.distributed; backend "nccl"
is RCCL over xGMI on MI355X, "gloo" for CPU tests).

SCORE shards documents (contiguous ranges per rank, the reference's Spark
partitions, LanguageDetectorModel.scala:225-238): no collective on the data
path; labels are gathered at the end only when the caller asks for them.

FIT has one exchange step.  Counts are sums over documents
(LanguageDetector.scala:59-63) and presence needs the global key set
(:79-87), so every rank counts its shard on its GPU, then:
  1. all_gather of the per-rank distinct-key lists (packed u64 sort keys),
  2. the sorted union U -- identical on every rank,
  3. each rank scatters its counts into a dense [|U|, L] int64 block,
  4. all_reduce(SUM) of that block (exact integer sums),
  5. every rank loads the global counts into a device table and builds the
     same probability / top-K table (computeProbabilities + filterTopGrams).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) share of n units for rank."""
    return n * rank // world, n * (rank + 1) // world


# ---------------------------------------------------------------- key codes
def sort_keys(keys: Sequence[bytes]) -> np.ndarray:
    """Gram keys (1..7 bytes) -> int64 codes ordered as (length, bytes):
    length in the top byte, the bytes big-endian below it."""
    out = np.empty(len(keys), dtype=np.int64)
    for i, k in enumerate(keys):
        n = len(k)
        if not 1 <= n <= 7:
            raise ValueError(f"gram key of {n} bytes outside the device path's 1..7")
        out[i] = (n << 56) | int.from_bytes(k.ljust(7, b"\0"), "big")
    return out


def keys_of(codes: np.ndarray) -> List[bytes]:
    out = []
    for c in codes.tolist():
        n = c >> 56
        out.append((c & ((1 << 56) - 1)).to_bytes(7, "big")[:n])
    return out


# ------------------------------------------------------------------- merge
def merge_counts(keys: Sequence[bytes], counts: np.ndarray, n_langs: int, group=None, device=None
                 ) -> Tuple[List[bytes], np.ndarray]:
    """All-reduce per-rank (gram -> count[L]) tables into the global one.
    Returns (keys sorted by (length, bytes), int64 counts [U, L]), identical
    on every rank."""
    import torch
    import torch.distributed as dist

    backend = dist.get_backend(group)
    dev = torch.device("cpu") if backend == "gloo" else (device or torch.device("cuda", torch.cuda.current_device()))
    world = dist.get_world_size(group)
    local = torch.from_numpy(sort_keys(keys)).to(dev)
    counts = np.ascontiguousarray(counts, dtype=np.int64).reshape(len(keys), n_langs)

    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([len(keys)], dtype=torch.int64, device=dev), group=group)
    mx = int(max(int(s.item()) for s in sizes))
    padded = torch.full((max(mx, 1),), -1, dtype=torch.int64, device=dev)
    padded[:len(keys)] = local
    gathered = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(gathered, padded, group=group)
    allk = torch.cat([g[:int(s.item())] for g, s in zip(gathered, sizes)])
    union = torch.unique(allk, sorted=True)

    dense = torch.zeros((union.numel(), n_langs), dtype=torch.int64, device=dev)
    if len(keys):
        pos = torch.searchsorted(union, local)
        dense[pos] = torch.from_numpy(counts).to(dev)
    dist.all_reduce(dense, op=dist.ReduceOp.SUM, group=group)
    codes = union.cpu().numpy()
    return keys_of(codes), dense.cpu().numpy()


def merge_counts_device(local, group=None):
    """The FIT merge on the GPUs: `local` is this rank's DeviceCounts; the
    keys/counts stay in HBM (ldgpu_counts_export_device), the exchange is
    all_gather + all_reduce(SUM) (RCCL over xGMI with backend "nccl"), and the
    result is loaded into a new DeviceCounts (ldgpu_counts_add_device).
    Returns the merged DeviceCounts, identical on every rank."""
    import torch
    import torch.distributed as dist

    from .runtime import DeviceCounts

    keys, cnt = local.export_device()
    gpu = keys.device
    backend = dist.get_backend(group)
    dev = torch.device("cpu") if backend == "gloo" else gpu
    world = dist.get_world_size(group)
    k = keys.to(dev)
    c = cnt.to(dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([k.numel()], dtype=torch.int64, device=dev), group=group)
    mx = int(max(int(x.item()) for x in sizes))
    padded = torch.full((max(mx, 1),), -1, dtype=torch.int64, device=dev)
    padded[:k.numel()] = k
    gathered = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(gathered, padded, group=group)
    union = torch.unique(torch.cat([g[:int(x.item())] for g, x in zip(gathered, sizes)]), sorted=True)
    dense = torch.zeros((union.numel(), local.L), dtype=torch.int64, device=dev)
    if k.numel():
        dense[torch.searchsorted(union, k)] = c
    dist.all_reduce(dense, op=dist.ReduceOp.SUM, group=group)
    merged = DeviceCounts(local.L, local.gram_lengths, capacity_hint=int(union.numel()), device=local.device)
    if union.numel():
        merged.add_device(union.to(gpu), dense.to(gpu))
    return merged


def fit_distributed(rows: Sequence[Tuple[str, str]], supported_languages: Sequence[str],
                    gram_lengths: Sequence[int], profile_size: int, group=None,
                    device: Optional[int] = None) -> Dict[bytes, List[float]]:
    """LanguageDetector.computeGramProbabilities over all ranks: `rows` are
    this rank's training rows; every rank returns the same table."""
    from .api import LanguageDetector

    local = LanguageDetector.count_grams(rows, gram_lengths, supported_languages, device=device)
    merged = merge_counts_device(local, group=group)
    local.close()
    try:
        return merged.fit_table(profile_size)
    finally:
        merged.close()


def score_sharded(model, texts: Sequence[str], group=None, gather: bool = True):
    """Score this rank's contiguous share of `texts` (no collective on the data
    path); with gather=True every rank receives all labels (one all_gather)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_range(len(texts), rank, world)
    labels, _ = model.predict_indices(list(texts[lo:hi]))
    if not gather:
        return labels
    backend = dist.get_backend(group)
    dev = torch.device("cpu") if backend == "gloo" else torch.device("cuda", torch.cuda.current_device())
    mx = max(shard_range(len(texts), r, world)[1] - shard_range(len(texts), r, world)[0] for r in range(world))
    buf = torch.full((max(mx, 1),), -1, dtype=torch.int32, device=dev)
    buf[:hi - lo] = torch.from_numpy(labels.astype(np.int32)).to(dev)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    parts = []
    for r in range(world):
        a, b = shard_range(len(texts), r, world)
        parts.append(out[r][:b - a].cpu().numpy())
    return np.concatenate(parts) if parts else np.zeros(0, dtype=np.int32)
