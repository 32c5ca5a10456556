"""Multi-GPU execution: one process per GPU (torch.distributed; backend "nccl"
is RCCL over xGMI on MI355X, "gloo" for CPU tests and one-GPU rehearsals).

SCORE shards documents (contiguous ranges per rank, the reference's Spark
partitions, LanguageDetectorModel.scala:225-238): no collective on the data
path; labels are gathered at the end only when the caller asks for them.

FIT has one exchange step, and it runs inside libldgpu.so behind the C ABI
(ldgpu_counts_merge, include/ldgpu.h), so a Spark executor reaches it the same
way this module does.  Counts are sums over documents
(LanguageDetector.scala:59-63) and presence needs the global key set (:79-87):
  1. every rank counts its shard on its GPU (ldgpu_count*),
  2. owner exchange: gram g belongs to rank owner(g) = a hash of its key; one
     all-to-all moves each rank's count rows to the owners, and every rank
     then holds the global counts of the grams it owns (bit-exact sums),
  3. ldgpu_fit_table_size runs the global top-K over the shards: a
     (language, class) histogram all-reduce, an all-gather of each rank's
     threshold-class tie candidates, an all-gather of the chosen rows -- every
     rank builds the same probability / top-K table.
The communicator (ldgpu_comm) is RCCL when the torch group is "nccl" (the
unique id travels through the group) and otherwise the host transport, whose
all-gather / all-to-all callbacks are served here by torch.distributed (gloo).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib


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


def packed_keys(keys: Sequence[bytes]) -> np.ndarray:
    """The device's packed u64 gram keys (ldgpu_common.h): bytes
    little-endian in bits 0..55, the length in bits 56..63."""
    out = np.empty(len(keys), dtype=np.uint64)
    for i, k in enumerate(keys):
        out[i] = (len(k) << 56) | int.from_bytes(k, "little")
    return out


def owner_of(packed: np.ndarray, world: int) -> np.ndarray:
    """The merge's owner rank of each packed key: the high 32 bits of
    (low 32 bits of mix64(key)) * world -- the same function as the device's
    owner_of (ldgpu_fit.hip), restated here for the protocol's CPU test."""
    with np.errstate(over="ignore"):
        k = packed.astype(np.uint64)
        k ^= k >> np.uint64(31)
        k *= np.uint64(0x7FB5D329728EA185)
        k ^= k >> np.uint64(27)
        k *= np.uint64(0x81DADEF4BC2DD44D)
        k ^= k >> np.uint64(33)
        return (((k & np.uint64(0xFFFFFFFF)) * np.uint64(world)) >> np.uint64(32)).astype(np.int64)


# ----------------------------------------------------------- communicators
class Communicator:
    """An ldgpu_comm spanning the ranks of a torch.distributed group.

    transport "rccl": RCCL over xGMI (rank 0's ldgpu_comm_unique_id reaches
    the others through the group); "host": the library's host transport with
    all-gather / all-to-all served by the group (gloo); "auto": RCCL when the
    group's backend is nccl."""

    def __init__(self, group=None, device: Optional[int] = None, transport: str = "auto", variant: str = "product"):
        """variant: the library of the count tables it merges (handles of the
        diagnostics library need a communicator of the same library)."""
        import torch.distributed as dist

        self.lib = _lib.load(variant=variant)
        self.ctx = _lib.context(device, variant)
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if transport == "auto":
            transport = "rccl" if dist.get_backend(group) == "nccl" else "host"
        self.transport = transport
        out = ctypes.c_void_p()
        if transport == "rccl":
            uid = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
            if self.rank == 0:
                _lib.check(self.lib.ldgpu_comm_unique_id(uid), self.lib)
            box = [bytes(uid)]
            if self.world > 1:
                dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                           group=group)
            uid = (ctypes.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(box[0])
            _lib.check(self.lib.ldgpu_comm_create_rccl(self.ctx, uid, self.rank, self.world, ctypes.byref(out)),
                       self.lib)
        elif transport == "host":
            self._fns = (_lib.ALLGATHER_FN(self._allgather), _lib.ALLTOALLV_FN(self._alltoallv))
            self._coll = _lib.HostColl(None, *self._fns)
            _lib.check(self.lib.ldgpu_comm_create_host(self.ctx, self.rank, self.world, ctypes.byref(self._coll),
                                                       ctypes.byref(out)), self.lib)
        else:
            raise ValueError(f"unknown transport {transport!r}")
        self.h = out.value

    # host transport callbacks (called from inside libldgpu.so)
    def _allgather(self, _user, send, nbytes, recv) -> int:
        try:
            import torch
            import torch.distributed as dist
            n = int(nbytes)
            src = np.ctypeslib.as_array((ctypes.c_uint8 * max(n, 1)).from_address(send))[:n]
            t = torch.from_numpy(src.copy())
            parts = [torch.empty(n, dtype=torch.uint8) for _ in range(self.world)]
            dist.all_gather(parts, t, group=self.group)
            dst = np.ctypeslib.as_array((ctypes.c_uint8 * max(n * self.world, 1)).from_address(recv))
            for r, part in enumerate(parts):
                dst[r * n:(r + 1) * n] = part.numpy()
            return 0
        except Exception:  # noqa: BLE001 -- reported to the library as a failed collective
            return 1

    def _alltoallv(self, _user, send, send_bytes, recv, recv_bytes) -> int:
        try:
            import torch
            import torch.distributed as dist
            sb = [int(send_bytes[r]) for r in range(self.world)]
            rb = [int(recv_bytes[r]) for r in range(self.world)]
            src = np.ctypeslib.as_array((ctypes.c_uint8 * max(sum(sb), 1)).from_address(send))[:sum(sb)]
            out = torch.empty(sum(rb), dtype=torch.uint8)
            dist.all_to_all_single(out, torch.from_numpy(src.copy()), rb, sb, group=self.group)
            if sum(rb):
                dst = np.ctypeslib.as_array((ctypes.c_uint8 * sum(rb)).from_address(recv))
                dst[:] = out.numpy()
            return 0
        except Exception:  # noqa: BLE001
            return 1

    def close(self):
        if getattr(self, "h", None):
            self.lib.ldgpu_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def merge_counts_device(local, comm: Optional[Communicator] = None, group=None):
    """The FIT merge (ldgpu_counts_merge): `local` is this rank's DeviceCounts;
    afterwards it holds the global counts of the grams this rank owns, and its
    fit_table() is the global table (collective).  Returns `local`."""
    if comm is None:
        comm = Communicator(group, device=local.device, variant=getattr(local, "variant", "product"))
    local._check(local.lib.ldgpu_counts_merge(local.h, comm.h))
    local.comm = comm  # the merged table's fit_table() runs its collectives
    return local


def merge_counts(keys: Sequence[bytes], counts: np.ndarray, n_langs: int, group=None
                 ) -> Tuple[List[bytes], np.ndarray]:
    """The owner-exchange protocol of ldgpu_counts_merge on host arrays (keys
    + int64 counts [n, L] of this rank's shard): returns this rank's OWNED
    grams with their global counts, sorted by (length, bytes).  Restates the
    device merge step by step for the CPU multi-process test."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    counts = np.ascontiguousarray(counts, dtype=np.int64).reshape(len(keys), n_langs)
    owner = owner_of(packed_keys(keys), world) if len(keys) else np.zeros(0, dtype=np.int64)
    order = np.argsort(owner, kind="stable")
    codes = sort_keys(keys)[order] if len(keys) else np.zeros(0, dtype=np.int64)
    rows = counts[order]
    send_n = np.bincount(owner, minlength=world).astype(np.int64)
    all_n = [torch.zeros(world, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(all_n, torch.from_numpy(send_n), group=group)
    rank = dist.get_rank(group)
    recv_n = [int(all_n[r][rank]) for r in range(world)]
    rk = torch.empty(sum(recv_n), dtype=torch.int64)
    dist.all_to_all_single(rk, torch.from_numpy(np.ascontiguousarray(codes)), recv_n, send_n.tolist(), group=group)
    rr = torch.empty((sum(recv_n), n_langs), dtype=torch.int64)
    dist.all_to_all_single(rr, torch.from_numpy(np.ascontiguousarray(rows)), recv_n, send_n.tolist(), group=group)
    u, inv = np.unique(rk.numpy(), return_inverse=True)
    glob = np.zeros((len(u), n_langs), dtype=np.int64)
    np.add.at(glob, inv, rr.numpy())
    return keys_of(u), glob


def fit_distributed(rows: Sequence[Tuple[str, str]], supported_languages: Sequence[str],
                    gram_lengths: Sequence[int], profile_size: int, group=None,
                    device: Optional[int] = None, transport: str = "auto") -> Dict[bytes, List[float]]:
    """LanguageDetector.computeGramProbabilities over all ranks: `rows` are
    this rank's training rows; every rank returns the same table."""
    from .api import LanguageDetector

    local = LanguageDetector.count_grams(rows, gram_lengths, supported_languages, device=device)
    comm = Communicator(group, device=device, transport=transport)
    try:
        merge_counts_device(local, comm)
        return local.fit_table(profile_size)
    finally:
        local.close()
        comm.close()


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
