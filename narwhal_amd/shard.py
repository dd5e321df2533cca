"""Sharding of independent units over GPUs -- one process per GPU.

Units never exchange data: triples (configs 2/5), whole certificates (config 3; a certificate's
votes are never split) and whole batches (config 4).  The only collective is an optional
all-gather of per-shard verdict words (RCCL over xGMI on GPUs, gloo in the CPU tests); it is not
needed for correctness because each rank already holds its own verdicts.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of n units for `rank`, cut on whole 64-unit verdict words: every shard
    starts on a multiple of 64, each holds ceil(ceil(n / 64) / world) words except the tail, so
    shards can differ by up to 64 * world - 1 units (the last ones may be short or empty)."""
    words = (n + 63) // 64
    per = (words + world - 1) // world
    lo = min(n, rank * per * 64)
    hi = min(n, (rank + 1) * per * 64)
    return lo, hi


def cert_cuts(offsets: Sequence[int], world: int) -> List[int]:
    """Vote-index cut points (world + 1 of them) on certificate boundaries, balanced by votes."""
    offs = np.asarray(offsets, dtype=np.int64)
    nv = int(offs[-1])
    cuts = [0]
    for r in range(1, world):
        target = nv * r // world
        c = int(np.searchsorted(offs, target, side="left"))
        cuts.append(int(offs[min(c, len(offs) - 1)]))
    cuts.append(nv)
    return cuts


def merge_words(parts: Sequence[np.ndarray], counts: Sequence[int]) -> np.ndarray:
    """Concatenate per-shard verdict bit arrays (uint64 words, counts[i] valid bits each) into
    one bool array of sum(counts) verdicts."""
    out = []
    for w, c in zip(parts, counts):
        bits = np.unpackbits(np.ascontiguousarray(w).view(np.uint8), bitorder="little")[:c].astype(bool)
        out.append(bits)
    return np.concatenate(out) if out else np.zeros(0, dtype=bool)


def all_gather_words(words, world: int, group=None):
    """All-gather equal-length verdict word tensors from every rank (RCCL on GPU tensors,
    gloo on CPU tensors).  Returns the list of per-rank tensors."""
    import torch
    import torch.distributed as dist
    parts = [torch.empty_like(words) for _ in range(world)]
    dist.all_gather(parts, words, group=group)
    return parts
