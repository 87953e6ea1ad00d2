"""Batch split across GPUs: contiguous packet ranges, no
collective.  Fixed-size batches split by packet count; variable-size
batches split at the prefix sum of ALIGN(L, 64) so every rank gets equal
bytes.  Each shard's descriptors are rebased to a shard-local chunk, and its
frames are generated from their GLOBAL indices, so shards are byte-identical
slices of the single-GPU batch.  The CPU analogue is mTCP's per-core RSS
queue sharding (mtcp/src/dpdk_module.c:644-676).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import pktgen


@dataclass
class Shard:
    rank: int
    world: int
    first_index: int      # global index of the shard's first packet
    count: int
    desc: np.ndarray      # shard-local descriptors (offsets rebased to 0)
    nbytes: int           # shard chunk size (multiple of 64)


def bounds(n: int, size, world: int, seed: int = 0) -> list[int]:
    """world+1 packet boundaries."""
    if size != "bimodal":
        return [n * r // world for r in range(world + 1)]
    lens = pktgen.lengths(n, size, seed)
    padded = (lens.astype(np.int64) + 63) & ~63
    csum = np.concatenate([[0], np.cumsum(padded)])
    total = int(csum[-1])
    cuts = [int(np.searchsorted(csum, total * r // world, side="left")) for r in range(world + 1)]
    cuts[0], cuts[-1] = 0, n
    return cuts


def make_shard(n: int, size, rank: int, world: int, seed: int = 0, off_shift: int = 6) -> Shard:
    b = bounds(n, size, world, seed)
    first, count = b[rank], b[rank + 1] - b[rank]
    lens = pktgen.lengths(count, size, seed, first_index=first)
    desc, nbytes = pktgen.layout_from_lengths(lens, off_shift)
    return Shard(rank, world, first, count, desc, nbytes)
