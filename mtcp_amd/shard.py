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


def core_groups(cpus, sysfs: str = "/sys") -> list[list[int]]:
    """`cpus` grouped into physical cores (sysfs
    devices/system/cpu/cpuN/topology/thread_siblings_list), ordered by each
    core's lowest cpu id; a cpu whose topology sysfs does not give is a core
    of its own."""
    import os
    from .gpu import parse_cpulist
    cpus = set(cpus)
    seen: set[int] = set()
    groups: list[list[int]] = []
    for c in sorted(cpus):
        if c in seen:
            continue
        try:
            with open(os.path.join(sysfs, "devices", "system", "cpu", f"cpu{c}", "topology",
                                   "thread_siblings_list")) as f:
                sib = parse_cpulist(f.read()) & cpus
        except (OSError, ValueError):
            sib = set()
        g = sorted(sib | {c})
        seen.update(g)
        groups.append(g)
    return groups


def split_cpus(cpus, index: int, k: int, sysfs: str = "/sys") -> set[int]:
    """The `index`-th of `k` disjoint shares of `cpus`, in whole physical
    cores (no two shares hold SMT siblings of one core): the share-nothing
    split mTCP makes of a node's cores among its per-queue threads
    (mtcp/src/core.c:1195-1213, one thread per core; dpdk_module.c:644-676,
    one queue per thread).  bench.py gives every rank whose GPU sits on the
    same node one share, so that the ranks' concurrent CPU baselines do not
    time the same cores.  With fewer cores than shares the shares wrap."""
    groups = core_groups(cpus, sysfs)
    if not groups or k <= 1:
        return set(cpus)
    if len(groups) < k:
        return set(groups[index % len(groups)])
    lo, hi = len(groups) * index // k, len(groups) * (index + 1) // k
    return {c for g in groups[lo:hi] for c in g}
