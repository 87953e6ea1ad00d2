"""Host-side layout of synthetic packet batches (BASELINE.json configs).

Frame lengths follow SURVEY §8(d): "X B packet" = frame length L as get_rptr
returns it (mtcp/src/dpdk_module.c:467); packet i sits at
sum_{j<i} ALIGN(L_j, 64), the PSIO chunk layout (io_engine/lib/pslib.c:146).
The bytes themselves are written on the GPU by mtcp_gpu_pktgen_dev
(include/mtcp_gpu_pktgen.h).
"""
from __future__ import annotations

import numpy as np

from ._types import DESC_DTYPE

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def lengths(n: int, size, seed: int = 0, first_index: int = 0) -> np.ndarray:
    """Frame lengths: an int for fixed-size batches, or "bimodal" for
    L in {64, 1500} with p = 0.5 per packet (config C3), a pure function of
    (seed, global packet index)."""
    if size == "bimodal":
        with np.errstate(over="ignore"):
            i = np.arange(first_index, first_index + n, dtype=np.uint64)
            z = i * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed) * np.uint64(0xD6E8FEB86659FD93)
            z = _mix(z)
        return np.where((z & np.uint64(1)) == 1, 1500, 64).astype(np.uint16)
    return np.full(n, int(size), dtype=np.uint16)


def layout_from_lengths(lens: np.ndarray, off_shift: int = 6):
    """Descriptors for a contiguous 64 B-aligned chunk; returns (desc, bytes)."""
    padded = (lens.astype(np.uint64) + np.uint64(63)) & ~np.uint64(63)
    ends = np.cumsum(padded, dtype=np.uint64)
    starts = ends - padded
    desc = np.zeros(len(lens), dtype=DESC_DTYPE)
    desc["offset"] = (starts >> np.uint64(off_shift)).astype(np.uint32)
    desc["len"] = lens
    total = int(ends[-1]) if len(lens) else 0
    return desc, total


def layout(n: int, size, off_shift: int = 6, seed: int = 0, first_index: int = 0):
    return layout_from_lengths(lengths(n, size, seed, first_index), off_shift)
