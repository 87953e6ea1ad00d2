"""Move frames of a chunk to chosen start alignments (test helper).

The reference's checksum and parse results do not depend on where a frame
sits in memory, so a frame moved to another (even) start must get exactly
the record it had before: that is how the 2- and 4-byte-aligned starts the
ABI accepts (include/mtcp_gpu.h mtcp_gpu_desc) are pinned to the golden
vectors.
"""
import numpy as np

from mtcp_amd import DESC_DTYPE


def repack(buf: np.ndarray, desc: np.ndarray, off_shift: int, phase) -> tuple:
    """Copy frame i to phase(i) bytes past the start of a fresh 128 B line
    (phase(i) in 0..127).  Returns (buf, desc) with byte offsets
    (off_shift 0); the buffer is padded to a multiple of 128 B."""
    n = len(desc)
    lens = desc["len"].astype(np.int64)
    src = desc["offset"].astype(np.int64) << off_shift
    offs = np.zeros(n, np.int64)
    pos = 0
    for i in range(n):
        pos = ((pos + 127) & ~127) + int(phase(i))
        offs[i] = pos
        pos += int(lens[i])
    out = np.zeros(((pos + 127) & ~127) + 128, np.uint8)
    for i in range(n):
        out[offs[i]:offs[i] + lens[i]] = buf[src[i]:src[i] + lens[i]]
    d = np.zeros(n, dtype=DESC_DTYPE)
    d["offset"] = offs.astype(np.uint32)
    d["len"] = desc["len"]
    return out, d
