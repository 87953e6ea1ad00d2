"""Which build a PMC traffic figure belongs to.

bench.py reports `roofline.traffic` from a rocprofv3 PMC profile of a
previous run (tools/profile_config.sh -> profiles/traffic_<cfg>.json).  The
profile records two keys:
  lib_sha256     the exact libmtcp_gpu.so that was profiled;
  rx_source_key  the sources that decide the rx kernels' code and their
                 dispatch (rx_kernels.hpp, rx_wave.hpp — C1's quad kernel —, rx_span.hpp,
                 mtcp_gpu.hip, dispatch.hpp, include/mtcp_gpu.h, the Makefile's flags).
bench.py uses the figure when the loaded library is the profiled one, or
when it differs only outside those sources (e.g. a small-batch kernel or
host-path change), and says which; otherwise the figure is reported stale.
(Hashing the rx_kernel symbols' machine code instead was tried: their bytes
move when an unrelated kernel in the same code object changes.)
"""
from __future__ import annotations

import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RX_SOURCES = ("mtcp_amd/csrc/rx_kernels.hpp", "mtcp_amd/csrc/rx_wave.hpp", "mtcp_amd/csrc/rx_span.hpp",
              "mtcp_amd/csrc/mtcp_gpu.hip", "mtcp_amd/csrc/dispatch.hpp", "include/mtcp_gpu.h", "Makefile")


def rx_source_key(root: str = ROOT) -> str:
    h = hashlib.sha256()
    for rel in RX_SOURCES:
        h.update(rel.encode())
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def lib_sha256(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()
