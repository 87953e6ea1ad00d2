"""mtcp_amd — MI355X (gfx950) offload of mTCP's software (--disable-hwcsum)
per-packet path: IPv4/TCP checksums, Eth/IP/TCP header parse + rx verdict,
RSS Toeplitz hash, tx checksum fill.

The product is libmtcp_gpu.so (HIP kernels + the C ABI of include/mtcp_gpu.h);
this package is its Python view for tests and benchmarks.
"""
from ._types import (DESC_DTYPE, RESULT16_DTYPE, RESULT_DTYPE, RX_ERROR_VERDICTS,  # noqa: F401
                     VERDICTS, compact_of)
from . import pktgen  # noqa: F401

__all__ = ["DESC_DTYPE", "RESULT_DTYPE", "RESULT16_DTYPE", "VERDICTS", "RX_ERROR_VERDICTS",
           "compact_of", "pktgen"]
# `from mtcp_amd import gpu` loads libmtcp_gpu.so (and raises if it was not built).
