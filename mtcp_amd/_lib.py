"""ctypes binding of libmtcp_gpu.so (the C ABI in include/mtcp_gpu.h).

The library is the product: HIP kernels for gfx950 plus the C ABI.  There is
no Python or CPU fallback — if the shared object is missing this module raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libmtcp_gpu.so")

# Every symbol include/mtcp_gpu.h and include/mtcp_gpu_pktgen.h declare.
EXPORTS = (
    "mtcp_gpu_abi_version", "mtcp_gpu_strerror", "mtcp_gpu_device_count", "mtcp_gpu_device_pci_bus_id",
    "mtcp_gpu_open",
    "mtcp_gpu_close", "mtcp_gpu_reserve", "mtcp_gpu_dev_ioctl", "mtcp_gpu_stream", "mtcp_gpu_set_wait_limit",
    "mtcp_gpu_wait_limit",
    "mtcp_gpu_record_size", "mtcp_gpu_last_kernel", "mtcp_gpu_rx_chunk_dev",
    "mtcp_gpu_rx_ptrs_dev", "mtcp_gpu_rx_chunk", "mtcp_gpu_rx_ptrs", "mtcp_gpu_tx_fill_dev",
    "mtcp_gpu_tx_fill", "mtcp_gpu_rx_chunk_flow_dev", "mtcp_gpu_rx_ptrs_flow_dev", "mtcp_gpu_rx_chunk_hint_dev",
    "mtcp_gpu_tx_fill_ptrs_dev", "mtcp_gpu_tx_fill_ptrs", "mtcp_gpu_tx_fill_ptrs_for",
    "mtcp_gpu_host_register", "mtcp_gpu_host_unregister", "mtcp_gpu_sync",
    "mtcp_gpu_flow_hash_dev", "mtcp_gpu_flow_hash", "mtcp_gpu_rss_queue_map_dev",
    "mtcp_gpu_addr_pool_search", "mtcp_gpu_pktgen_dev",
    "mtcp_gpu_rxq_create", "mtcp_gpu_rxq_destroy", "mtcp_gpu_rxq_push", "mtcp_gpu_rxq_push_chunk",
    "mtcp_gpu_rxq_pending", "mtcp_gpu_rxq_flush", "mtcp_gpu_rxq_flush_async", "mtcp_gpu_rxq_wait", "mtcp_gpu_rxq_wait_for", "mtcp_gpu_rxq_get", "mtcp_gpu_rxq_get16", "mtcp_gpu_rxq_frame", "mtcp_gpu_rxq_reset",
)

_lib = None


class MtcpGpuError(RuntimeError):
    def __init__(self, code: int, what: str):
        msg = lib().mtcp_gpu_strerror(code).decode()
        super().__init__(f"{what} failed: {msg} ({code})")
        self.code = code


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make lib` (hipcc --offload-arch=gfx950); "
            "mtcp_amd has no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i32, u16p = (ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64,
                               ctypes.c_int, ctypes.c_void_p)
    sig = {
        "mtcp_gpu_abi_version": ([], i32),
        "mtcp_gpu_strerror": ([i32], ctypes.c_char_p),
        "mtcp_gpu_device_count": ([], i32),
        "mtcp_gpu_device_pci_bus_id": ([i32, ctypes.c_char_p, i32], i32),
        "mtcp_gpu_open": ([ctypes.POINTER(vp), i32, vp, i32, u32], i32),
        "mtcp_gpu_close": ([vp], None),
        "mtcp_gpu_reserve": ([vp, u64, u32], i32),
        "mtcp_gpu_dev_ioctl": ([vp, i32, i32, vp], i32),
        "mtcp_gpu_stream": ([vp], vp),
        "mtcp_gpu_set_wait_limit": ([vp, u32], i32),
        "mtcp_gpu_wait_limit": ([vp], u32),
        "mtcp_gpu_record_size": ([vp], u32),
        "mtcp_gpu_last_kernel": ([vp], ctypes.c_char_p),
        "mtcp_gpu_sync": ([vp], i32),
        "mtcp_gpu_rx_chunk_dev": ([vp, vp, u64, vp, u32, u32, vp, vp], i32),
        "mtcp_gpu_rx_ptrs_dev": ([vp, vp, u16p, u32, vp, vp], i32),
        "mtcp_gpu_rx_chunk": ([vp, vp, u64, vp, u32, u32, vp], i32),
        "mtcp_gpu_rx_ptrs": ([vp, vp, u16p, u32, vp], i32),
        "mtcp_gpu_tx_fill_dev": ([vp, vp, u64, vp, u32, u32, vp], i32),
        "mtcp_gpu_tx_fill": ([vp, vp, u64, vp, u32, u32, ctypes.POINTER(u32)], i32),
        "mtcp_gpu_rx_chunk_flow_dev": ([vp, vp, u64, vp, u32, u32, vp, vp, vp], i32),
        "mtcp_gpu_rx_ptrs_flow_dev": ([vp, vp, u16p, u32, vp, vp, vp], i32),
        "mtcp_gpu_rx_chunk_hint_dev": ([vp, vp, u64, vp, u32, u32, vp, vp, vp, vp], i32),
        "mtcp_gpu_tx_fill_ptrs_dev": ([vp, vp, u16p, u32, vp], i32),
        "mtcp_gpu_tx_fill_ptrs": ([vp, vp, u16p, u32, ctypes.POINTER(u32)], i32),
        "mtcp_gpu_tx_fill_ptrs_for": ([vp, vp, u16p, u32, ctypes.POINTER(u32), u32], i32),
        "mtcp_gpu_host_register": ([vp, u64], i32),
        "mtcp_gpu_host_unregister": ([vp], i32),
        "mtcp_gpu_flow_hash_dev": ([vp, vp, u32, vp, vp], i32),
        "mtcp_gpu_flow_hash": ([vp, vp, u32, vp], i32),
        "mtcp_gpu_rss_queue_map_dev": ([vp, u32, u32, u32, ctypes.c_uint16, i32, i32, vp, vp],
                                       i32),
        "mtcp_gpu_addr_pool_search": ([vp, i32, i32, u32, i32, u32, ctypes.c_uint16, i32, vp, u32,
                                       ctypes.POINTER(u32)], i32),
        "mtcp_gpu_pktgen_dev": ([vp, u64, vp, u32, u32, u64, u64, vp], i32),
        "mtcp_gpu_rxq_create": ([ctypes.POINTER(vp), vp, u32, u64], i32),
        "mtcp_gpu_rxq_destroy": ([vp], None),
        "mtcp_gpu_rxq_push": ([vp, vp, ctypes.c_uint16], i32),
        "mtcp_gpu_rxq_push_chunk": ([vp, vp, vp, u32, u32], i32),
        "mtcp_gpu_rxq_pending": ([vp], u32),
        "mtcp_gpu_rxq_flush": ([vp, ctypes.POINTER(u32)], i32),
        "mtcp_gpu_rxq_flush_async": ([vp], i32),
        "mtcp_gpu_rxq_wait": ([vp, ctypes.POINTER(u32)], i32),
        "mtcp_gpu_rxq_wait_for": ([vp, ctypes.POINTER(u32), u32], i32),
        "mtcp_gpu_rxq_get": ([vp, u32, ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(vp)], vp),
        "mtcp_gpu_rxq_get16": ([vp, u32, ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(vp)], vp),
        "mtcp_gpu_rxq_frame": ([vp, u32, ctypes.POINTER(ctypes.c_uint16)], vp),
        "mtcp_gpu_rxq_reset": ([vp], None),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise MtcpGpuError(rc, what)
