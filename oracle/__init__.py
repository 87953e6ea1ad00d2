"""TEST INFRASTRUCTURE ONLY — ctypes view of the C oracle (oracle/mtcp_oracle.c).

The oracle is the CPU restatement of mTCP's --disable-hwcsum rx/tx path used
as the parity checker and as bench.py's "port" CPU baseline.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product (mtcp_amd, libmtcp_gpu.so) never does.

`ref` below exposes oracle/_ref/libref_rx.so when it was built in this
container (the reference's own rx code compiled from /root/reference); it is
optional on the GPU box.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmtcp_oracle.so")
REF_LIB_PATH = os.path.join(HERE, "_ref", "libref_rx.so")

# Must match include/mtcp_gpu.h (mtcp_gpu_desc / mtcp_gpu_result).
DESC_DTYPE = np.dtype([("offset", "<u4"), ("len", "<u2"), ("flags", "u1"), ("rsvd", "u1")])
RESULT_DTYPE = np.dtype([
    ("saddr", "<u4"), ("daddr", "<u4"), ("sport", "<u2"), ("dport", "<u2"),
    ("seq", "<u4"), ("ack_seq", "<u4"), ("window", "<u2"), ("ip_len", "<u2"),
    ("ip_csum", "<u2"), ("tcp_csum", "<u2"), ("rss_hash", "<u4"),
    ("payload_len", "<u2"), ("ihl_doff", "u1"), ("tcp_flags", "u1"),
    ("verdict", "u1"), ("rss_queue", "u1"), ("eth_type", "<u2"),
])
assert DESC_DTYPE.itemsize == 8 and RESULT_DTYPE.itemsize == 40

KEY_0X05 = bytes([0x05] * 40)
KEY_MICROSOFT = bytes([
    0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
    0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
    0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa])


class RssCfg(ctypes.Structure):
    _fields_ = [("cache", ctypes.c_uint32 * 96), ("num_queues", ctypes.c_int),
                ("endian_check", ctypes.c_int)]


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64, u16, i32 = (ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64,
                                  ctypes.c_uint16, ctypes.c_int)
        L.oracle_ip_fast_csum.argtypes = [vp, ctypes.c_uint]
        L.oracle_ip_fast_csum.restype = u16
        L.oracle_tcp_calc_checksum.argtypes = [vp, u16, u32, u32]
        L.oracle_tcp_calc_checksum.restype = u16
        L.oracle_build_key_cache.argtypes = [vp, vp, i32]
        L.oracle_get_rss_hash.argtypes = [vp, u32, u32, u16, u16]
        L.oracle_get_rss_hash.restype = u32
        L.oracle_get_rss_cpu_core.argtypes = [vp, u32, u32, u16, u16, i32, i32]
        L.oracle_get_rss_cpu_core.restype = i32
        L.oracle_rss_cfg_init.argtypes = [ctypes.POINTER(RssCfg), vp, i32, i32]
        L.oracle_rx_packet.argtypes = [vp, u32, ctypes.POINTER(RssCfg), vp]
        L.oracle_rx_packet.restype = i32
        L.oracle_rx_chunk.argtypes = [vp, u64, vp, u32, u32, ctypes.POINTER(RssCfg), vp]
        L.oracle_tx_fill.argtypes = [vp, u64, vp, u32, u32]
        L.oracle_tx_fill.restype = u32
        L.oracle_pktgen.argtypes = [vp, u64, vp, u32, u32, u64, u64]
        L.oracle_bench_rx.argtypes = [vp, u64, vp, u32, u32, ctypes.POINTER(RssCfg), vp,
                                      i32, i32]
        L.oracle_bench_rx.restype = ctypes.c_double
        L.oracle_hash_flow.argtypes = [vp]
        L.oracle_hash_flow.restype = u32
        L.oracle_flow_bins.argtypes = [vp, u32, vp]
        L.oracle_addr_pool_search.argtypes = [vp, i32, i32, u32, i32, u32, u16, i32, vp, u32]
        L.oracle_addr_pool_search.restype = u32
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def rss_cfg(key: bytes | None = None, num_queues: int = 1, endian_check: int = 1) -> RssCfg:
    cfg = RssCfg()
    kb = None if key is None else (ctypes.c_uint8 * 40).from_buffer_copy(key)
    lib().oracle_rss_cfg_init(ctypes.byref(cfg), kb, num_queues, endian_check)
    return cfg


def ip_fast_csum(hdr: bytes, ihl: int) -> int:
    b = np.frombuffer(bytes(hdr) + b"\0" * 64, dtype=np.uint8)
    return lib().oracle_ip_fast_csum(_ptr(b), ihl)


def tcp_calc_checksum(seg: bytes, length: int, saddr: int, daddr: int) -> int:
    b = np.frombuffer(bytes(seg) + b"\0" * 2, dtype=np.uint8)
    return lib().oracle_tcp_calc_checksum(_ptr(b), length, saddr, daddr)


def key_cache(key: bytes) -> np.ndarray:
    out = np.zeros(96, dtype=np.uint32)
    kb = np.frombuffer(key, dtype=np.uint8)
    lib().oracle_build_key_cache(_ptr(kb), _ptr(out), 96)
    return out


def rss_hash(cache: np.ndarray, sip: int, dip: int, sp: int, dp: int) -> int:
    return lib().oracle_get_rss_hash(_ptr(cache), sip, dip, sp, dp)


def rss_cpu_core(cache: np.ndarray, sip, dip, sp, dp, nq: int, endian: int) -> int:
    return lib().oracle_get_rss_cpu_core(_ptr(cache), sip, dip, sp, dp, nq, endian)


def rx_chunk(buf: np.ndarray, desc: np.ndarray, off_shift: int = 0,
             rss: RssCfg | None = None) -> np.ndarray:
    out = np.zeros(len(desc), dtype=RESULT_DTYPE)
    lib().oracle_rx_chunk(_ptr(buf), buf.nbytes, _ptr(desc), len(desc), off_shift,
                          ctypes.byref(rss) if rss is not None else None, _ptr(out))
    return out


def tx_fill(buf: np.ndarray, desc: np.ndarray, off_shift: int = 0) -> int:
    return lib().oracle_tx_fill(_ptr(buf), buf.nbytes, _ptr(desc), len(desc), off_shift)


def pktgen(buf: np.ndarray, desc: np.ndarray, off_shift: int, seed: int,
           first_index: int = 0) -> None:
    lib().oracle_pktgen(_ptr(buf), buf.nbytes, _ptr(desc), len(desc), off_shift, seed,
                        first_index)


ADDR_ENTRY_DTYPE = np.dtype([("saddr", "<u4"), ("sport", "<u2"), ("rsvd", "<u2")])


def hash_flow(key12: bytes) -> int:
    """HashFlow (mtcp/src/tcp_stream.c:56-90) of a 12-byte stream key."""
    b = (ctypes.c_uint8 * 12).from_buffer_copy(key12)
    return lib().oracle_hash_flow(ctypes.cast(b, ctypes.c_void_p))


def flow_bins(res: np.ndarray) -> np.ndarray:
    res = np.ascontiguousarray(res, dtype=RESULT_DTYPE)
    bins = np.zeros(len(res), dtype=np.uint32)
    lib().oracle_flow_bins(_ptr(res), len(res), _ptr(bins))
    return bins


def addr_pool_search(key: bytes | None, core: int, num_queues: int, saddr_base: int,
                     num_addr: int, daddr: int, dport: int, endian_check: int = 1,
                     max_out: int | None = None) -> np.ndarray:
    """CreateAddressPoolPerCore's search (mtcp/src/addr_pool.c:103-180)."""
    if max_out is None:
        max_out = num_addr * 64511 // max(num_queues, 1)
    out = np.zeros(max(max_out, 1), dtype=ADDR_ENTRY_DTYPE)
    kb = None
    if key is not None:
        kb = (ctypes.c_uint8 * 40).from_buffer_copy(key)
    n = lib().oracle_addr_pool_search(ctypes.cast(kb, ctypes.c_void_p) if kb else None, core,
                                      num_queues, saddr_base, num_addr, daddr, dport,
                                      endian_check, _ptr(out), max_out)
    return out[:min(n, max_out)]


def bench_rx(buf, desc, off_shift, rss, nthreads, reps, out=None) -> float:
    if out is None:
        out = np.zeros(len(desc), dtype=RESULT_DTYPE)
    return lib().oracle_bench_rx(_ptr(buf), buf.nbytes, _ptr(desc), len(desc), off_shift,
                                 ctypes.byref(rss) if rss is not None else None, _ptr(out),
                                 nthreads, reps)


# ---- the reference's own code (optional: only where oracle/_ref was built) ----
_ref = None


def ref_available() -> bool:
    return os.path.exists(REF_LIB_PATH)


def ref() -> ctypes.CDLL:
    global _ref
    if _ref is None:
        R = ctypes.CDLL(REF_LIB_PATH)
        R.ref_bench_rx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        R.ref_bench_rx.restype = ctypes.c_double
        R.ref_rx_packet.argtypes = [ctypes.c_void_p, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_uint16)]
        R.ref_rx_packet.restype = ctypes.c_int
        _ref = R
    return _ref


def ref_bench_rx(buf, desc, off_shift, rss: bool, nthreads, reps) -> float:
    return ref().ref_bench_rx(_ptr(buf), _ptr(desc), len(desc), off_shift, int(rss),
                              nthreads, reps)
