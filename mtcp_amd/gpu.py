"""Python view of the C ABI (include/mtcp_gpu.h) for tests and bench.py.

Device memory and streams come from PyTorch-ROCm (plumbing only); every
computation runs in libmtcp_gpu.so's gfx950 kernels.  Mirrors the
reference's operator boundary: `dev_ioctl` answers like
io_module_func.dev_ioctl (mtcp/src/include/io_module.h:67, :80-87), rx calls
return one verdict per packet in place of ProcessPacket's return value
(mtcp/src/eth_in.c:9-56).
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import numpy as np

from ._lib import check, lib
from ._types import ADDR_ENTRY_DTYPE, DESC_DTYPE, MAX_PORT, MIN_PORT, RESULT16_DTYPE, RESULT_DTYPE

F_RSS = 0x1
F_RSS_ENDIAN = 0x2
F_COMPACT = 0x4

PKT_TX_IP_CSUM = 0x01
PKT_TX_TCP_CSUM = 0x02
PKT_RX_TCP_LROSEG = 0x03
PKT_TX_TCPIP_CSUM = 0x04
PKT_RX_IP_CSUM = 0x05
PKT_RX_TCP_CSUM = 0x06
PKT_TX_TCPIP_CSUM_PEEK = 0x07


def _stream_handle(stream) -> int | None:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream   # torch.cuda.Stream


def _dptr(t) -> int:
    if not t.is_cuda:
        raise ValueError("device-resident entry points take GPU tensors")
    return t.data_ptr()


class Context:
    """One mtcp_gpu_ctx (one per mTCP thread; not re-entrant).

    The `*_dev` methods take GPU tensors and a `stream`: a torch.cuda.Stream
    or a raw hipStream_t handle; None (the default) orders the call after
    the work PyTorch has queued on its current stream, as a torch op would."""

    def __init__(self, device: int = 0, rss: bool = False, rss_key: bytes | None = None,
                 rss_queues: int = 1, rss_endian: bool = True, compact: bool = False):
        L = lib()
        self._h = ctypes.c_void_p()
        flags = (F_RSS if rss else 0) | (F_RSS_ENDIAN if (rss and rss_endian) else 0)
        flags |= F_COMPACT if compact else 0
        key = None
        if rss_key is not None:
            if len(rss_key) != 40:
                raise ValueError("RSS key must be 40 bytes (util/rss.c:84-90)")
            self._key = (ctypes.c_uint8 * 40).from_buffer_copy(rss_key)
            key = ctypes.cast(self._key, ctypes.c_void_p)
        check(L.mtcp_gpu_open(ctypes.byref(self._h), device, key, rss_queues, flags),
              "mtcp_gpu_open")
        self.device = device
        self.compact = compact
        # the rx records this context writes (numpy dtype of one record)
        self.result_dtype = RESULT16_DTYPE if compact else RESULT_DTYPE

    @property
    def record_size(self) -> int:
        return lib().mtcp_gpu_record_size(self._h)

    @property
    def last_kernel(self) -> str:
        """The kernel the last rx / tx launch dispatched (mtcp_gpu_last_kernel)."""
        return lib().mtcp_gpu_last_kernel(self._h).decode()

    # -- lifetime ----------------------------------------------------------
    def close(self) -> None:
        if self._h:
            lib().mtcp_gpu_close(self._h)
            self._h = ctypes.c_void_p()

    @property
    def wait_limit(self) -> int:
        """The bound of every wait of this context's synchronous calls, in us
        (0: none; mtcp_gpu_set_wait_limit)."""
        return lib().mtcp_gpu_wait_limit(self._h)

    @wait_limit.setter
    def wait_limit(self, timeout_us: int) -> None:
        check(lib().mtcp_gpu_set_wait_limit(self._h, timeout_us), "mtcp_gpu_set_wait_limit")

    def reserve(self, max_bytes: int, max_pkts: int) -> None:
        """Allocate the host calls' device staging and load the kernels now
        (mtcp_gpu_reserve), instead of on the first host-buffer call."""
        check(lib().mtcp_gpu_reserve(self._h, max_bytes, max_pkts), "mtcp_gpu_reserve")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return lib().mtcp_gpu_stream(self._h) or 0

    def sync(self) -> None:
        check(lib().mtcp_gpu_sync(self._h), "mtcp_gpu_sync")

    def dev_ioctl(self, cmd: int, nif: int = 0) -> int:
        return lib().mtcp_gpu_dev_ioctl(self._h, nif, cmd, None)

    # -- device-resident ---------------------------------------------------
    @contextlib.contextmanager
    def _ordered(self, stream):
        """The stream handle for one device call.  None: PyTorch's current
        stream OF THIS CONTEXT'S DEVICE (whatever device is current); when
        that is the legacy default stream, which the C-ABI cannot name (NULL
        there means the context's own non-blocking stream), the call is
        ordered by synchronizing that device's default stream before and the
        context's stream after."""
        if stream is not None:
            yield _stream_handle(stream)
            return
        import torch
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream:
            yield cur.cuda_stream
            return
        cur.synchronize()
        yield None
        torch.cuda.ExternalStream(lib().mtcp_gpu_stream(self._h), device=self.device).synchronize()

    def rx_chunk_dev(self, buf, desc, n: int, off_shift: int, out, stream=None, hint=None) -> None:
        """hint: (min_len, max_len) of the batch's frames -> mtcp_gpu_rx_chunk_hint_dev."""
        with self._ordered(stream) as st:
            if hint is None:
                check(lib().mtcp_gpu_rx_chunk_dev(self._h, _dptr(buf), buf.numel() * buf.element_size(),
                                                  _dptr(desc), n, off_shift, _dptr(out),
                                                  st), "mtcp_gpu_rx_chunk_dev")
            else:
                h = (ctypes.c_uint16 * 2)(*hint)
                check(lib().mtcp_gpu_rx_chunk_hint_dev(self._h, _dptr(buf), buf.numel() * buf.element_size(),
                                                       _dptr(desc), n, off_shift, _dptr(out), None,
                                                       ctypes.cast(h, ctypes.c_void_p), st),
                      "mtcp_gpu_rx_chunk_hint_dev")

    def rx_ptrs_dev(self, ptrs, lens, n: int, out, stream=None) -> None:
        with self._ordered(stream) as st:
            check(lib().mtcp_gpu_rx_ptrs_dev(self._h, _dptr(ptrs), _dptr(lens), n, _dptr(out),
                                             st), "mtcp_gpu_rx_ptrs_dev")

    def rx_chunk_flow_dev(self, buf, desc, n: int, off_shift: int, out, bins, stream=None) -> None:
        with self._ordered(stream) as st:
            check(lib().mtcp_gpu_rx_chunk_flow_dev(self._h, _dptr(buf), buf.numel() * buf.element_size(),
                                                   _dptr(desc), n, off_shift, _dptr(out), _dptr(bins),
                                                   st), "mtcp_gpu_rx_chunk_flow_dev")

    def rx_ptrs_flow_dev(self, ptrs, lens, n: int, out, bins, stream=None) -> None:
        with self._ordered(stream) as st:
            check(lib().mtcp_gpu_rx_ptrs_flow_dev(self._h, _dptr(ptrs), _dptr(lens), n, _dptr(out),
                                                  _dptr(bins), st),
                  "mtcp_gpu_rx_ptrs_flow_dev")

    def tx_fill_ptrs_dev(self, ptrs, lens, n: int, stream=None) -> None:
        with self._ordered(stream) as st:
            check(lib().mtcp_gpu_tx_fill_ptrs_dev(self._h, _dptr(ptrs), _dptr(lens), n,
                                                  st), "mtcp_gpu_tx_fill_ptrs_dev")

    def tx_fill_dev(self, buf, desc, n: int, off_shift: int, stream=None) -> None:
        with self._ordered(stream) as st:
            check(lib().mtcp_gpu_tx_fill_dev(self._h, _dptr(buf), buf.numel() * buf.element_size(),
                                             _dptr(desc), n, off_shift, st),
                  "mtcp_gpu_tx_fill_dev")

    # -- host memory ---------------------------------------------------------
    def rx_chunk(self, buf: np.ndarray, desc: np.ndarray, off_shift: int = 0,
                 out: np.ndarray | None = None) -> np.ndarray:
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        if out is None:
            out = np.zeros(len(desc), dtype=self.result_dtype)
        if out.dtype.itemsize != self.result_dtype.itemsize:
            raise ValueError("out must hold this context's records (compact: 16 B)")
        check(lib().mtcp_gpu_rx_chunk(self._h, buf.ctypes.data, buf.nbytes, desc.ctypes.data,
                                      len(desc), off_shift, out.ctypes.data), "mtcp_gpu_rx_chunk")
        return out

    def rx_ptrs(self, frames: list) -> np.ndarray:
        n = len(frames)
        arrs = [np.ascontiguousarray(np.frombuffer(bytes(f), dtype=np.uint8)) for f in frames]
        ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
        lens = np.array([a.nbytes for a in arrs], dtype=np.uint16)
        out = np.zeros(n, dtype=self.result_dtype)
        check(lib().mtcp_gpu_rx_ptrs(self._h, ctypes.cast(ptrs, ctypes.c_void_p),
                                     lens.ctypes.data, n, out.ctypes.data), "mtcp_gpu_rx_ptrs")
        return out

    def tx_fill(self, buf: np.ndarray, desc: np.ndarray, off_shift: int = 0) -> int:
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        cnt = ctypes.c_uint32(0)
        check(lib().mtcp_gpu_tx_fill(self._h, buf.ctypes.data, buf.nbytes, desc.ctypes.data,
                                     len(desc), off_shift, ctypes.byref(cnt)), "mtcp_gpu_tx_fill")
        return cnt.value

    def tx_fill_ptrs(self, buf: np.ndarray, offsets, lens, timeout_us: int | None = None) -> int:
        """mtcp_gpu_tx_fill_ptrs over frames of the host array `buf` at byte
        `offsets` (a DPDK-style pointer burst into one host buffer); fills
        `buf` in place and returns the number of frames filled.  With
        timeout_us: mtcp_gpu_tx_fill_ptrs_for (MtcpGpuError ETIMEDOUT past
        the limit, the context abandoned; 0: the context's wait limit)."""
        offsets = np.asarray(offsets, dtype=np.int64)
        n = len(offsets)
        ptrs = (ctypes.c_void_p * max(n, 1))(*[buf.ctypes.data + int(o) for o in offsets])
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        cnt = ctypes.c_uint32(0)
        if timeout_us is None:
            check(lib().mtcp_gpu_tx_fill_ptrs(self._h, ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data,
                                              n, ctypes.byref(cnt)), "mtcp_gpu_tx_fill_ptrs")
        else:
            check(lib().mtcp_gpu_tx_fill_ptrs_for(self._h, ctypes.cast(ptrs, ctypes.c_void_p),
                                                  lens.ctypes.data, n, ctypes.byref(cnt), timeout_us),
                  "mtcp_gpu_tx_fill_ptrs_for")
        return cnt.value

    # -- flow-table hash (HashFlow, mtcp/src/tcp_stream.c:56-90) -------------
    def flow_hash_dev(self, res, n: int, bins, stream=None) -> None:
        with self._ordered(stream) as st:
            check(lib().mtcp_gpu_flow_hash_dev(self._h, _dptr(res), n, _dptr(bins),
                                               st), "mtcp_gpu_flow_hash_dev")

    def flow_hash(self, res: np.ndarray) -> np.ndarray:
        res = np.ascontiguousarray(res, dtype=RESULT_DTYPE)
        bins = np.zeros(len(res), dtype=np.uint32)
        check(lib().mtcp_gpu_flow_hash(self._h, res.ctypes.data, len(res), bins.ctypes.data),
              "mtcp_gpu_flow_hash")
        return bins

    # -- RSS-friendly address pool (mtcp/src/addr_pool.c:103-180) ------------
    def rss_queue_map_dev(self, saddr_base_h: int, num_addr: int, daddr_h: int, dport_h: int,
                          num_queues: int, endian_check: bool, queue, stream=None) -> None:
        if queue.numel() * queue.element_size() < num_addr * (MAX_PORT - MIN_PORT):
            raise ValueError("queue buffer too small")
        with self._ordered(stream) as st:
            check(lib().mtcp_gpu_rss_queue_map_dev(self._h, saddr_base_h, num_addr, daddr_h, dport_h,
                                                   num_queues, int(endian_check), _dptr(queue),
                                                   st),
                  "mtcp_gpu_rss_queue_map_dev")

    def addr_pool_search(self, core: int, num_queues: int, saddr_base: int, num_addr: int,
                         daddr: int, dport: int, endian_check: bool = True,
                         max_out: int | None = None) -> np.ndarray:
        """CreateAddressPoolPerCore's entries for `core` (network-order arguments,
        as the reference's); returns the ADDR_ENTRY_DTYPE records in pool order."""
        if max_out is None:
            max_out = num_addr * (MAX_PORT - MIN_PORT) // max(num_queues, 1)
        out = np.zeros(max(max_out, 1), dtype=ADDR_ENTRY_DTYPE)
        found = ctypes.c_uint32(0)
        check(lib().mtcp_gpu_addr_pool_search(self._h, core, num_queues, saddr_base, num_addr,
                                              daddr, dport, int(endian_check), out.ctypes.data,
                                              max_out, ctypes.byref(found)),
              "mtcp_gpu_addr_pool_search")
        return out[:min(found.value, max_out)]


def parse_cpulist(text: str) -> set[int]:
    """The kernel's cpulist format ("0-3,8,10-11") as a set of cpu ids."""
    cpus: set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def device_pci_bus_id(device: int) -> str:
    """PCI address of `device` ("0000:a7:00.0"), lower case as sysfs names it."""
    buf = ctypes.create_string_buffer(64)
    check(lib().mtcp_gpu_device_pci_bus_id(device, buf, len(buf)), "mtcp_gpu_device_pci_bus_id")
    return buf.value.decode().lower()


def device_local_cpus(device: int, sysfs: str = "/sys") -> tuple[str, set[int]]:
    """The cpus on `device`'s side of the host (sysfs
    bus/pci/devices/<bdf>/local_cpulist): where a process that stages frames
    for this GPU should run so that its host buffers (first-touched by it) sit
    on the GPU's socket.  mTCP keeps each thread and its memory on one node
    the same way (mtcp_core_affinitize, mtcp/src/cpu.c:54-79; DPDK queues on
    the NIC's socket, dpdk_module.c:660-663; gpu_module.c picks the GPU by the
    thread's node, gpu_topo.h).  An empty set when sysfs does not tell."""
    bdf = device_pci_bus_id(device)
    try:
        with open(os.path.join(sysfs, "bus", "pci", "devices", bdf, "local_cpulist")) as f:
            return bdf, parse_cpulist(f.read())
    except (OSError, ValueError):
        return bdf, set()


def host_register(arr: np.ndarray) -> None:
    check(lib().mtcp_gpu_host_register(arr.ctypes.data, arr.nbytes), "mtcp_gpu_host_register")


def host_unregister(arr: np.ndarray) -> None:
    check(lib().mtcp_gpu_host_unregister(arr.ctypes.data), "mtcp_gpu_host_unregister")


def pktgen_dev(buf, desc, n: int, off_shift: int, seed: int, first_index: int = 0,
               stream=None) -> None:
    """Synthetic frames on the GPU (include/mtcp_gpu_pktgen.h)."""
    check(lib().mtcp_gpu_pktgen_dev(_dptr(buf), buf.numel() * buf.element_size(), _dptr(desc),
                                    n, off_shift, seed, first_index, _stream_handle(stream)),
          "mtcp_gpu_pktgen_dev")


def results_view(t) -> np.ndarray:
    """A device result buffer (uint8 tensor of n*40 bytes) as a numpy record array."""
    return t.cpu().numpy().view(RESULT_DTYPE)
