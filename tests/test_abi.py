"""CPU-side checks of the drop-in boundary: libmtcp_gpu.so loads, exports
every symbol include/*.h declares, mirrors the reference's dev_ioctl command
values, and fails loudly (no CPU fallback) when no GPU is present."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in sorted(f for f in os.listdir(os.path.join(ROOT, "include")) if f.endswith(".h")):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(mtcp_gpu_\w+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    from mtcp_amd import _lib
    lib = _lib.lib()
    decl = declared_functions()
    assert decl == set(_lib.EXPORTS), decl ^ set(_lib.EXPORTS)
    for name in decl:
        assert hasattr(lib, name), name
    assert lib.mtcp_gpu_abi_version() == 5
    assert lib.mtcp_gpu_strerror(-22) == b"invalid argument"


def test_ioctl_constants_match_reference():
    """io_module.h:80-87 command values."""
    hdr = open(os.path.join(ROOT, "include", "mtcp_gpu.h")).read()
    want = {"PKT_TX_IP_CSUM": 0x01, "PKT_TX_TCP_CSUM": 0x02, "PKT_RX_TCP_LROSEG": 0x03,
            "PKT_TX_TCPIP_CSUM": 0x04, "PKT_RX_IP_CSUM": 0x05, "PKT_RX_TCP_CSUM": 0x06,
            "PKT_TX_TCPIP_CSUM_PEEK": 0x07, "DRV_NAME": 0x08}
    for k, v in want.items():
        m = re.search(r"#define MTCP_GPU_%s\s+(0x[0-9a-fA-F]+)" % k, hdr)
        assert m and int(m.group(1), 16) == v, k


def test_struct_layouts():
    from mtcp_amd import DESC_DTYPE, RESULT_DTYPE
    assert DESC_DTYPE.itemsize == 8          # == struct ps_pkt_info (ps.h:181-185)
    assert RESULT_DTYPE.itemsize == 40
    assert RESULT_DTYPE.fields["verdict"][1] == 36
    assert RESULT_DTYPE.fields["eth_type"][1] == 38
    from mtcp_amd import RESULT16_DTYPE
    assert RESULT16_DTYPE.itemsize == 16       # mtcp_gpu_result16 (MTCP_GPU_F_COMPACT)
    assert RESULT16_DTYPE.fields["verdict"][1] == 14
    assert RESULT16_DTYPE.fields["rss_hash"][1] == 0
    hdr = open(os.path.join(ROOT, "include", "mtcp_gpu.h")).read()
    assert re.search(r"uint8_t\s+verdict;\s+/\* 14 \*/", hdr)


def test_compact_projection_keeps_same_named_fields():
    import numpy as np
    from mtcp_amd import RESULT16_DTYPE, RESULT_DTYPE, compact_of
    r = np.zeros(3, RESULT_DTYPE)
    r["verdict"] = [0, 9, 4]
    r["tcp_csum"] = [0, 0x1234, 0]
    r["rss_hash"] = [1, 2, 0xFFFFFFFF]
    r["ihl_doff"] = [0x55, 0x85, 5]
    c = compact_of(r)
    assert c.dtype == RESULT16_DTYPE
    for f in RESULT16_DTYPE.names:
        assert np.array_equal(c[f], r[f]), f


def test_no_gpu_no_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from mtcp_amd import gpu
    from mtcp_amd._lib import MtcpGpuError
    with pytest.raises(MtcpGpuError):
        gpu.Context(0)


def test_default_stream_is_the_contexts_device(monkeypatch):
    """with stream=None a device call is ordered on PyTorch's
    current stream of the CONTEXT's device, not of whatever device is current
    (a context on device 1 must never be queued on device 0's stream)."""
    import torch
    from mtcp_amd import gpu
    asked = []

    class _S:
        cuda_stream = 0xBEEF

    def fake_current_stream(device=None):
        asked.append(device)
        return _S()

    monkeypatch.setattr(torch.cuda, "current_stream", fake_current_stream)
    ctx = object.__new__(gpu.Context)
    ctx._h = ctypes.c_void_p()
    ctx.device = 3
    with ctx._ordered(None) as st:
        assert st == 0xBEEF
    assert asked == [3]
    with ctx._ordered(0x1234) as st:                # an explicit stream is used as given
        assert st == 0x1234
    assert asked == [3]
