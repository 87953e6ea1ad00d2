#!/usr/bin/env python3
"""PCIe-inclusive alternatives on one GPU, C2 frames in pinned host memory:
(a) mtcp_gpu_rx_chunk — DMA staging, 3 streams (what bench.py reports);
(b) the rx kernel reading the registered host chunk directly (zero copy,
    mtcp_gpu_rx_chunk_dev on the host pointer), records to device memory;
(c) as (b) with the records written straight into registered host memory."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtcp_amd import gpu, pktgen  # noqa: E402
from mtcp_amd._lib import lib  # noqa: E402

n, seed = 1 << 20, 2
dev = torch.device("cuda", 0)
desc, nbytes = pktgen.layout(n, 1500, 6, seed)
d_buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
gpu.pktgen_dev(d_buf, d_desc, n, 6, seed)
host = d_buf.cpu().numpy()
del d_buf
frame_bytes = int(desc["len"].astype(np.int64).sum())
ctx = gpu.Context(0)
gpu.host_register(host)
out_h = np.zeros(n, dtype=gpu.RESULT_DTYPE)
gpu.host_register(out_h)
d_out = torch.empty(n * 40, dtype=torch.uint8, device=dev)
L = lib()


def best(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    b = None
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        b = dt if b is None else min(b, dt)
    return frame_bytes / b / 1e9


def staged():
    ctx.rx_chunk(host, desc, 6, out_h)


def zc_dev_out():
    rc = L.mtcp_gpu_rx_chunk_dev(ctx._h, host.ctypes.data, host.nbytes, d_desc.data_ptr(), n, 6,
                                 d_out.data_ptr(), None)
    assert rc == 0, rc
    ctx.sync()


def zc_host_out():
    rc = L.mtcp_gpu_rx_chunk_dev(ctx._h, host.ctypes.data, host.nbytes, d_desc.data_ptr(), n, 6,
                                 out_h.ctypes.data, None)
    assert rc == 0, rc
    ctx.sync()


res = {"staged_dma_GBs": best(staged), "zero_copy_dev_out_GBs": best(zc_dev_out),
       "zero_copy_host_out_GBs": best(zc_host_out)}
ref = out_h.copy()
staged()
same = bool(np.array_equal(ref.view(np.uint8), out_h.view(np.uint8)))
print(json.dumps({**{k: round(v, 2) for k, v in res.items()}, "records_equal": same}))
gpu.host_unregister(out_h)
gpu.host_unregister(host)
