#!/usr/bin/env python3
"""Why does tx fill time differently in bench.py and tools/rx_variants?
Times mtcp_gpu_tx_fill_dev and mtcp_gpu_rx_chunk_dev on the same torch
buffer, on a torch stream and on the context's own stream."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtcp_amd import gpu, pktgen  # noqa: E402

n, seed = 1 << 20, 2
dev = torch.device("cuda", 0)
desc, nbytes = pktgen.layout(n, 1500, 6, seed)
d_buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
d_out = torch.empty(n * 40, dtype=torch.uint8, device=dev)
gpu.pktgen_dev(d_buf, d_desc, n, 6, seed)
torch.cuda.synchronize()
ctx = gpu.Context(0)
ts = torch.cuda.Stream(dev)
own = torch.cuda.ExternalStream(ctx.stream)


def t(fn, stream, reps=50):
    for _ in range(5):
        fn(stream)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(reps):
        fn(stream)
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


tx = lambda s: ctx.tx_fill_dev(d_buf, d_desc, n, 6, stream=s)
rx = lambda s: ctx.rx_chunk_dev(d_buf, d_desc, n, 6, d_out, stream=s)
res = {"tx_torch_stream_us": t(tx, ts), "tx_ctx_stream_us": t(tx, own),
       "rx_torch_stream_us": t(rx, ts), "rx_ctx_stream_us": t(rx, own),
       "tx_torch_stream_again_us": t(tx, ts)}
print(json.dumps({k: round(v, 2) for k, v in res.items()}))
