"""One batch shape through mtcp_gpu_rx_chunk_dev, launched `reps` times back
to back, for a rocprofv3 kernel trace of the dispatched small-batch kernel:
  rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/small_batch_trace.py 1500 4096 200 [graph]
The per-dispatch durations (profiles/r2/small_batch_trace_*.csv) are the
kernel's own begin->end; HIP events over the same back-to-back launches
(printed here) add the launch gaps.  "graph": the launches are captured in
one HIP graph and replayed, so they reach the GPU back to back (as from an
io_module thread calling the C ABI directly), not at the Python call's rate."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtcp_amd import gpu, pktgen  # noqa: E402

size = sys.argv[1] if len(sys.argv) > 1 else "1500"
size = size if size == "bimodal" else int(size)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
graph = len(sys.argv) > 4 and sys.argv[4] == "graph"
dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
desc, nbytes = pktgen.layout(n, size, 6, 7)
b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
d = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
o = torch.empty(n * 40, dtype=torch.uint8, device=dev)
gpu.pktgen_dev(b, d, n, 6, 7, stream=st)
with gpu.Context(0, rss=size == "bimodal", rss_queues=8) as ctx:
    for _ in range(20):
        ctx.rx_chunk_dev(b, d, n, 6, o, stream=st)
    torch.cuda.synchronize()
    kernel = ctx.last_kernel
    run = None
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                ctx.rx_chunk_dev(b, d, n, 6, o, stream=st)
        g.replay()
        torch.cuda.synchronize()
        run = g.replay
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    if run:
        run()
    else:
        for _ in range(reps):
            ctx.rx_chunk_dev(b, d, n, 6, o, stream=st)
    e1.record(st)
    torch.cuda.synchronize()
frame_bytes = int(desc["len"].astype(np.int64).sum())
us = e0.elapsed_time(e1) / reps * 1e3
print(json.dumps({"size": size, "n": n, "reps": reps, "graph": graph, "kernel": kernel,
                  "frame_bytes": frame_bytes,
                  "events_us_per_launch": round(us, 2), "GBs": round(frame_bytes / us / 1e3, 1)}))
