"""Per-launch time of every rx kernel over batch sizes — a wavefront, a row
or a quad per packet (rx_wave.hpp), rx_kernel (64 packets per wave) — each
forced with MTCP_GPU_SCHED at context open, and the dispatched choice, on
the same frames; HIP events on the launch stream over back-to-back launches.
The crossovers set mtcp_gpu.hip pick_sched.
  python tools/small_batch_probe.py [sizes...]    (default: 64 1500 bimodal 9000)
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtcp_amd import gpu, pktgen  # noqa: E402

dev = torch.device("cuda", 0)
# a non-null stream: the kernels and the events share it
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
sizes = [s if s == "bimodal" else int(s) for s in sys.argv[1:]] or [64, 1500, "bimodal", 9000]
NS = [64, 1024, 4096, 16384, 32768, 65536, 131072]
for size in sizes:
    for n in NS:
        desc, nbytes = pktgen.layout(n, size, 6, 7)
        b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        d = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
        o = torch.empty(n * 40, dtype=torch.uint8, device=dev)
        gpu.pktgen_dev(b, d, n, 6, 7, stream=st)
        frame_bytes = int(desc["len"].astype(np.int64).sum())
        line = {"size": size, "n": n, "frame_bytes": frame_bytes}
        ref = None
        for sched in ("wave", "row", "quad", "big", "auto"):
            os.environ["MTCP_GPU_SCHED"] = sched
            with gpu.Context(0, rss=size == "bimodal", rss_queues=8) as ctx:
                for _ in range(10):
                    ctx.rx_chunk_dev(b, d, n, 6, o, stream=st)
                torch.cuda.synchronize()
                reps = 100 if n <= 65536 else 20
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(reps):
                    ctx.rx_chunk_dev(b, d, n, 6, o, stream=st)
                e1.record(st)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / reps * 1e3
                line[f"{sched}_us"] = round(us, 2)
                line[f"{sched}_GBs"] = round(frame_bytes / us / 1e3, 1)
                rec = o.cpu()
                if ref is None:
                    ref = rec
                line["records_equal"] = line.get("records_equal", True) and bool(torch.equal(ref, rec))
        os.environ.pop("MTCP_GPU_SCHED", None)
        print(json.dumps(line), flush=True)
        del b, d, o
