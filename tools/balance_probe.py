"""How much of C3's time is per-wave work imbalance?  C3 draws each frame's
size (64 B or 1500 B) independently, so the large-frame count a wave gets
over its 8 passes varies (std ~4.4 %), and the launch ends with the most
loaded waves.  This times the dispatched rx kernel (RSS on, as C3) on
1 M frames whose sizes are
  random     C3 itself (pktgen "bimodal")
  alternate  64 / 1500 by packet parity: every run of 8 packets, hence every
             wave's pass, holds exactly 4 large frames
  runs8      the random sizes, permuted inside each aligned block of 512
             packets so that every run of 8 holds as many large frames as
             the block's average allows (same multiset of sizes per block)
with HIP events on the launch stream over back-to-back launches.
  python tools/balance_probe.py [reps]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtcp_amd import gpu, pktgen  # noqa: E402

N = 1 << 20
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)


def runs8(lens):
    out = lens.copy()
    blk = 512
    for b0 in range(0, len(lens), blk):
        big = int((lens[b0:b0 + blk] == 1500).sum())
        # deal large frames round-robin over the 64 runs of 8 in the block
        runs = np.zeros((blk // 8, 8), dtype=np.uint16) + 64
        for j in range(big):
            runs[j % (blk // 8), j // (blk // 8)] = 1500
        out[b0:b0 + blk] = runs.reshape(-1)
    return out


rnd = pktgen.lengths(N, "bimodal", 7)
cases = {
    "random": rnd,
    "alternate": np.where(np.arange(N) % 2 == 1, 1500, 64).astype(np.uint16),
    "runs8": runs8(rnd),
}
for rnd_round in range(3):
    for name, lens in cases.items():
        desc, nbytes = pktgen.layout_from_lengths(lens, 6)
        b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        d = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
        o = torch.empty(N * 40, dtype=torch.uint8, device=dev)
        gpu.pktgen_dev(b, d, N, 6, 7, stream=st)
        frame_bytes = int(lens.astype(np.int64).sum())
        with gpu.Context(0, rss=True, rss_queues=8) as ctx:
            for _ in range(10):
                ctx.rx_chunk_dev(b, d, N, 6, o, stream=st)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                ctx.rx_chunk_dev(b, d, N, 6, o, stream=st)
            e1.record(st)
            torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print(json.dumps({"round": rnd_round, "case": name, "frame_bytes": frame_bytes,
                          "chunk_bytes": nbytes, "us": round(us, 2),
                          "frac": round(frame_bytes / us / 1e3 / 8000, 4)}), flush=True)
        del b, d, o
