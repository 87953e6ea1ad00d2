#!/usr/bin/env python3
"""Size-mix soak (a checking tool, not product code): large batches of
IMIX, bimodal, uniform mid-size and random-length frames through the
automatic dispatch (without and with the size hint) and every forced
kernel, each compared with the oracle
field by field (40 B records, RSS on).  One JSON line per batch.
  usage: python tools/mix_soak.py [n]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402  (the checker)
from mtcp_amd import RESULT_DTYPE, gpu, pktgen  # noqa: E402

SCHEDS = ("auto", "auto_hint", "wave", "row", "quad", "oct", "span", "big")


def lengths(kind, n, rng):
    if kind == "imix":
        r = rng.integers(0, 12, n)
        return np.where(r < 7, 64, np.where(r < 11, 576, 1500)).astype(np.uint16)
    if kind == "random":
        return rng.integers(1, 2049, n).astype(np.uint16)
    if kind == "bimodal":
        return pktgen.lengths(n, "bimodal", int(rng.integers(1 << 30)))
    return np.full(n, int(kind), np.uint16)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    rng = np.random.default_rng(2024)
    for kind in ("imix", "random", "bimodal", "128", "256", "384", "512", "768"):
        t0 = time.time()
        desc, nbytes = pktgen.layout_from_lengths(lengths(kind, n, rng), 6)
        buf = np.zeros(nbytes, np.uint8)
        seed = int(rng.integers(1 << 30))
        oracle.pktgen(buf, desc, 6, seed, 0)
        want = oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(None, 8, 1))
        b = torch.from_numpy(buf).to("cuda:0")
        d = torch.from_numpy(desc.view(np.uint8).copy()).to("cuda:0")
        bad, kernels = {}, {}
        for sched in SCHEDS:
            if sched.startswith("auto"):
                os.environ.pop("MTCP_GPU_SCHED", None)
            else:
                os.environ["MTCP_GPU_SCHED"] = sched
            out = torch.full((n * 40,), 0xEE, dtype=torch.uint8, device="cuda:0")
            with gpu.Context(0, rss=True, rss_queues=8, rss_endian=True) as ctx:
                # auto_hint: the batch's true {min, max} length (mtcp_gpu_size_hint)
                hint = (int(desc["len"].min()), int(desc["len"].max())) if sched == "auto_hint" else None
                ctx.rx_chunk_dev(b, d, n, 6, out, hint=hint)
                torch.cuda.synchronize()
                kernels[sched] = ctx.last_kernel
            got = out.cpu().numpy().view(RESULT_DTYPE)
            bad[sched] = int(sum((got[f] != want[f]).sum() for f in RESULT_DTYPE.names))
        os.environ.pop("MTCP_GPU_SCHED", None)
        print(json.dumps({"probe": "mix_soak", "mix": kind, "frames": n, "bytes": nbytes,
                          "tcp_ok": int((want["verdict"] == 0).sum()), "field_mismatches": bad,
                          "kernels": kernels, "seconds": round(time.time() - t0, 1)}), flush=True)
        del b, d
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
