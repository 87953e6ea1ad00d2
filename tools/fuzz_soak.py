#!/usr/bin/env python3
"""Fuzz soak (a checking tool, not product code): many seeds of the fuzz
frames of tests/fuzz_frames.py through every kernel the library dispatches
(MTCP_GPU_SCHED wave / row / quad / oct / span / big), compared with the oracle field by
field — rx over the chunk and over a pointer burst (40 B records, the RSS key
and queue count drawn per seed), rx into 16 B records, and the tx fill byte
for byte.  Prints a progress line every 10 seeds and one summary line.
  usage: python tools/fuzz_soak.py [first_seed] [n_seeds] [frames]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402  (the checker)
from mtcp_amd import RESULT_DTYPE, RESULT16_DTYPE, compact_of, gpu  # noqa: E402
from tests.fuzz_frames import fuzz_batch  # noqa: E402

DEV = "cuda:0"
SCHEDS = ("wave", "row", "quad", "oct", "span", "big")


def to_dev(a):
    a = np.ascontiguousarray(a).view(np.uint8)
    pad = (-a.nbytes) % 16
    if pad:
        a = np.concatenate([a, np.zeros(pad, np.uint8)])
    return torch.from_numpy(a.copy()).to(DEV)


def mismatches(got, want, dtype):
    return sum(int((got[f] != want[f]).sum()) for f in dtype.names)


def main():
    first = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    rng = np.random.default_rng(first)
    totals = {"batches": 0, "frames": 0, "rx_mismatch": 0, "ptrs_mismatch": 0,
              "compact_mismatch": 0, "tx_mismatch_bytes": 0}
    verdicts = np.zeros(12, np.int64)
    kernels = {}                      # rx kernels the chunk launches dispatched, and how often
    t0 = time.time()
    for seed in range(first, first + count):
        aligned = bool(seed & 1)
        buf, desc = fuzz_batch(frames, seed, aligned)
        key = oracle.KEY_MICROSOFT if rng.random() < .5 else None
        nq = int(rng.integers(1, 17))
        endian = int(rng.integers(0, 2))
        want = oracle.rx_chunk(buf, desc, 0, oracle.rss_cfg(key, nq, endian))
        verdicts += np.bincount(want["verdict"], minlength=12)
        want16 = compact_of(want)
        tx_want = buf.copy()
        oracle.tx_fill(tx_want, desc, 0)
        n = len(desc)
        for sched in SCHEDS:
            os.environ["MTCP_GPU_SCHED"] = sched
            b = to_dev(buf)
            d = to_dev(desc)
            with gpu.Context(0, rss=True, rss_key=key, rss_queues=nq, rss_endian=bool(endian)) as ctx:
                out = torch.zeros(n * 40, dtype=torch.uint8, device=DEV)
                ctx.rx_chunk_dev(b, d, n, 0, out)
                kernels[ctx.last_kernel] = kernels.get(ctx.last_kernel, 0) + 1
                ptrs = torch.from_numpy(desc["offset"].astype(np.int64) + b.data_ptr()).to(DEV)
                lens = torch.from_numpy(desc["len"].view(np.int16).copy()).to(DEV)
                outp = torch.zeros(n * 40, dtype=torch.uint8, device=DEV)
                ctx.rx_ptrs_dev(ptrs, lens, n, outp)
                torch.cuda.synchronize()
                totals["rx_mismatch"] += mismatches(out.cpu().numpy().view(RESULT_DTYPE), want, RESULT_DTYPE)
                totals["ptrs_mismatch"] += mismatches(outp.cpu().numpy().view(RESULT_DTYPE), want,
                                                      RESULT_DTYPE)
            with gpu.Context(0, rss=True, rss_key=key, rss_queues=nq, rss_endian=bool(endian),
                             compact=True) as ctx:
                out16 = torch.zeros(n * 16, dtype=torch.uint8, device=DEV)
                ctx.rx_chunk_dev(b, d, n, 0, out16)
                torch.cuda.synchronize()
                totals["compact_mismatch"] += mismatches(out16.cpu().numpy().view(RESULT16_DTYPE), want16,
                                                         RESULT16_DTYPE)
            with gpu.Context(0) as ctx:
                ctx.tx_fill_dev(b, d, n, 0)
                torch.cuda.synchronize()
                got = b.cpu().numpy()[:buf.nbytes]
                totals["tx_mismatch_bytes"] += int((got != tx_want).sum())
            totals["batches"] += 1
            totals["frames"] += n
        os.environ.pop("MTCP_GPU_SCHED", None)
        if (seed - first + 1) % 10 == 0:
            print(json.dumps({"progress_seeds": seed - first + 1, "elapsed_s": round(time.time() - t0, 1),
                              **totals}), flush=True)
    print(json.dumps({"probe": "fuzz_soak", "first_seed": first, "seeds": count,
                      "frames_per_batch": frames, "scheds": SCHEDS, **totals,
                      "verdicts_seen": verdicts.tolist(), "kernels": kernels,
                      "seconds": round(time.time() - t0, 1)}),
          flush=True)
    bad = sum(v for k, v in totals.items() if "mismatch" in k)
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
