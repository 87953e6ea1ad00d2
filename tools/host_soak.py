#!/usr/bin/env python3
"""Host-path soak (a checking tool, not product code): many seeds of the fuzz
frames of tests/fuzz_frames.py through the HOST entry points of the C ABI —
mtcp_gpu_rx_chunk over sorted and shuffled descriptors, mtcp_gpu_rx_ptrs,
mtcp_gpu_tx_fill and mtcp_gpu_tx_fill_ptrs (the report mode both use since
round 6) — each on a context without and with a wait limit (the bounded form
stages every byte through pinned bounce buffers), compared with the oracle
field by field and byte for byte.  Prints a progress line every 10 seeds and
one summary line; exit status 1 on any mismatch.
  usage: python tools/host_soak.py [first_seed] [n_seeds] [frames]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402  (the checker)
from mtcp_amd import RESULT_DTYPE, gpu  # noqa: E402
from tests.fuzz_frames import fuzz_batch  # noqa: E402


def mismatches(got, want):
    return sum(int((got[f] != want[f]).sum()) for f in RESULT_DTYPE.names)


def main():
    first = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    rng = np.random.default_rng(first)
    totals = {"batches": 0, "frames": 0, "rx_mismatch": 0, "rx_unsorted_mismatch": 0, "ptrs_mismatch": 0,
              "tx_mismatch_bytes": 0, "tx_ptrs_mismatch_bytes": 0, "tx_count_mismatch": 0}
    t0 = time.time()
    for seed in range(first, first + count):
        aligned = bool(seed & 1)
        buf, desc = fuzz_batch(frames, seed, aligned)
        key = oracle.KEY_MICROSOFT if rng.random() < .5 else None
        nq = int(rng.integers(1, 17))
        endian = int(rng.integers(0, 2))
        want = oracle.rx_chunk(buf, desc, 0, oracle.rss_cfg(key, nq, endian))
        perm = rng.permutation(len(desc))
        tx_want = buf.copy()
        n_want = oracle.tx_fill(tx_want, desc, 0)
        # the pointer forms take even frame starts inside the buffer (as DPDK's mbufs)
        ok = (desc["offset"] % 2 == 0) & (desc["offset"].astype(np.int64) + desc["len"] <= buf.nbytes)
        pdesc = desc[ok]
        pwant = oracle.rx_chunk(buf, pdesc, 0, oracle.rss_cfg(key, nq, endian))
        ptx_want = buf.copy()
        oracle.tx_fill(ptx_want, pdesc, 0)
        frames_list = [buf[int(o):int(o) + int(ln)].tobytes() for o, ln in zip(pdesc["offset"], pdesc["len"])]
        for limit in (0, 5_000_000):
            with gpu.Context(0, rss=True, rss_key=key, rss_queues=nq, rss_endian=bool(endian)) as ctx:
                ctx.wait_limit = limit
                got = ctx.rx_chunk(buf, desc, 0)
                totals["rx_mismatch"] += mismatches(got, want)
                got = ctx.rx_chunk(buf, desc[perm], 0)
                totals["rx_unsorted_mismatch"] += mismatches(got, want[perm])
                got = ctx.rx_ptrs(frames_list)
                totals["ptrs_mismatch"] += mismatches(got, pwant)
            with gpu.Context(0) as ctx:
                ctx.wait_limit = limit
                host = buf.copy()
                n = ctx.tx_fill(host, desc, 0)
                totals["tx_mismatch_bytes"] += int((host != tx_want).sum())
                totals["tx_count_mismatch"] += int(n != n_want)
                host = buf.copy()
                ctx.tx_fill_ptrs(host, pdesc["offset"].astype(np.int64), pdesc["len"])
                totals["tx_ptrs_mismatch_bytes"] += int((host != ptx_want).sum())
            totals["batches"] += 1
            totals["frames"] += len(desc)
        if (seed - first + 1) % 10 == 0:
            print(json.dumps({"progress_seeds": seed - first + 1, "elapsed_s": round(time.time() - t0, 1),
                              **totals}), flush=True)
    print(json.dumps({"probe": "host_soak", "first_seed": first, "seeds": count, "frames_per_batch": frames,
                      "limits_us": [0, 5_000_000], **totals, "seconds": round(time.time() - t0, 1)}), flush=True)
    bad = sum(v for k, v in totals.items() if "mismatch" in k)
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
