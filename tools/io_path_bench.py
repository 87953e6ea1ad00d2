#!/usr/bin/env python3
"""Rate of the io_module path: mTCP's rx loop
(core.c:763-777) over gpu_module.c wrapping a PSIO-like backend that serves
64-frame bursts from host memory (tests/c/rxloop.c).  Every frame is copied
into the rxq's pinned staging, 64 bursts (4096 frames) go to the GPU per
launch (H2D, rx kernel, D2H of the records), and get_rptr serves the staged
frames.  Frames come from the GPU generator (include/mtcp_gpu_pktgen.h),
copied to host memory first.  Prints one JSON line per frame size.
  usage: python tools/io_path_bench.py [n_frames]
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mtcp_amd import gpu, pktgen  # noqa: E402


def run(n, size, seed, tmp, mode):
    desc, nbytes = pktgen.layout(n, size, 6, seed)
    dev = torch.device("cuda", 0)
    d_buf = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    gpu.pktgen_dev(d_buf, d_desc, n, 6, seed)
    host = d_buf.cpu().numpy()
    bdesc = desc.copy()
    bdesc["offset"] = desc["offset"] << 6          # rxloop takes byte offsets
    chunk, dpath, opath = (os.path.join(tmp, x) for x in ("chunk.bin", "desc.bin", "out.bin"))
    host.tofile(chunk)
    bdesc.tofile(dpath)
    exe = os.path.join(ROOT, "tests", "c", "rxloop")
    best = None
    for _ in range(3):
        r = subprocess.run([exe, chunk, dpath, opath] + (["timing"] if mode == "timing" else []),
                           capture_output=True, text=True, check=True)
        st = json.loads(r.stdout.strip().splitlines()[-1])
        if best is None or st["seconds"] < best["seconds"]:
            best = st
    s = best["seconds"]
    return {"probe": "io_module_path", "mode": mode, "frame_size": size, "frames": n,
            "bursts_per_launch": 64, "burst": 64, "seconds": s,
            "mpkt_per_s": round(n / s / 1e6, 3), "GBs": round(best["frame_bytes"] / s / 1e9, 3),
            "rx_errors": best["rx_errors"], "changed": best["changed"],
            "ioctl_rx_tcp": best["ioctl_rx_tcp"],
            "note": "one mTCP thread: copy into pinned staging + H2D + rx kernel + D2H per 4096 "
                    "frames, get_rptr from staging; mode timing: the first 64 B of each served "
                    "frame read (as ProcessPacket's parse would), mode verify: every served frame "
                    "compared with the original; wall clock of the rx loop, best of 3"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
    with tempfile.TemporaryDirectory() as tmp:
        for size, seed in ((1500, 2), (64, 1), ("bimodal", 3)):
            for mode in ("timing", "verify"):
                print(json.dumps(run(n, size, seed, tmp, mode)), flush=True)


if __name__ == "__main__":
    main()
