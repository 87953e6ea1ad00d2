#!/usr/bin/env python3
"""Frame-size sweep of the rx path (a measurement tool, not product code):
for each fixed frame size, a batch of ~1.5 GB of synthetic frames resident
in HBM, 20 back-to-back mtcp_gpu_rx_chunk_dev launches captured in one HIP
graph, replayed 6 times (3 rounds interleaved with the other kernel
choices of --scheds), HIP events on the launch stream, the median replay's
per-launch time (the C function called with its arguments bound
once: a Python call per launch would time the host for the few-µs
batches), next to the box's read ceiling on the same buffer
(tools/libstream_ceiling.so).  One JSON line per size: the kernel the
dispatcher picked, its time, Σ L / t against 8 TB/s and against the stream.
  usage: python tools/size_sweep.py [--n N] [--no-ceiling] [--ptrs] [--compact] [--hint]
                                    [--scheds auto,auto_hint,wave,...] [sizes...]
  --ptrs: the same frames as a pointer burst (mtcp_gpu_rx_ptrs_dev).
  --hint: pass the batch's (min, max) frame length (mtcp_gpu_rx_chunk_hint_dev),
  as an io_module's rxq does.
  --compact: 16 B records (MTCP_GPU_F_COMPACT) instead of 40 B.
  sizes: bytes, or "bimodal" (C3's 64 / 1500 B mix) or "imix" (64 / 576 /
  1500 B, 7 : 4 : 1); --n fixes the batch (default ~1.5 GB of slots, <= 8 M).
  MTCP_GPU_SCHED=wave|row|quad|oct|span|big forces a kernel (mtcp_gpu.hip)."""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mtcp_amd import _lib, gpu, pktgen  # noqa: E402

SIZES = [64, 128, 256, 384, 512, 768, 1024, 1500, 2048, 4096, 9000]


def ceiling_us(buf, nbytes, stream):
    f = ctypes.CDLL(os.path.join(ROOT, "tools", "libstream_ceiling.so")).stream_ceiling_us
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                  ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]
    us, shape = ctypes.c_float(0.0), ctypes.c_int(0)
    if f(buf.data_ptr(), nbytes, 20, stream.cuda_stream, ctypes.byref(us), ctypes.byref(shape)) != 0:
        raise RuntimeError("stream_ceiling_us failed")
    return float(us.value)


def lengths(n, size):
    if size == "imix":
        r = np.random.default_rng(5).integers(0, 12, n)
        return np.where(r < 7, 64, np.where(r < 11, 576, 1500)).astype(np.uint16)
    return pktgen.lengths(n, size if size == "bimodal" else int(size), 7)


def _graph_times(fn, args, ctx, stream, reps=20):
    """Capture `reps` back-to-back launches in one HIP graph (the C function
    called with its arguments bound once); returns (graph, return codes)."""
    rcs = []
    launch = lambda: rcs.append(fn(ctx._h, *args))  # noqa: E731
    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for _ in range(reps):
            launch()
    g.replay()
    torch.cuda.synchronize()
    return g, rcs


def _replay_us(g, stream, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    g.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    args = sys.argv[1:]
    fixed_n, ceiling, ptrs, compact, hinted, scheds = None, True, False, False, False, None
    while args[:1] in (["--n"], ["--no-ceiling"], ["--ptrs"], ["--compact"], ["--hint"], ["--scheds"]):
        if args[0] == "--n":
            fixed_n, args = int(args[1]), args[2:]
        elif args[0] == "--scheds":
            scheds, args = args[1].split(","), args[2:]
        elif args[0] == "--hint":
            hinted, args = True, args[1:]
        elif args[0] == "--ptrs":
            ptrs, args = True, args[1:]
        elif args[0] == "--compact":
            compact, args = True, args[1:]
        else:
            ceiling, args = False, args[1:]
    sizes = args or SIZES
    # --scheds a,b,...: every kernel choice in ONE process on the same buffer,
    # the timings interleaved round by round (separate processes differ by up
    # to ~9 % for the same kernel); "auto" / "auto_hint" = the dispatcher
    # without / with the size hint, any other name = MTCP_GPU_SCHED forced
    if scheds is None:
        scheds = [os.environ.get("MTCP_GPU_SCHED", "auto") + ("_hint" if hinted else "")]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    L = _lib.lib()
    st = stream.cuda_stream
    for size in sizes:
        slot = 1600 if size in ("bimodal", "imix") else (int(size) + 63) & ~63
        n = fixed_n or min((3 << 29) // slot, 1 << 23)   # ~1.5 GB of slots, at most 8 M frames
        desc, nbytes = pktgen.layout_from_lengths(lengths(n, size), 6)
        buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        d = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
        rec = 16 if compact else 40
        out = torch.empty(n * rec, dtype=torch.uint8, device=dev)
        gpu.pktgen_dev(buf, d, n, 6, 7, stream=stream)
        hint = (ctypes.c_uint16 * 2)(int(desc["len"].min()), int(desc["len"].max()))
        ceil = ceiling_us(buf, nbytes, stream) if ceiling else float("nan")
        runs = []
        saved = os.environ.get("MTCP_GPU_SCHED")
        for sc in scheds:
            if sc.startswith("auto"):
                os.environ.pop("MTCP_GPU_SCHED", None)
            else:
                os.environ["MTCP_GPU_SCHED"] = sc
            ctx = gpu.Context(0, compact=compact)          # reads MTCP_GPU_SCHED at open
            if ptrs:
                p = torch.from_numpy((desc["offset"].astype(np.int64) << 6) + buf.data_ptr()).to(dev)
                ln = torch.from_numpy(desc["len"].view(np.int16).copy()).to(dev)
                fn, fargs = L.mtcp_gpu_rx_ptrs_dev, (p.data_ptr(), ln.data_ptr(), n, out.data_ptr(), st)
                keep = (p, ln)
            else:
                fn = L.mtcp_gpu_rx_chunk_hint_dev
                fargs = (buf.data_ptr(), nbytes, d.data_ptr(), n, 6, out.data_ptr(), None,
                         ctypes.cast(hint, ctypes.c_void_p) if sc.endswith("_hint") else None, st)
                keep = ()
            g, rcs = _graph_times(fn, fargs, ctx, stream)
            if any(rcs):
                raise SystemExit(f"{sc}: launch failed: {[r for r in rcs if r][0]}")
            sha = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
            runs.append(dict(sched=sc, ctx=ctx, g=g, keep=keep, kernel=ctx.last_kernel, sha=sha, us=[]))
        if saved is None:
            os.environ.pop("MTCP_GPU_SCHED", None)
        else:
            os.environ["MTCP_GPU_SCHED"] = saved
        for _ in range(3):                                  # interleaved rounds
            for r in runs:
                for _ in range(2):
                    r["us"].append(_replay_us(r["g"], stream))
        fb = int(desc["len"].astype(np.int64).sum())
        for r in runs:
            us = sorted(r["us"])[len(r["us"]) // 2]
            print(json.dumps({"probe": "size_sweep", "mode": "ptrs" if ptrs else "chunk",
                              "sched": r["sched"], "frame_size": size, "frames": n, "kernel": r["kernel"],
                              "us_per_launch": round(us, 2), "us_min": round(min(r["us"]), 2),
                              "GBs": round(fb / us / 1e3, 1),
                              "gpkt_per_s": round(n / us / 1e3, 3), "frac_of_8TBs": round(fb / us / 8e6, 4),
                              "ceiling_us": round(ceil, 2), "frac_of_ceiling": round(ceil / us, 4),
                              "records_MB": round(n * rec / 1e6, 1), "records_sha": r["sha"]}),
                  flush=True)
            del r["g"]
            r["ctx"].close()
        del buf, d, out, runs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
