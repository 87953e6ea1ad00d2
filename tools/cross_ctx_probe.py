"""Does one context's shutdown wait for ANOTHER context's work on the same
device?  Context A queues a 1 s mtcp_gpu_debug_stall (tests/c's testing
library); context B, meanwhile, creates an rxq, checks a batch, destroys the
rxq and closes.  Prints one JSON line with each of B's call times: a call
that frees device memory through a device-wide synchronisation waits for
A's stall (about 1 s)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    assert torch.cuda.is_available()
    from mtcp_amd import gpu, pktgen
    from mtcp_amd._lib import lib
    L = lib()
    T = ctypes.CDLL(os.path.join(ROOT, "tests", "c", "libmtcp_gpu_testing.so"))
    T.mtcp_gpu_debug_stall.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    desc, nbytes = pktgen.layout(256, 1500, 6, 3)
    buf = np.random.default_rng(1).integers(0, 256, nbytes, dtype=np.uint8)
    base = buf.ctypes.data
    out = {}
    a = gpu.Context(0)
    b = gpu.Context(0)
    b.reserve(1 << 20, 1024)
    q = ctypes.c_void_p()
    assert L.mtcp_gpu_rxq_create(ctypes.byref(q), b._h, 256, 256 * 2048) == 0
    assert T.mtcp_gpu_debug_stall(a._h, 1_000_000) == 0
    t0 = time.monotonic()
    for d in desc:
        assert L.mtcp_gpu_rxq_push(q, base + (int(d["offset"]) << 6), int(d["len"])) == 0
    n = ctypes.c_uint32()
    assert L.mtcp_gpu_rxq_flush(q, ctypes.byref(n)) == 0
    out["b_flush_s"] = time.monotonic() - t0
    t1 = time.monotonic()
    L.mtcp_gpu_rxq_destroy(q)
    out["b_rxq_destroy_s"] = time.monotonic() - t1
    t1 = time.monotonic()
    b.close()
    out["b_close_s"] = time.monotonic() - t1
    t1 = time.monotonic()
    assert L.mtcp_gpu_sync(a._h) == 0
    out["a_sync_after_s"] = time.monotonic() - t1
    out["since_stall_s"] = time.monotonic() - t0
    a.close()
    print(json.dumps({k: round(v, 4) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
