"""The steps of test_gpu_rxq.py::test_a_shutdown_does_not_wait_for_another_contexts_work,
each timed: context A has a 1 s mtcp_gpu_debug_stall queued while context B
opens, creates an rxq, checks 512 golden frames, destroys the rxq and
closes, and C opens, reserves and closes.  One JSON line of step -> seconds."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    assert torch.cuda.is_available()
    from mtcp_amd import gpu
    from mtcp_amd._lib import lib
    from tests.golden_io import load_golden
    L = lib()
    T = ctypes.CDLL(os.path.join(ROOT, "tests", "c", "libmtcp_gpu_testing.so"))
    T.mtcp_gpu_debug_stall.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    g = load_golden()
    base = g.buf.ctypes.data
    part = g.desc[:512]
    out = {}

    def step(name, fn):
        t0 = time.monotonic()
        r = fn()
        out[name] = round(time.monotonic() - t0, 4)
        return r

    def check(ctx, tag):
        q = ctypes.c_void_p()
        step(tag + "rxq_create", lambda: L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, 512, 512 * 2048))
        step(tag + "push", lambda: [L.mtcp_gpu_rxq_push(q, base + int(d["offset"]), int(d["len"])) for d in part])
        n = ctypes.c_uint32()
        step(tag + "flush", lambda: L.mtcp_gpu_rxq_flush(q, ctypes.byref(n)))
        return q

    if "--after-abandon" in sys.argv:
        # test_tx_fill_ptrs_for_gives_up_and_abandons first: a tx fill that
        # times out behind an 800 ms host-stream stall, the context abandoned
        from mtcp_amd._lib import MtcpGpuError
        T.mtcp_gpu_debug_stall.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        offs = g.desc[:64]["offset"].astype("int64")
        z = gpu.Context(0)
        host = g.buf.copy()
        z.tx_fill_ptrs(host, offs, g.desc[:64]["len"], timeout_us=2_000_000)
        assert T.mtcp_gpu_debug_stall(z._h, 800 * 1000) == 0
        try:
            z.tx_fill_ptrs(host, offs, g.desc[:64]["len"], timeout_us=30_000)
        except MtcpGpuError:
            pass
        z.close()
        with gpu.Context(0) as fresh:
            fresh.tx_fill_ptrs(host, offs, g.desc[:64]["len"], timeout_us=2_000_000)
        time.sleep(1.0)                          # the 800 ms stall is over
    a = gpu.Context(0)
    first = gpu.Context(0)
    L.mtcp_gpu_rxq_destroy(check(first, "first_"))
    first.close()
    assert T.mtcp_gpu_debug_stall(a._h, 1_000_000) == 0
    b = step("b_open", lambda: gpu.Context(0))
    q = check(b, "b_")
    step("b_rxq_destroy", lambda: L.mtcp_gpu_rxq_destroy(q))
    step("b_close", b.close)
    c = step("c_open", lambda: gpu.Context(0))
    step("c_reserve", lambda: c.reserve(1 << 20, 1024))
    step("c_close", c.close)
    step("a_sync", lambda: L.mtcp_gpu_sync(a._h))
    a.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
