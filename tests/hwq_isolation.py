"""Child process of tests/test_gpu_bounded.py::test_one_threads_stall_does_not_delay_another
(run as `python -m tests.hwq_isolation`; GPU box only).

Two mTCP threads' GPU resources as gpu_module.c sets them up with
MTCP_GPU_TX=1 (mtcp_amd/io_module/gpu_module.c gpu_init_handle): per thread
a compact context with a wait limit, kernels loaded at init, two pipelined
rxqs, tx fills of the frames get_wptr handed out.  No torch in this process,
so the process's HIP streams are exactly the contexts' (mtcp_gpu.h: one per
context).  Both threads check an aggregate and fill a tx burst (every stream
the threads use exists); then thread A's context gets a 1 s stall with its
next aggregate queued behind it, and thread B checks an aggregate and fills
a burst.  Prints one JSON line: how long B took, whether B's records and
frames are the oracle's, and whether A's stall was still running when B
was done.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from mtcp_amd import RESULT16_DTYPE, compact_of  # noqa: E402
from mtcp_amd._lib import lib  # noqa: E402
from tests.golden_io import load_golden  # noqa: E402

F_COMPACT = 0x4
AGG = 512


class Thread:
    """One mTCP thread's GPU context and rxqs (gpu_module.c's per-thread state)."""

    def __init__(self, L, wait_us):
        self.L = L
        self.h = ctypes.c_void_p()
        assert L.mtcp_gpu_open(ctypes.byref(self.h), 0, None, 1, F_COMPACT) == 0
        assert L.mtcp_gpu_set_wait_limit(self.h, wait_us) == 0
        assert L.mtcp_gpu_reserve(self.h, 0, 0) == 0
        self.q = []
        for _ in range(2):
            q = ctypes.c_void_p()
            assert L.mtcp_gpu_rxq_create(ctypes.byref(q), self.h, 4096, 4096 * 2048) == 0
            self.q.append(q)

    def push(self, k, buf, desc):
        L, q = self.L, self.q[k]
        L.mtcp_gpu_rxq_reset(q)
        for d in desc:
            assert L.mtcp_gpu_rxq_push(q, buf.ctypes.data + int(d["offset"]), int(d["len"])) == 0

    def records(self, k, n):
        out = np.zeros(n, RESULT16_DTYPE)
        for i in range(n):
            res = ctypes.c_void_p()
            self.L.mtcp_gpu_rxq_get16(self.q[k], i, None, ctypes.byref(res))
            out[i] = np.frombuffer(ctypes.string_at(res.value, 16), RESULT16_DTYPE)[0]
        return out

    def tx_fill(self, host, desc):
        ptrs = (ctypes.c_void_p * len(desc))(*[host.ctypes.data + int(o) for o in desc["offset"]])
        lens = np.ascontiguousarray(desc["len"])
        cnt = ctypes.c_uint32(0)
        rc = self.L.mtcp_gpu_tx_fill_ptrs_for(self.h, ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data,
                                              len(desc), ctypes.byref(cnt), 0)
        return rc, cnt.value


def main():
    L = lib()
    T = ctypes.CDLL(os.path.join(ROOT, "tests", "c", "libmtcp_gpu_testing.so"))
    T.mtcp_gpu_debug_stall.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    # the HIP runtime libmtcp_gpu.so loaded (its path from this process's maps)
    hip_path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    hip = ctypes.CDLL(hip_path)
    hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
    g = load_golden()
    part = g.desc[:AGG]
    want40 = oracle.rx_chunk(g.buf, part, 0)
    want_rx = compact_of(want40)
    # a descriptor the reference finds misaligned is restaged at an aligned
    # slot by the rxq (gpu_module.c copies frames): its record is not compared
    cmp = want40["verdict"] != 11
    tx_desc = g.desc[:64]
    tx_want = g.buf.copy()
    oracle.tx_fill(tx_want, tx_desc, 0)

    a, b = Thread(L, 2_000_000), Thread(L, 2_000_000)
    for t in (a, b):                 # every stream each thread uses exists from here on
        t.push(0, g.buf, part)
        n = ctypes.c_uint32()
        assert L.mtcp_gpu_rxq_flush(t.q[0], ctypes.byref(n)) == 0 and n.value == AGG
        host = g.buf.copy()
        assert t.tx_fill(host, tx_desc)[0] == 0 and np.array_equal(host, tx_want)

    a_stream = L.mtcp_gpu_stream(a.h)
    assert T.mtcp_gpu_debug_stall(a.h, 1_000_000) == 0
    a.push(1, g.buf, part)
    assert L.mtcp_gpu_rxq_flush_async(a.q[1]) == 0        # A's next aggregate, behind the stall

    t0 = time.monotonic()
    b.push(1, g.buf, part)
    n = ctypes.c_uint32()
    rc_rx = L.mtcp_gpu_rxq_flush(b.q[1], ctypes.byref(n))
    host = g.buf.copy()
    rc_tx, filled = b.tx_fill(host, tx_desc)
    b_s = time.monotonic() - t0
    a_busy = hip.hipStreamQuery(a_stream) != 0                # hipErrorNotReady: A's stall still runs
    b_records_ok = rc_rx == 0 and n.value == AGG and b.records(1, AGG)[cmp].tobytes() == want_rx[cmp].tobytes()
    b_tx_ok = rc_tx == 0 and np.array_equal(host, tx_want)

    n_a = ctypes.c_uint32()
    rc_a = L.mtcp_gpu_rxq_wait(a.q[1], ctypes.byref(n_a))
    a_records_ok = rc_a == 0 and a.records(1, AGG)[cmp].tobytes() == want_rx[cmp].tobytes()
    for t in (a, b):
        for q in t.q:
            L.mtcp_gpu_rxq_destroy(q)
        L.mtcp_gpu_close(t.h)
    print(json.dumps({"b_s": round(b_s, 4), "b_records_ok": bool(b_records_ok), "b_tx_ok": bool(b_tx_ok),
                      "a_busy_after_b": bool(a_busy), "a_records_ok": bool(a_records_ok),
                      "b_tx_filled": filled}), flush=True)


if __name__ == "__main__":
    main()
