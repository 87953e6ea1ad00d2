"""include/mtcp_gpu_rxq.h on the GPU: frames pushed one by one (as
gpu_module.c does with the wrapped backend's get_rptr pointers), checked by
a synchronous flush or by flush_async + wait, served by rxq_get: NULL
exactly for the checksum failures (ip_in.c:35-36, tcp_in.c:1167-1173) and
the frames whose headers claim bytes past the frame (TRUNCATED), the staged
frame byte for byte otherwise, and every result record equal to the
oracle's for the same frame."""
import ctypes
import os

import numpy as np
import pytest

import oracle
from mtcp_amd import RESULT_DTYPE

torch = pytest.importorskip("torch")

V_IP_CSUM_BAD, V_TCP_CSUM_BAD, V_TRUNCATED, V_BAD_DESC = 4, 9, 10, 11
EINVAL, ETIMEDOUT, EIO = -22, -110, -5
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _testing_lib():
    """tests/c/libmtcp_gpu_testing.so: mtcp_gpu_debug_stall, the fault
    injection the product library does not export (built by build())."""
    T = ctypes.CDLL(os.path.join(ROOT, "tests", "c", "libmtcp_gpu_testing.so"))
    T.mtcp_gpu_debug_stall.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    T.mtcp_gpu_debug_stall.restype = ctypes.c_int
    return T


def _busy(handle: int) -> bool:
    """Work is still queued or running on the HIP stream `handle` (read from
    the device, not inferred from how long a call took)."""
    return not torch.cuda.ExternalStream(handle, device=0).query()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sync", "async"])
def test_rxq_serves_the_oracle_verdicts(golden, mode):
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    from mtcp_amd import gpu
    from mtcp_amd._lib import lib
    L = lib()
    buf, desc = golden.buf, golden.desc
    want = oracle.rx_chunk(buf, desc, 0)
    base = buf.ctypes.data
    agg = 1000                                     # frames per flush
    with gpu.Context(0) as ctx:
        q = ctypes.c_void_p()
        assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, agg, agg * 2048) == 0
        try:
            for first in range(0, len(desc), agg):
                L.mtcp_gpu_rxq_reset(q)
                part = desc[first:first + agg]
                for d in part:
                    assert L.mtcp_gpu_rxq_push(q, base + int(d["offset"]), int(d["len"])) == 0
                assert L.mtcp_gpu_rxq_pending(q) == len(part)
                n_done = ctypes.c_uint32()
                if mode == "sync":
                    assert L.mtcp_gpu_rxq_flush(q, ctypes.byref(n_done)) == 0
                else:
                    assert L.mtcp_gpu_rxq_flush_async(q) == 0
                    # in flight: the staging is the GPU's until rxq_wait
                    assert L.mtcp_gpu_rxq_push(q, base, 64) == EINVAL
                    assert L.mtcp_gpu_rxq_flush_async(q) == EINVAL
                    L.mtcp_gpu_rxq_reset(q)                  # refused silently
                    assert L.mtcp_gpu_rxq_pending(q) == len(part)
                    assert L.mtcp_gpu_rxq_wait(q, ctypes.byref(n_done)) == 0
                assert n_done.value == len(part) and L.mtcp_gpu_rxq_pending(q) == 0
                for i, d in enumerate(part):
                    k = first + i
                    ln = ctypes.c_uint16()
                    res = ctypes.c_void_p()
                    p = L.mtcp_gpu_rxq_get(q, i, ctypes.byref(ln), ctypes.byref(res))
                    got = np.frombuffer(ctypes.string_at(res.value, 40), dtype=RESULT_DTYPE)[0]
                    if want["verdict"][k] != V_BAD_DESC:
                        assert got.tobytes() == want[k].tobytes(), k
                    drop = got["verdict"] in (V_IP_CSUM_BAD, V_TCP_CSUM_BAD, V_TRUNCATED)
                    assert (p is None) == drop, k
                    assert ln.value == d["len"]
                    if p is not None:
                        frame = buf[int(d["offset"]):int(d["offset"]) + int(d["len"])]
                        assert ctypes.string_at(p, int(d["len"])) == frame.tobytes(), k
        finally:
            L.mtcp_gpu_rxq_destroy(q)


@pytest.mark.gpu
def test_rxq_wait_for_abandons_a_flush_that_does_not_finish(golden):
    """mtcp_gpu_rxq_wait_for: a flush queued behind 300 ms of
    mtcp_gpu_debug_stall is not in after 20 ms — MTCP_GPU_ETIMEDOUT, no
    results served, the staged frames still served raw by rxq_frame, resets
    and pushes taken again, further flushes refused (the abandoned one may
    still write its results); with no limit, wait_for is rxq_wait."""
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    import time
    from mtcp_amd import gpu
    from mtcp_amd._lib import lib
    L, T = lib(), _testing_lib()
    buf, desc = golden.buf, golden.desc
    base = buf.ctypes.data
    part = desc[:256]
    with gpu.Context(0) as ctx:
        assert T.mtcp_gpu_debug_stall(ctx._h, 20 * 1000 * 1000) == EINVAL     # over the 10 s cap
        q = ctypes.c_void_p()
        assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, 256, 256 * 2048) == 0
        try:
            for d in part:
                assert L.mtcp_gpu_rxq_push(q, base + int(d["offset"]), int(d["len"])) == 0
            n_done = ctypes.c_uint32()
            assert L.mtcp_gpu_rxq_flush_async(q) == 0
            assert L.mtcp_gpu_rxq_wait_for(q, ctypes.byref(n_done), 0) == 0      # no limit: rxq_wait
            assert n_done.value == len(part)
            L.mtcp_gpu_rxq_reset(q)
            for d in part:
                assert L.mtcp_gpu_rxq_push(q, base + int(d["offset"]), int(d["len"])) == 0
            assert T.mtcp_gpu_debug_stall(ctx._h, 300 * 1000) == 0
            t0 = time.monotonic()
            assert L.mtcp_gpu_rxq_flush_async(q) == 0
            assert L.mtcp_gpu_rxq_wait_for(q, ctypes.byref(n_done), 20 * 1000) == ETIMEDOUT
            assert time.monotonic() - t0 < 0.02 + 0.2          # the contract: within the limit
            assert _busy(ctx.stream)                           # it gave up; the flush still waits
            assert n_done.value == 0
            ln = ctypes.c_uint16()
            assert L.mtcp_gpu_rxq_get(q, 0, ctypes.byref(ln), None) is None
            p = L.mtcp_gpu_rxq_frame(q, 3, ctypes.byref(ln))
            o, n = int(part[3]["offset"]), int(part[3]["len"])
            assert ln.value == n and ctypes.string_at(p, n) == buf[o:o + n].tobytes()
            L.mtcp_gpu_rxq_reset(q)
            assert L.mtcp_gpu_rxq_pending(q) == 0
            assert L.mtcp_gpu_rxq_push(q, base + int(part[0]["offset"]), int(part[0]["len"])) == 0
            assert L.mtcp_gpu_rxq_flush_async(q) == EIO
            assert L.mtcp_gpu_sync(ctx._h) == 0                  # the stall ends by itself
            assert not _busy(ctx.stream)
        finally:
            L.mtcp_gpu_rxq_destroy(q)


@pytest.mark.gpu
@pytest.mark.parametrize("stall_ms,leaks", [(400, True), (60, False)])
def test_rxq_destroy_right_after_a_timeout(golden, stall_ms, leaks):
    """mtcp_gpu_rxq_destroy straight after MTCP_GPU_ETIMEDOUT, no
    mtcp_gpu_sync first.  The abandoned flush may still write the staging:
    destroy waits for it at most MTCP_GPU_RXQ_DESTROY_WAIT_US (100 ms).  A
    400 ms stall outlasts that, so destroy returns within its bound without
    freeing (the buffers are leaked, the flush lands in them later) and the
    flush is still running then; a 60 ms stall ends within it, so destroy
    waited for the flush and freed: the stream is idle when it returns.
    Either way the context stays usable."""
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    import time
    from mtcp_amd import gpu
    from mtcp_amd._lib import lib
    L, T = lib(), _testing_lib()
    buf, desc = golden.buf, golden.desc
    base = buf.ctypes.data
    with gpu.Context(0) as ctx:
        q = ctypes.c_void_p()
        assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, 256, 256 * 2048) == 0
        for d in desc[:256]:
            assert L.mtcp_gpu_rxq_push(q, base + int(d["offset"]), int(d["len"])) == 0
        assert T.mtcp_gpu_debug_stall(ctx._h, stall_ms * 1000) == 0
        assert L.mtcp_gpu_rxq_flush_async(q) == 0
        assert L.mtcp_gpu_rxq_wait_for(q, None, 10 * 1000) == -110
        t0 = time.monotonic()
        L.mtcp_gpu_rxq_destroy(q)
        dt = time.monotonic() - t0
        # what destroy did, read from the stream: when it leaked the buffers
        # the flush was still running; when it freed them it had waited for it
        assert _busy(ctx.stream) == leaks
        assert dt < 0.1 + 0.2, dt                        # the contract: never past its bound
        assert L.mtcp_gpu_sync(ctx._h) == 0
        # the context still works: a fresh rxq checks frames
        q = ctypes.c_void_p()
        assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, 64, 64 * 2048) == 0
        try:
            for d in desc[:64]:
                assert L.mtcp_gpu_rxq_push(q, base + int(d["offset"]), int(d["len"])) == 0
            n = ctypes.c_uint32()
            assert L.mtcp_gpu_rxq_flush(q, ctypes.byref(n)) == 0 and n.value == 64
        finally:
            L.mtcp_gpu_rxq_destroy(q)


@pytest.mark.gpu
def test_tx_fill_ptrs_for_gives_up_and_abandons(golden):
    """mtcp_gpu_tx_fill_ptrs_for (gpu_module.c's send_pkts): a fill whose
    report is not in within the limit answers MTCP_GPU_ETIMEDOUT in about
    the limit, leaves the caller's frames untouched (nothing is written
    before the report), and abandons the context: every later call answers
    EIO without touching the device, and closing it does not wait for the
    stalled work.  A fresh context fills the same frames as the reference."""
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    import time
    from mtcp_amd import gpu
    from mtcp_amd._lib import MtcpGpuError, lib
    L, T = lib(), _testing_lib()
    part = golden.desc[:64]
    offs = part["offset"].astype(np.int64)
    want = golden.buf.copy()
    oracle.tx_fill(want, part, 0)
    ctx = gpu.Context(0)
    host = golden.buf.copy()
    assert ctx.tx_fill_ptrs(host, offs, part["len"], timeout_us=2_000_000) > 0   # a healthy fill
    assert np.array_equal(host, want)
    host = golden.buf.copy()
    handle = ctx.stream
    assert T.mtcp_gpu_debug_stall(ctx._h, 800 * 1000) == 0   # the stream tx fills run on
    t0 = time.monotonic()
    with pytest.raises(MtcpGpuError) as e:
        ctx.tx_fill_ptrs(host, offs, part["len"], timeout_us=30_000)
    assert e.value.code == ETIMEDOUT
    assert time.monotonic() - t0 < 0.03 + 0.2                # the contract: within the limit
    assert _busy(handle)                                     # it did not wait for the stall
    assert np.array_equal(host, golden.buf)                  # nothing written
    with pytest.raises(MtcpGpuError) as e:                   # abandoned: EIO, no device call
        ctx.tx_fill_ptrs(host, offs, part["len"], timeout_us=30_000)
    assert e.value.code == EIO
    assert L.mtcp_gpu_sync(ctx._h) == EIO
    ctx.close()                                              # host state only
    assert _busy(handle)                                     # close did not wait either
    torch.cuda.ExternalStream(handle, device=0).synchronize()
    assert np.array_equal(host, golden.buf)                  # nothing written later either
    with gpu.Context(0) as fresh:
        assert fresh.tx_fill_ptrs(host, offs, part["len"], timeout_us=2_000_000) > 0
        assert np.array_equal(host, want)


@pytest.mark.gpu
@pytest.mark.parametrize("size,kernel", [(512, "rx_group_kernel<oct>"), ("bimodal", "rx_wave_kernel")])
def test_rxq_passes_its_size_hint(size, kernel):
    """An rxq sees every length at push and launches its aggregate with the
    aggregate's {min, max} (mtcp_gpu_rx_chunk_hint_dev): 4 096 frames of
    512 B, with NULL pushes between them (the wrapped backend's own NULLs,
    length 0, not counted in the hint), take the uniform kernel (8 lanes per
    packet); a 64 / 1500 B aggregate keeps the mix's (a wave per packet).
    Every served record equals the oracle's."""
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    from mtcp_amd import gpu, pktgen
    from mtcp_amd._lib import lib
    L = lib()
    n, seed = 4096, 29
    desc, nbytes = pktgen.layout(n, size, 6, seed)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, seed, 0)
    want = oracle.rx_chunk(buf, desc, 6)
    base = buf.ctypes.data
    with gpu.Context(0) as ctx:
        q = ctypes.c_void_p()
        assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, n + 64, (n + 64) * 2048) == 0
        try:
            null_at = set(range(0, n, 97))
            order = []
            for i, d in enumerate(desc):
                if i in null_at:
                    assert L.mtcp_gpu_rxq_push(q, None, 0) == 0
                    order.append(-1)
                assert L.mtcp_gpu_rxq_push(q, base + (int(d["offset"]) << 6), int(d["len"])) == 0
                order.append(i)
            n_done = ctypes.c_uint32()
            assert L.mtcp_gpu_rxq_flush(q, ctypes.byref(n_done)) == 0 and n_done.value == len(order)
            assert ctx.last_kernel.startswith(kernel), ctx.last_kernel
            for j, i in enumerate(order):
                ln, res = ctypes.c_uint16(), ctypes.c_void_p()
                L.mtcp_gpu_rxq_get(q, j, ctypes.byref(ln), ctypes.byref(res))
                got = np.frombuffer(ctypes.string_at(res.value, 40), dtype=RESULT_DTYPE)[0]
                if i < 0:
                    assert got["verdict"] == V_TRUNCATED         # a 0-byte frame (the oracle's too)
                else:
                    assert got.tobytes() == want[i].tobytes(), i
        finally:
            L.mtcp_gpu_rxq_destroy(q)


@pytest.mark.gpu
def test_a_shutdown_does_not_wait_for_another_contexts_work(golden):
    """Two mTCP threads on one GPU: thread B has checked a batch through its
    rxq when thread A's context gets 1 s of work queued
    (mtcp_gpu_debug_stall); B then destroys its rxq and closes its context.
    Neither release waits for A: the library parks its buffers
    (mtcp_amd/csrc/park.hpp) instead of hipFree / hipHostFree, which wait for
    every stream on the device (tools/free_sync_probe.py; before parking B's
    rxq destroy took the whole second, profiles/r5/cross_ctx.jsonl).  Once A
    is done, a fresh context's rxq of the same size gets B's parked buffers
    and checks frames exactly as fresh ones.  (New work of B's is checked in
    a fresh process by test_gpu_bounded.py::test_one_threads_stall_does_not_delay_another:
    here earlier tests' abandoned contexts keep streams alive, and past
    GPU_MAX_HW_QUEUES streams HIP lets two contexts share a hardware queue.)"""
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    import time
    from mtcp_amd import gpu
    from mtcp_amd._lib import lib
    L, T = lib(), _testing_lib()
    buf, desc = golden.buf, golden.desc
    base = buf.ctypes.data
    part = desc[:512]
    want = oracle.rx_chunk(buf, part, 0)

    def check(ctx):
        q = ctypes.c_void_p()
        assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, 512, 512 * 2048) == 0
        for d in part:
            assert L.mtcp_gpu_rxq_push(q, base + int(d["offset"]), int(d["len"])) == 0
        n = ctypes.c_uint32()
        assert L.mtcp_gpu_rxq_flush(q, ctypes.byref(n)) == 0 and n.value == len(part)
        for i in range(len(part)):
            res = ctypes.c_void_p()
            L.mtcp_gpu_rxq_get(q, i, None, ctypes.byref(res))
            got = np.frombuffer(ctypes.string_at(res.value, 40), dtype=RESULT_DTYPE)[0]
            if want["verdict"][i] != V_BAD_DESC:
                assert got.tobytes() == want[i].tobytes(), i
        return q

    a = gpu.Context(0)
    try:
        b = gpu.Context(0)
        q = check(b)
        assert T.mtcp_gpu_debug_stall(a._h, 1_000_000) == 0
        L.mtcp_gpu_rxq_destroy(q)
        b.close()
        # read from the device: A's stall was still running when B's
        # releases had returned, so they did not wait for it
        assert _busy(a.stream)
        assert L.mtcp_gpu_sync(a._h) == 0
        with gpu.Context(0) as d:                            # B's parked buffers, reused
            L.mtcp_gpu_rxq_destroy(check(d))
    finally:
        a.close()


@pytest.mark.gpu
def test_parked_buffers_under_concurrent_threads(golden):
    """Four threads (as four mTCP threads on one GPU) each open a context,
    create an rxq of one of two sizes, check 256 frames, destroy the rxq and
    close the context, 12 times over: the parked buffers (park.hpp) move
    between threads and contexts under its lock, and every batch's records
    are the oracle's, whichever thread's buffers it got."""
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    import threading
    from mtcp_amd import gpu
    from mtcp_amd._lib import lib
    L = lib()
    buf, desc = golden.buf, golden.desc
    base = buf.ctypes.data
    errors = []

    def worker(t):
        try:
            for it in range(12):
                first = (t * 12 + it) * 97 % (len(desc) - 256)
                part = desc[first:first + 256]
                want = oracle.rx_chunk(buf, part, 0)
                cap = 256 if (t + it) % 2 else 512           # frames; golden frames reach 16 000 B
                with gpu.Context(0) as ctx:
                    q = ctypes.c_void_p()
                    assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, cap, cap * 65536) == 0
                    try:
                        for d in part:
                            assert L.mtcp_gpu_rxq_push(q, base + int(d["offset"]), int(d["len"])) == 0
                        n = ctypes.c_uint32()
                        assert L.mtcp_gpu_rxq_flush(q, ctypes.byref(n)) == 0 and n.value == 256
                        for i in range(256):
                            res = ctypes.c_void_p()
                            L.mtcp_gpu_rxq_get(q, i, None, ctypes.byref(res))
                            got = np.frombuffer(ctypes.string_at(res.value, 40), dtype=RESULT_DTYPE)[0]
                            if want["verdict"][i] != V_BAD_DESC:
                                assert got.tobytes() == want[i].tobytes(), (t, it, i)
                    finally:
                        L.mtcp_gpu_rxq_destroy(q)
        except Exception as e:                     # noqa: BLE001 - reported below
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads)
    assert not errors, errors[:3]
