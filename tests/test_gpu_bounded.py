"""The context wait limit (mtcp_gpu_set_wait_limit, ABI 5) on the MI355X.

mTCP's rx loop never waits on a device (mtcp/src/core.c:763-777) and a
device without the offload just answers dev_ioctl with -1
(mtcp/src/dpdk_module.c:809-816).  A context with a wait limit keeps every
synchronous call of the C ABI to that: each host-memory entry point
(rx_chunk, rx_ptrs, tx_fill, tx_fill_ptrs, flow_hash, addr_pool_search,
reserve, close) gives up at the limit with MTCP_GPU_ETIMEDOUT, writes nothing
into the caller's memory then or later, and abandons the context; a fresh
context gives the reference's results.  Without a stall the bounded calls
(which go through pinned bounce buffers) give exactly the unbounded calls'
results.

What happened is read from the device, not from how long a call took: the
stall is still running when a call has returned (the context's stream is
busy), and the caller's buffers still hold their sentinel after the stall
has ended.  The one wall-clock bound per test is the contract itself: a
call returns within its limit (+ 200 ms of slack for a loaded box).
"""
import ctypes
import os
import time

import numpy as np
import pytest

import oracle
from mtcp_amd import DESC_DTYPE, RESULT_DTYPE, pktgen
from tests.golden_io import compare_results

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ETIMEDOUT, EIO = -110, -5
LIMIT_US = 30_000
STALL_US = 600_000
SLACK_S = 0.2
SENTINEL = 0xA5


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    from mtcp_amd import gpu as g
    return g


def stall_lib():
    T = ctypes.CDLL(os.path.join(ROOT, "tests", "c", "libmtcp_gpu_testing.so"))
    T.mtcp_gpu_debug_stall.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    T.mtcp_gpu_debug_stall.restype = ctypes.c_int
    T.mtcp_gpu_debug_stall_stream.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    T.mtcp_gpu_debug_stall_stream.restype = ctypes.c_int
    return T


def stream_busy(handle: int) -> bool:
    """Work is still queued or running on the HIP stream `handle`."""
    return not torch.cuda.ExternalStream(handle, device=0).query()


def stream_wait(handle: int) -> None:
    torch.cuda.ExternalStream(handle, device=0).synchronize()


def unfilled(golden, desc):
    """The golden frames with every frame's iph->check zeroed: a tx fill
    then changes every frame it fills (ip_out.c:145,164)."""
    host = golden.buf.copy()
    for o, ln in zip(desc["offset"].astype(np.int64), desc["len"]):
        if ln >= 26:
            host[o + 24:o + 26] = 0
    return host


def ptr_array(base: int, offsets):
    offs = [base + int(o) for o in offsets]
    return (ctypes.c_void_p * max(len(offs), 1))(*offs)


# ---- the calls, each with its caller-owned buffers ---------------------------
# Every case builds its inputs, calls the C ABI once and returns
# (rc, {name: caller buffer that must not change on a timeout}, check) where
# check() verifies a successful call against the reference.

def case_rx_chunk(L, ctx, golden):
    out = np.full(len(golden.desc) * 40, SENTINEL, np.uint8)
    rc = L.mtcp_gpu_rx_chunk(ctx._h, golden.buf.ctypes.data, golden.buf.nbytes, golden.desc.ctypes.data,
                             len(golden.desc), 0, out.ctypes.data)
    return rc, {"out": out}, lambda: not compare_results(out.view(RESULT_DTYPE), golden)


def case_rx_chunk_unsorted(L, ctx, golden):
    perm = np.random.default_rng(5).permutation(len(golden.desc))
    desc = np.ascontiguousarray(golden.desc[perm])
    out = np.full(len(desc) * 40, SENTINEL, np.uint8)
    rc = L.mtcp_gpu_rx_chunk(ctx._h, golden.buf.ctypes.data, golden.buf.nbytes, desc.ctypes.data,
                             len(desc), 0, out.ctypes.data)
    inv = np.argsort(perm)
    return rc, {"out": out}, lambda: not compare_results(out.view(RESULT_DTYPE)[inv], golden)


def case_rx_ptrs(L, ctx, golden):
    d = golden.desc[:500]
    ptrs = ptr_array(golden.buf.ctypes.data, d["offset"])
    lens = np.ascontiguousarray(d["len"])
    out = np.full(len(d) * 40, SENTINEL, np.uint8)
    rc = L.mtcp_gpu_rx_ptrs(ctx._h, ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, len(d), out.ctypes.data)
    want = oracle.rx_chunk(golden.buf, d, 0, oracle.rss_cfg(None, golden.rss_num_queues, 1))
    return rc, {"out": out}, lambda: out.view(RESULT_DTYPE).tobytes() == want.tobytes()


def case_tx_fill(L, ctx, golden):
    host = unfilled(golden, golden.desc)
    want = host.copy()
    cnt = ctypes.c_uint32(0xFFFF)
    rc = L.mtcp_gpu_tx_fill(ctx._h, host.ctypes.data, host.nbytes, golden.desc.ctypes.data, len(golden.desc), 0,
                            ctypes.byref(cnt))
    n = oracle.tx_fill(want, golden.desc, 0)
    return rc, {"frames": host}, lambda: np.array_equal(host, want) and cnt.value == n


def case_tx_fill_ptrs(L, ctx, golden):
    d = golden.desc[:64]
    host = unfilled(golden, d)
    want = host.copy()
    ptrs = ptr_array(host.ctypes.data, d["offset"])
    lens = np.ascontiguousarray(d["len"])
    cnt = ctypes.c_uint32(0)
    # timeout 0: the context's wait limit
    rc = L.mtcp_gpu_tx_fill_ptrs_for(ctx._h, ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, len(d),
                                     ctypes.byref(cnt), 0)
    oracle.tx_fill(want, d, 0)
    return rc, {"frames": host}, lambda: np.array_equal(host, want)


def case_flow_hash(L, ctx, golden):
    res = np.ascontiguousarray(golden.expect)
    bins = np.full(len(res), 0xA5A5A5A5, np.uint32)
    rc = L.mtcp_gpu_flow_hash(ctx._h, res.ctypes.data, len(res), bins.ctypes.data)
    ok = golden.meta["ref_ub"] == 0
    return rc, {"bins": bins}, lambda: np.array_equal(bins[ok], golden.flow_bins[ok])


def case_addr_pool(L, ctx, golden):
    from mtcp_amd._types import ADDR_ENTRY_DTYPE
    args = (1, 4, 0x0A00000A, 4, 0x0B00000A, 0x5000, 1)       # core, nq, saddr, num_addr, daddr, dport, endian
    out = np.full(4 * 64511 * ADDR_ENTRY_DTYPE.itemsize, SENTINEL, np.uint8).view(ADDR_ENTRY_DTYPE)
    found = ctypes.c_uint32(0xFFFF)
    rc = L.mtcp_gpu_addr_pool_search(ctx._h, *args, out.ctypes.data, len(out), ctypes.byref(found))
    want = oracle.addr_pool_search(None, *args)
    return rc, {"entries": out.view(np.uint8), "found": np.frombuffer(found, np.uint8)}, \
        lambda: (found.value == len(want) and np.array_equal(out["saddr"][:len(want)], want["saddr"])
                 and np.array_equal(out["sport"][:len(want)], want["sport"]))


CASES = {"rx_chunk": case_rx_chunk, "rx_chunk_unsorted": case_rx_chunk_unsorted, "rx_ptrs": case_rx_ptrs,
         "tx_fill": case_tx_fill, "tx_fill_ptrs": case_tx_fill_ptrs, "flow_hash": case_flow_hash,
         "addr_pool_search": case_addr_pool}


@pytest.mark.parametrize("name", sorted(CASES))
def test_bounded_calls_give_the_reference_results(gpu, golden, name):
    """With a (generous) wait limit every host call goes through the pinned
    bounce buffers; its results are the reference's / the oracle's, as the
    unbounded call's are."""
    from mtcp_amd._lib import lib
    L = lib()
    with gpu.Context(0, rss=True, rss_queues=golden.rss_num_queues) as ctx:
        ctx.wait_limit = 5_000_000
        assert ctx.wait_limit == 5_000_000
        rc, _, check = CASES[name](L, ctx, golden)
        assert rc == 0
        assert check(), name
        rc, _, check = CASES[name](L, ctx, golden)          # the bounce buffers reused
        assert rc == 0 and check(), name


@pytest.mark.parametrize("size,n", [(1500, 150000), ("bimodal", 300000)])
def test_bounded_pipeline_over_several_stages(gpu, size, n):
    """A bounded host rx over more than one 64 MiB stage (three streams,
    each stage's batch copied out of its bounce buffer before the stage is
    reused): every record equals the device path's."""
    seed = 47
    desc, nbytes = pktgen.layout(n, size, 6, seed)
    b = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    d = torch.from_numpy(desc.view(np.uint8).copy()).to("cuda:0")
    gpu.pktgen_dev(b, d, n, 6, seed)
    out = torch.zeros(n * 40, dtype=torch.uint8, device="cuda:0")
    with gpu.Context(0, rss=True, rss_queues=5) as ctx:
        ctx.rx_chunk_dev(b, d, n, 6, out)
        torch.cuda.synchronize()
        dev = out.cpu().numpy().view(RESULT_DTYPE)
        host = b.cpu().numpy()
        ctx.wait_limit = 10_000_000
        got = ctx.rx_chunk(host, desc, 6)
    assert nbytes > 2 * (64 << 20) or n > 2 * (1 << 16)
    assert got.tobytes() == dev.tobytes()


@pytest.mark.parametrize("name", sorted(CASES))
def test_each_host_call_gives_up_at_the_limit(gpu, golden, name):
    """A call queued behind 600 ms of stall on the context's stream, with a
    30 ms limit: MTCP_GPU_ETIMEDOUT within the limit; the stall is still
    running when it returns; the caller's buffers hold their sentinel then
    AND after the stall has ended (no copy the call gave up on lands in
    them); the context is abandoned (EIO, no device call); closing it does
    not wait; a fresh context gives the reference's results."""
    from mtcp_amd._lib import lib
    L, T = lib(), stall_lib()
    ctx = gpu.Context(0, rss=True, rss_queues=golden.rss_num_queues)
    handle = ctx.stream
    rc, _, check = CASES[name](L, ctx, golden)             # unbounded: stages sized, kernels loaded
    assert rc == 0 and check()
    ctx.wait_limit = LIMIT_US
    assert T.mtcp_gpu_debug_stall(ctx._h, STALL_US) == 0
    t0 = time.monotonic()
    rc, bufs, _ = CASES[name](L, ctx, golden)
    dt = time.monotonic() - t0
    assert rc == ETIMEDOUT, rc
    assert dt < LIMIT_US / 1e6 + SLACK_S, dt               # the contract: within the limit
    assert stream_busy(handle)                              # it did not wait for the stall
    before = {k: v.copy() for k, v in bufs.items()}
    untouched = {k: v.tobytes() for k, v in bufs.items()}
    assert L.mtcp_gpu_sync(ctx._h) == EIO                   # abandoned
    assert L.mtcp_gpu_rx_chunk(ctx._h, golden.buf.ctypes.data, golden.buf.nbytes, golden.desc.ctypes.data,
                               1, 0, bufs[next(iter(bufs))].ctypes.data) == EIO
    ctx.close()                                             # host state only: no wait
    assert stream_busy(handle)
    stream_wait(handle)                                     # the stall and what was queued behind it end
    for k, v in bufs.items():
        assert v.tobytes() == untouched[k], f"{name}: {k} written after the call gave up"
        assert np.array_equal(v, before[k])
    with gpu.Context(0, rss=True, rss_queues=golden.rss_num_queues) as fresh:
        fresh.wait_limit = 5_000_000
        rc, _, check = CASES[name](L, fresh, golden)
        assert rc == 0 and check(), name


def test_bounded_pipeline_gives_up_mid_call(gpu):
    """The limit passes while a multi-stage host rx is still filling its
    stages (stage 0 waits behind the stall): ETIMEDOUT, and not one record
    of the batches that did run is written into the caller's results."""
    from mtcp_amd._lib import lib
    L, T = lib(), stall_lib()
    n, seed = 150000, 53
    desc, nbytes = pktgen.layout(n, 1500, 6, seed)
    host = np.zeros(nbytes, np.uint8)
    oracle.pktgen(host, desc, 6, seed, 0)
    out = np.full(n * 40, SENTINEL, np.uint8)
    ctx = gpu.Context(0)
    handle = ctx.stream
    ctx.wait_limit = 100_000
    assert T.mtcp_gpu_debug_stall(ctx._h, STALL_US) == 0
    t0 = time.monotonic()
    rc = L.mtcp_gpu_rx_chunk(ctx._h, host.ctypes.data, nbytes, desc.ctypes.data, n, 6, out.ctypes.data)
    dt = time.monotonic() - t0
    assert rc == ETIMEDOUT
    assert dt < 0.1 + SLACK_S + 0.2, dt                     # + the bounce copies of up to three stages
    ctx.close()
    stream_wait(handle)
    assert (out == SENTINEL).all()


def test_sync_times_out_without_abandoning(gpu, golden):
    """mtcp_gpu_sync with a limit: ETIMEDOUT while the stall runs, and the
    context stays usable (what sync waits for is the caller's own device
    work): after the stall, sync succeeds and a host call gives the
    reference's results on the same context."""
    from mtcp_amd._lib import lib
    L, T = lib(), stall_lib()
    with gpu.Context(0, rss=True, rss_queues=golden.rss_num_queues) as ctx:
        ctx.wait_limit = LIMIT_US
        assert T.mtcp_gpu_debug_stall(ctx._h, 300_000) == 0
        t0 = time.monotonic()
        assert L.mtcp_gpu_sync(ctx._h) == ETIMEDOUT
        assert time.monotonic() - t0 < LIMIT_US / 1e6 + SLACK_S
        assert stream_busy(ctx.stream)
        stream_wait(ctx.stream)
        assert L.mtcp_gpu_sync(ctx._h) == 0
        ctx.wait_limit = 5_000_000
        rc, _, check = case_rx_chunk(L, ctx, golden)
        assert rc == 0 and check()


def test_reserve_and_rxq_calls_are_bounded(gpu, golden):
    """mtcp_gpu_reserve and an rxq of a bounded context (the rxq takes the
    limit at create): behind the stall, reserve answers ETIMEDOUT within
    the limit; on another context, rxq_flush (flush_async + a wait with the
    context's limit) answers ETIMEDOUT, serves no verdicts, and the rxq's
    destroy returns without waiting for the stall."""
    from mtcp_amd._lib import lib
    L, T = lib(), stall_lib()
    a = gpu.Context(0)
    ha = a.stream
    a.wait_limit = LIMIT_US
    assert T.mtcp_gpu_debug_stall(a._h, STALL_US) == 0
    t0 = time.monotonic()
    assert L.mtcp_gpu_reserve(a._h, 1 << 20, 1024) == ETIMEDOUT
    assert time.monotonic() - t0 < LIMIT_US / 1e6 + SLACK_S
    assert stream_busy(ha)
    a.close()

    b = gpu.Context(0)
    hb = b.stream
    b.wait_limit = LIMIT_US
    q = ctypes.c_void_p()
    assert L.mtcp_gpu_rxq_create(ctypes.byref(q), b._h, 256, 256 * 2048) == 0
    base = golden.buf.ctypes.data
    for dsc in golden.desc[:256]:
        assert L.mtcp_gpu_rxq_push(q, base + int(dsc["offset"]), int(dsc["len"])) == 0
    assert T.mtcp_gpu_debug_stall(b._h, STALL_US) == 0
    n = ctypes.c_uint32(7)
    t0 = time.monotonic()
    assert L.mtcp_gpu_rxq_flush(q, ctypes.byref(n)) == ETIMEDOUT
    assert time.monotonic() - t0 < LIMIT_US / 1e6 + SLACK_S
    assert n.value == 0 and L.mtcp_gpu_rxq_get(q, 0, None, None) is None
    L.mtcp_gpu_rxq_destroy(q)
    assert stream_busy(hb)                                  # destroy did not wait for it
    b.close()
    stream_wait(ha)
    stream_wait(hb)


def test_close_with_a_caller_stream_launch_pending(gpu):
    """a context is closed while its launch on the
    CALLER's stream is still queued (behind a stall on that stream), and a
    context with a different RSS key is opened and used meanwhile.  The
    pending launch still computes with its own key: the device-side tables
    are shared per key and never freed or rewritten (rss_tables_for)."""
    T = stall_lib()
    n, seed = 4096, 59
    desc, nbytes = pktgen.layout(n, "bimodal", 6, seed)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, seed, 0)
    dev = torch.device("cuda", 0)
    b = torch.from_numpy(buf).to(dev)
    d = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    caller = torch.cuda.Stream(dev)
    out_a = torch.zeros(n * 40, dtype=torch.uint8, device=dev)
    out_b = torch.zeros(n * 40, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    a = gpu.Context(0, rss=True, rss_key=oracle.KEY_MICROSOFT, rss_queues=16, rss_endian=False)
    assert T.mtcp_gpu_debug_stall_stream(caller.cuda_stream, 400_000) == 0
    a.rx_chunk_dev(b, d, n, 6, out_a, stream=caller)
    a.close()                                               # the launch has not run yet
    assert not caller.query()
    for _ in range(4):                                      # new contexts, another key, busy
        with gpu.Context(0, rss=True, rss_queues=8) as c:
            c.rx_chunk_dev(b, d, n, 6, out_b)
            c.sync()
    caller.synchronize()
    got = out_a.cpu().numpy().view(RESULT_DTYPE)
    want = oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(oracle.KEY_MICROSOFT, 16, 0))
    assert got.tobytes() == want.tobytes()
    torch.cuda.synchronize()
    got_b = out_b.cpu().numpy().view(RESULT_DTYPE)
    assert got_b.tobytes() == oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(None, 8, 1)).tobytes()


def test_one_threads_stall_does_not_delay_another():
    """VERDICT r5 item 2, in the io_module's default configuration: two mTCP
    threads' GPU contexts (compact records, two pipelined rxqs each, tx
    fills on, as gpu_module.c with MTCP_GPU_TX=1), in a fresh process so
    that its streams are exactly theirs.  While thread A's context has a 1 s
    stall queued (behind it, A's next aggregate), thread B flushes an
    aggregate and fills a tx burst: B's records and frames are the oracle's,
    B is done in under 0.3 s, and A's stall is still running then (B's work
    went on a hardware queue of its own: one stream per context)."""
    import json
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-u", "-m", "tests.hwq_isolation"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=90)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["b_records_ok"] and r["b_tx_ok"], r
    assert r["a_busy_after_b"], r                          # A's stall outlasted all of B's work
    assert r["b_s"] < 0.3, r
    assert r["a_records_ok"], r                            # and A's aggregate, once its stall ended


def test_rxqs_of_an_abandoned_context_do_not_touch_the_device(gpu, golden):
    """A context abandoned by a tx fill that timed out (its own limit, the
    context without one) while one of its rxqs has a flush queued behind the
    same stall: the rxq's wait takes one look and gives up (no unbounded
    wait on the abandoned stream), its further flushes and a new rxq on the
    context answer EIO without touching the device, and its destroy returns
    within its bound while the stall still runs."""
    from mtcp_amd._lib import MtcpGpuError, lib
    L, T = lib(), stall_lib()
    ctx = gpu.Context(0)
    handle = ctx.stream
    base = golden.buf.ctypes.data
    q = ctypes.c_void_p()
    assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, 256, 256 * 2048) == 0
    for d in golden.desc[:256]:
        assert L.mtcp_gpu_rxq_push(q, base + int(d["offset"]), int(d["len"])) == 0
    assert T.mtcp_gpu_debug_stall(ctx._h, STALL_US) == 0
    assert L.mtcp_gpu_rxq_flush_async(q) == 0
    part = golden.desc[:64]
    host = golden.buf.copy()
    with pytest.raises(MtcpGpuError) as e:
        ctx.tx_fill_ptrs(host, part["offset"].astype(np.int64), part["len"], timeout_us=LIMIT_US)
    assert e.value.code == ETIMEDOUT
    t0 = time.monotonic()
    n = ctypes.c_uint32(7)
    assert L.mtcp_gpu_rxq_wait(q, ctypes.byref(n)) == ETIMEDOUT        # one look, no wait
    assert time.monotonic() - t0 < SLACK_S
    assert n.value == 0 and stream_busy(handle)
    assert L.mtcp_gpu_rxq_flush_async(q) == EIO
    q2 = ctypes.c_void_p()
    assert L.mtcp_gpu_rxq_create(ctypes.byref(q2), ctx._h, 64, 64 * 2048) == EIO
    t0 = time.monotonic()
    L.mtcp_gpu_rxq_destroy(q)
    assert time.monotonic() - t0 < 0.1 + SLACK_S                       # MTCP_GPU_RXQ_DESTROY_WAIT_US
    assert stream_busy(handle)
    ctx.close()
    stream_wait(handle)
    assert np.array_equal(host, golden.buf)                             # the tx fill wrote nothing


def test_park_best_fit():
    """park.hpp hands a parked buffer to the smallest
    request it covers up to twice over (a sweep of sizes reuses what it
    parked), a buffer handed out larger than asked goes back with its real
    size, pinned host and device buffers stay apart, and a buffer above
    kParkMaxBytes is freed rather than parked — unless the release belongs
    to a call bounded by a wait limit, which must not wait on the device:
    then it is parked and reused (tests/c/park_test.hip)."""
    import json
    import subprocess
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    p = subprocess.run([os.path.join(ROOT, "tests", "c", "park_test")], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["ok"] and r["best_fit_reused"] and r["small_not_reused"] and r["real_size_kept"], r
    assert r["smallest_wins"] and r["kinds_apart"] and r["big_freed"], r
    assert r["big_parked_when_bounded"] and r["big_reused"], r          # a bounded call never frees
    assert r["parked_after_release"] == 1 << 20 and r["parked_after_reuse"] == 0, r
    assert r["parked_after_lent_release"] == 1 << 20, r                 # its real size, not the 700 KiB asked


def test_host_code_under_asan_on_the_gpu(golden):
    """The C ABI's host code — staging, bounce buffers, gathers, parking,
    rxqs, bounded waits — built with AddressSanitizer on the host side
    (tests/c/asan_host.hip; the pool has no GPU ASan) and driven on the
    MI355X through every host entry point without and with a wait limit,
    over a multi-stage chunk, and through each bounded call giving up
    behind a stall: no ASan report, bounded and unbounded calls write the
    same bytes, every bounded call behind the stall answers ETIMEDOUT and
    leaves the caller's buffers untouched after the stall ends."""
    import json
    import subprocess
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    gold = os.path.join(ROOT, "tests", "golden")
    p = subprocess.run([os.path.join(ROOT, "tests", "c", "asan_host"), os.path.join(gold, "rx_buf.bin"),
                        os.path.join(gold, "rx_desc.bin")], capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0"))
    assert "AddressSanitizer" not in p.stderr, p.stderr[-3000:]
    assert p.returncode == 0, p.stdout[-1000:] + p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["ok"] and r["bounded_equals_unbounded"] and r["timeouts"] == 7, r
    assert r["frames"] == len(golden.desc)
