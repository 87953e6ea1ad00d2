"""Frames at every 2-byte alignment inside a 128 B line, through each phase-1
schedule the library dispatches (mtcp_gpu.hip launch_sched): size-sorted
rounds (average slot < 1 KiB, or <= 1536 B in batches of at most 64 K
packets), unrolled rounds (<= 1536 B in larger batches) and unrolled
rounds with line-aligned trips (> 1536 B, rx_kernel LALIGN, where the first
trip of a multi-trip frame starts (p16 & 127) / 16 chunks before the frame).
Multi-trip frames (> 1536 B) appear in all three.  Frames come from the
oracle's generator (valid checksums, a few corrupted), are moved to the
offsets under test, and every field of every record must equal the oracle's.
"""
import numpy as np
import pytest

import oracle
from mtcp_amd import DESC_DTYPE, RESULT_DTYPE, pktgen
from tests.test_gpu_parity import DEV, assert_same, dev_results, run_rx_dev, to_dev

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    from mtcp_amd import gpu as g
    return g


def _lengths(kind, n, rng):
    if kind == "jumbo":                      # average slot > 1536 B: LALIGN
        return rng.integers(1537, 9001, n)
    if kind == "mid":                        # 1024 .. 1536 B: unrolled, no LALIGN
        return np.where(rng.random(n) < 0.12, rng.integers(1537, 3000, n), rng.integers(900, 1200, n))
    return np.where(rng.random(n) < 0.08, rng.integers(1537, 9001, n), 64)   # < 1 KiB: sorted


def _unaligned_batch(kind, n=1536, seed=11):
    """Generator frames re-packed so that frame i starts at 2*(i % 64) mod 128."""
    rng = np.random.default_rng(seed)
    lens = _lengths(kind, n, rng).astype(np.uint16)
    desc64, nbytes = pktgen.layout_from_lengths(lens, 6)
    src = np.zeros(nbytes, np.uint8)
    oracle.pktgen(src, desc64, 6, seed, 0)
    offs = np.zeros(n, np.int64)
    pos = 0
    for i in range(n):
        pos = (pos + 127) & ~127                     # next line, then the alignment under test
        offs[i] = pos + 2 * (i % 64)
        pos = offs[i] + int(lens[i])
    buf = np.zeros(((pos + 127) & ~127) + 128, np.uint8)
    s0 = desc64["offset"].astype(np.int64) << 6
    for i in range(n):
        buf[offs[i]:offs[i] + lens[i]] = src[s0[i]:s0[i] + lens[i]]
    desc = np.zeros(n, dtype=DESC_DTYPE)
    desc["offset"] = offs.astype(np.uint32)
    desc["len"] = lens
    return buf, desc


# mtcp_gpu.hip launch_sched: slot > 1536 B -> unrolled + LALIGN; 1024..1536 B
# -> unrolled above kSortedUpToPkts (64 K) packets, sorted at or below it;
# < 1 KiB -> sorted.
@pytest.mark.parametrize("kind,slot_lo,slot_hi,n", [("jumbo", 1537, 1 << 30, 1536),
                                                    ("mid", 1024, 1536, (1 << 16) + 512),
                                                    ("mid", 1024, 1536, 1536),
                                                    ("small", 0, 1023, 1536)])
def test_unaligned_frames_every_schedule(gpu, kind, slot_lo, slot_hi, n, monkeypatch):
    monkeypatch.setenv("MTCP_GPU_SCHED", "big")        # rx_kernel's schedules (test_gpu_wave: the small kernels)
    buf, desc = _unaligned_batch(kind, n)
    padded = buf.nbytes + (-buf.nbytes) % 16
    assert slot_lo <= padded // len(desc) <= slot_hi        # the schedule under test is dispatched
    assert (desc["len"] > 1536).sum() > 50                    # multi-trip frames present
    with gpu.Context(0, rss=True, rss_queues=8) as ctx:
        got = run_rx_dev(ctx, buf, desc, 0)
    want = oracle.rx_chunk(buf, desc, 0, oracle.rss_cfg(None, 8, 1))
    assert_same(got, want, kind)
    assert (got["verdict"] == 0).mean() > 0.95


def test_unaligned_frames_pointer_burst(gpu):
    """The same frames as a (pointer, len) burst: rx_ptrs always streams with
    line-aligned trips, whatever the frame sizes."""
    buf, desc = _unaligned_batch("small", seed=12)
    b = to_dev(buf)
    ptrs = torch.from_numpy(desc["offset"].astype(np.int64) + b.data_ptr()).to(DEV)
    lens = torch.from_numpy(desc["len"].astype(np.int16)).to(DEV)
    out = dev_results(len(desc))
    with gpu.Context(0) as ctx:
        ctx.rx_ptrs_dev(ptrs, lens, len(desc), out)
        torch.cuda.synchronize()
    got = out.cpu().numpy().view(RESULT_DTYPE)
    assert_same(got, oracle.rx_chunk(buf, desc, 0), "pointer burst")


def test_maximum_length_frames(gpu):
    """Frames up to the u16 maximum (65 535 B: 43 trips, tot_len 65 521, a TCP
    sum of 32 760 words — still exact in 32 bits), at odd 2-byte alignments,
    with and without a flipped payload bit; chunk mode and pointer burst."""
    lens = np.array([65535, 65534, 65533, 40001, 16385, 9001, 1537, 65535] * 4, dtype=np.uint16)
    n = len(lens)
    desc64, nbytes = pktgen.layout_from_lengths(lens, 6)
    src = np.zeros(nbytes, np.uint8)
    oracle.pktgen(src, desc64, 6, 21, 0)
    offs, pos = np.zeros(n, np.int64), 0
    for i in range(n):
        pos = ((pos + 127) & ~127) + 2 * (7 * i % 64)
        offs[i] = pos
        pos += int(lens[i])
    buf = np.zeros(((pos + 127) & ~127) + 128, np.uint8)
    s0 = desc64["offset"].astype(np.int64) << 6
    for i in range(n):
        buf[offs[i]:offs[i] + lens[i]] = src[s0[i]:s0[i] + lens[i]]
    for i in range(1, n, 3):                               # a payload bit flip in every third
        buf[offs[i] + int(lens[i]) - 7] ^= 0x10
    desc = np.zeros(n, dtype=DESC_DTYPE)
    desc["offset"] = offs.astype(np.uint32)
    desc["len"] = lens
    want = oracle.rx_chunk(buf, desc, 0)
    assert (want["verdict"] == 9).sum() >= n // 3 - 1 and (want["verdict"] == 0).sum() >= n // 2
    with gpu.Context(0) as ctx:
        assert_same(run_rx_dev(ctx, buf, desc, 0), want, "max-length chunk")
        b = to_dev(buf)
        ptrs = torch.from_numpy(offs + b.data_ptr()).to(DEV)
        lt = torch.from_numpy(lens.view(np.int16).copy()).to(DEV)
        out = dev_results(n)
        ctx.rx_ptrs_dev(ptrs, lt, n, out)
        torch.cuda.synchronize()
    assert_same(out.cpu().numpy().view(RESULT_DTYPE), want, "max-length pointers")


def test_batches_larger_than_one_launch(gpu):
    """Batches beyond one launch's held passes (mtcp_gpu.hip launch: grid x 4
    waves x 64 x 8 packets, 1 M on a full MI355X) are cut into several
    launches; every record of every launch, the pointer-burst twin and the tx
    fill must still equal the oracle's."""
    n, seed = (1 << 20) + 4099, 31
    desc, nbytes = pktgen.layout(n, 64, 6, seed)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, seed, 0)
    want = oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(None, 8, 1))
    with gpu.Context(0, rss=True, rss_queues=8) as ctx:
        assert_same(run_rx_dev(ctx, buf, desc, 6), want, "split chunk")
        b = to_dev(buf)
        ptrs = torch.from_numpy((desc["offset"].astype(np.int64) << 6) + b.data_ptr()).to(DEV)
        lens = torch.from_numpy(desc["len"].view(np.int16).copy()).to(DEV)
        out = dev_results(n)
        ctx.rx_ptrs_dev(ptrs, lens, n, out)
        torch.cuda.synchronize()
        assert_same(out.cpu().numpy().view(RESULT_DTYPE), want, "split pointers")
        ctx.tx_fill_dev(b, to_dev(desc), n, 6)
        torch.cuda.synchronize()
    fixed = buf.copy()
    oracle.tx_fill(fixed, desc, 6)
    assert not np.array_equal(fixed, buf)                  # the batch has corrupted frames
    assert np.array_equal(b.cpu().numpy(), fixed)


@pytest.mark.parametrize("size,n", [(1500, 150000), ("bimodal", 300000), (9000, 20000)])
def test_host_pipeline_stages_match_device_path(gpu, size, n):
    """mtcp_gpu_rx_chunk on a host chunk far larger than one pipeline stage
    (64 MiB or 64 K descriptors, three streams): every record equals the
    device path's on the same frames, and a sample equals the oracle's."""
    seed = 41
    desc, nbytes = pktgen.layout(n, size, 6, seed)
    b = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    d = to_dev(desc)
    gpu.pktgen_dev(b, d, n, 6, seed)
    out = dev_results(n)
    with gpu.Context(0, rss=True, rss_queues=5) as ctx:
        ctx.rx_chunk_dev(b, d, n, 6, out)
        torch.cuda.synchronize()
        dev = out.cpu().numpy().view(RESULT_DTYPE)
        host = b.cpu().numpy()
        got = ctx.rx_chunk(host, desc, 6)
    assert nbytes > 2 * (64 << 20) or n > 2 * (1 << 16)
    assert_same(got, dev, f"host pipeline {size}")
    idx = np.sort(np.random.default_rng(1).choice(n, size=2000, replace=False))
    assert_same(got[idx], oracle.rx_chunk(host, desc[idx], 6, oracle.rss_cfg(None, 5, 1)), "sample")


def test_rss_queue_every_nq_and_endian(gpu):
    """GetRSSCPUCore for every queue count mTCP can run (1..16, MAX_CPUS) with
    and without the endian fix (mtcp/src/rss.c:90-103), both keys, on one
    bimodal batch: rss_hash and rss_queue of every packet equal the oracle's."""
    n, seed = 1 << 13, 43
    desc, nbytes = pktgen.layout(n, "bimodal", 6, seed)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, seed, 0)
    for key in (None, oracle.KEY_MICROSOFT):
        for nq in range(1, 17):
            for endian in (0, 1):
                want = oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(key, nq, endian))
                with gpu.Context(0, rss=True, rss_key=key, rss_queues=nq, rss_endian=bool(endian)) as ctx:
                    got = run_rx_dev(ctx, buf, desc, 6)
                assert np.array_equal(got["rss_hash"], want["rss_hash"]), (nq, endian)
                assert np.array_equal(got["rss_queue"], want["rss_queue"]), (nq, endian)


def test_host_pipeline_stage_growth_mid_call(gpu):
    """Small frames first (three 64 K-descriptor batches of 64 B frames size
    the stages at ~4 MiB), then 9000 B frames whose batches need 64 MiB: each
    stage grows while the stages' earlier batches may still be in flight.
    Every record equals the device path's on the same frames."""
    seed = 43
    n_small, n_big = 3 * (1 << 16), 20000
    lens = np.concatenate([np.full(n_small, 64), np.full(n_big, 9000)]).astype(np.uint16)
    desc = np.zeros(len(lens), dtype=DESC_DTYPE)
    slots = (lens.astype(np.int64) + 63) & ~63
    offs = np.concatenate([[0], np.cumsum(slots)[:-1]])
    desc["offset"] = (offs >> 6).astype(np.uint32)
    desc["len"] = lens
    nbytes = int(slots.sum())
    n = len(desc)
    b = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    d = to_dev(desc)
    gpu.pktgen_dev(b, d, n, 6, seed)
    out = dev_results(n)
    with gpu.Context(0, rss=True, rss_queues=3) as ctx:
        ctx.rx_chunk_dev(b, d, n, 6, out)
        torch.cuda.synchronize()
        dev = out.cpu().numpy().view(RESULT_DTYPE)
    host = b.cpu().numpy()
    with gpu.Context(0, rss=True, rss_queues=3) as fresh:   # empty stages: growth happens in this call
        got = fresh.rx_chunk(host, desc, 6)
    assert_same(got, dev, "stage growth")
    idx = np.sort(np.random.default_rng(2).choice(n, size=1000, replace=False))
    assert_same(got[idx], oracle.rx_chunk(host, desc[idx], 6, oracle.rss_cfg(None, 3, 1)), "sample")


@pytest.mark.parametrize("size,n", [(1500, (1 << 17) + 1000), (1500, (2 << 17) + 333), (2000, (1 << 17) + 77)])
def test_unrolled_partial_last_pass(gpu, size, n):
    """The unrolled schedule's workgroup descriptor loads (rx_kernel COOP: one
    LDS exchange and barrier per pass) on batches whose last pass leaves whole
    waves of a workgroup without a packet (they leave the pass loop while
    their siblings finish): rx and the tx fill equal the oracle.  (1 << 17
    packets fill one pass of the grid on a 256-CU MI355X: 512 workgroups x 4
    waves x 64.)"""
    seed = 41
    desc, nbytes = pktgen.layout(n, size, 6, seed)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, seed, 0)
    want = oracle.rx_chunk(buf, desc, 6)
    with gpu.Context(0) as ctx:
        got = run_rx_dev(ctx, buf, desc, 6)
        assert ctx.last_kernel.startswith("rx_kernel<unrolled"), ctx.last_kernel
        assert_same(got, want, f"{size} B x {n}")
        b = to_dev(buf)
        ctx.tx_fill_dev(b, to_dev(desc), n, 6)
        torch.cuda.synchronize()
    fixed = buf.copy()
    oracle.tx_fill(fixed, desc, 6)
    assert not np.array_equal(fixed, buf)
    assert np.array_equal(b.cpu().numpy(), fixed)
