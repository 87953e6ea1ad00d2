"""Small batches and the entry points added with the wave-per-packet kernel
(mtcp_amd/csrc/rx_wave.hpp), on the MI355X, bit-exact:

* every dispatched kernel — a wavefront, a 16-lane row or a 4-lane quad per
  packet (rx_wave.hpp), the chunk-parallel span kernel (rx_span.hpp) and
  rx_kernel's sorted / unrolled / line-aligned rounds, each forced with MTCP_GPU_SCHED (mtcp_gpu.hip pick_sched) — on the
  golden vectors and on config-shaped batches of 4 096 (one io_module
  aggregate) and 65 536 packets, against the reference's results and the
  oracle;
* frames at every even start (2-byte aligned, NET_IP_ALIGN-style), chunk and
  pointer modes, rx and tx;
* rx with HashFlow fused in (mtcp_gpu_rx_*_flow_dev) against the reference's
  own bins (tests/golden/rx_flowbins.bin) and the separate f3 kernel;
* the tx fill of pointer bursts (mtcp_gpu_tx_fill_ptrs[_dev]) against the
  reference's fills;
* mtcp_gpu_reserve(0, 0) / rxq creation on a context that already ran host
  calls (the staging it warms is then already allocated).
"""
import ctypes

import numpy as np
import pytest

import oracle
from mtcp_amd import DESC_DTYPE, RESULT_DTYPE, pktgen
from tests.fuzz_frames import fuzz_batch
from tests.golden_io import compare_results
from tests.repack import repack
from tests.test_gpu_parity import DEV, assert_same, dev_results, run_rx_dev, to_dev

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    from mtcp_amd import gpu as g
    return g


def ctx_for(gpu, monkeypatch, sched, **kw):
    """A context whose batches all take kernel `sched` (mtcp_gpu.hip
    MTCP_GPU_SCHED): "wave", "row", "quad" (rx_wave.hpp), "span" (rx_span.hpp)
    or "big" (rx_kernel)."""
    monkeypatch.setenv("MTCP_GPU_SCHED", sched)
    c = gpu.Context(0, **kw)
    monkeypatch.delenv("MTCP_GPU_SCHED")
    return c


def ptr_burst(b, desc):
    ptrs = torch.from_numpy(desc["offset"].astype(np.int64) + b.data_ptr()).to(DEV)
    lens = torch.from_numpy(desc["len"].view(np.int16).copy()).to(DEV)
    return ptrs, lens


SCHEDS = ["wave", "row", "quad", "oct", "span", "big"]


@pytest.mark.parametrize("sched", SCHEDS)
def test_golden_every_schedule(gpu, golden, monkeypatch, sched):
    rss = oracle.rss_cfg(oracle.KEY_0X05, golden.rss_num_queues, 1)
    want = oracle.rx_chunk(golden.buf, golden.desc, 0, rss)
    n = len(golden.desc)
    with ctx_for(gpu, monkeypatch, sched, rss=True, rss_queues=golden.rss_num_queues) as ctx:
        got = run_rx_dev(ctx, golden.buf, golden.desc, 0)
        b = to_dev(golden.buf)
        ptrs, lens = ptr_burst(b, golden.desc)
        out = dev_results(n)
        ctx.rx_ptrs_dev(ptrs, lens, n, out)
        torch.cuda.synchronize()
        got_p = out.cpu().numpy().view(RESULT_DTYPE)
        d = to_dev(golden.desc)
        ctx.tx_fill_dev(b, d, n, 0)
        torch.cuda.synchronize()
        filled = b.cpu().numpy()
    bad = compare_results(got, golden)
    assert not bad, bad
    assert_same(got, want, f"{sched} chunk vs oracle")
    assert not compare_results(got_p, golden)
    assert_same(got_p, want, f"{sched} pointers vs oracle")
    fixed = golden.buf.copy()
    assert oracle.tx_fill(fixed, golden.desc, 0) == golden.manifest["tx_filled"]
    assert np.array_equal(filled, fixed)


@pytest.mark.parametrize("n", [4096, 1 << 16])
@pytest.mark.parametrize("size,rss", [(1500, False), ("bimodal", True), (64, False), (9000, False)])
def test_small_batches_every_schedule(gpu, monkeypatch, n, size, rss):
    """One io_module aggregate (4 096 frames) and 64 K frames through every
    kernel, each equal to the oracle."""
    if size == 9000 and n > 4096:
        n = 16384
    seed = 61
    desc, nbytes = pktgen.layout(n, size, 6, seed)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, seed, 0)
    want = oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(None, 8, 1) if rss else None)
    kw = dict(rss=True, rss_queues=8, rss_endian=True) if rss else {}
    for sched in SCHEDS:
        with ctx_for(gpu, monkeypatch, sched, **kw) as ctx:
            assert_same(run_rx_dev(ctx, buf, desc, 6), want, f"{sched} {size} x {n}")
    assert (want["verdict"] == 0).mean() > 0.99


def imix_lengths(n, seed):
    """64 / 576 / 1500 B frames in the ratio 7 : 4 : 1 (simple IMIX)."""
    r = np.random.default_rng(seed).integers(0, 12, n)
    return np.where(r < 7, 64, np.where(r < 11, 576, 1500)).astype(np.uint16)


@pytest.mark.parametrize("n,size,kernel", [
    (2048, 64, "rx_wave"), (2049, 64, "rx_group_kernel<quad"), (1 << 17, 64, "rx_group_kernel<quad"),
    ((1 << 17) + 1, 64, "rx_group_kernel<quad"), ((1 << 17) + 1, 128, "rx_span_kernel"),
    (8192, 1500, "rx_wave"), (8193, 1500, "rx_group_kernel<row"), (32768, 512, "rx_group_kernel<row"),
    (32769, 512, "rx_span_kernel"), (32769, 640, "rx_span_kernel"), (32769, 704, "rx_group_kernel<oct"),
    (65536, 1500, "rx_group_kernel<oct"), (65537, 1500, "rx_kernel"), (65536, 4096, "rx_wave"),
    (65537, 4096, "rx_kernel"), (16384, 4032, "rx_wave"), (32768, 4032, "rx_group_kernel<row"),
    ((1 << 18) + 3, "imix", "rx_span_kernel"), (16384, 2048, "rx_wave"), (16385, 2048, "rx_group_kernel<row"),
    # with the caller's size hint (mtcp_gpu_rx_chunk_hint_dev): one size class
    ((1 << 16), "256h", "rx_group_kernel<oct"), ((1 << 16) + 1, "256h", "rx_group_kernel<quad"),
    ((1 << 17) + 1, "256h", "rx_span_kernel"), (4096, "512h", "rx_group_kernel<oct"), (2048, "512h", "rx_wave"),
    (16384, "256h", "rx_group_kernel<oct"), (4096, "imixh", "rx_wave"), ((1 << 16) + 1, "512h", "rx_span_kernel"),
    ((1 << 16), "512h", "rx_group_kernel<oct"), ((1 << 16), 512, "rx_span_kernel"),
    ((1 << 16) + 1, "768h", "rx_span_kernel"), ((1 << 16) + 1, 768, "rx_kernel"),
    ((1 << 16) + 1, "1024h", "rx_kernel"), ((1 << 17) + 1, "bimodalh", "rx_kernel<sorted>"),
    ((1 << 17) + 1, "imixh", "rx_span_kernel")])
def test_dispatch_boundaries(gpu, monkeypatch, n, size, kernel):
    """The automatic kernel choice (mtcp_gpu.hip pick_sched) on both sides of
    each boundary it draws — small frames: wave up to 2 048, quad up to
    128 K, then quads for 64 B slots and the span kernel for larger ones; MTU
    frames: wave up to 8 192, row up to 32 K, 8 lanes per packet up to 64 K
    (slots <= 2 KiB), rx_kernel above; 4 KiB slots and up: wave up to 64 K;
    past 32 K frames of <= 640 B slots the span kernel; 2 KiB slots wave up
    to 16 K; and, with a size hint saying the batch is of one size class
    (mtcp_gpu_rx_chunk_hint_dev), 8 lanes per packet for 256-640 B slots
    from 4 K to 64 K frames, quads for 256 B slots up to 128 K, the span
    kernel for 768 B slots past 64 K, while a hinted mix (bimodal, IMIX)
    keeps the mix's kernel — each the kernel it should be, and equal to the
    oracle."""
    monkeypatch.delenv("MTCP_GPU_SCHED", raising=False)
    seed = 67
    hinted = isinstance(size, str) and size.endswith("h")
    size = size[:-1] if hinted else size
    if size == "imix":
        desc, nbytes = pktgen.layout_from_lengths(imix_lengths(n, seed), 6)
    else:
        desc, nbytes = pktgen.layout(n, size if size == "bimodal" else int(size), 6, seed)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, seed, 0)
    want = oracle.rx_chunk(buf, desc, 6)
    hint = (int(desc["len"].min()), int(desc["len"].max())) if hinted else None
    with gpu.Context(0) as ctx:
        assert_same(run_rx_dev(ctx, buf, desc, 6, hint=hint), want, f"auto {size} x {n} hint {hint}")
        assert ctx.last_kernel.startswith(kernel), ctx.last_kernel


@pytest.mark.parametrize("sizes", ["imix", "ragged"])
def test_span_kernel_mixed_sizes(gpu, monkeypatch, sizes):
    """rx_span_kernel on the batches it exists for — an IMIX, and frames of
    every length 1 .. 2 000 B with empty descriptors, out-of-buffer ones and
    runs of one-chunk frames between them — chunk and pointer modes, with RSS
    and the fused flow bins, equal to the oracle."""
    rng = np.random.default_rng(73)
    n = 20000 + 37
    if sizes == "imix":
        lens = imix_lengths(n, 73)
    else:
        lens = rng.integers(1, 2001, n).astype(np.uint16)
        lens[rng.random(n) < .1] = 0
        lens[rng.random(n) < .1] = 14
    desc, nbytes = pktgen.layout_from_lengths(lens, 6)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, 73, 0)
    if sizes == "ragged":
        bad = rng.random(n) < .01
        desc["offset"][bad] = (nbytes >> 6) + 5                     # past the buffer
    want = oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(None, 8, 1))
    with ctx_for(gpu, monkeypatch, "span", rss=True, rss_queues=8, rss_endian=True) as ctx:
        got = run_rx_dev(ctx, buf, desc, 6)
        assert ctx.last_kernel == "rx_span_kernel"
        b = to_dev(buf)
        bdesc = desc.copy()
        bdesc["offset"] = desc["offset"].astype(np.int64) << 6
        ok = desc["offset"].astype(np.int64) << 6 < nbytes
        bdesc["offset"][~ok] = 0
        ptrs, lns = ptr_burst(b, bdesc)
        out = dev_results(n)
        bins = torch.zeros(n, dtype=torch.int32, device=DEV)
        ctx.rx_ptrs_flow_dev(ptrs, lns, n, out, bins)
        torch.cuda.synchronize()
    assert_same(got, want, f"span {sizes} chunk")
    gp = out.cpu().numpy().view(RESULT_DTYPE)
    assert_same(gp[ok], want[ok], f"span {sizes} pointers")
    assert np.array_equal(bins.cpu().numpy().view(np.uint32)[ok], oracle.flow_bins(want)[ok])


def test_short_trip_kernel_with_jumbo_frames(gpu, monkeypatch):
    """A batch whose average slot is at most 2 KiB takes the wave kernel's
    2-load trips (mtcp_gpu.hip kWaveShortUpToSlot): its jumbo frames then
    need several trips and the masked segment sum; with the fuzz frames'
    padded and truncated datagrams spliced in, every kernel equals the
    oracle, chunk and pointer modes."""
    rng = np.random.default_rng(71)
    n = 4096
    lens = np.where(rng.random(n) < .06, rng.integers(2049, 16001, n),
                    np.where(rng.random(n) < .5, 1500, rng.integers(54, 1400, n))).astype(np.uint16)
    desc, nbytes = pktgen.layout_from_lengths(lens, 6)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, 71, 0)
    fb, fd = fuzz_batch(512, 72, True)                # padded / truncated datagrams, 64 B slots
    base = nbytes
    buf = np.concatenate([buf, fb])
    fd = fd.copy()
    fd["offset"] = (fd["offset"] >> 6) + (base >> 6)     # byte offsets -> 64 B units
    desc = np.concatenate([desc, fd])
    assert buf.nbytes // len(desc) <= 2048
    want = oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(None, 8, 1))
    assert (want["verdict"] == 0).sum() > 3000
    for sched in SCHEDS:
        with ctx_for(gpu, monkeypatch, sched, rss=True, rss_queues=8, rss_endian=True) as ctx:
            assert_same(run_rx_dev(ctx, buf, desc, 6), want, f"{sched} short trips, chunk")
            b = to_dev(buf)
            bdesc = desc.copy()
            bdesc["offset"] = desc["offset"] << 6
            ptrs, lns = ptr_burst(b, bdesc)
            out = dev_results(len(desc))
            ctx.rx_ptrs_dev(ptrs, lns, len(desc), out)
            torch.cuda.synchronize()
            assert_same(out.cpu().numpy().view(RESULT_DTYPE), want, f"{sched} short trips, pointers")


@pytest.mark.parametrize("key,nq,endian", [(None, 8, 1), ("ms", 16, 0), ("ms", 5, 1)])
@pytest.mark.parametrize("sched", ["wave", "row"])
def test_small_kernels_toeplitz_both_keys(gpu, monkeypatch, key, nq, endian, sched):
    """RSS in the small-batch kernels — the wave kernel's lane-parallel
    Toeplitz (key windows from the key words, no table), the grouped kernels'
    LDS tables — for both keys of util/rss.c."""
    k = oracle.KEY_MICROSOFT if key == "ms" else None
    n, seed = 8192, 62
    desc, nbytes = pktgen.layout(n, "bimodal", 6, seed)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, seed, 0)
    want = oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(k, nq, endian))
    with ctx_for(gpu, monkeypatch, sched, rss=True, rss_key=k, rss_queues=nq,
                 rss_endian=bool(endian)) as ctx:
        got = run_rx_dev(ctx, buf, desc, 6)
    assert_same(got, want, f"toeplitz key={key} nq={nq} endian={endian}")
    assert len(np.unique(got["rss_queue"])) == nq


def _even_phase(i):
    return (2 * i) % 128


@pytest.mark.parametrize("sched", SCHEDS)
def test_golden_at_every_even_start(gpu, golden, monkeypatch, sched):
    """The golden frames at every 2-byte alignment inside a 128 B line: the
    reference's records (chunk and pointer modes) and its tx fills."""
    buf, desc = repack(golden.buf, golden.desc, 0, _even_phase)
    n = len(desc)
    with ctx_for(gpu, monkeypatch, sched, rss=True, rss_queues=golden.rss_num_queues) as ctx:
        got = run_rx_dev(ctx, buf, desc, 0)
        b = to_dev(buf)
        ptrs, lens = ptr_burst(b, desc)
        out = dev_results(n)
        ctx.rx_ptrs_dev(ptrs, lens, n, out)
        ctx.tx_fill_dev(b, to_dev(desc), n, 0)
        torch.cuda.synchronize()
        got_p = out.cpu().numpy().view(RESULT_DTYPE)
        filled = b.cpu().numpy()
    assert not compare_results(got, golden), compare_results(got, golden)
    assert not compare_results(got_p, golden), compare_results(got_p, golden)
    want_fill = buf.copy()
    oracle.tx_fill(want_fill, desc, 0)
    assert np.array_equal(filled, want_fill)
    # odd starts are refused
    d = desc[:64].copy()
    d["offset"] += 1
    with ctx_for(gpu, monkeypatch, sched) as ctx:
        assert (run_rx_dev(ctx, buf, d, 0)["verdict"] == 11).all()


@pytest.mark.parametrize("sched", SCHEDS)
def test_fused_flow_bins_golden(gpu, golden, monkeypatch, sched):
    """rx + HashFlow in one launch: the reference's bins for the golden chunk
    (HashFlow over the keys it handed to StreamHTSearch, golden_flow.c)."""
    n = len(golden.desc)
    b = to_dev(golden.buf)
    d = to_dev(golden.desc)
    with ctx_for(gpu, monkeypatch, sched, rss=True, rss_queues=golden.rss_num_queues) as ctx:
        out = dev_results(n)
        bins = torch.full((n,), 7, dtype=torch.int32, device=DEV)
        ctx.rx_chunk_flow_dev(b, d, n, 0, out, bins)
        ptrs, lens = ptr_burst(b, golden.desc)
        out_p = dev_results(n)
        bins_p = torch.full((n,), 7, dtype=torch.int32, device=DEV)
        ctx.rx_ptrs_flow_dev(ptrs, lens, n, out_p, bins_p)
        torch.cuda.synchronize()
    got = out.cpu().numpy().view(RESULT_DTYPE)
    assert not compare_results(got, golden)
    assert np.array_equal(out.cpu().numpy(), out_p.cpu().numpy())
    gb = bins.cpu().numpy().view(np.uint32)
    ok = golden.meta["ref_ub"] == 0
    assert np.array_equal(gb[ok], golden.flow_bins[ok])
    assert np.array_equal(gb, oracle.flow_bins(got))
    assert np.array_equal(bins_p.cpu().numpy().view(np.uint32), gb)


@pytest.mark.parametrize("size,n", [(1500, 1 << 20), ("bimodal", (1 << 20) + 77), (1500, 3000)])
def test_fused_flow_bins_equal_separate_pass(gpu, size, n):
    """At full size (and past one launch's held passes) the fused bins equal
    f3's separate kernel over the same records."""
    seed = 63
    desc, nbytes = pktgen.layout(n, size, 6, seed)
    b = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    d = to_dev(desc)
    gpu.pktgen_dev(b, d, n, 6, seed)
    out = dev_results(n)
    bins = torch.full((n,), 7, dtype=torch.int32, device=DEV)
    sep = torch.full((n,), 9, dtype=torch.int32, device=DEV)
    out2 = dev_results(n)
    with gpu.Context(0, rss=size == "bimodal", rss_queues=8) as ctx:
        ctx.rx_chunk_flow_dev(b, d, n, 6, out, bins)
        ctx.rx_chunk_dev(b, d, n, 6, out2)
        ctx.flow_hash_dev(out, n, sep)
        torch.cuda.synchronize()
    assert torch.equal(out, out2)
    assert torch.equal(bins, sep)
    assert (bins.cpu().numpy().view(np.uint32) != 0xFFFFFFFF).mean() > 0.99


@pytest.mark.parametrize("sched", ["wave", "row", "quad", "oct"])
def test_tx_fill_ptrs_golden(gpu, golden, monkeypatch, sched):
    """mtcp_gpu_tx_fill_ptrs (host frames, e.g. a DPDK m_table burst) and
    _dev (device-accessible frames): exactly the reference's fills, and only
    the two check fields of the filled frames change."""
    n = len(golden.desc)
    offs = golden.desc["offset"].astype(np.int64)
    want = golden.buf.copy()
    assert oracle.tx_fill(want, golden.desc, 0) == golden.manifest["tx_filled"]
    with ctx_for(gpu, monkeypatch, sched) as ctx:
        host = golden.buf.copy()
        assert ctx.tx_fill_ptrs(host, offs, golden.desc["len"]) == golden.manifest["tx_filled"]
        assert np.array_equal(host, want)
        # the bounded form (gpu_module.c's send_pkts) fills the same bytes
        host = golden.buf.copy()
        assert ctx.tx_fill_ptrs(host, offs, golden.desc["len"], timeout_us=2_000_000) == \
            golden.manifest["tx_filled"]
        assert np.array_equal(host, want)
        # a 64-frame burst (MAX_PKT_BURST) at 2-byte-aligned starts
        buf2, d2 = repack(golden.buf, golden.desc[:64], 0, _even_phase)
        w2 = buf2.copy()
        k = oracle.tx_fill(w2, d2, 0)
        h2 = buf2.copy()
        assert ctx.tx_fill_ptrs(h2, d2["offset"].astype(np.int64), d2["len"]) == k
        assert np.array_equal(h2, w2)
        b = to_dev(golden.buf)
        ptrs, lens = ptr_burst(b, golden.desc)
        ctx.tx_fill_ptrs_dev(ptrs, lens, n)
        torch.cuda.synchronize()
        assert np.array_equal(b.cpu().numpy(), want)


def test_reserve_and_rxq_after_host_calls(gpu, golden):
    """mtcp_gpu_reserve(ctx, 0, 0) — which mtcp_gpu_rxq_create
    calls — on a context whose stage 0 a host call already allocated."""
    from mtcp_amd._lib import lib
    L = lib()
    with gpu.Context(0, rss=True, rss_queues=golden.rss_num_queues) as ctx:
        got = ctx.rx_chunk(golden.buf, golden.desc, 0)           # allocates stage 0
        assert not compare_results(got, golden)
        ctx.reserve(0, 0)
        q = ctypes.c_void_p()
        assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, 64, 64 * 2048) == 0
        L.mtcp_gpu_rxq_destroy(q)
        ctx.reserve(4096, 64)
        ctx.reserve(0, 0)
        got = ctx.rx_chunk(golden.buf, golden.desc, 0)
        assert not compare_results(got, golden)


def max_length_frames(n=64, seed=7):
    """n IPv4/TCP frames of 65 535 B down to 65 472 B (tot_len up to 65 521,
    the u16 limit of desc.len) whose payload is all 0xFF, the checksums
    filled by the oracle's tx fill and every eighth frame's payload bit
    flipped after it: the largest one's-complement sums any kernel meets
    (rx_span_kernel's per-frame LDS sum of 4 096 chunks x up to 524 280 is
    about 2.15e9, below 2^32)."""
    rng = np.random.default_rng(seed)
    lens = (65535 - np.arange(n)).astype(np.uint16)
    slots = (lens.astype(np.int64) + 63) & ~63
    offs = np.concatenate([[0], np.cumsum(slots)[:-1]])
    buf = np.full(int(slots.sum()), 0xFF, np.uint8)
    desc = np.zeros(n, DESC_DTYPE)
    desc["offset"] = (offs >> 6).astype(np.uint32)
    desc["len"] = lens
    for i in range(n):
        f = buf[offs[i]:offs[i] + int(lens[i])]
        f[0:12] = rng.integers(0, 256, 12, dtype=np.uint8)
        f[12:14] = (0x08, 0x00)
        tot = int(lens[i]) - 14
        f[14:34] = (0x45, 0, tot >> 8, tot & 0xFF, 0, 1, 0x40, 0, 64, 6, 0, 0, *rng.integers(0, 256, 8))
        f[34:54] = (*rng.integers(0, 256, 12), 0x50, 0x10, 0xFF, 0xFF, 0, 0, 0, 0)
    assert oracle.tx_fill(buf, desc, 6) == n
    for i in range(0, n, 8):
        buf[offs[i] + 60000] ^= 0x10
    return buf, desc


@pytest.mark.parametrize("sched", SCHEDS)
def test_max_length_frames_every_schedule(gpu, monkeypatch, sched):
    """frames at the u16 length limit, all-0xFF payload, through
    every kernel (a forced span included) and the pointer path: equal to the
    oracle, TCP_OK except the flipped ones (TCP_CSUM_BAD)."""
    buf, desc = max_length_frames()
    want = oracle.rx_chunk(buf, desc, 6)
    assert (want["verdict"][::8] == 9).all() and (np.delete(want["verdict"], np.s_[::8]) == 0).all()
    n = len(desc)
    with ctx_for(gpu, monkeypatch, sched) as ctx:
        assert_same(run_rx_dev(ctx, buf, desc, 6), want, f"{sched} max-length chunk")
        b = to_dev(buf)
        pd = desc.copy()
        pd["offset"] = (desc["offset"].astype(np.int64) << 6).astype(np.uint32)
        ptrs, lens = ptr_burst(b, pd)
        out = dev_results(n)
        ctx.rx_ptrs_dev(ptrs, lens, n, out)
        torch.cuda.synchronize()
        assert_same(out.cpu().numpy().view(RESULT_DTYPE), want, f"{sched} max-length pointers")


@pytest.mark.parametrize("n,size,hint", [
    (1 << 16, "bimodal", (700, 800)),       # a mix claimed uniform: 8 lanes per packet on it
    ((1 << 17) + 1, "imix", (700, 800)),    # the span kernel on an IMIX claimed uniform 768 B
    (4096, "bimodal", (256, 300)),          # 8 lanes at 4 K
    ((1 << 16) + 1, 256, (0, 0)),           # empty hint
    ((1 << 16) + 1, 256, (900, 100)),       # min > max
    ((1 << 16) + 1, 256, (1, 65535)),       # a hint wider than the batch
])
def test_records_never_depend_on_the_hint(gpu, monkeypatch, n, size, hint):
    """mtcp_gpu_size_hint only chooses a kernel: a hint that is wrong, empty
    or inverted still gives the oracle's records, byte for byte (every
    kernel is exact for any frame mix; include/mtcp_gpu.h)."""
    monkeypatch.delenv("MTCP_GPU_SCHED", raising=False)
    seed = 71
    if size == "imix":
        desc, nbytes = pktgen.layout_from_lengths(imix_lengths(n, seed), 6)
    else:
        desc, nbytes = pktgen.layout(n, size, 6, seed)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, seed, 0)
    want = oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(None, 8, 1))
    with gpu.Context(0, rss=True, rss_queues=8, rss_endian=True) as ctx:
        assert_same(run_rx_dev(ctx, buf, desc, 6, hint=hint), want, f"{size} x {n} hint {hint}")
