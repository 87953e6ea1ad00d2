"""The compact 16 B record (MTCP_GPU_F_COMPACT, include/mtcp_gpu.h
mtcp_gpu_result16) on the MI355X, bit-exact.

Every field of the compact record equals the same-named field of the 40 B
record, so the oracle's (and the reference's golden) 40 B records projected
onto the 16 B layout (mtcp_amd.compact_of) are the expectation:

* every kernel (wave / row / quad / rx_kernel, forced with MTCP_GPU_SCHED),
  chunk and pointer modes, with and without RSS, on the golden vectors and on
  config-shaped batches, with the flow bins fused in (the compact record has
  no 4-tuple: the bin is computed in phase 2 and held beside it);
* the host entry points (staged pipeline, pointer gather);
* the 1 M-packet C3 batch (rx_kernel's sorted schedule with RSS, the kernel
  the compact bench line measures) against the 40 B run of the same frames;
* an rxq on a compact context (the io_module's rxqs): the same NULL set;
* flow_hash entry points refuse a compact context (they read the 4-tuple).
The caller the compact record serves only needs the verdict: mTCP's own
offload pattern reads one checksum bit per frame (dpdk_module.c:473-479).
"""
import ctypes

import numpy as np
import pytest

import oracle
from mtcp_amd import RESULT16_DTYPE, RESULT_DTYPE, compact_of, pktgen
from tests.golden_io import compare_results
from tests.test_gpu_parity import DEV, to_dev

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SCHEDS = ["wave", "row", "quad", "oct", "span", "big"]


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    from mtcp_amd import gpu as g
    return g


def ctx_for(gpu, monkeypatch, sched, **kw):
    if sched != "auto":
        monkeypatch.setenv("MTCP_GPU_SCHED", sched)
    c = gpu.Context(0, compact=True, **kw)
    monkeypatch.delenv("MTCP_GPU_SCHED", raising=False)
    return c


def assert_same16(got, want, what=""):
    assert got.dtype == RESULT16_DTYPE and len(got) == len(want)
    for f in RESULT16_DTYPE.names:
        diff = np.nonzero(got[f] != want[f])[0]
        assert len(diff) == 0, (
            f"{what} field {f}: {len(diff)} mismatches, first #{diff[0]} got {got[f][diff[0]]} "
            f"want {want[f][diff[0]]} (verdict got {got['verdict'][diff[0]]} "
            f"want {want['verdict'][diff[0]]})")


def rx16(ctx, b, d, n, off_shift, ptrs=None, bins=None):
    out = torch.full((n * 16,), 0xEE, dtype=torch.uint8, device=DEV)   # every byte must be written
    if ptrs is not None:
        if bins is not None:
            ctx.rx_ptrs_flow_dev(ptrs[0], ptrs[1], n, out, bins)
        else:
            ctx.rx_ptrs_dev(ptrs[0], ptrs[1], n, out)
    elif bins is not None:
        ctx.rx_chunk_flow_dev(b, d, n, off_shift, out, bins)
    else:
        ctx.rx_chunk_dev(b, d, n, off_shift, out)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(RESULT16_DTYPE)


def padded(buf):
    pad = (-buf.nbytes) % 16
    return np.concatenate([buf, np.zeros(pad, np.uint8)]) if pad else buf


@pytest.mark.parametrize("sched", ["auto"] + SCHEDS)
@pytest.mark.parametrize("rss", [False, True])
def test_compact_golden_every_kernel(gpu, golden, monkeypatch, sched, rss):
    n = len(golden.desc)
    cfg = oracle.rss_cfg(oracle.KEY_0X05, golden.rss_num_queues, 1) if rss else None
    want40 = oracle.rx_chunk(golden.buf, golden.desc, 0, cfg)
    want = compact_of(want40)
    b, d = to_dev(padded(golden.buf)), to_dev(golden.desc)
    ptrs = (torch.from_numpy(golden.desc["offset"].astype(np.int64) + b.data_ptr()).to(DEV),
            torch.from_numpy(golden.desc["len"].view(np.int16).copy()).to(DEV))
    bins = torch.zeros(n, dtype=torch.int32, device=DEV)
    kw = dict(rss=True, rss_queues=golden.rss_num_queues) if rss else {}
    with ctx_for(gpu, monkeypatch, sched, **kw) as ctx:
        assert ctx.record_size == 16
        got = rx16(ctx, b, d, n, 0)
        kernel = ctx.last_kernel
        got_f = rx16(ctx, b, d, n, 0, bins=bins)
        bins_c = bins.cpu().numpy().view(np.uint32).copy()
        got_p = rx16(ctx, b, d, n, 0, ptrs=ptrs, bins=bins)
        bins_p = bins.cpu().numpy().view(np.uint32).copy()
    assert kernel, "mtcp_gpu_last_kernel names the dispatched kernel"
    if sched in ("wave", "row", "quad", "oct", "span"):
        assert kernel.startswith({"wave": "rx_wave", "row": "rx_group_kernel<row", "quad": "rx_group_kernel<quad",
                                  "oct": "rx_group_kernel<oct", "span": "rx_span_kernel"}[sched]), kernel
    elif sched == "big":
        assert kernel.startswith("rx_kernel"), kernel
    for g, what in ((got, "chunk"), (got_f, "chunk+bins"), (got_p, "ptrs+bins")):
        assert_same16(g, want, f"{sched} {what} vs oracle")
    # the reference's own values where they are defined (ref-UB frames aside)
    ok = golden.meta["ref_ub"] == 0
    ref16 = compact_of(golden.expect)
    for f in RESULT16_DTYPE.names:
        if f in ("rss_hash", "rss_queue") and not rss:
            continue
        assert np.array_equal(got[f][ok], ref16[f][ok]), f
    want_bins = oracle.flow_bins(want40)
    assert np.array_equal(bins_c, want_bins) and np.array_equal(bins_p, want_bins)
    assert np.array_equal(bins_c[ok], golden.flow_bins[ok])


@pytest.mark.parametrize("sched", SCHEDS)
@pytest.mark.parametrize("size,n", [(64, 4096), ("bimodal", 65536), (1500, 65536), (9000, 4096)])
def test_compact_config_batches(gpu, monkeypatch, sched, size, n):
    seed = 11
    desc, nbytes = pktgen.layout(n, size, 6, seed)
    b = torch.zeros(nbytes, dtype=torch.uint8, device=DEV)
    d = to_dev(desc)
    gpu.pktgen_dev(b, d, n, 6, seed)
    host = b.cpu().numpy()
    want = compact_of(oracle.rx_chunk(host, desc, 6, oracle.rss_cfg(None, 8, 1)))
    with ctx_for(gpu, monkeypatch, sched, rss=True, rss_queues=8) as ctx:
        got = rx16(ctx, b, d, n, 6)
    assert_same16(got, want, f"{sched} {size} x {n}")


def test_compact_host_entry_points(gpu, golden):
    cfg = oracle.rss_cfg(oracle.KEY_0X05, golden.rss_num_queues, 1)
    want = compact_of(oracle.rx_chunk(golden.buf, golden.desc, 0, cfg))
    with gpu.Context(0, rss=True, rss_queues=golden.rss_num_queues, compact=True) as ctx:
        got = ctx.rx_chunk(golden.buf, golden.desc, 0)
        frames = [golden.buf[int(o):int(o) + int(n)] for o, n in
                  zip(golden.desc["offset"][:2000], golden.desc["len"][:2000])]
        got_p = ctx.rx_ptrs(frames)
        with pytest.raises(ValueError):
            ctx.rx_chunk(golden.buf, golden.desc, 0, np.zeros(len(golden.desc), RESULT_DTYPE))
    assert got.dtype == RESULT16_DTYPE
    assert_same16(got, want, "host chunk")
    assert_same16(got_p, want[:2000], "host ptrs")


def test_compact_c3_full_size_equals_full_records(gpu):
    """1 M bimodal packets with RSS (the C3 bench config): the compact run's
    records equal the 40 B run's, field by field, for every packet."""
    n, seed = 1 << 20, 3
    desc, nbytes = pktgen.layout(n, "bimodal", 6, seed)
    b = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    d = to_dev(desc)
    gpu.pktgen_dev(b, d, n, 6, seed)
    out40 = torch.empty(n * 40, dtype=torch.uint8, device=DEV)
    with gpu.Context(0, rss=True, rss_queues=8) as ctx:
        ctx.rx_chunk_dev(b, d, n, 6, out40)
        torch.cuda.synchronize()
    with gpu.Context(0, rss=True, rss_queues=8, compact=True) as ctx:
        got = rx16(ctx, b, d, n, 6)
        assert ctx.last_kernel == "rx_kernel<sorted>"
    full = out40.cpu().numpy().view(RESULT_DTYPE)
    assert_same16(got, compact_of(full), "C3 compact vs 40 B")
    assert (got["verdict"] == 0).mean() > 0.99


def test_compact_rxq_drops_the_same_frames(gpu, golden):
    """mtcp_gpu_rxq on a compact context (gpu_module.c opens its contexts so):
    the same NULL set as the reference's checksum drops + ref-UB frames; the
    record handed back is the 16 B one."""
    from mtcp_amd._lib import lib
    L = lib()
    ok = golden.meta["ref_ub"] == 0
    ref_v = golden.expect["verdict"]
    with gpu.Context(0, compact=True) as ctx:
        q = ctypes.c_void_p()
        assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, len(golden.desc), golden.buf.nbytes * 2) == 0
        try:
            assert L.mtcp_gpu_rxq_push_chunk(q, golden.buf.ctypes.data, golden.desc.ctypes.data,
                                             len(golden.desc), 0) == 0
            done = ctypes.c_uint32()
            assert L.mtcp_gpu_rxq_flush(q, ctypes.byref(done)) == 0
            assert done.value == len(golden.desc)
            nulls = np.zeros(len(golden.desc), bool)
            verdicts = np.zeros(len(golden.desc), np.uint8)
            for i in range(len(golden.desc)):
                ln, res, res40 = ctypes.c_uint16(), ctypes.c_void_p(), ctypes.c_void_p(1)
                p = L.mtcp_gpu_rxq_get16(q, i, ctypes.byref(ln), ctypes.byref(res))
                nulls[i] = p is None
                verdicts[i] = ctypes.cast(res, ctypes.POINTER(ctypes.c_uint8))[14]
                # the 40 B accessor never hands out a 16 B record
                assert L.mtcp_gpu_rxq_get(q, i, None, ctypes.byref(res40)) == p
                assert res40.value is None
        finally:
            L.mtcp_gpu_rxq_destroy(q)
    drop = (ok & np.isin(ref_v, [4, 9])) | (golden.meta["ref_ub"] == 1)
    assert np.array_equal(nulls, drop)
    # and rxq_get16 on a 40 B context: no record
    with gpu.Context(0) as ctx:
        q = ctypes.c_void_p()
        assert L.mtcp_gpu_rxq_create(ctypes.byref(q), ctx._h, 64, 64 * 2048) == 0
        try:
            assert L.mtcp_gpu_rxq_push_chunk(q, golden.buf.ctypes.data, golden.desc.ctypes.data, 64, 0) == 0
            assert L.mtcp_gpu_rxq_flush(q, None) == 0
            res16 = ctypes.c_void_p(1)
            L.mtcp_gpu_rxq_get16(q, 0, None, ctypes.byref(res16))
            assert res16.value is None
        finally:
            L.mtcp_gpu_rxq_destroy(q)
    assert np.array_equal(verdicts[ok], ref_v[ok])


def test_compact_refuses_flow_hash_and_misaligned_out(gpu):
    from mtcp_amd._lib import MtcpGpuError
    with gpu.Context(0, compact=True) as ctx:
        res = torch.zeros(64 * 40, dtype=torch.uint8, device=DEV)
        bins = torch.zeros(64, dtype=torch.int32, device=DEV)
        with pytest.raises(MtcpGpuError):
            ctx.flow_hash_dev(res, 64, bins)
        desc, nbytes = pktgen.layout(64, 64, 6, 1)
        b = torch.zeros(nbytes, dtype=torch.uint8, device=DEV)
        d = to_dev(desc)
        out = torch.zeros(64 * 16 + 8, dtype=torch.uint8, device=DEV)
        with pytest.raises(MtcpGpuError):
            ctx.rx_chunk_dev(b, d, 64, 6, out[8:])      # 16 B records need 16 B alignment
