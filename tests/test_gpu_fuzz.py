"""Randomised parity: tens of thousands of frames with random lengths (1 B to
20 000 B), random bytes, and headers drawn to hit every branch of the
reference's chain (ethertypes, ihl 0..15, version, tot_len shorter / longer
than the frame, protocols, doff 0..15), checksums made valid by the oracle's
tx fill for the frames that qualify, then single-bit corruptions.  GPU and
oracle must agree on every field of every record (rx, both RSS keys), and on
every byte after a tx fill.  Layouts: PSIO 64 B slots, 2-byte-aligned
offsets anywhere in a line, and a pointer burst; each through every kernel
the library dispatches (mtcp_gpu.hip pick_sched, forced with MTCP_GPU_SCHED:
a wavefront, a row or a quad per packet, and rx_kernel)."""
import numpy as np
import pytest

import oracle
from mtcp_amd import RESULT_DTYPE
from tests.fuzz_frames import fuzz_batch
from tests.test_gpu_parity import DEV, assert_same, dev_results, run_rx_dev, to_dev

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    from mtcp_amd import gpu as g
    return g


SCHEDS = ["wave", "row", "quad", "oct", "span", "big"]


@pytest.mark.parametrize("sched", SCHEDS)
@pytest.mark.parametrize("seed,aligned,key,nq,endian", [
    (101, True, None, 16, 1), (102, False, oracle.KEY_MICROSOFT, 7, 0), (103, False, None, 3, 1)],
    ids=["psio-key05-nq16", "unaligned-microsoft-nq7-noendian", "unaligned-key05-nq3"])
def test_fuzz_rx_matches_oracle(gpu, seed, aligned, key, nq, endian, sched, monkeypatch):
    buf, desc = fuzz_batch(6000, seed, aligned)
    want = oracle.rx_chunk(buf, desc, 0, oracle.rss_cfg(key, nq, endian))
    seen = np.bincount(want["verdict"], minlength=12)
    assert (seen[:11] > 0).sum() >= 10, seen                  # nearly every branch is taken
    monkeypatch.setenv("MTCP_GPU_SCHED", sched)
    with gpu.Context(0, rss=True, rss_key=key, rss_queues=nq, rss_endian=bool(endian)) as ctx:
        assert_same(run_rx_dev(ctx, buf, desc, 0), want, f"fuzz {seed} chunk")
        b = to_dev(buf)
        ptrs = torch.from_numpy(desc["offset"].astype(np.int64) + b.data_ptr()).to(DEV)
        lens = torch.from_numpy(desc["len"].view(np.int16).copy()).to(DEV)
        out = dev_results(len(desc))
        ctx.rx_ptrs_dev(ptrs, lens, len(desc), out)
        torch.cuda.synchronize()
    assert_same(out.cpu().numpy().view(RESULT_DTYPE), want, f"fuzz {seed} pointers")


@pytest.mark.parametrize("sched", SCHEDS)
@pytest.mark.parametrize("seed,aligned", [(201, True), (202, False)])
def test_fuzz_tx_fill_matches_oracle(gpu, seed, aligned, sched, monkeypatch):
    buf, desc = fuzz_batch(6000, seed, aligned)
    want = buf.copy()
    n_want = oracle.tx_fill(want, desc, 0)
    b = to_dev(buf)
    monkeypatch.setenv("MTCP_GPU_SCHED", sched)
    with gpu.Context(0) as ctx:
        ctx.tx_fill_dev(b, to_dev(desc), len(desc), 0)
        torch.cuda.synchronize()
        got = b.cpu().numpy()[:buf.nbytes]
        host = buf.copy()
        n_host = ctx.tx_fill(host, desc, 0)
    assert n_host == n_want > len(desc) // 4
    assert np.array_equal(got, want)
    assert np.array_equal(host, want)


@pytest.mark.parametrize("sched", ["wave", "row", "quad", "oct"])
def test_fuzz_tx_fill_ptrs_matches_oracle(gpu, sched, monkeypatch):
    """The pointer-burst tx fill (host frames: staged, filled, check fields
    written back; device frames: filled in place) on the fuzz frames."""
    buf, desc = fuzz_batch(3000, 203, False)
    want = buf.copy()
    n_want = oracle.tx_fill(want, desc, 0)
    monkeypatch.setenv("MTCP_GPU_SCHED", sched)
    with gpu.Context(0) as ctx:
        host = buf.copy()
        assert ctx.tx_fill_ptrs(host, desc["offset"].astype(np.int64), desc["len"]) == n_want
        b = to_dev(buf)
        ptrs = torch.from_numpy(desc["offset"].astype(np.int64) + b.data_ptr()).to(DEV)
        lens = torch.from_numpy(desc["len"].view(np.int16).copy()).to(DEV)
        ctx.tx_fill_ptrs_dev(ptrs, lens, len(desc))
        torch.cuda.synchronize()
        dev = b.cpu().numpy()[:buf.nbytes]
    assert np.array_equal(host, want)
    assert np.array_equal(dev, want)
