"""Error behaviour of the C ABI on a GPU box: arguments the kernels' address
arithmetic relies on are rejected with MTCP_GPU_EINVAL before anything is
launched (the reference's own code has no such checks: its callers exit or
read out of bounds, SURVEY §8b "Errors"), empty batches succeed with null
pointers, and a rejected call leaves the context usable."""
import numpy as np
import pytest

from mtcp_amd import pktgen
from tests.test_gpu_parity import DEV, dev_results, to_dev

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

EINVAL = -22


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    from mtcp_amd import gpu
    c = gpu.Context(0)
    yield c
    c.close()


def test_rejects_what_the_kernel_assumes(ctx):
    from mtcp_amd._lib import lib
    L = lib()
    n = 64
    desc, nbytes = pktgen.layout(n, 64, 6, 1)
    b = torch.zeros(nbytes + 64, dtype=torch.uint8, device=DEV)
    d = to_dev(desc)
    from mtcp_amd import gpu
    gpu.pktgen_dev(b, d, n, 6, 1)
    out = dev_results(n)
    h, pb, pd, po = ctx._h, b.data_ptr(), d.data_ptr(), out.data_ptr()
    assert L.mtcp_gpu_rx_chunk_dev(h, pb + 1, nbytes, pd, n, 6, po, None) == EINVAL      # 16 B base
    assert L.mtcp_gpu_rx_chunk_dev(h, pb, nbytes + 4, pd, n, 6, po, None) == EINVAL      # length % 16
    assert L.mtcp_gpu_rx_chunk_dev(h, pb, nbytes, pd, n, 17, po, None) == EINVAL         # off_shift
    assert L.mtcp_gpu_rx_chunk_dev(h, pb, nbytes, pd + 4, n, 6, po, None) == EINVAL      # desc align
    assert L.mtcp_gpu_rx_chunk_dev(h, pb, nbytes, pd, n, 6, po + 4, None) == EINVAL      # out align
    assert L.mtcp_gpu_rx_chunk_dev(h, None, nbytes, pd, n, 6, po, None) == EINVAL
    assert L.mtcp_gpu_rx_chunk_dev(None, pb, nbytes, pd, n, 6, po, None) == EINVAL
    assert L.mtcp_gpu_rx_ptrs_dev(h, pd, None, n, po, None) == EINVAL
    assert L.mtcp_gpu_tx_fill_dev(h, pb, nbytes, None, n, 6, None) == EINVAL
    assert L.mtcp_gpu_flow_hash_dev(h, None, n, po, None) == EINVAL
    # empty batches: nothing to read, null pointers allowed
    assert L.mtcp_gpu_rx_chunk_dev(h, None, 0, None, 0, 6, None, None) == 0
    assert L.mtcp_gpu_rx_ptrs_dev(h, None, None, 0, None, None) == 0
    # the context still works after the rejections
    ctx.rx_chunk_dev(b, d, n, 6, out)
    torch.cuda.synchronize()
    from mtcp_amd import RESULT_DTYPE
    got = out.cpu().numpy().view(RESULT_DTYPE)
    assert got["ip_len"].tolist() == [50] * n


def test_descriptor_past_the_buffer_is_a_verdict_not_a_fault(ctx):
    """Descriptors are data: one that points past buf_len gets BAD_DESC and
    nothing outside the buffer is read."""
    n = 256
    desc, nbytes = pktgen.layout(n, 1500, 6, 2)
    b = torch.zeros(nbytes, dtype=torch.uint8, device=DEV)
    d = desc.copy()
    d["offset"][::7] = 0xFFFFFFFF                   # 256 GiB past the base with off_shift 6
    d["len"][1::7] = 65535
    out = dev_results(n)
    ctx.rx_chunk_dev(b, to_dev(d), n, 6, out)
    torch.cuda.synchronize()
    from mtcp_amd import RESULT_DTYPE
    v = out.cpu().numpy().view(RESULT_DTYPE)["verdict"]
    pos = desc["offset"].astype(np.int64) << 6
    past = (d["offset"] == 0xFFFFFFFF) | (pos + d["len"].astype(np.int64) > nbytes)
    assert past.sum() > n // 7
    assert (v[past] == 11).all()                     # MTCP_GPU_V_BAD_DESC
    assert (v[~past] != 11).all()


def test_context_on_another_device_orders_on_its_own_stream():
    """a Context opened on device d, called with stream=None while
    another device is current, queues its kernel on device d's current stream
    and gives the oracle's records (needs two GPUs; the pool's boxes have one)."""
    import numpy as np
    import torch
    import oracle
    from mtcp_amd import RESULT_DTYPE, gpu, pktgen
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU visible")
    d = torch.cuda.device_count() - 1
    n, seed = 4096, 9
    desc, nbytes = pktgen.layout(n, 1500, 6, seed)
    dev = torch.device("cuda", d)
    b = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    dd = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    out = torch.zeros(n * 40, dtype=torch.uint8, device=dev)
    torch.cuda.set_device(0)
    gpu.pktgen_dev(b, dd, n, 6, seed, stream=torch.cuda.current_stream(d))
    with gpu.Context(d) as ctx:
        ctx.rx_chunk_dev(b, dd, n, 6, out)
        torch.cuda.synchronize(d)
    got = out.cpu().numpy().view(RESULT_DTYPE)
    want = oracle.rx_chunk(b.cpu().numpy(), desc, 6)
    assert got.tobytes() == want.tobytes()
