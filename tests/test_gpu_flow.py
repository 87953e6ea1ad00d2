"""SURVEY §8 f3/f4 on the GPU, through the C ABI: HashFlow of the flow-table
key (mtcp/src/tcp_stream.c:56-90 over tcp_in.c:1180-1186) and the
RSS-friendly address-pool search (mtcp/src/addr_pool.c:103-180).  Bit-exact
against the reference's golden vectors and the oracle."""
import numpy as np
import pytest

import oracle
from mtcp_amd import RESULT_DTYPE, pktgen
from tests.golden_io import pool_case_entries, pool_entries_equal

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    from mtcp_amd import gpu as g
    return g


def to_dev(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(DEV)


def test_flow_hash_golden_rx(gpu, golden):
    # input: the reference's own rx results; expected: the reference's
    # HashFlow of the key it handed to StreamHTSearch
    ok = golden.meta["ref_ub"] == 0
    with gpu.Context() as ctx:
        host = ctx.flow_hash(golden.expect)
        d_res = to_dev(golden.expect)
        d_bins = torch.zeros(len(golden.expect), dtype=torch.int32, device=DEV)
        ctx.flow_hash_dev(d_res, len(golden.expect), d_bins)
        torch.cuda.synchronize()
        dev = d_bins.cpu().numpy().view(np.uint32)
    assert np.array_equal(host[ok], golden.flow_bins[ok])
    assert np.array_equal(dev, host)


def test_flow_hash_cases(gpu, golden):
    # every key of flow_cases.bin as the stream key of a TCP_OK result
    c = golden.flow_cases
    res = np.zeros(len(c), dtype=RESULT_DTYPE)
    k = c["key"]
    # key = saddr(stream) | daddr(stream) | sport | dport = iph->daddr | iph->saddr | dest | source
    res["daddr"] = k[:, 0:4].copy().view("<u4")[:, 0]
    res["saddr"] = k[:, 4:8].copy().view("<u4")[:, 0]
    res["dport"] = k[:, 8:10].copy().view("<u2")[:, 0]
    res["sport"] = k[:, 10:12].copy().view("<u2")[:, 0]
    res["verdict"] = 0
    res["verdict"][::7] = 9                       # not TCP_OK: no flow lookup
    with gpu.Context() as ctx:
        got = ctx.flow_hash(res)
    want = c["hash"].copy()
    want[::7] = 0xFFFFFFFF
    assert np.array_equal(got, want)


def test_flow_hash_full_size_vs_oracle(gpu):
    # 1 M generated packets: rx on the GPU, HashFlow on the GPU, oracle on both
    n, size, seed = 1 << 20, "bimodal", 3
    desc, total = pktgen.layout(n, size, seed=seed)
    buf = torch.zeros((total + 15) & ~15, dtype=torch.uint8, device=DEV)
    d_desc = to_dev(desc)
    gpu.pktgen_dev(buf, d_desc, n, 6, seed)
    out = torch.zeros(n * 40, dtype=torch.uint8, device=DEV)
    bins = torch.zeros(n, dtype=torch.int32, device=DEV)
    with gpu.Context() as ctx:
        ctx.rx_chunk_dev(buf, d_desc, n, 6, out)
        ctx.flow_hash_dev(out, n, bins, stream=ctx.stream)
        ctx.sync()
    res = out.cpu().numpy().view(RESULT_DTYPE)
    got = bins.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, oracle.flow_bins(res))
    ok = res["verdict"] == 0
    assert ok.sum() > n * 0.99 and (got[~ok] == 0xFFFFFFFF).all()
    assert len(np.unique(got[ok])) > 100000       # spread over the 131072 bins


def test_addr_pool_search_golden(gpu, golden):
    with gpu.Context() as ctx:           # the context's key: 0x05 x 40 (mtcp/src/rss.c:18-24)
        for c, saddr, sport in pool_case_entries(golden):
            got = ctx.addr_pool_search(int(c["core"]), int(c["nq"]), int(c["saddr_base"]),
                                       int(c["num_addr"]), int(c["daddr"]), int(c["dport"]),
                                       bool(c["endian"]))
            assert pool_entries_equal(got, saddr, sport), dict(zip(c.dtype.names, c.tolist()))


def test_addr_pool_search_microsoft_key_vs_oracle(gpu):
    key = oracle.KEY_MICROSOFT
    with gpu.Context(rss_key=key) as ctx:
        for core, nq, num_addr, endian in [(0, 4, 3, 1), (7, 8, 2, 0), (2, 5, 1, 1)]:
            args = (core, nq, 0x0100A8C0, num_addr, 0x0101A8C0, 0x5000, endian)
            got = ctx.addr_pool_search(*args)
            want = oracle.addr_pool_search(key, *args)
            assert len(got) == len(want) and np.array_equal(got["saddr"], want["saddr"])
            assert np.array_equal(got["sport"], want["sport"])
            # max_out truncation keeps the first entries
            part = ctx.addr_pool_search(*args, max_out=100)
            assert np.array_equal(part, got[:100])


def test_rss_queue_map_vs_oracle(gpu):
    num_addr, nq = 2, 6
    base_h, daddr_h, dport_h = 0x0A000010, 0x0A0000FE, 443
    q = torch.zeros(num_addr * 64511 + 3, dtype=torch.uint8, device=DEV)
    cache = oracle.key_cache(oracle.KEY_0X05)
    with gpu.Context() as ctx:
        ctx.rss_queue_map_dev(base_h, num_addr, daddr_h, dport_h, nq, True, q)
        ctx.sync()
    got = q.cpu().numpy()
    assert (got[num_addr * 64511:] == 0).all()    # nothing past the candidates
    rng = np.random.default_rng(5)
    for g in rng.integers(0, num_addr * 64511, 2000):
        i, port = divmod(int(g), 64511)
        want = oracle.rss_cpu_core(cache, daddr_h, base_h + i, dport_h, 1025 + port, nq, 1)
        assert got[g] == want, (i, port)


@pytest.mark.parametrize("key_name,num_addr,nq,endian", [("0x05", 3, 5, 1), ("microsoft", 3, 16, 0),
                                                         ("microsoft", 2, 3, 1), ("0x05", 1, 1, 0)])
def test_rss_queue_map_every_candidate(gpu, key_name, num_addr, nq, endian):
    """The queue map (the split Toeplitz: a per-address part and two port-byte
    tables, flow_kernels.hpp) equals GetRSSCPUCore (rss.c:90-103, the oracle)
    on EVERY candidate, across address edges inside a workgroup's tile and
    the batch's ragged end; nothing written past the candidates."""
    key = oracle.KEY_0X05 if key_name == "0x05" else oracle.KEY_MICROSOFT
    base_h, daddr_h, dport_h = 0xC0A80A01, 0x0A000005, 8080
    total = num_addr * 64511
    q = torch.full((total + 64,), 0xAA, dtype=torch.uint8, device=DEV)
    cache = oracle.key_cache(key)
    with gpu.Context(rss_key=key) as ctx:
        ctx.rss_queue_map_dev(base_h, num_addr, daddr_h, dport_h, nq, bool(endian), q)
        ctx.sync()
    got = q.cpu().numpy()
    assert (got[total:] == 0xAA).all()
    want = np.empty(total, np.uint8)
    for i in range(num_addr):
        for port in range(64511):
            want[i * 64511 + port] = oracle.rss_cpu_core(cache, daddr_h, base_h + i, dport_h, 1025 + port,
                                                         nq, endian)
    bad = np.nonzero(got[:total] != want)[0]
    assert len(bad) == 0, (len(bad), bad[:10])


def test_rss_queue_map_more_tiles_than_the_grid(gpu):
    """200 addresses = 12.9 M candidates = 3 150 tiles of 4 096, more than
    the launch's 8 workgroups per CU: the kernel walks the extra tiles
    grid-stride.  A sample of 30 000 candidates from everywhere plus every
    candidate of the first and the last address equal the oracle's
    GetRSSCPUCore (rss.c:90-103); nothing written past the end."""
    num_addr, nq = 200, 7
    base_h, daddr_h, dport_h = 0x0A010001, 0xAC100002, 5201
    total = num_addr * 64511
    q = torch.full((total + 64,), 0xAA, dtype=torch.uint8, device=DEV)
    cache = oracle.key_cache(oracle.KEY_0X05)
    with gpu.Context() as ctx:
        ctx.rss_queue_map_dev(base_h, num_addr, daddr_h, dport_h, nq, True, q)
        ctx.sync()
    got = q.cpu().numpy()
    assert (got[total:] == 0xAA).all()
    rng = np.random.default_rng(11)
    idx = np.unique(np.concatenate([rng.integers(0, total, 30000), np.arange(64511),
                                    np.arange(total - 64511, total)]))
    for g in idx:
        i, port = divmod(int(g), 64511)
        want = oracle.rss_cpu_core(cache, daddr_h, base_h + i, dport_h, 1025 + port, nq, 1)
        assert got[g] == want, (i, port)
