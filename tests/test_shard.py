"""Batch split across ranks, checked on CPU with the oracle:
world_size-2 gloo processes each process their shard; the gathered results
equal the single-batch results packet for packet."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from mtcp_amd import pktgen, shard


def _full(n, size, seed):
    desc, nbytes = pktgen.layout(n, size, 6, seed)
    buf = np.zeros(nbytes, np.uint8)
    oracle.pktgen(buf, desc, 6, seed, 0)
    return buf, desc


@pytest.mark.parametrize("size", [1500, "bimodal"])
def test_bounds_balance(size):
    b = shard.bounds(10000, size, 4, seed=3)
    assert b[0] == 0 and b[-1] == 10000 and all(x <= y for x, y in zip(b, b[1:]))
    if size == "bimodal":
        lens = pktgen.lengths(10000, size, 3)
        padded = (lens.astype(np.int64) + 63) & ~63
        per = [padded[b[r]:b[r + 1]].sum() for r in range(4)]
        assert max(per) - min(per) <= 2 * 1536


def _worker(rank, world, port, size, n, seed, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = shard.make_shard(n, size, rank, world, seed)
    buf = np.zeros(s.nbytes, np.uint8)
    oracle.pktgen(buf, s.desc, 6, seed, s.first_index)
    res = oracle.rx_chunk(buf, s.desc, 6, oracle.rss_cfg(None, 4, 1))
    import torch
    t = torch.from_numpy(res.view(np.uint8).copy())
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([t.numel()]))
    mx = int(max(x.item() for x in sizes))
    pad = torch.zeros(mx, dtype=torch.uint8)
    pad[:t.numel()] = t
    gathered = [torch.zeros(mx, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(gathered, pad)
    if rank == 0:
        out = b"".join(g[:int(sz.item())].numpy().tobytes() for g, sz in zip(gathered, sizes))
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("size,world", [(1500, 2), ("bimodal", 2), ("bimodal", 4)])
def test_two_rank_shards_equal_full_batch(size, world):
    n, seed = 3000, 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000) + 7 * world
    procs = [ctx.Process(target=_worker, args=(r, world, port, size, n, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    buf, desc = _full(n, size, seed)
    want = oracle.rx_chunk(buf, desc, 6, oracle.rss_cfg(None, 4, 1))
    assert got == want.tobytes()


def _fake_topology(root, ncores, smt):
    """A sysfs tree with `ncores` physical cores of `smt` threads each,
    numbered the Linux way (siblings ncores apart)."""
    for c in range(ncores):
        sib = ",".join(str(c + t * ncores) for t in range(smt))
        for t in range(smt):
            d = root / "devices" / "system" / "cpu" / f"cpu{c + t * ncores}" / "topology"
            d.mkdir(parents=True)
            (d / "thread_siblings_list").write_text(sib + "\n")


def test_split_cpus_gives_disjoint_whole_cores(tmp_path):
    """bench.py's N > 1 CPU baseline: ranks on one node split its cores in
    whole physical cores (no two ranks time SMT siblings of one core)."""
    _fake_topology(tmp_path, 64, 2)
    node = set(range(128))
    shares = [shard.split_cpus(node, i, 4, str(tmp_path)) for i in range(4)]
    assert set().union(*shares) == node
    for i, s in enumerate(shares):
        assert len(s) == 32
        prim = sorted(c for c in s if c < 64)
        assert prim == list(range(16 * i, 16 * i + 16))
        assert {c - 64 for c in s if c >= 64} == set(prim)      # siblings travel together
        for t in shares[i + 1:]:
            assert not s & t


def test_split_cpus_edge_cases(tmp_path):
    _fake_topology(tmp_path, 4, 1)
    assert shard.split_cpus({0, 1, 2, 3}, 0, 1, str(tmp_path)) == {0, 1, 2, 3}
    # more ranks than cores: the shares wrap
    assert [shard.split_cpus({0, 1}, i, 4, str(tmp_path)) for i in range(4)] == [{0}, {1}, {0}, {1}]
    # no topology in sysfs: every cpu is its own core
    assert shard.split_cpus({5, 6, 7, 8}, 1, 2, str(tmp_path / "none")) == {7, 8}


def _cpu_baseline_worker(rank, world, port, q):
    """One bench.py rank's N > 1 CPU-baseline leg on the CPU: its shard of a
    C4-shaped batch in host memory, the reference's rx code (or the oracle)
    on its share of the cores, all ranks at once."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.sched_setaffinity(0, shard.split_cpus(os.sched_getaffinity(0), rank, world))
    s = shard.make_shard(4096 * world, 1500, rank, world, 4)
    buf = np.zeros(s.nbytes, np.uint8)
    oracle.pktgen(buf, s.desc, 6, 4, s.first_index)
    r = bench.cpu_baseline_ranks(buf, s.desc, bench.CONFIGS["c4"], 2048, world, rank)
    if rank == 0:
        q.put(r)
    else:
        assert r is None
    dist.barrier()
    dist.destroy_process_group()


def test_cpu_baseline_at_n_ranks():
    """bench.py's CPU baseline at N > 1: every rank
    times its own shard at once; rank 0 reports each rank and the host
    aggregate (all sample bytes / the slowest rank's time), with cores."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000) + 101
    procs = [ctx.Process(target=_cpu_baseline_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    r = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert r["kind"] in ("reference", "port") and r["unit"] == "GB/s"
    assert [x["rank"] for x in r["per_rank"]] == [0, 1]
    assert r["cores"] == sum(x["cores"] for x in r["per_rank"]) >= 2
    slowest = max(x["seconds"] for x in r["per_rank"])
    assert abs(r["value"] - 2 * 2048 * 1500 / slowest / 1e9) < 0.01 * r["value"]   # seconds rounded to 1 us
    assert r["value"] <= sum(x["GB/s"] for x in r["per_rank"]) + 1e-3


def test_split_cpus_eight_shares(tmp_path):
    """bench.py --gpus 8: the ranks whose GPUs share a node split its cores.
    An 8-GPU node with 4 GPUs per socket (64 cores + SMT per socket): each of
    the 4 ranks gets 16 whole cores; the one-GPU box's 16-cpu share (8 cores
    + SMT) rehearsing 8 ranks: one whole core each, disjoint."""
    _fake_topology(tmp_path, 128, 2)
    socket0 = set(range(64)) | set(range(128, 192))
    shares = [shard.split_cpus(socket0, i, 4, str(tmp_path)) for i in range(4)]
    assert set().union(*shares) == socket0 and all(len(s) == 32 for s in shares)
    assert all(not (a & b) for i, a in enumerate(shares) for b in shares[i + 1:])
    box = set(range(8)) | set(range(128, 136))
    shares = [shard.split_cpus(box, i, 8, str(tmp_path)) for i in range(8)]
    assert shares == [{i, 128 + i} for i in range(8)]
