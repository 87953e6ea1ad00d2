"""The multi-GPU batch split (SURVEY §8 e) on the device.

* C4's per-GPU shard — 2 M x 1500 B of a 16 M batch over 8 GPUs, generated
  from its global packet indices — runs as two launches of rx_kernel's
  unrolled schedule (mtcp_gpu.hip launch: 1 M packets per launch on a full
  MI355X).  Every packet's verdict is the one the generator's corruption
  rule predicts, and every record equals the oracle's.  Ranks 0 and 7
  (first and last shard).
* bench.py's N > 1 path itself (torch.distributed.run, gloo, shard /
  generate / rx / barriers) with two ranks sharing device 0
  (MTCP_BENCH_DEVICE=0): the records the ranks dump, concatenated, equal one
  launch over the whole batch.  The CPU analogue of the split is mTCP's
  per-core RSS queues (mtcp/src/dpdk_module.c:644-676).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from mtcp_amd import RESULT_DTYPE, pktgen, shard
from tests.test_gpu_parity import DEV, V_TCP_OK, _expected_verdicts, assert_same, dev_results, to_dev

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    from mtcp_amd import gpu as g
    return g


@pytest.mark.parametrize("rank", [0, 7])
def test_c4_shard_two_launches(gpu, rank):
    seed, world = 4, 8
    sh = shard.make_shard(1 << 24, 1500, rank, world, seed)
    n = sh.count
    assert n == 1 << 21 and sh.first_index == rank * n
    b = torch.empty(sh.nbytes, dtype=torch.uint8, device=DEV)
    d = to_dev(sh.desc)
    gpu.pktgen_dev(b, d, n, 6, seed, sh.first_index)
    out = dev_results(n)
    with gpu.Context(0) as ctx:
        ctx.rx_chunk_dev(b, d, n, 6, out)
        torch.cuda.synchronize()
    got = out.cpu().numpy().view(RESULT_DTYPE)
    want_v, ip_flip = _expected_verdicts(n, seed, sh.desc["len"], first_index=sh.first_index)
    ok = ~ip_flip
    assert np.array_equal(got["verdict"][ok], want_v[ok])
    assert np.all(got["verdict"][ip_flip] != V_TCP_OK)
    # every record of the 2 M-packet shard (two launches of 1 M, mtcp_gpu.hip
    # kHeldPasses) against the oracle's threaded form (round 4: a 1 % sample
    # plus the launch boundary)
    host = b.cpu().numpy()
    want = np.zeros(n, RESULT_DTYPE)
    oracle.bench_rx(host, sh.desc, 6, None, min(16, len(os.sched_getaffinity(0))), 1, want)
    assert_same(got, want, f"c4 shard {rank}")


def _bench_ranks(tmp_path, config, per_gpu, world=2, launcher="torchrun"):
    """bench.py's N-rank path.  launcher "torchrun": the driver's form
    (python -m torch.distributed.run ... bench.py --gpus N); "self": plain
    `python3 bench.py --gpus N`, which starts its own ranks (bench.py
    self_launch) — WORLD_SIZE is removed from the environment."""
    dump = tmp_path / f"{config}_{launcher}"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MTCP_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--config", config,
            "--per-gpu", str(per_gpu), "--steps", "3", "--warmup", "1", "--cpu-baseline", "off",
            "--pcie", "off", "--dump-records", str(dump)]
    if launcher == "torchrun":
        port = 29600 + os.getpid() % 300
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", f"--master-port={port}", *args]
    else:
        cmd = [sys.executable, *args]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    json_lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(json_lines) == 1, p.stdout[-2000:]
    line = json.loads(json_lines[0])
    recs, metas = [], []
    for r in range(world):
        metas.append(json.load(open(dump / f"shard_rank{r}.json")))
        recs.append(np.fromfile(dump / f"records_rank{r}.bin", dtype=RESULT_DTYPE))
    return line, metas, recs


@pytest.mark.parametrize("config,size,rss,per_gpu,launcher",
                         [("c2", 1500, False, 1 << 17, "torchrun"),
                          ("c3", "bimodal", True, 1 << 17, "torchrun"),
                          ("c2", 1500, False, 1 << 17, "self")])
def test_bench_two_ranks_equal_one_launch(gpu, tmp_path, config, size, rss, per_gpu, launcher):
    line, metas, recs = _bench_ranks(tmp_path, config, per_gpu, launcher=launcher)
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["config"]["packets_total"] == 2 * per_gpu
    # the measured read ceiling of the slowest rank's GPU, next to its kernel
    rc = line["roofline"]["read_ceiling"]
    assert rc["us"] > 0 and rc["kernel_frac_of_ceiling"] > 0, rc
    first = 0
    for m, r in zip(metas, recs):
        assert m["first_index"] == first and m["count"] == len(r)
        first += m["count"]
    assert first == 2 * per_gpu
    seed = {"c2": 2, "c3": 3}[config]
    n = 2 * per_gpu
    desc, nbytes = pktgen.layout(n, size, 6, seed)
    b = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    d = to_dev(desc)
    gpu.pktgen_dev(b, d, n, 6, seed)
    out = dev_results(n)
    kw = dict(rss=True, rss_queues=8, rss_endian=True) if rss else {}
    with gpu.Context(0, **kw) as ctx:
        ctx.rx_chunk_dev(b, d, n, 6, out)
        torch.cuda.synchronize()
    whole = out.cpu().numpy().view(RESULT_DTYPE)
    assert_same(np.concatenate(recs), whole, f"{config} ranks vs one launch")
    if size == "bimodal":                  # the byte-balanced split of shard.bounds
        cut = metas[1]["first_index"]
        assert cut == shard.bounds(n, size, 2, seed)[1]


def test_bench_default_n2_runs_c4_with_cpu_baseline(gpu, tmp_path):
    """The driver's N > 1 form without --config, launcher-less: the ranks run
    BASELINE's multi-GPU config C4 (here at a reduced per-GPU count) and the
    line carries the same-run CPU baseline of every rank on its own cores."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MTCP_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--per-gpu", str(1 << 17),
           "--steps", "3", "--warmup", "1", "--cpu-sample", str(1 << 14), "--pcie", "off"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["workload"].startswith("c4: 256 K x 1500 B")
    assert line["config"]["packets_total"] == 2 << 17
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] in ("reference", "port")
    assert [r["rank"] for r in cb["per_rank"]] == [0, 1]
    assert cb["cores"] == sum(r["cores"] for r in cb["per_rank"])
    # the two ranks share device 0's node: disjoint halves of its cores
    assert line["host_cpus"]["shared_with_ranks"] == [0, 1]


def _bench_line(cmd, env, timeout=300):
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def _clean_env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MASTER_ADDR="127.0.0.1", **kw)
    return env


def test_bench_default_n1_carries_c4_per_gpu(gpu):
    """the N = 1 default line (C2) also times C4's
    per-GPU step — rank 0's 2 M x 1500 B shard, two launches — in the same
    run, so the driver's 1 -> 8 ratio can be read on identical per-GPU work."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
           "--cpu-baseline", "off", "--pcie", "off", "--small-batch", "off", "--ceiling", "off"]
    line = _bench_line(cmd, _clean_env())
    assert line["n_gpus"] == 1 and line["config"]["workload"].startswith("c2: 1 M x 1500 B")
    c4 = line["c4_per_gpu"]
    assert "error" not in c4, c4
    assert c4["packets"] == 1 << 21 and c4["launches_per_step"] == 2 and c4["value"] > 0
    assert c4["tcp_ok_fraction"] > 0.99
    assert line["run"]["wall_s_max_rank"] > 0 and line["run"]["host_rss_gb_max_rank"] > 0


def test_bench_driver_form_eight_ranks_on_one_device(gpu):
    """the driver's exact `python3 bench.py --gpus 8`
    form, rehearsed with all eight ranks on device 0 (MTCP_BENCH_DEVICE=0)
    at a reduced per-GPU count, every leg on: one JSON line, C4's workload
    over 8 ranks, the CPU baseline of every rank on its own disjoint core
    share at once, the PCIe-inclusive leg of all 8 ranks, the run's wall time
    and host memory.  (The timings mean nothing: 8 ranks share one GPU.)"""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--per-gpu", str(1 << 14),
           "--steps", "3", "--warmup", "1", "--cpu-sample", str(1 << 13)]
    line = _bench_line(cmd, _clean_env(MTCP_BENCH_DEVICE="0"))
    assert line["n_gpus"] == 8 and line["config"]["workload"].startswith("c4: 128 K x 1500 B")
    assert line["config"]["packets_total"] == 8 << 14 and line["scaling"] == "weak"
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and [r["rank"] for r in cb["per_rank"]] == list(range(8))
    assert cb["cores"] == sum(r["cores"] for r in cb["per_rank"])
    assert line["host_cpus"]["shared_with_ranks"] == list(range(8))
    assert line["pcie_inclusive"]["n_gpus"] == 8 and line["pcie_inclusive"]["value"] > 0
    assert "c4_per_gpu" not in line
    assert line["run"]["wall_s_max_rank"] > 0
    # every rank's own view: all eight on the one device
    ro = line["roofline"]
    assert [r["rank"] for r in ro["per_rank"]] == list(range(8))
    assert all(r["device"] == 0 and r["kern_ms"] > 0 and r["wall_ms"] > 0 for r in ro["per_rank"])
    assert len({r["gpu_pci"] for r in ro["per_rank"]}) == 1 == ro["distinct_gpus"]
    assert ro["kern_ms_spread"] >= 1.0
    assert line["config"]["note"].startswith("MTCP_BENCH_DEVICE=0") and "warning" not in line["config"]
