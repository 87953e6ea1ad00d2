#!/usr/bin/env python3
"""bench.py — device-resident throughput of mTCP's software rx path on MI355X.

One step = one launch of the rx kernel (IPv4 + TCP checksum over every
segment byte, Eth/IP/TCP header parse and verdict, per-packet RSS when the
config asks for it) over one resident batch of synthetic frames.  Frames are
generated on the GPU (include/mtcp_gpu_pktgen.h) and stay in HBM; results
(40 B per packet) are written to HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1..c5|f1|f3|f4] [--strong]

Without --config the workload is BASELINE.json's config for that N: C2
(1 M x 1500 B) on one GPU, C4 (2 M x 1500 B per GPU, 16 M at N = 8) on
N > 1; config.workload names the total.

MTCP_BENCH_DEVICE=d in the environment puts every rank on device d (a
rehearsal of the N > 1 path on a one-GPU box; the timings then mean
nothing), and --dump-records DIR writes each rank's result records after the
timed steps (tests/test_gpu_shard.py compares them with one launch over the
whole batch).

Multi-GPU: one process per GPU, weak scaling (--strong: the whole batch
split N ways) — each rank processes its own contiguous shard of one global
batch (batch split, no collective on the data path; gloo carries only the
barrier and the max of the per-rank times).  Rank 0 prints ONE JSON line.
Under torch.distributed.run (WORLD_SIZE set) each process is one rank;
`python bench.py --gpus N` with no launcher starts its N ranks itself
(self_launch) and forwards that line.

The CPU baseline times the reference's own rx code (oracle/_ref/libref_rx.so,
compiled from /root/reference) or, where that was not built, the oracle's C
restatement, on a bounded sample of the same frames copied to host memory:
at N = 1 on rank 0 with 1 core and with its GPU-local share; at N > 1 on
every rank at once, each on its own disjoint GPU-local cores, reported per
rank and as the host aggregate.
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import sys
import time

T_START = time.perf_counter()

import numpy as np
import torch
import torch.distributed as dist

from mtcp_amd import _codeobj, pktgen, shard

METRIC = "device-resident Gpkt/s + payload GB/s checksummed, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

# BASELINE.json configs; per_gpu = packets per rank (weak scaling)
CONFIGS = {
    # C1 is the reference's CPU-runnable case; on the GPU it is launch-bound
    # (64 K x 64 B = 4 MB per launch), reported for completeness beside the
    # reference's code on the same frames
    "c1": dict(size=64, per_gpu=1 << 16, rss=False, seed=1, graph=True,
               desc="64 K x 64 B TCP segments, checksum + parse"),
    "c2": dict(size=1500, per_gpu=1 << 20, rss=False, seed=2,
               desc="1 M x 1500 B (MTU) packets, IP+TCP checksum + header parse"),
    "c3": dict(size="bimodal", per_gpu=1 << 20, rss=True, seed=3,
               desc="1 M packets bimodal 64 B / 1500 B + RSS Toeplitz hash"),
    "c4": dict(size=1500, per_gpu=1 << 21, total=1 << 24, rss=False, seed=4,
               desc="16 M x 1500 B packets sharded across 8 MI355X (2 M per GPU)"),
    "c5": dict(size=9000, per_gpu=1 << 19, total=1 << 22, rss=False, seed=5,
               desc="4 M x 9000 B jumbo frames (512 K per GPU), checksum + parse"),
}

# what each config computes, for config.workload (the sizes come from the run)
WHAT = {"c1": "TCP segments, checksum + parse", "c2": "packets, IP+TCP checksum + header parse",
        "c3": "packets, IP+TCP checksum + header parse + RSS Toeplitz hash",
        "c4": "packets, IP+TCP checksum + header parse",
        "c5": "jumbo frames, checksum + parse"}


def default_config(gpus: int) -> str:
    """The workload of `bench.py --gpus N` without --config: BASELINE.json's
    configs[1] (C2, 1 M x 1500 B, the metric's own single-GPU config) at
    N = 1; its multi-GPU config C4 (2 M x 1500 B per GPU, 16 M at N = 8)
    at N > 1."""
    return "c2" if gpus <= 1 else "c4"


def _count(n: int) -> str:
    if n % (1 << 20) == 0:
        return f"{n >> 20} M"
    if n % (1 << 10) == 0:
        return f"{n >> 10} K"
    return str(n)


def workload(config: str, world: int, per_gpu_override=None, strong: bool = False) -> dict:
    """Packets per rank and in total, and the scaling, of one run.  Weak (the
    default): every rank processes the config's per-GPU batch, so C4 at N
    GPUs is N x 2 M (16 M at N = 8).  --strong: the config's whole batch
    (C4 16 M, C5 4 M; C1-C3 their one-GPU batch) split N ways, as SURVEY
    §8(d) phrases C4.  --per-gpu overrides the per-rank count (tests)."""
    cfg = CONFIGS[config]
    size = cfg["size"]
    if per_gpu_override:
        per_gpu, scaling = per_gpu_override, "weak"
        total = per_gpu * world
    elif strong:
        total, scaling = cfg.get("total", cfg["per_gpu"]), "strong"
        per_gpu = total // world
    else:
        per_gpu, scaling = cfg["per_gpu"], "weak"
        total = per_gpu * world
    sz = "bimodal 64 B / 1500 B" if size == "bimodal" else f"{size} B"
    desc = (f"{config}: {_count(total)} x {sz} {WHAT[config]}, "
            + (f"{_count(per_gpu)} per GPU x {world} MI355X (batch split)" if world > 1 else "1 MI355X"))
    return {"config": config, "per_gpu": per_gpu, "total": total, "scaling": scaling, "desc": desc}


# SURVEY §8(f) rows beside the rx path, each measured on one GPU (not the
# headline line): f1 tx checksum fill over the C2 batch, f3 HashFlow over the
# rx records of the C2 batch, f4 the RSS queue map of CreateAddressPoolPerCore's
# candidate space (num_addr x 64511 ports).
ROWS = {
    "f1": "tx checksum fill (ip_out.c:94,164, tcp_out.c:211,329) over 1 M x 1500 B frames",
    "f3": "HashFlow (tcp_stream.c:56-90) over 1 M rx records of the C2 batch",
    "f4": "RSS queue of 64 addresses x 64511 ports (addr_pool.c:155-178, rss.c:90-103)",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS) + sorted(ROWS),
                    help="default: c2 at --gpus 1, c4 (2 M x 1500 B per GPU) at --gpus N > 1")
    ap.add_argument("--strong", action="store_true",
                    help="split the config's whole batch N ways (C4: 16 M) instead of N x its per-GPU batch")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--cpu-sample", type=int, default=1 << 20,
                    help="packets in the CPU sample (default: the whole 1-GPU batch, "
                         "larger than the host L3, so the CPU streams from DRAM like the GPU)")
    ap.add_argument("--pcie", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="launch the K timed steps from one HIP graph (auto: for C1, whose "
                         "~4 us launches would otherwise be timed at the Python call's rate)")
    ap.add_argument("--small-batch", default="on", choices=["on", "off"],
                    help="N=1: also time one 4 096-frame aggregate (graph-captured launches)")
    ap.add_argument("--pcie-max-bytes", type=int, default=1 << 30,
                    help="frame bytes per rank in the PCIe-inclusive leg (a prefix of the "
                         "shard, staged to host memory piece by piece)")
    ap.add_argument("--per-gpu", type=int, default=None,
                    help="packets per GPU (default: the config's; tests use smaller batches)")
    ap.add_argument("--dump-records", default=None,
                    help="directory: each rank writes its result records there")
    ap.add_argument("--prewarm-s", type=float, default=1.0,
                    help="seconds of untimed launches of the step before the read ceiling and the "
                         "warmup steps: a box whose GPU sat idle ran its first second 3-4 %% slow, "
                         "read stream and kernel alike (profiles/r6/c2_cold_box.jsonl)")
    ap.add_argument("--ceiling", default="on", choices=["on", "off"],
                    help="time a plain read stream over the same frame buffer (tools/libstream_ceiling.so) "
                         "and report the kernel against it (roofline.read_ceiling)")
    ap.add_argument("--numa", default="on", choices=["on", "off"],
                    help="run each rank on the cpus local to its GPU (sysfs local_cpulist), so the "
                         "host buffers of the CPU-baseline and PCIe-inclusive legs sit on its socket")
    ap.add_argument("--c4-per-gpu", default="auto", choices=["auto", "on", "off"],
                    help="N = 1: also time C4's per-GPU step (2 M x 1500 B, two launches; what each "
                         "rank of `--gpus N` runs) in the same run, so that the 1 -> N ratio can "
                         "compare identical per-GPU work (auto: on for the default C2 line)")
    ap.add_argument("--record", default="full", choices=["full", "compact"],
                    help="rx result record: the 40 B mtcp_gpu_result (default, the headline) or "
                         "the 16 B mtcp_gpu_result16 of a MTCP_GPU_F_COMPACT context")
    a = ap.parse_args()
    if a.config is None:
        a.config = default_config(a.gpus)
    return a


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_prefix(d_buf, desc, max_pkts=None, max_bytes=None):
    """The shard's first frames copied to host memory, in pieces of 256 MiB
    (no full-shard host copy: at N = 8 every rank stages at once)."""
    n = len(desc)
    if max_pkts is not None:
        n = min(n, max_pkts)
    ends = (desc["offset"][:n].astype(np.int64) << 6) + ((desc["len"][:n].astype(np.int64) + 63) & ~63)
    if max_bytes is not None:
        n = max(1, int(np.searchsorted(ends, max_bytes, side="right")))
    end = int(ends[n - 1])
    host = np.empty(end, np.uint8)
    step = 256 << 20
    for o in range(0, end, step):
        host[o:o + step] = d_buf[o:min(o + step, end)].cpu().numpy()
    return host, desc[:n]


def bind_to_device(device: int, mode: str, world: int = 1, rank: int = 0) -> dict:
    """Restrict this rank to the cpus local to its GPU before any host buffer
    is touched (mode "on"), as mTCP keeps each thread and its memory on one
    node (mtcp/src/cpu.c:54-79) and gpu_module.c picks the GPU on the
    thread's node (gpu_topo.h).  With N > 1 ranks, the ranks whose GPUs
    share a node split its cores (whole physical cores, shard.split_cpus),
    so that their concurrent CPU baselines run on disjoint cores.  Returns
    what was done, for the JSON line."""
    from mtcp_amd import gpu
    allowed = os.sched_getaffinity(0)
    info = {"binding": "off"}
    use = set(allowed)
    bdf = None
    if mode == "on":
        bdf, local = gpu.device_local_cpus(device)
        info = {"binding": "cpus local to the GPU", "gpu_pci": bdf}
        if local & allowed:
            use = local & allowed
        else:
            info["binding"] = "none (sysfs gives no local cpus)"
    if world > 1:
        sets = [None] * world
        dist.all_gather_object(sets, sorted(use))
        peers = [r for r in range(world) if sets[r] == sets[rank]]
        use = shard.split_cpus(use, peers.index(rank), len(peers))
        info["shared_with_ranks"] = peers
    if use != allowed:
        os.sched_setaffinity(0, use)
    info["cpus"] = len(use)
    return info


def read_ceiling(d_buf, nbytes, stream, reps=20):
    """The box's read-only streaming ceiling on this rank's own frame buffer
    (SURVEY §8(d)), measured now: the fastest of eight plain non-temporal
    grid-stride read streams over all `nbytes` (slot padding included),
    tools/stream_ceiling.hip.  Measurement infrastructure, outside the timed
    region; None when the probe library is not built."""
    import ctypes
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "libstream_ceiling.so")
    if not os.path.exists(path):
        return None
    f = ctypes.CDLL(path).stream_ceiling_us
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                  ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]
    f.restype = ctypes.c_int
    us, shape = ctypes.c_float(0.0), ctypes.c_int(0)
    if f(d_buf.data_ptr(), nbytes, reps, stream.cuda_stream, ctypes.byref(us), ctypes.byref(shape)) != 0:
        raise RuntimeError("stream_ceiling_us failed")
    return float(us.value), int(shape.value)


def gpu_identity(device: int) -> dict:
    """The GPU a rank runs on: its PCI address and NUMA node (sysfs), so that
    an N-GPU line shows N distinct GPUs and where each sits."""
    from mtcp_amd import gpu
    bdf = gpu.device_pci_bus_id(device)
    try:
        node = int(open(os.path.join("/sys/bus/pci/devices", bdf, "numa_node")).read().strip())
    except (OSError, ValueError):
        node = -1
    return {"gpu_pci": bdf, "numa_node": node}


def rank_summary(per_rank: list, forced_device) -> dict:
    """What the N ranks' own measurements say, for roofline: each rank's GPU
    (pci, node), its event-timed launch and wall time, its own read ceiling
    and the kernel's fraction of it; the spread of the launch times (max /
    min); and how many distinct GPUs the ranks ran on.  Fewer GPUs than ranks
    without MTCP_BENCH_DEVICE (a launcher that mapped two ranks to one GPU)
    is flagged, so such a line cannot pass for an N-GPU number."""
    kern = [r["kern_ms"] for r in per_rank]
    distinct = len({r["gpu_pci"] for r in per_rank})
    out = {"per_rank": sorted(per_rank, key=lambda r: r["rank"]),
           "kern_ms_spread": round(max(kern) / min(kern), 4) if min(kern) > 0 else None,
           "distinct_gpus": distinct}
    if distinct < len(per_rank):
        if forced_device is not None:
            out["note"] = (f"MTCP_BENCH_DEVICE={forced_device}: every rank on one device (a rehearsal "
                           f"of the N-rank path; the timings are not an N-GPU measurement)")
        else:
            out["warning"] = (f"{len(per_rank)} ranks ran on {distinct} distinct GPU(s): ranks shared a GPU, "
                              f"this is not a {len(per_rank)}-GPU measurement")
    return out


def patch_ceiling(d_buf, d_desc, n, stream, reps=20):
    """The f1 row's ceiling, measured now on its own frames: the tx fill's
    access pattern without its arithmetic (read every frame, write the two
    u16 check fields of each, the bytes unchanged), fastest of four shapes,
    tools/stream_ceiling.hip patch_walk.  None when the probe library is not
    built."""
    import ctypes
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "libstream_ceiling.so")
    if not os.path.exists(path):
        return None
    f = ctypes.CDLL(path).patch_ceiling_us
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                  ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]
    f.restype = ctypes.c_int
    us, shape = ctypes.c_float(0.0), ctypes.c_int(0)
    if f(d_buf.data_ptr(), d_desc.data_ptr(), n, 6, reps, stream.cuda_stream, ctypes.byref(us),
         ctypes.byref(shape)) != 0:
        raise RuntimeError("patch_ceiling_us failed")
    return float(us.value), int(shape.value)


def lib_sha256() -> str:
    """Identity of the product library whose kernels this run measures: the
    committed PMC traffic figure (profiles/traffic_*.json) counts when it was
    collected on the same build, or on one whose rx_kernel sources are the
    same (mtcp_amd/_codeobj.py)."""
    from mtcp_amd import _lib
    return _codeobj.lib_sha256(_lib.LIB_PATH)


def pmc_traffic(name: str):
    """HBM bytes per launch of the dominant kernel from the committed
    rocprofv3 PMC profile (profiles/traffic_<name>.json: FETCH_SIZE x 2 +
    WRITE_SIZE, separate passes, tools/profile_config.sh), when it was taken
    on this build or one with the same rx sources; else (None, why)."""
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", f"traffic_{name}.json")
    if not os.path.exists(tpath):
        return None, "no PMC profile for this config"
    tj = json.load(open(tpath))
    if tj.get("lib_sha256") == lib_sha256():
        return tj.get("hbm_bytes_per_launch"), f"rocprofv3 PMC of this build ({os.path.relpath(tpath)})"
    if tj.get("rx_source_key") == _codeobj.rx_source_key():
        return tj.get("hbm_bytes_per_launch"), (f"rocprofv3 PMC of a build with the same rx sources "
                                                f"({os.path.relpath(tpath)}; the library differs elsewhere)")
    return None, (f"stale: {os.path.relpath(tpath)} was collected on another build "
                  f"({tj.get('hbm_bytes_per_launch')} B per launch there)")


def cpu_share() -> int:
    n = len(os.sched_getaffinity(0))
    return max(1, min(n, 16))   # the GPU box's CPU share per GPU is 16


def cpu_baseline(host_buf, desc, cfg, sample_n):
    """Rank-0 CPU baseline over a bounded sample of the same frames."""
    import oracle   # test infrastructure: the baseline leg only
    n = min(sample_n, len(desc))
    d = desc[:n].copy()
    end = (int(d["offset"][-1]) << 6) + ((int(d["len"][-1]) + 63) & ~63)
    buf = np.ascontiguousarray(host_buf[:end])
    nbytes = int(d["len"].astype(np.int64).sum())
    cores_all = cpu_share()
    kind = "reference" if oracle.ref_available() else "port"

    def measure(with_rss):
        runs = {}
        for cores in sorted({1, cores_all}):
            reps = 5
            if kind == "reference":
                best = oracle.ref_bench_rx(buf.copy(), d, 6, with_rss, cores, reps)
            else:
                rss = oracle.rss_cfg(None, 8, 1) if with_rss else None
                best = oracle.bench_rx(buf, d, 6, rss, cores, reps)
            runs[cores] = dict(gbs=nbytes / best / 1e9, mpps=n / best / 1e6, seconds=best)
        return runs

    def per_core(runs):
        return {str(c): {"GB/s": round(v["gbs"], 3), "Mpkt/s": round(v["mpps"], 3)}
                for c, v in runs.items()}

    runs = measure(cfg["rss"])
    best_cores = max(runs, key=lambda c: runs[c]["gbs"])
    r = runs[best_cores]
    extra = {}
    if cfg["rss"]:
        # also without the per-packet Toeplitz hash (mTCP's own
        # rx path does not hash per packet in software; the NIC does)
        extra["without_rss"] = {"per_core_count": per_core(measure(False)),
                                "note": "the same frames and code with GetRSSCPUCore not called"}
    return {
        "value": round(r["gbs"], 3), "unit": "GB/s", "cores": best_cores, "kind": kind,
        "mpkt_per_s": round(r["mpps"], 3),
        "sample": f"first {n} packets of the same batch ({nbytes} frame bytes), best of 5 "
                  f"after warm-up, one pinned thread per core on contiguous shards "
                  f"({'mtcp/src eth_in/ip_in/tcp_in/tcp_util compiled from /root/reference' if kind == 'reference' else 'oracle/mtcp_oracle.c restatement'}, gcc -O3)",
        "per_core_count": per_core(runs),
        "cpu_model": cpu_model(),
        **extra,
    }


def cpu_baseline_ranks(host_buf, desc, cfg, sample_n, world, rank):
    """N > 1: the reference's rx code on every rank's own GPU-local core share
    at the same time (bind_to_device gave the ranks disjoint cores), each
    over the first frames of its own shard — the host doing the same job on
    the cores that feed these GPUs, as mTCP runs one share-nothing thread
    per core and queue (mtcp/src/core.c:1195-1213, dpdk_module.c:644-676).
    The ranks start together after a barrier; each reports its best of 5
    after a warm-up.  Rank 0 returns the per-rank figures and the host
    aggregate (every rank's sample bytes / the slowest rank's time); the
    other ranks return None."""
    import oracle   # test infrastructure: the baseline leg only
    n = min(sample_n, len(desc))
    d = desc[:n].copy()
    end = (int(d["offset"][-1]) << 6) + ((int(d["len"][-1]) + 63) & ~63)
    buf = np.ascontiguousarray(host_buf[:end])
    nbytes = int(d["len"].astype(np.int64).sum())
    cores = cpu_share()
    kind = "reference" if oracle.ref_available() else "port"
    dist.barrier()
    try:
        if kind == "reference":
            best = oracle.ref_bench_rx(buf, d, 6, cfg["rss"], cores, 5)
        else:
            best = oracle.bench_rx(buf, d, 6, oracle.rss_cfg(None, 8, 1) if cfg["rss"] else None, cores, 5)
    except Exception as exc:   # every rank still joins the gather below: no hang
        print(f"bench.py rank {rank}: cpu baseline failed: {exc!r}", file=sys.stderr)
        best = -1.0
    mine = torch.tensor([nbytes, n, best, cores, float(ord(kind[0]))], dtype=torch.float64)
    rows = [torch.zeros(5, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(rows, mine)
    if rank != 0:
        return None
    rows = [r.tolist() for r in rows]
    failed = [i for i, r in enumerate(rows) if r[2] <= 0]
    if failed:
        return {"value": None, "error": f"the CPU baseline failed on ranks {failed} (their stderr says why)"}
    kinds = {"reference" if int(r[4]) == ord("r") else "port" for r in rows}
    total_bytes = sum(r[0] for r in rows)
    total_pkts = sum(r[1] for r in rows)
    slowest = max(r[2] for r in rows)
    return {
        "value": round(total_bytes / slowest / 1e9, 3), "unit": "GB/s",
        "cores": int(sum(r[3] for r in rows)), "kind": kind if len(kinds) == 1 else "mixed",
        "mpkt_per_s": round(total_pkts / slowest / 1e6, 3),
        "scope": f"host aggregate: {world} ranks at once, each on its own GPU-local cores",
        "per_rank": [{"rank": i, "cores": int(r[3]), "GB/s": round(r[0] / r[2] / 1e9, 3),
                      "Mpkt/s": round(r[1] / r[2] / 1e6, 3), "seconds": round(r[2], 6)}
                     for i, r in enumerate(rows)],
        "sample": f"each rank the first {n} packets of its own shard, best of 5 after warm-up, "
                  f"one pinned thread per core on contiguous pieces, all ranks started together "
                  f"({'mtcp/src eth_in/ip_in/tcp_in/tcp_util compiled from /root/reference' if kind == 'reference' else 'oracle/mtcp_oracle.c restatement'}, gcc -O3); "
                  f"aggregate = all ranks' sample bytes / the slowest rank's time",
        "cpu_model": cpu_model(),
    }


def pcie_inclusive(ctx, host_buf, desc, nbytes, world):
    """Host frames -> H2D -> kernel -> D2H of results, pipelined on 3 streams.
    Every rank runs its own shard at the same time (each GPU has its own PCIe
    link); a rep's time is the max over ranks, the best rep is reported."""
    from mtcp_amd import gpu
    gpu.host_register(host_buf)
    try:
        out = np.zeros(len(desc), dtype=ctx.result_dtype)
        gpu.host_register(out)
        try:
            ctx.rx_chunk(host_buf, desc, 6, out)   # warm-up (allocates stages)
            best = None
            for _ in range(3):
                if world > 1:
                    dist.barrier()
                t0 = time.perf_counter()
                ctx.rx_chunk(host_buf, desc, 6, out)
                dt = time.perf_counter() - t0
                if world > 1:
                    t = torch.tensor([dt], dtype=torch.float64)
                    dist.all_reduce(t, op=dist.ReduceOp.MAX)
                    dt = float(t[0])
                best = dt if best is None else min(best, dt)
            # the same with a context wait limit (mtcp_gpu_set_wait_limit):
            # every byte through pinned bounce buffers, so that a call that
            # gives up at its limit leaves the caller's memory alone
            ctx.wait_limit = 10_000_000
            try:
                ctx.rx_chunk(host_buf, desc, 6, out)   # warm-up (allocates the bounce buffers)
                best_b = None
                for _ in range(3):
                    if world > 1:
                        dist.barrier()
                    t0 = time.perf_counter()
                    ctx.rx_chunk(host_buf, desc, 6, out)
                    dt = time.perf_counter() - t0
                    if world > 1:
                        t = torch.tensor([dt], dtype=torch.float64)
                        dist.all_reduce(t, op=dist.ReduceOp.MAX)
                        dt = float(t[0])
                    best_b = dt if best_b is None else min(best_b, dt)
            finally:
                ctx.wait_limit = 0
        finally:
            gpu.host_unregister(out)
    finally:
        gpu.host_unregister(host_buf)
    total_bytes, total_pkts = nbytes, len(desc)
    if world > 1:
        tb = torch.tensor([nbytes, len(desc)], dtype=torch.int64)
        dist.all_reduce(tb)
        total_bytes, total_pkts = int(tb[0]), int(tb[1])
    return {"value": round(total_bytes / best / 1e9, 3), "unit": "GB/s",
            "gpkt_per_s": round(total_pkts / best / 1e9, 5), "n_gpus": world,
            "packets_per_rank": len(desc),
            "note": "pinned host chunk in, host results out; H2D + kernel + D2H overlapped "
                    "on 3 streams, 64 MiB stages; each rank its shard's first frames (at most "
                    "--pcie-max-bytes), all ranks at once, wall clock max over ranks, best of 3",
            "bounded": {"value": round(total_bytes / best_b / 1e9, 3), "unit": "GB/s",
                        "note": "the same calls on a context with a wait limit (mtcp_gpu_set_wait_limit): "
                                "the chunk is first copied into pinned bounce buffers by the calling "
                                "thread and the records come back through them"}}


def small_batch(ctx, dev, stream, n=4096, size=1500, launches=100, reps=5):
    """One io_module aggregate (4 096 x 1500 B frames, the batch the
    io_module backend launches; mTCP's bursts are <= 64 frames,
    dpdk_module.c:71) through mtcp_gpu_rx_chunk_dev: `launches` back-to-back
    launches captured in one HIP graph, so that the per-launch time is the
    kernel's and not the Python call's; median over `reps` replays."""
    from mtcp_amd import gpu
    desc, nbytes = pktgen.layout(n, size, 6, 7)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    o = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    gpu.pktgen_dev(b, d, n, 6, 7, stream=stream)
    for _ in range(5):
        ctx.rx_chunk_dev(b, d, n, 6, o, stream=stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for _ in range(launches):
            ctx.rx_chunk_dev(b, d, n, 6, o, stream=stream)
    g.replay()
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        g.replay()
        e1.record(stream)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1e3 / launches)
    us = sorted(times)[len(times) // 2]
    frame_bytes = int(desc["len"].astype(np.int64).sum())
    return {"frames": n, "frame_size": size, "us_per_launch": round(us, 2),
            "GBs": round(frame_bytes / us / 1e3, 1), "gpkt_per_s": round(n / us / 1e3, 3),
            "kernel": "mg::" + ctx.last_kernel,
            "note": f"{launches} launches of mtcp_gpu_rx_chunk_dev captured in a HIP graph, "
                    f"HIP events over a replay, median of {reps}"}


def _timed(step, steps, warmup, stream):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, ev0.elapsed_time(ev1) / steps / 1e3


def c4_per_gpu(ctx, dev, stream, steps, warmup):
    """C4's per-GPU step on this one GPU, in the N = 1 run: the 2 M x 1500 B
    shard rank 0 of `bench.py --gpus 8` processes (frames 0 .. 2 M of C4's
    seed-4 stream, byte-identical to that rank's shard), timed exactly as the
    N > 1 ranks time it — one mtcp_gpu_rx_chunk_dev call per step (two
    launches of 1 M, mtcp_gpu.hip kHeldPasses), K direct calls between HIP
    events on the launch stream.  Value / N-GPU line's value / N is then the
    scaling of identical per-GPU work."""
    from mtcp_amd import _lib, gpu
    cfg = CONFIGS["c4"]
    sh = shard.make_shard(cfg["per_gpu"], cfg["size"], 0, 1, cfg["seed"])
    d_buf = torch.empty(sh.nbytes, dtype=torch.uint8, device=dev)
    d_desc = torch.from_numpy(sh.desc.view(np.uint8).copy()).to(dev)
    d_out = torch.empty(sh.count * 40, dtype=torch.uint8, device=dev)
    gpu.pktgen_dev(d_buf, d_desc, sh.count, 6, cfg["seed"], sh.first_index, stream=stream)
    frame_bytes = int(sh.desc["len"].astype(np.int64).sum())
    rx_fn = _lib.lib().mtcp_gpu_rx_chunk_dev
    rx_args = (ctx._h, d_buf.data_ptr(), sh.nbytes, d_desc.data_ptr(), sh.count, 6, d_out.data_ptr(),
               stream.cuda_stream)
    rcs = []
    wall, kern = _timed(lambda: rcs.append(rx_fn(*rx_args)), steps, warmup, stream)
    if any(rc != 0 for rc in rcs):
        raise RuntimeError(f"mtcp_gpu_rx_chunk_dev failed ({[rc for rc in rcs if rc][0]})")
    ok = float((d_out.view(-1, 40)[:, 36] == 0).float().mean())
    del d_buf, d_desc, d_out
    torch.cuda.empty_cache()
    return {"value": round(frame_bytes / wall / 1e9, 2), "unit": "GB/s",
            "ms_per_step": round(wall * 1e3, 5), "gpkt_per_s": round(sh.count / wall / 1e9, 4),
            "packets": sh.count, "frame_bytes": frame_bytes, "launches_per_step": 2,
            "kernel": "mg::" + ctx.last_kernel, "avg_step_ms_events": round(kern * 1e3, 5),
            "frac": round(frame_bytes / kern / 1e9 / HBM_PEAK_GBS, 4), "tcp_ok_fraction": round(ok, 5),
            "note": "C4's per-GPU step (rank 0's 2 M x 1500 B shard of the 16 M batch) on this GPU in "
                    "the same run, timed as each rank of --gpus N times it: the N-GPU line's value "
                    "/ N / this value is the scaling of identical per-GPU work"}


def _cpu_time(fn, reps=3):
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best


def run_row(args):
    """One §8(f) row on one GPU; prints one JSON line of the headline's shape."""
    from mtcp_amd import gpu
    if int(os.environ.get("WORLD_SIZE", "1")) != 1 or args.gpus != 1:
        raise SystemExit("the f-row benches run on one GPU")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    host_cpus = bind_to_device(0, args.numa)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    want_cpu = args.cpu_baseline in ("on", "auto")
    line = {"metric": f"{args.config}: " + ROWS[args.config], "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "data": "synthetic", "config": {"workload": args.config},
            "host_cpus": host_cpus}
    n, seed = 1 << 20, 2
    if args.config in ("f1", "f3"):
        desc, nbytes = pktgen.layout(n, 1500, 6, seed)
        d_buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
        gpu.pktgen_dev(d_buf, d_desc, n, 6, seed, stream=stream)
        frame_bytes = int(desc["len"].astype(np.int64).sum())
    ctx = gpu.Context(0)
    if args.config == "f1":
        # idempotent after the first fill: every step rewrites the same checks
        step = lambda: ctx.tx_fill_dev(d_buf, d_desc, n, 6, stream=stream)
        # the access pattern's own ceiling on these frames, measured now,
        # before the fill's launches (as read_ceiling is for rx)
        try:
            ceil = patch_ceiling(d_buf, d_desc, n, stream)
        except Exception as exc:      # never costs the line
            ceil = repr(exc)
        wall, kern = _timed(step, args.steps, args.warmup, stream)
        algo = frame_bytes + 4 * n
        line.update(value=round(frame_bytes / wall / 1e9, 2), unit="GB/s", dtype="u8",
                    ms_per_step=round(wall * 1e3, 5), gpkt_per_s=round(n / wall / 1e9, 4))
        traffic, traffic_note = pmc_traffic("f1")
        line["roofline"] = {"bound": "hbm", "achieved": round(algo / kern / 1e9, 2),
                            "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(algo / kern / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                            "traffic_source": traffic_note,
                            "kernel": "mg::" + ctx.last_kernel,
                            "avg_launch_ms": round(kern * 1e3, 5),
                            "algorithmic_bytes_per_launch": algo,
                            "note": "sum L read + 4 B of check fields written per frame"}
        # the access pattern's own ceiling: a 2 x 2-byte patch per frame
        # costs a write granule and a dirty sector per frame,
        # measured in this run on these frames (tools/stream_ceiling.hip)
        if isinstance(ceil, tuple):
            cus, shape = ceil
            line["roofline"]["ceiling"] = {
                "us": round(cus, 2), "kernel_frac_of_ceiling": round(cus / (kern * 1e6), 4),
                "what": f"the fill's access pattern without its arithmetic on the same {n} frames: each "
                        f"16-lane row reads its frame ({shape // 10} loads per lane), lanes 1 and 3 write "
                        f"the u16 at bytes 24 and 50 back (values unchanged); fastest of 4 shapes "
                        f"({shape % 10} WG/CU won), 20 launches, HIP events, measured before the fill; "
                        f"tools/stream_ceiling.hip patch_walk"}
        elif ceil is not None:
            line["roofline"]["ceiling"] = {"error": ceil}
        if want_cpu:
            import oracle   # test infrastructure: the baseline leg only
            host = d_buf.cpu().numpy()
            m = 1 << 18
            sub = desc[:m]
            end = (int(sub["offset"][-1]) << 6) + 1536
            hb = np.ascontiguousarray(host[:end])
            t = _cpu_time(lambda: oracle.tx_fill(hb, sub, 6))
            sb = int(sub["len"].astype(np.int64).sum())
            line["cpu_baseline"] = {"value": round(sb / t / 1e9, 3), "unit": "GB/s", "cores": 1,
                                    "kind": "port", "sample": f"first {m} frames, best of 3 "
                                    "(oracle/mtcp_oracle.c tx fill, gcc -O3)"}
    elif args.config == "f3":
        d_out = torch.empty(n * 40, dtype=torch.uint8, device=dev)
        ctx.rx_chunk_dev(d_buf, d_desc, n, 6, d_out, stream=stream)
        bins = torch.empty(n, dtype=torch.int32, device=dev)
        step = lambda: ctx.flow_hash_dev(d_out, n, bins, stream=stream)
        wall, kern = _timed(step, args.steps, args.warmup, stream)
        algo = n * (40 + 4)
        line.update(value=round(n / wall / 1e9, 4), unit="Gpkt/s", dtype="u32",
                    ms_per_step=round(wall * 1e3, 5))
        traffic, traffic_note = pmc_traffic("f3")
        line["roofline"] = {"bound": "hbm", "achieved": round(algo / kern / 1e9, 2),
                            "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(algo / kern / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                            "traffic_source": traffic_note, "kernel": "mg::flow_hash_kernel",
                            "avg_launch_ms": round(kern * 1e3, 5),
                            "algorithmic_bytes_per_launch": algo,
                            "note": "40 B record read (its 12 key bytes and verdict span the "
                                    "record's lines) + 4 B bin written per packet"}
        # HashFlow fused into the rx pass (mtcp_gpu_rx_chunk_flow_dev): the
        # bin leaves with the record, so the record is never read back
        rx_step = lambda: ctx.rx_chunk_dev(d_buf, d_desc, n, 6, d_out, stream=stream)
        fused_step = lambda: ctx.rx_chunk_flow_dev(d_buf, d_desc, n, 6, d_out, bins, stream=stream)
        _, k_rx = _timed(rx_step, args.steps, args.warmup, stream)
        _, k_fused = _timed(fused_step, args.steps, args.warmup, stream)
        line["fused_rx_flow"] = {"rx_us": round(k_rx * 1e6, 2), "rx_flow_fused_us": round(k_fused * 1e6, 2),
                                 "rx_then_flow_us": round((k_rx + kern) * 1e6, 2),
                                 "saved_us": round((k_rx + kern - k_fused) * 1e6, 2),
                                 "note": "HIP events per launch, C2 batch (1 M x 1500 B): rx alone, "
                                         "rx with the bin fused, rx followed by the separate "
                                         "flow_hash kernel"}
        if want_cpu:
            import oracle
            res = d_out.cpu().numpy().view(gpu.RESULT_DTYPE)
            t = _cpu_time(lambda: oracle.flow_bins(res))
            line["cpu_baseline"] = {"value": round(n / t / 1e9, 4), "unit": "Gpkt/s", "cores": 1,
                                    "kind": "port", "sample": f"the same {n} records, best of 3 "
                                    "(oracle/mtcp_oracle.c HashFlow, gcc -O3)"}
    else:
        num_addr, nq = 64, 16
        total = num_addr * (gpu.MAX_PORT - gpu.MIN_PORT)
        queue = torch.empty(total, dtype=torch.uint8, device=dev)
        base_h, daddr_h, dport_h = 0x0A000001, 0xC0A80001, 80
        step = lambda: ctx.rss_queue_map_dev(base_h, num_addr, daddr_h, dport_h, nq, True, queue,
                                             stream=stream)
        # a launch is a few us: the K steps are captured in one HIP graph and
        # replayed (a direct Python call per launch would time the host)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for _ in range(args.steps):
                step()
        graph.replay()
        torch.cuda.synchronize()
        wall, kern = _timed(graph.replay, 1, 0, stream)
        wall, kern = wall / args.steps, kern / args.steps
        line.update(value=round(total / wall / 1e9, 3), unit="Gcandidates/s", dtype="u32",
                    ms_per_step=round(wall * 1e3, 5))
        line["config"]["launch"] = "hip_graph"
        # per candidate: 1 B written (the queue byte) — the HBM-side bytes;
        # 3 LDS byte reads (C(i) ^ t_hi[port >> 8] ^ t_lo[port & 255], then the
        # queue of the 7-bit value, flow_kernels.hpp): at ds_read_b32's
        # 128 B/clk/CU x 256 CUs x 2.4 GHz = 78.6 TB/s (MI355X_MICROARCH.md
        # §LDS; a byte read costs a dword read's cycle) that is 3 x 4 B per
        # candidate
        lds_peak = 128 * 256 * 2.4e9 / 1e9
        lds_bytes = 12 * total
        line["roofline"] = {"bound": "hbm", "achieved": round(total / kern / 1e9, 2), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(total / kern / 1e9 / HBM_PEAK_GBS, 4),
                            "traffic": None, "kernel": "mg::rss_queue_map_kernel",
                            "avg_launch_ms": round(kern * 1e3, 5), "algorithmic_bytes_per_launch": total,
                            "lds": {"bytes_per_launch": lds_bytes, "achieved_GBs": round(lds_bytes / kern / 1e9, 1),
                                    "peak_GBs": round(lds_peak, 1),
                                    "frac": round(lds_bytes / kern / 1e9 / lds_peak, 4),
                                    "note": "3 ds_read_u8 per candidate, priced as ds_read_b32 (128 B/clk/CU)"},
                            "note": "1 B written per candidate is the only HBM traffic (the nibble tables "
                                    "come from L2); at this size (4.1 MB) a launch is near the empty-kernel "
                                    "floor (DESIGN §9: 2.0-2.7 us), so neither bound is reached"}
        import socket
        import struct
        b_n = struct.unpack("<I", socket.inet_aton("10.0.0.1"))[0]
        d_n = struct.unpack("<I", socket.inet_aton("192.168.0.1"))[0]
        p_n = struct.unpack("<H", struct.pack(">H", 80))[0]
        t_gpu = _cpu_time(lambda: ctx.addr_pool_search(3, nq, b_n, num_addr, d_n, p_n, True))
        line["search_end_to_end"] = {"value": round(total / t_gpu / 1e9, 3), "unit": "Gcandidates/s",
                                     "note": "mtcp_gpu_addr_pool_search host call: queue map, "
                                             "count / scan / emit compaction, D2H of one core's "
                                             "entries; wall clock, best of 3"}
        if want_cpu:
            import oracle
            t = _cpu_time(lambda: oracle.addr_pool_search(None, 3, nq, b_n, num_addr, d_n, p_n, 1))
            line["cpu_baseline"] = {"value": round(total / t / 1e9, 4), "unit": "Gcandidates/s",
                                    "cores": 1, "kind": "port",
                                    "sample": "the same search (core 3 of 16 queues, 64 addresses), "
                                              "best of 3 (oracle/mtcp_oracle.c, gcc -O3)"}
    ctx.close()
    print(json.dumps(line), flush=True)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(argv, n, port):
    """The rank launcher bench.py starts for `--gpus N` without one:
    torch.distributed.run, one process per GPU on this node, rendezvous on
    127.0.0.1 (the container's hostname may not resolve)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__), *argv]


def self_launch(args, argv) -> int:
    """`python bench.py --gpus N` (N > 1) with no WORLD_SIZE in the
    environment: start the N rank processes here, as mTCP starts its own
    per-core workers (mtcp_create_context -> pthread_create /
    rte_eal_remote_launch, mtcp/src/core.c:1195-1213).  Nothing in this
    parent touches the GPU (no torch.cuda call: the ranks are fresh child
    processes, never an exec of a process that initialised HIP).  The ranks'
    JSON line (rank 0 prints one) is forwarded to stdout, everything else to
    stderr; the exit status is the launcher's (non-zero if any rank failed)."""
    import subprocess
    if "MTCP_BENCH_DEVICE" not in os.environ:
        # device_count() does not initialise HIP on this image; a clear error
        # beats N ranks dying in set_device
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but {ndev} GPU(s) visible "
                  f"(MTCP_BENCH_DEVICE=d puts every rank on device d)", file=sys.stderr)
            return 2
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.Popen(launch_cmd(argv, args.gpus, _free_port()), env=env,
                         stdout=subprocess.PIPE, text=True, bufsize=1)
    lines = 0
    for ln in p.stdout:
        if ln.startswith("{"):
            sys.stdout.write(ln)
            sys.stdout.flush()
            lines += 1
        else:
            sys.stderr.write(ln)
    rc = p.wait()
    if rc == 0 and lines != 1:
        print(f"bench.py: the ranks printed {lines} JSON lines, expected 1", file=sys.stderr)
        return 3
    return rc


def main():
    args = parse()
    if args.config in ROWS:
        return run_row(args)
    cfg = CONFIGS[args.config]
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(self_launch(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    device = int(os.environ.get("MTCP_BENCH_DEVICE", local_rank))
    if "MTCP_BENCH_DEVICE" not in os.environ and device >= torch.cuda.device_count() == 1:
        # a launcher that gives each rank only its own GPU (HIP_VISIBLE_DEVICES
        # per rank): that one device is this rank's (device_count() does not
        # initialise HIP on this image)
        device = 0
    torch.cuda.set_device(device)
    from mtcp_amd import gpu   # loads libmtcp_gpu.so (raises if not built)
    host_cpus = bind_to_device(device, args.numa, world, rank)

    wl = workload(args.config, world, args.per_gpu, args.strong)
    per_gpu, n_total = wl["per_gpu"], wl["total"]
    sh = shard.make_shard(n_total, cfg["size"], rank, world, cfg["seed"])
    dev = torch.device("cuda", device)
    # a dedicated (non-null) stream: the kernel and the timing events share it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    d_buf = torch.empty(sh.nbytes, dtype=torch.uint8, device=dev)
    d_desc = torch.from_numpy(sh.desc.view(np.uint8).copy()).to(dev)
    compact = args.record == "compact"
    rec_bytes = 16 if compact else 40
    d_out = torch.empty(sh.count * rec_bytes, dtype=torch.uint8, device=dev)
    gpu.pktgen_dev(d_buf, d_desc, sh.count, 6, cfg["seed"], sh.first_index, stream=stream)
    frame_bytes = int(sh.desc["len"].astype(np.int64).sum())

    ctx = gpu.Context(device, rss=cfg["rss"], rss_queues=8, rss_endian=True, compact=compact)
    # One step = one mtcp_gpu_rx_chunk_dev call, issued as a C caller would:
    # the C-ABI function with its arguments bound once (the Python wrapper's
    # per-call argument handling, ~5-10 us, is otherwise on the critical path
    # of the first timed launch); every return code is checked after the
    # timed region.
    from mtcp_amd import _lib
    rx_fn = _lib.lib().mtcp_gpu_rx_chunk_dev
    rx_args = (ctx._h, d_buf.data_ptr(), sh.nbytes, d_desc.data_ptr(), sh.count, 6, d_out.data_ptr(),
               stream.cuda_stream)
    step_rcs = []
    step = lambda: step_rcs.append(rx_fn(*rx_args))

    # bring the device to its steady state first (untimed; every launch's
    # return code is still checked below)
    t_warm = time.perf_counter()
    while time.perf_counter() - t_warm < args.prewarm_s:
        for _ in range(50):
            step()
        torch.cuda.synchronize()
    ceiling = my_ceiling_us = None
    if args.ceiling == "on":
        # The box's read ceiling on this rank's own frame buffer, measured
        # right before the kernel so that both see the same device state
        # (a cold device runs its first launches a few us slow: C2 at
        # --steps 20 --warmup 5 averaged 243 us after nothing, 239 us after
        # 200 launches).  Every rank times its own GPU; the slowest GPU's
        # stream is the ceiling the slowest rank's launches (kern_ms_max)
        # are compared with.
        try:
            ceiling = read_ceiling(d_buf, sh.nbytes, stream)
        except Exception as exc:   # never costs the headline line
            ceiling = repr(exc)
        my_ceiling_us = ceiling[0] if isinstance(ceiling, tuple) else None
        if world > 1:
            t = torch.tensor([ceiling[0] if isinstance(ceiling, tuple) else -1.0], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if isinstance(ceiling, tuple):
                ceiling = (float(t[0]), ceiling[1])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # C1's launches (~4 us of kernel) are shorter than a Python call into the
    # C ABI: its K steps are captured in one HIP graph and replayed, as a C
    # caller (the io_module) would issue them back to back; every other
    # config's launch is ~0.1-0.7 ms and is timed from direct calls
    use_graph = args.graph == "on" or (args.graph == "auto" and cfg.get("graph", False))
    if use_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for _ in range(args.steps):
                step()
        graph.replay()                       # untimed: the first replay uploads the graph
        torch.cuda.synchronize()
        run_steps = graph.replay
    else:
        def run_steps():
            for _ in range(args.steps):
                step()
    # HIP events on the launch stream bracket the timed region: average launch
    # duration = their interval / K (back-to-back launches, no host sync between)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if world > 1:
        # A barrier releases the ranks up to a few hundred µs apart, which a
        # short timed region (K x 0.24 ms) would count as lost scaling.  The
        # ranks share one host and so one CLOCK_MONOTONIC (perf_counter):
        # after the barrier they agree on a start instant 5 ms past the
        # latest rank's clock and spin until it; each rank's time runs from
        # that common instant (a rank arriving late is charged for it).
        tt = torch.tensor([t0], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t0 = float(tt[0]) + 5e-3
        while time.perf_counter() < t0:
            pass
    ev0.record(stream)
    run_steps()
    ev1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()     # this rank's completion; the max over ranks is taken below
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    # this rank's own view (roofline.per_rank): which GPU, its launches, its
    # wall time and its own read ceiling
    mine = dict(rank=rank, device=device, **gpu_identity(device), kern_ms=round(kern_ms, 5),
                wall_ms=round(elapsed * 1e3, 3),
                read_ceiling_us=round(my_ceiling_us, 2) if my_ceiling_us else None,
                kernel_frac_of_ceiling=round(my_ceiling_us / (kern_ms * 1e3), 4) if my_ceiling_us else None)
    per_rank = [mine]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
    else:
        kern_ms_max = kern_ms

    bad = [rc for rc in step_rcs if rc != 0]
    if bad:
        raise SystemExit(f"bench.py: mtcp_gpu_rx_chunk_dev failed in the timed steps ({bad[0]})")
    kernel = ctx.last_kernel                 # the kernel the timed launches dispatched
    # verdict summary of the last step (sanity: corruption rate ~1/1024 + 1/4096)
    recs = d_out.view(-1, rec_bytes)
    v_at, pl_at = (14, 8) if compact else (36, 32)   # verdict, payload_len (include/mtcp_gpu.h)
    res = recs[:, v_at].cpu().numpy()
    ok_frac = float((res == 0).mean())
    # TCP payload bytes (payload_len of the records, tcp_in.c:1144): the
    # metric's "payload GB/s" without the 54+ B of headers per frame
    payload = int(recs[:, pl_at:pl_at + 2].contiguous().view(torch.int16).to(torch.int64)
                  .bitwise_and(0xFFFF).sum())
    if args.dump_records:
        os.makedirs(args.dump_records, exist_ok=True)
        d_out.cpu().numpy().tofile(os.path.join(args.dump_records, f"records_rank{rank}.bin"))
        json.dump({"rank": rank, "world": world, "first_index": sh.first_index, "count": sh.count},
                  open(os.path.join(args.dump_records, f"shard_rank{rank}.json"), "w"))

    if world > 1:
        tb = torch.tensor([frame_bytes, sh.count, payload], dtype=torch.int64)
        dist.all_reduce(tb)
        total_bytes, total_pkts, total_payload = int(tb[0]), int(tb[1]), int(tb[2])
    else:
        total_bytes, total_pkts, total_payload = frame_bytes, sh.count, payload
    ms_per_step = elapsed / args.steps * 1e3
    gbs = total_bytes * args.steps / elapsed / 1e9
    gpps = total_pkts * args.steps / elapsed / 1e9
    payload_gbs = total_payload * args.steps / elapsed / 1e9

    extra = {}
    # the CPU baseline at every N: rank 0 alone at N = 1 (1 core and its
    # share), every rank at once on its own cores at N > 1 (a collective step)
    want_cpu = args.cpu_baseline in ("on", "auto")
    want_pcie = args.pcie in ("on", "auto")     # every rank: a collective step when N > 1
    if want_cpu:
        host, hdesc = host_prefix(d_buf, sh.desc, max_pkts=args.cpu_sample)
        if world == 1:
            try:
                extra["cpu_baseline"] = cpu_baseline(host, hdesc, cfg, args.cpu_sample)
            except Exception as exc:   # report, never fake
                extra["cpu_baseline"] = {"value": None, "error": repr(exc)}
        else:
            cb = cpu_baseline_ranks(host, hdesc, cfg, args.cpu_sample, world, rank)   # collective
            if rank == 0:
                extra["cpu_baseline"] = cb
        del host
    want_c4 = args.c4_per_gpu == "on" or (args.c4_per_gpu == "auto" and world == 1 and args.config == "c2"
                                          and not args.per_gpu and not compact)
    if world == 1 and want_c4:
        try:
            extra["c4_per_gpu"] = c4_per_gpu(ctx, dev, stream, args.steps, args.warmup)
        except Exception as exc:      # never costs the headline line
            extra["c4_per_gpu"] = {"error": repr(exc)}
    if rank == 0 and world == 1 and args.small_batch != "off":
        try:
            extra["small_batch"] = small_batch(ctx, dev, stream)
        except Exception as exc:      # never costs the headline line
            extra["small_batch"] = {"error": repr(exc)}
    if want_pcie:
        host, hdesc = host_prefix(d_buf, sh.desc, max_bytes=args.pcie_max_bytes)
        extra["pcie_inclusive"] = pcie_inclusive(ctx, host, hdesc,
                                                 int(hdesc["len"].astype(np.int64).sum()), world)
        del host
    ctx.close()

    # the run's own footprint (the 8-GPU default run's wall time
    # and host memory): wall seconds from process start, peak host RSS, the
    # max over ranks
    run = torch.tensor([time.perf_counter() - T_START,
                        resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(run, op=dist.ReduceOp.MAX)

    if rank == 0:
        # per-GPU roofline of the slowest rank's launches (N > 1: the max
        # over ranks of the event-timed average launch)
        achieved = frame_bytes / (kern_ms_max / 1e3) / 1e9
        # C4's per-GPU step is two launches of C2's shape (1 M x 1500 B each):
        # the per-launch figure is C2's
        traffic, traffic_note = pmc_traffic(f"{'c2' if args.config == 'c4' else args.config}"
                                            f"{'_compact' if compact else ''}")
        if traffic is not None and args.config == "c4":
            # a C4 step (the unit of avg_launch_ms and of the algorithmic
            # bytes here) is two launches of C2's shape: C2's per-launch
            # traffic scaled by the frame bytes
            traffic = round(traffic * frame_bytes / CONFIGS["c2"]["per_gpu"] / 1500)
            traffic_note += "; C2's per-launch figure x the C4 step's frame bytes / C2's"
        line = {
            "metric": METRIC, "value": round(gbs, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True, "scaling": wl["scaling"], "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (GPU splitmix64 frames, include/mtcp_gpu_pktgen.h)",
            "gpkt_per_s": round(gpps, 4), "payload_gbs": round(payload_gbs, 2),
            "config": {"workload": wl["desc"], "packets_per_gpu": per_gpu,
                       "packets_total": total_pkts, "frame_bytes_total": total_bytes,
                       "rss": cfg["rss"], "parallelism": f"batch split x{world} (no collective)",
                       "launch": "hip_graph" if use_graph else "direct",
                       "record": f"{rec_bytes} B ({'mtcp_gpu_result16, MTCP_GPU_F_COMPACT' if compact else 'mtcp_gpu_result'})"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_note,
                         "kernel": "mg::" + kernel, "avg_launch_ms": round(kern_ms_max, 5),
                         "algorithmic_bytes_per_launch": frame_bytes},
            "tcp_ok_fraction": round(ok_frac, 5),
            "host_cpus": host_cpus,
            "run": {"wall_s_max_rank": round(float(run[0]), 1), "host_rss_gb_max_rank": round(float(run[1]), 2),
                    "note": "each rank's seconds from its start to the end of its legs and its peak "
                            "resident host memory, the max over ranks"},
        }
        ranks = rank_summary(per_rank, os.environ.get("MTCP_BENCH_DEVICE"))
        for k in ("note", "warning"):
            if k in ranks:
                line["config"][k] = ranks.pop(k)
        line["roofline"].update(ranks)
        if isinstance(ceiling, tuple):
            cus, shape = ceiling
            line["roofline"]["read_ceiling"] = {
                "us": round(cus, 2), "GBs": round(sh.nbytes / cus / 1e3, 1),
                "algorithmic_GBs": round(frame_bytes / cus / 1e3, 1),
                "frac_of_peak": round(frame_bytes / cus / 1e3 / HBM_PEAK_GBS, 4),
                "kernel_frac_of_ceiling": round(cus / (kern_ms_max * 1e3), 4),
                "what": f"plain non-temporal read stream of the same {sh.nbytes} B frame buffer "
                        f"(slot padding included), fastest of 8 shapes ({shape // 10} loads per lane, "
                        f"{shape % 10} WG/CU), 20 launches, HIP events; tools/stream_ceiling.hip"}
        elif ceiling is not None:
            line["roofline"]["read_ceiling"] = {"error": ceiling}
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
