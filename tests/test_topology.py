"""gpu_module.c's device choice (mtcp_amd/io_module/gpu_topo.h) on a faked
sysfs topology — CPU only.  mTCP binds each thread's memory to its core's
NUMA node (mtcp/src/cpu.c:54-79) and DPDK keeps each port's queues on the
NIC's socket (mtcp/src/dpdk_module.c:660-663); the thread's GPU context opens
a device on the core's node, the node's cpus dealt round-robin over its
devices, so that an 8-GPU host's threads use all eight PCIe links from
NUMA-local memory.  (Unmeasured on hardware: the pool's boxes have one GPU.)"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def topo_exe(tmp_path_factory):
    exe = tmp_path_factory.mktemp("topo") / "topo_test"
    subprocess.run(["gcc", "-std=gnu99", "-O2", "-Wall", "-Werror", "-o", str(exe),
                    os.path.join(ROOT, "tests", "c", "topo_test.c")], check=True)
    return str(exe)


def fake_sysfs(root, nodes, devices):
    """nodes: {node: cpulist string}; devices: {bdf: numa_node}."""
    for n, cl in nodes.items():
        d = root / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cl + "\n")
    for bdf, n in devices.items():
        d = root / "bus" / "pci" / "devices" / bdf
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{n}\n")
    return str(root)


def run(exe, sysfs, ncpu, bdfs):
    out = subprocess.run([exe, sysfs, str(ncpu), *bdfs], check=True, capture_output=True,
                         text=True).stdout.split("\n")
    return [tuple(int(x) for x in ln.split()) for ln in out if ln.strip()]


def test_eight_gpus_two_sockets(topo_exe, tmp_path):
    # an MI355X node: 2 sockets, SMT siblings listed as a second range, 4 GPUs
    # per socket, enumerated interleaved across the sockets (device order of
    # HIP need not follow the sockets)
    nodes = {0: "0-63,128-191", 1: "64-127,192-255"}
    bdfs = [f"0000:{b:02x}:00.0" for b in (0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xe5, 0xf5)]
    dev_nodes = [0, 1, 0, 1, 0, 1, 0, 1]
    sysfs = fake_sysfs(tmp_path, nodes, dict(zip(bdfs, dev_nodes)))
    rows = run(topo_exe, sysfs, 256, [b.upper() for b in bdfs])   # hipDeviceGetPCIBusId may print upper case
    per_dev = [0] * 8
    for cpu, node, rank, dev in rows:
        want_node = 0 if cpu < 64 or 128 <= cpu < 192 else 1
        assert node == want_node
        assert dev_nodes[dev] == node, (cpu, dev)
        per_dev[dev] += 1
    assert per_dev == [32] * 8                       # the node's cpus dealt evenly
    # consecutive cores of a node go to different GPUs (one link per thread)
    assert len({rows[c][3] for c in range(4)}) == 4
    # the node's cpus in list order: cpu 128 (SMT sibling of 0) is rank 64
    assert rows[128][2] == 64 and rows[128][3] == rows[0][3]


def test_node_without_gpu_and_unknown_topology(topo_exe, tmp_path):
    nodes = {0: "0-7", 1: "8-15"}
    devs = {"0000:05:00.0": 0, "0000:06:00.0": 0, "0000:07:00.0": -1}
    sysfs = fake_sysfs(tmp_path / "a", nodes, devs)
    rows = run(topo_exe, sysfs, 16, list(devs))
    for cpu, node, rank, dev in rows:
        if node == 0:
            assert dev in (0, 1)
        else:                                         # no device on node 1: cpu mod ndev
            assert dev == cpu % 3
    # no sysfs topology at all (containers): the round-2 rule, cpu mod ndev
    rows = run(topo_exe, str(tmp_path / "missing"), 12, list(devs))
    assert [r[3] for r in rows] == [c % 3 for c in range(12)]
    assert all(r[1] == -1 for r in rows)


def test_cpulist_parser_edges(topo_exe, tmp_path):
    sysfs = fake_sysfs(tmp_path, {0: "0,2,4-5", 3: "1,3, 6-7"}, {"0000:01:00.0": 3})
    rows = run(topo_exe, sysfs, 8, ["0000:01:00.0"])
    assert [r[1] for r in rows] == [0, 3, 0, 3, 0, 0, 3, 3]
    assert [r[2] for r in rows] == [0, 0, 1, 1, 2, 3, 2, 3]
    assert [r[3] for r in rows] == [0 % 1] * 8


def test_bench_host_binding_reads_local_cpulist(tmp_path, monkeypatch):
    """bench.py --numa on: a rank runs on its GPU's local_cpulist (the same
    sysfs file family gpu_topo.h reads), parsed in the kernel's list format."""
    from mtcp_amd import gpu
    assert gpu.parse_cpulist("64-127,192-255\n") == set(range(64, 128)) | set(range(192, 256))
    assert gpu.parse_cpulist("0,2,4-5") == {0, 2, 4, 5}
    assert gpu.parse_cpulist("") == set()
    bdf = "0000:f4:00.0"
    d = tmp_path / "bus" / "pci" / "devices" / bdf
    d.mkdir(parents=True)
    (d / "local_cpulist").write_text("8-11,40\n")
    monkeypatch.setattr(gpu, "device_pci_bus_id", lambda device: bdf)
    assert gpu.device_local_cpus(0, sysfs=str(tmp_path)) == (bdf, {8, 9, 10, 11, 40})
    # a device sysfs does not describe: no binding
    monkeypatch.setattr(gpu, "device_pci_bus_id", lambda device: "0000:01:00.0")
    assert gpu.device_local_cpus(0, sysfs=str(tmp_path)) == ("0000:01:00.0", set())
