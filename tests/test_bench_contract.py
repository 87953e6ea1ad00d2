"""bench.py keeps the driver's contract (CPU-only checks): the metric string is
BASELINE.json's, every BASELINE config has a bench config of the stated
shape, the default run is the configs[1] workload on one GPU, and the f-row
benches refuse multi-GPU runs rather than reporting a partial number."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


def test_metric_and_configs_follow_baseline(bench):
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert bench.METRIC == base["metric"]
    assert bench.HBM_PEAK_GBS == 8000.0
    c = bench.CONFIGS
    assert (c["c1"]["size"], c["c1"]["per_gpu"]) == (64, 1 << 16)
    assert (c["c2"]["size"], c["c2"]["per_gpu"], c["c2"]["rss"]) == (1500, 1 << 20, False)
    assert (c["c3"]["size"], c["c3"]["per_gpu"], c["c3"]["rss"]) == ("bimodal", 1 << 20, True)
    assert (c["c4"]["size"], c["c4"]["per_gpu"] * 8) == (1500, 16 << 20)
    assert (c["c5"]["size"], c["c5"]["per_gpu"] * 8) == (9000, 4 << 20)


def test_default_run_is_c2_on_one_gpu(bench, monkeypatch):
    monkeypatch.setattr("sys.argv", ["bench.py"])
    a = bench.parse()
    assert (a.config, a.gpus) == ("c2", 1)
    assert a.steps > 0 and a.warmup >= 0


@pytest.mark.parametrize("gpus", [2, 4, 8])
def test_default_run_on_n_gpus_is_c4(bench, monkeypatch, gpus):
    """`bench.py --gpus N` (the driver's form) runs BASELINE.json's
    multi-GPU config: C4's 2 M x 1500 B per GPU, 16 M in total at N = 8."""
    monkeypatch.setattr("sys.argv", ["bench.py", "--gpus", str(gpus)])
    a = bench.parse()
    assert a.config == "c4" and not a.strong
    w = bench.workload(a.config, gpus)
    assert (w["per_gpu"], w["total"], w["scaling"]) == (1 << 21, gpus << 21, "weak")
    assert w["desc"].startswith(f"c4: {2 * gpus} M x 1500 B")
    assert f"2 M per GPU x {gpus} MI355X" in w["desc"]


def test_workload_arithmetic(bench):
    w = bench.workload("c2", 1)
    assert (w["per_gpu"], w["total"], w["scaling"]) == (1 << 20, 1 << 20, "weak")
    assert w["desc"].startswith("c2: 1 M x 1500 B") and w["desc"].endswith("1 MI355X")
    w = bench.workload("c4", 8)
    assert (w["per_gpu"], w["total"]) == (1 << 21, 1 << 24)
    assert w["desc"].startswith("c4: 16 M x 1500 B")
    # --strong: C4's 16 M batch split N ways
    for n in (1, 2, 4, 8):
        w = bench.workload("c4", n, strong=True)
        assert (w["total"], w["per_gpu"] * n, w["scaling"]) == (1 << 24, 1 << 24, "strong")
    w = bench.workload("c5", 8, strong=True)
    assert (w["total"], w["per_gpu"]) == (4 << 20, 512 << 10)
    w = bench.workload("c3", 2, strong=True)
    assert (w["total"], w["per_gpu"]) == (1 << 20, 1 << 19) and "bimodal" in w["desc"]
    # --per-gpu (tests) overrides, weak
    w = bench.workload("c4", 2, per_gpu_override=1 << 17)
    assert (w["total"], w["scaling"]) == (1 << 18, "weak") and w["desc"].startswith("c4: 256 K")


def test_rows_refuse_multi_gpu(bench, monkeypatch):
    monkeypatch.setattr("sys.argv", ["bench.py", "--config", "f1", "--gpus", "2"])
    with pytest.raises(SystemExit):
        bench.run_row(bench.parse())


class _FakeRanks:
    """Stands in for the launcher process: records the command, prints what
    a 2-rank run prints (launcher chatter and rank 0's one JSON line)."""
    seen = {}

    def __init__(self, cmd, env=None, stdout=None, text=None, bufsize=None):
        _FakeRanks.seen = dict(cmd=cmd, env=env)
        self.stdout = iter(["launcher: starting 2 ranks\n", '{"metric": "m", "n_gpus": 2}\n'])

    def wait(self):
        return 0


def test_self_launch_starts_n_ranks(bench, monkeypatch, capsys):
    """`bench.py --gpus N` without WORLD_SIZE: the parent starts
    torch.distributed.run with N ranks on 127.0.0.1 and a free port, the
    same arguments, and forwards the ranks' single JSON line to stdout."""
    import subprocess
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("MTCP_BENCH_DEVICE", "0")
    monkeypatch.setattr(subprocess, "Popen", _FakeRanks)
    argv = ["--gpus", "2", "--config", "c2", "--steps", "3"]
    monkeypatch.setattr("sys.argv", ["bench.py", *argv])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    cmd = _FakeRanks.seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "127.0.0.1" in cmd
    port = [c for c in cmd if c.startswith("--master-port=")]
    assert len(port) == 1 and 0 < int(port[0].split("=")[1]) < 65536
    assert cmd[-len(argv):] == argv and cmd[-len(argv) - 1].endswith("bench.py")
    assert _FakeRanks.seen["env"]["MASTER_ADDR"] == "127.0.0.1"
    out, err = capsys.readouterr()
    assert out.strip().splitlines() == ['{"metric": "m", "n_gpus": 2}']
    assert "launcher: starting" in err


def test_self_launch_fails_when_a_rank_fails(tmp_path):
    """The real path end to end on a GPU-less host: the parent launches two
    ranks (both pointed at device 0), they fail at their first GPU call, and
    the parent exits non-zero without printing a JSON line."""
    import subprocess
    import sys
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present (tests/test_gpu_shard.py runs this path there)")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MTCP_BENCH_DEVICE"] = "0"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--per-gpu", "4096", "--cpu-baseline", "off", "--pcie", "off"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_self_launch_refuses_more_gpus_than_visible(tmp_path):
    import subprocess
    import sys
    import torch
    if torch.cuda.device_count() >= 64:
        pytest.skip("64 GPUs visible")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MTCP_BENCH_DEVICE")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "GPU(s) visible" in p.stderr


def test_read_ceiling_probe_is_built_and_exported(bench, monkeypatch):
    """bench.py's read-ceiling leg (roofline.read_ceiling) loads
    tools/libstream_ceiling.so, which build() makes; on by default."""
    import ctypes
    path = os.path.join(ROOT, "tools", "libstream_ceiling.so")
    assert os.path.exists(path), "run __graft_entry__.build()"
    assert hasattr(ctypes.CDLL(path), "stream_ceiling_us")
    monkeypatch.setattr("sys.argv", ["bench.py"])
    a = bench.parse()
    assert (a.ceiling, a.numa) == ("on", "on")


def _rank(r, pci, kern, node=0):
    return {"rank": r, "device": r, "gpu_pci": pci, "numa_node": node, "kern_ms": kern, "wall_ms": 10.0,
            "read_ceiling_us": 220.0, "kernel_frac_of_ceiling": round(0.22 / kern, 4)}


def test_rank_summary_shape(bench):
    """the N > 1 line carries every rank's GPU (pci,
    NUMA node), event-timed launch, wall time and own read ceiling, the
    launch spread and the number of distinct GPUs; ranks sharing a GPU are
    flagged unless MTCP_BENCH_DEVICE forced it (then a note says so)."""
    eight = [_rank(r, f"0000:{0x10 * (r + 1):02x}:00.0", 0.24 + 0.001 * r, r // 4) for r in reversed(range(8))]
    s = bench.rank_summary(eight, None)
    assert [r["rank"] for r in s["per_rank"]] == list(range(8))
    assert set(s["per_rank"][0]) == {"rank", "device", "gpu_pci", "numa_node", "kern_ms", "wall_ms",
                                     "read_ceiling_us", "kernel_frac_of_ceiling"}
    assert s["distinct_gpus"] == 8 and "warning" not in s and "note" not in s
    assert s["kern_ms_spread"] == round(0.247 / 0.24, 4)
    shared = [_rank(r, "0000:10:00.0" if r < 2 else f"0000:{0x10 * (r + 1):02x}:00.0", 0.24) for r in range(8)]
    s = bench.rank_summary(shared, None)
    assert s["distinct_gpus"] == 7 and "7 distinct" in s["warning"] and "not a 8-GPU" in s["warning"]
    one = [_rank(r, "0000:10:00.0", 0.24) for r in range(8)]
    s = bench.rank_summary(one, "0")
    assert s["distinct_gpus"] == 1 and "warning" not in s and s["note"].startswith("MTCP_BENCH_DEVICE=0")
    s = bench.rank_summary([_rank(0, "0000:10:00.0", 0.24)], None)
    assert s["distinct_gpus"] == 1 and s["kern_ms_spread"] == 1.0 and "warning" not in s
