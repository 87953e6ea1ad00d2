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


def test_rows_refuse_multi_gpu(bench, monkeypatch):
    monkeypatch.setattr("sys.argv", ["bench.py", "--config", "f1", "--gpus", "2"])
    with pytest.raises(SystemExit):
        bench.run_row(bench.parse())
