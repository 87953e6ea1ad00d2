"""The kernel choice (mtcp_amd/csrc/dispatch.hpp: pick_sched, big_schedule,
narrow_batch) on the CPU: the header is plain C++, compiled here with g++
into tests/c/dispatch_test.cpp, and asked for the kernel of each batch.

* every boundary tests/test_gpu_wave.py::test_dispatch_boundaries checks on
  the MI355X, here without a GPU;
* the choices the MI355X itself reported (mtcp_gpu_last_kernel) for the 84
  cells of the round-5 dispatch map, with and without the size hint;
* the rules' invariants: tx never takes the span kernel, a launch only the
  small kernels implement never takes rx_kernel, a forced kernel is kept,
  a mix's hint changes nothing, pointer bursts count as 1 KiB slots.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from mtcp_amd import pktgen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AUTO, WAVE, ROW, QUAD, BIG, SPAN, OCT = range(7)


@pytest.fixture(scope="module")
def choose(tmp_path_factory):
    exe = tmp_path_factory.mktemp("dispatch") / "dispatch_test"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    "-o", str(exe), os.path.join(ROOT, "tests", "c", "dispatch_test.cpp")], check=True)

    def run(cases):
        """cases: (n, slot, min_len, max_len, rx, small_only, forced, ptrs)"""
        inp = "".join(" ".join(str(int(v)) for v in c) + "\n" for c in cases)
        out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True).stdout
        return out.splitlines()
    return run


def imix_lengths(n, seed):
    r = np.random.default_rng(seed).integers(0, 12, n)
    return np.where(r < 7, 64, np.where(r < 11, 576, 1500)).astype(np.uint16)


def batch(n, size):
    """(average slot, min_len, max_len) of the batches the GPU tests build."""
    if size == "imix":
        desc, nbytes = pktgen.layout_from_lengths(imix_lengths(n, 67), 6)
    else:
        desc, nbytes = pktgen.layout(n, size if size == "bimodal" else int(size), 6, 67)
    return nbytes // n, int(desc["len"].min()), int(desc["len"].max())


def test_gpu_test_boundaries_on_the_cpu(choose):
    from tests.test_gpu_wave import test_dispatch_boundaries
    params = next(m for m in test_dispatch_boundaries.pytestmark if m.name == "parametrize").args[1]
    cases, want = [], []
    for n, size, kernel in params:
        hinted = isinstance(size, str) and size.endswith("h")
        slot, lo, hi = batch(n, size[:-1] if hinted else size)
        cases.append((n, slot, lo if hinted else 0, hi if hinted else 0, 1, 0, AUTO, 0))
        want.append(kernel)
    got = choose(cases)
    bad = [(c[0], c[1], c[2:4], g, w) for c, g, w in zip(cases, got, want) if not g.startswith(w)]
    assert not bad, bad
    assert len(cases) >= 35


def test_the_hardware_map_choices(choose):
    """The kernel the MI355X reported for every cell of the round-5 dispatch
    map (profiles/r5/dispatch_map.jsonl: `auto` without, `auto_hint` with the
    batch's {min, max} length) is the one these rules give."""
    path = os.path.join(ROOT, "profiles", "r5", "dispatch_map.jsonl")
    if not os.path.exists(path):
        pytest.skip("profiles/r5/dispatch_map.jsonl not in this tree")
    rows = [json.loads(ln) for ln in open(path)]
    rows = [r for r in rows if r["sched"] in ("auto", "auto_hint")]
    cases = []
    for r in rows:
        slot, lo, hi = _sweep_batch(r["frames"], r["frame_size"])
        hinted = r["sched"] == "auto_hint"
        cases.append((r["frames"], slot, lo if hinted else 0, hi if hinted else 0, 1, 0, AUTO, 0))
    got = choose(cases)
    bad = [(r["frames"], r["frame_size"], r["sched"], g, r["kernel"]) for r, g in zip(rows, got) if g != r["kernel"]]
    assert not bad, bad
    assert len(rows) == 168


def _sweep_batch(n, size):
    """tools/size_sweep.py's batch of n frames of `size` (its `lengths`)."""
    if size == "imix":
        r = np.random.default_rng(5).integers(0, 12, n)
        lens = np.where(r < 7, 64, np.where(r < 11, 576, 1500)).astype(np.uint16)
    else:
        lens = pktgen.lengths(n, size if size == "bimodal" else int(size), 7)
    desc, nbytes = pktgen.layout_from_lengths(lens, 6)
    return nbytes // n, int(desc["len"].min()), int(desc["len"].max())


def test_rules_invariants(choose):
    sizes = [64, 128, 256, 512, 768, 1024, 1500, 2048, 4096, 9000]
    ns = [1, 64, 2048, 2049, 4096, 8192, 8193, 16384, 16385, 32768, 32769, 65536, 65537, 131072, 131073,
          262144, 1 << 20, 1 << 22]
    base = [(n, (s + 63) & ~63, s, s) for n in ns for s in sizes]
    # tx (rx = 0): never the span kernel; small_only: never rx_kernel
    got = choose([(n, sl, lo, hi, 0, 0, AUTO, 0) for n, sl, lo, hi in base])
    assert not any(g == "rx_span_kernel" for g in got)
    got = choose([(n, sl, lo, hi, 1, 1, AUTO, 0) for n, sl, lo, hi in base])
    assert not any(g.startswith("rx_kernel") for g in got)
    # a forced kernel is kept (span for rx; big unless small_only)
    for forced, name in ((WAVE, "rx_wave"), (ROW, "rx_group_kernel<row>"), (QUAD, "rx_group_kernel<quad>"),
                         (OCT, "rx_group_kernel<oct>"), (SPAN, "rx_span_kernel"), (BIG, "rx_kernel")):
        got = choose([(n, sl, 0, 0, 1, 0, forced, 0) for n, sl, lo, hi in base])
        assert all(g.startswith(name) for g in got), (forced, set(got))
    got = choose([(n, sl, 0, 0, 0, 1, BIG, 0) for n, sl, lo, hi in base])
    assert set(got) == {"rx_group_kernel<row>"}
    # a hint that spans more than 2x (a mix) changes nothing
    mixed = [(n, sl, 64, 1500) for n, sl, lo, hi in base]
    assert choose([(n, sl, lo, hi, 1, 0, AUTO, 0) for n, sl, lo, hi in mixed]) == \
        choose([(n, sl, 0, 0, 1, 0, AUTO, 0) for n, sl, lo, hi in mixed])
    # an inverted or empty hint is no hint
    assert choose([(n, sl, 900, 100, 1, 0, AUTO, 0) for n, sl, lo, hi in base]) == \
        choose([(n, sl, 0, 0, 1, 0, AUTO, 0) for n, sl, lo, hi in base])
    # pointer bursts: 1 KiB slots, the sorted line-aligned rounds for rx_kernel
    got = choose([(n, 1024, 0, 0, 1, 0, AUTO, 1) for n in ns])
    assert all(g in ("rx_wave_kernel<2 loads>", "rx_group_kernel<row>", "rx_group_kernel<oct>",
                     "rx_kernel<sorted,line-aligned>") for g in got), set(got)
    # the headline configs' kernels: C2 / C4 / C5 unrolled (line-aligned for
    # jumbo), C3's bimodal 800 B average the sorted rounds, C1 quads
    got = choose([(1 << 20, 1536, 0, 0, 1, 0, AUTO, 0), (1 << 21, 1536, 0, 0, 1, 0, AUTO, 0),
                  (1 << 19, 9024, 0, 0, 1, 0, AUTO, 0), (1 << 20, 800, 0, 0, 1, 0, AUTO, 0),
                  (1 << 16, 64, 0, 0, 1, 0, AUTO, 0)])
    assert got == ["rx_kernel<unrolled>", "rx_kernel<unrolled>", "rx_kernel<unrolled,line-aligned>",
                   "rx_kernel<sorted>", "rx_group_kernel<quad>"]


def test_small_hinted_batches_keep_the_wave_kernel(choose):
    """a hinted batch of at most 2 048 frames with 256-320 B slots
    (a small io_module aggregate) takes the wave kernel as the same batch
    without a hint does; the quad rule starts above 2 048 frames, where the
    dispatch map measured it."""
    for n in (1, 64, 512, 2048):
        for s in (200, 256, 300):
            sl = (s + 63) & ~63
            hinted, plain = choose([(n, sl, s, s, 1, 0, AUTO, 0), (n, sl, 0, 0, 1, 0, AUTO, 0)])
            assert hinted == plain and hinted.startswith("rx_wave_kernel"), (n, s, hinted, plain)
    got = choose([(4096, 256, 256, 256, 1, 0, AUTO, 0)])
    assert got[0].startswith("rx_group_kernel<oct>"), got
