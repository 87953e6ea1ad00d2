"""The bounded waits of the C ABI (mtcp_amd/csrc/wait.hpp: Deadline, poll)
on the CPU: tests/c/wait_test.cpp drives poll with fake device queries.
A wait without a bound runs until the work is done; with one it gives up
with MTCP_GPU_ETIMEDOUT at (not before) its deadline; a runtime error is
MTCP_GPU_EIO at once; work found done after the deadline still counts."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OK, EIO, ETIMEDOUT = 0, -5, -110


def test_poll_rules(tmp_path):
    exe = tmp_path / "wait_test"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I/opt/rocm/include", "-o", str(exe), os.path.join(ROOT, "tests", "c", "wait_test.cpp")],
                   check=True)
    r = json.loads(subprocess.run([str(exe)], capture_output=True, text=True, check=True,
                                  timeout=60).stdout.strip())
    assert r["ready_after_100"] == [OK, 100]
    rc, polled, ms = r["never_ready_20ms"]
    assert rc == ETIMEDOUT and polled and 20.0 <= ms < 2000.0
    assert r["error"] == [EIO, 1]
    assert r["done_after_deadline"] == [OK, 1]
    assert r["unbounded"] == [0, 0]
