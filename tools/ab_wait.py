#!/usr/bin/env python3
"""A/B of gpu_module's wait (a checking tool): the bounded wait polls the
aggregate's event (MTCP_GPU_WAIT_TIMEOUT_MS, default 2000) against the
blocking hipEventSynchronize (MTCP_GPU_WAIT_TIMEOUT_MS=0), io path timing
mode, 1500 B and 64 B frames, 1 and 2 threads, interleaved three times.
  usage: python tools/ab_wait.py [n_frames]"""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import io_path_bench as iop  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    host = iop.host_topology()
    os.environ["RXLOOP_CPUS"] = ",".join(map(str, host["gpu_local_cpus"]))
    with tempfile.TemporaryDirectory() as tmp:
        for rep in range(3):
            for size, seed in ((1500, 2), (64, 1)):
                for threads in (1, 2):
                    for wait in ("0", "2000"):
                        os.environ["MTCP_GPU_WAIT_TIMEOUT_MS"] = wait
                        r = iop.run(n, size, seed, tmp, "timing", threads, True)
                        print(json.dumps({"probe": "ab_wait", "rep": rep, "frame_size": size,
                                          "threads": threads, "wait_timeout_ms": wait,
                                          "mpkt_per_s": r["mpkt_per_s"]}), flush=True)


if __name__ == "__main__":
    main()
