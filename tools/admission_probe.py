#!/usr/bin/env python3
"""What gpu_module.c's admission default (two offloading mTCP threads per
GPU) does to a deployment of many threads: mTCP's rx loop
over gpu_module.c (tests/c/rxloop.c, 1500 B frames, threads on the GPU's
NUMA node, software threads running the reference's own rx chain) at 8, 12
and 16 threads with MTCP_GPU_THREADS default (2), 1 and 0 (no offload),
interleaved and rotated per rep so that drifts of the box hit every limit
alike.  Each line also carries what the run cost the host: the CPU seconds
the threads used per million frames (getrusage of the child) and how often
the box's CPU quota throttled the process meanwhile (cgroup cpu.stat), so a
slow run can be told apart from a throttled one.

  python tools/admission_probe.py [reps] > gpurun_out/admission.jsonl
  (ADM_THREADS=1,2,4,8,16: other thread counts)
"""
import json
import os
import resource
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import io_path_bench as iob  # noqa: E402


def cgroup():
    """The process's cgroup v2 directory (or None)."""
    try:
        for ln in open("/proc/self/cgroup"):
            if ln.startswith("0::"):
                d = "/sys/fs/cgroup" + ln.strip()[3:]
                return d if os.path.isdir(d) else "/sys/fs/cgroup"
    except OSError:
        pass
    return None


def cpu_stat(d):
    out = {}
    try:
        for ln in open(os.path.join(d, "cpu.stat")):
            k, v = ln.split()
            out[k] = int(v)
    except (OSError, TypeError, ValueError):
        pass
    return out


THREADS = tuple(int(t) for t in os.environ.get("ADM_THREADS", "8,12,16").split(","))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    n = 1 << 18
    cg = cgroup()
    quota = None
    try:
        quota = open(os.path.join(cg, "cpu.max")).read().strip()
    except (OSError, TypeError):
        pass
    host = iob.host_topology()
    host.update({"cgroup": cg, "cpu_max": quota, "os_cpu_count": os.cpu_count()})
    print(json.dumps(host), flush=True)
    import oracle
    if oracle.ref_available():
        os.environ["RXLOOP_REF"] = oracle.REF_LIB_PATH
    os.environ["RXLOOP_CPUS"] = ",".join(map(str, host["gpu_local_cpus"]))
    limits = ("default", "1", "0")
    with tempfile.TemporaryDirectory() as tmp:
        for rep in range(reps):
            for threads in THREADS:
                order = limits[rep % 3:] + limits[:rep % 3]
                for limit in order:
                    os.environ["RXLOOP_PASSES"] = str(4 * threads)
                    os.environ.pop("MTCP_GPU_THREADS", None)
                    if limit != "default":
                        os.environ["MTCP_GPU_THREADS"] = limit
                    ru0 = resource.getrusage(resource.RUSAGE_CHILDREN)
                    st0 = cpu_stat(cg)
                    r = iob.run(n, 1500, 2, tmp, "timing", threads, True, reps=1)
                    ru1 = resource.getrusage(resource.RUSAGE_CHILDREN)
                    st1 = cpu_stat(cg)
                    cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
                    share = r["frames"] / threads
                    per = r["thread_seconds_offload"] or []
                    print(json.dumps({
                        "probe": "admission_paired", "rep": rep, "threads": threads, "gpu_threads": limit,
                        "offloading_threads": r["offloading_threads"], "mpkt_per_s": r["mpkt_per_s"],
                        "GBs": r["GBs"], "frames": r["frames"],
                        "cpu_s_per_mframe": round(cpu_s / (r["frames"] / 1e6), 4),
                        "throttled_periods": st1.get("nr_throttled", 0) - st0.get("nr_throttled", 0),
                        "throttled_ms": round((st1.get("throttled_usec", 0) - st0.get("throttled_usec", 0)) / 1e3, 1),
                        "offload_thread_mpps": [round(share / s / 1e6, 2) for s, o in per if o],
                        "sw_thread_mpps": [round(share / s / 1e6, 2) for s, o in per if not o]}), flush=True)
    os.environ.pop("MTCP_GPU_THREADS", None)


if __name__ == "__main__":
    main()
