#!/usr/bin/env python3
"""Summarize tools/profile_config.sh output for one config into a JSON file
for profiles/: the config's kernel's average duration (kernel trace), HBM traffic per
launch from PMC (FETCH_SIZE x 2 per the gfx950 correction of
MI355X_MICROARCH.md §HBM, cross-checked against TCC_EA0_RDREQ_128B x 128 B;
WRITE_SIZE as is), and the algorithmic bytes."""
import csv
import glob
import json
import statistics
import sys

src, cfg, out = sys.argv[1], sys.argv[2], sys.argv[3]
# algorithmic bytes per launch: sum L (rx), sum L + 4 B of check fields per frame (f1)
algo = {"c1": 65536 * 64, "c2": 1572864000, "c3": 819090368, "c3_compact": 819090368, "c5": 4718592000,
        "f1": 1572864000 + 4 * (1 << 20), "f3": (1 << 20) * (40 + 4)}[cfg]
# the config's dominant kernel: C1's 64 K small frames take the quad kernel
# (mtcp_gpu.hip pick_sched), f3 is the separate HashFlow kernel
KERNEL = {"c1": "rx_group_kernel", "f3": "flow_hash_kernel"}.get(cfg, "rx_kernel")


def rows(pattern):
    r = []
    for f in glob.glob(pattern):
        r += list(csv.DictReader(open(f)))
    return r


def kname(r):
    return r["Kernel_Name"].split("(")[0]


stats = {r["Name"]: r for r in rows(f"{src}/trace/run_kernel_stats.csv")}
rx = [k for k in stats if k.startswith(KERNEL)][0]
trace = [r for r in rows(f"{src}/trace/run_kernel_trace.csv") if kname(r).startswith(KERNEL)]
trace.sort(key=lambda r: int(r["Start_Timestamp"]))
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace]
# the bench's own line under the profiler (same process): HIP-event average
# over its timed steps; the trace's last `steps` launches are those steps
bench = None
try:
    bench = json.loads([ln for ln in open(f"{src}/trace.log") if ln.startswith("{")][-1])
except (OSError, IndexError, ValueError):
    pass
steps = bench["steps"] if bench else len(durs)
timed = durs[-steps:]


def pmc(sub, counter):
    v = [float(r["Counter_Value"]) for r in rows(f"{src}/{sub}/run_counter_collection.csv")
         if kname(r).startswith(KERNEL) and r["Counter_Name"] == counter]
    return statistics.median(v) if v else None


fetch = pmc("fetch", "FETCH_SIZE")
write = pmc("write", "WRITE_SIZE")
rd128 = pmc("rdreq", "TCC_EA0_RDREQ_128B_sum")
rd64 = pmc("rdreq", "TCC_EA0_RDREQ_64B_sum")
rdall = pmc("rdreq", "TCC_EA0_RDREQ_sum")
read_fetch = fetch * 1024 * 2 if fetch is not None else None
read_req = rd128 * 128 + (rd64 or 0) * 64 + max(0.0, (rdall or 0) - rd128 - (rd64 or 0)) * 32 \
    if rd128 is not None else None
wbytes = write * 1024 if write is not None else None
res = {
    "config": cfg,
    "kernel": rx,
    "launches": len(durs),
    "avg_duration_ns": statistics.mean(durs),
    "median_duration_ns": statistics.median(durs),
    "timed_steps": len(timed),
    "timed_avg_duration_ns": statistics.mean(timed),
    "bench_events_avg_launch_ns_same_run": bench["roofline"]["avg_launch_ms"] * 1e6 if bench else None,
    "note_launches": f"all {KERNEL} launches of the run (for rx_kernel: the generator's tx fill, "
                     "pktgen uses the kernel in fill mode), the warm-up steps and the timed steps; "
                     "timed_* = the last `steps` launches, the ones bench.py's HIP events bracket",
    "stats_row": stats[rx],
    "algorithmic_bytes_per_launch": algo,
    "achieved_GBs_from_trace": algo / statistics.median(durs),
    "pmc": {"FETCH_SIZE_KB": fetch, "WRITE_SIZE_KB": write, "TCC_EA0_RDREQ_sum": rdall,
            "TCC_EA0_RDREQ_128B_sum": rd128, "TCC_EA0_RDREQ_64B_sum": rd64},
    "hbm_read_bytes_per_launch": read_fetch,
    "hbm_read_bytes_per_launch_rdreq": read_req,
    "hbm_write_bytes_per_launch": wbytes,
    "hbm_bytes_per_launch": (read_fetch or 0) + (wbytes or 0),
    "note": "read bytes = FETCH_SIZE x 1024 x 2 (gfx950: FETCH_SIZE reports half of a 16 B/lane "
            "streaming read, MI355X_MICROARCH.md §HBM); cross-check: TCC_EA0_RDREQ_128B x 128 B",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: res[k] for k in ("config", "avg_duration_ns", "timed_avg_duration_ns",
                                      "bench_events_avg_launch_ns_same_run", "achieved_GBs_from_trace",
                                      "hbm_read_bytes_per_launch", "hbm_read_bytes_per_launch_rdreq",
                                      "hbm_write_bytes_per_launch")}))
