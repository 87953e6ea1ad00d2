#!/usr/bin/env python3
"""Copy one GPU session's evidence from gpurun_out/ into profiles/<round>/.

For each config: the bench JSON line (gpurun_out/b<cfg>.log), the rocprofv3
kernel-stats CSV and the trace+PMC summary (tools/profile_config.sh output in
gpurun_out/prof_<cfg>, summarized by tools/summarize_profile.py), and the
per-launch HBM traffic that bench.py reports as roofline.traffic
(profiles/traffic_<cfg>.json).
  usage: tools/update_profiles.py ROUND [configs...]   e.g. r3 c2 c3 c3_compact c5 f1
         tools/update_profiles.py --traffic [configs...]
The --traffic form runs ON THE GPU BOX inside tools/round_evidence.sh, right
after the PMC passes and before the bench lines: it writes
profiles/traffic_<cfg>.json (which bench.py reads in the same session, so the
committed bench lines quote the traffic of the build they measured) and
copies them to gpurun_out/ (the only directory that comes back).
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def summarize(c, summ):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{c}")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "summarize_profile.py"), src, c, summ],
                   check=True)
    return src


def write_traffic(c, src, summ, source):
    s = json.load(open(summ))
    t = {
        "config": c,
        # bench.py uses the figure on this build or one with the same rx sources (mtcp_amd/_codeobj.py)
        "lib_sha256": open(os.path.join(src, "lib.sha256")).read().strip(),
        "rx_source_key": open(os.path.join(src, "rx_source.key")).read().strip(),
        "hbm_bytes_per_launch": s["hbm_bytes_per_launch"],
        "hbm_read_bytes_per_launch": s["hbm_read_bytes_per_launch"],
        "hbm_write_bytes_per_launch": s["hbm_write_bytes_per_launch"],
        "avg_duration_ns_trace": s["timed_avg_duration_ns"],
        "source": source,
    }
    path = os.path.join(ROOT, "profiles", f"traffic_{c}.json")
    json.dump(t, open(path, "w"), indent=1)
    return path


if sys.argv[1] == "--traffic":
    for c in sys.argv[2:]:
        src = os.path.join(ROOT, "gpurun_out", f"prof_{c}")
        summ = os.path.join(src, "summary.json")
        summarize(c, summ)
        path = write_traffic(c, src, summ, f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of this build, separate "
                                           f"passes, FETCH_SIZE x2 gfx950 correction (gpurun_out/prof_{c})")
        shutil.copy(path, os.path.join(ROOT, "gpurun_out", os.path.basename(path)))
    sys.exit(0)

rnd = sys.argv[1]
cfgs = sys.argv[2:] or ["c2", "c3", "c5"]
dst = os.path.join(ROOT, "profiles", rnd)
os.makedirs(dst, exist_ok=True)
for c in cfgs:
    summ = os.path.join(dst, f"summary_{c}.json")
    src = summarize(c, summ)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"kernel_stats_{c}.csv"))
    blog = os.path.join(ROOT, "gpurun_out", f"b{c}.log")
    if os.path.exists(blog):
        line = [ln for ln in open(blog) if ln.startswith("{")][-1]
        json.dump(json.loads(line), open(os.path.join(dst, f"bench_{c}.json"), "w"), indent=1)
    write_traffic(c, src, summ, f"profiles/{rnd}/summary_{c}.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                                "separate passes, FETCH_SIZE x2 gfx950 correction)")
