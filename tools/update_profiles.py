#!/usr/bin/env python3
"""Copy one GPU session's evidence from gpurun_out/ into profiles/<round>/.

For each config: the bench JSON line (gpurun_out/b<N>.log), the rocprofv3
kernel-stats CSV and the trace+PMC summary (tools/profile_config.sh output in
gpurun_out/prof_c<N>, summarized by tools/summarize_profile.py), and the
per-launch HBM traffic that bench.py reports as roofline.traffic
(profiles/traffic_c<N>.json).
  usage: tools/update_profiles.py ROUND [configs...]   e.g. r1 c2 c3 c5
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1]
cfgs = sys.argv[2:] or ["c2", "c3", "c5"]
dst = os.path.join(ROOT, "profiles", rnd)
os.makedirs(dst, exist_ok=True)
for c in cfgs:
    src = os.path.join(ROOT, "gpurun_out", f"prof_{c}")
    summ = os.path.join(dst, f"summary_{c}.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "summarize_profile.py"), src, c, summ],
                   check=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"kernel_stats_{c}.csv"))
    line = [ln for ln in open(os.path.join(ROOT, "gpurun_out", f"b{c[1:]}.log")) if ln.startswith("{")][-1]
    json.dump(json.loads(line), open(os.path.join(dst, f"bench_{c}.json"), "w"), indent=1)
    s = json.load(open(summ))
    json.dump({
        "config": c,
        # bench.py uses the figure on this build or one with the same rx_kernel sources (mtcp_amd/_codeobj.py)
        "lib_sha256": open(os.path.join(src, "lib.sha256")).read().strip(),
        "rx_source_key": open(os.path.join(src, "rx_source.key")).read().strip(),
        "hbm_bytes_per_launch": s["hbm_bytes_per_launch"],
        "hbm_read_bytes_per_launch": s["hbm_read_bytes_per_launch"],
        "hbm_write_bytes_per_launch": s["hbm_write_bytes_per_launch"],
        "source": f"profiles/{rnd}/summary_{c}.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate "
                  "passes, FETCH_SIZE x2 gfx950 correction)",
    }, open(os.path.join(ROOT, "profiles", f"traffic_{c}.json"), "w"), indent=1)
