#!/usr/bin/env python3
"""Summary of tools/dispatch_map.sh: for each (batch size, frame size) the
automatic choice against the fastest forced kernel, and whether every
kernel's records hashed the same.
  usage: python3 tools/dispatch_map.py gpurun_out/dispatch_map.jsonl"""
import collections
import json
import sys


def main():
    rows = collections.defaultdict(dict)
    for line in open(sys.argv[1]):
        d = json.loads(line)
        rows[(d["frames"], str(d["frame_size"]))][d["sched"]] = d
    worst = []
    for (n, size) in sorted(rows, key=lambda k: (k[0], k[1])):
        r = rows[(n, size)]
        # the automatic choice with the size hint when the run has it (what an
        # io_module's rxq passes), else without
        key = "auto_hint" if "auto_hint" in r else "auto"
        if key not in r:
            continue
        forced = {k: v for k, v in r.items() if not k.startswith("auto")}
        best = min(forced.items(), key=lambda kv: kv[1]["us_per_launch"])
        a = r[key]
        ratio = a["us_per_launch"] / best[1]["us_per_launch"]
        same = len({v["records_sha"] for v in r.values()}) == 1
        worst.append(ratio)
        row = {"n": n, "size": size, "auto": key, "auto_kernel": a["kernel"], "auto_us": a["us_per_launch"],
               "best": best[0], "best_us": best[1]["us_per_launch"], "auto_over_best": round(ratio, 3),
               "records_identical": same}
        if key == "auto_hint" and "auto" in r:
            row["unhinted_kernel"], row["unhinted_us"] = r["auto"]["kernel"], r["auto"]["us_per_launch"]
        print(json.dumps(row))
    if worst:
        print(json.dumps({"cells": len(worst), "auto_within_5pct": sum(w <= 1.05 for w in worst),
                          "auto_within_10pct": sum(w <= 1.10 for w in worst), "worst": round(max(worst), 3)}))


if __name__ == "__main__":
    main()
