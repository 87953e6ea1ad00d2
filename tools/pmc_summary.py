#!/usr/bin/env python3
"""Average each PMC counter per kernel over the pass directories of pmc_passes.sh."""
import collections
import csv
import glob
import json
import sys

out = sys.argv[1]
agg = collections.defaultdict(list)
dur = collections.defaultdict(list)
for f in glob.glob(f"{out}/pass*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
        dur[r["Kernel_Name"].split("(")[0][:60]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
res = collections.defaultdict(dict)
for (k, c), v in sorted(agg.items()):
    res[k][c] = sum(v) / len(v)
for k in res:
    res[k]["_avg_duration_ns"] = sum(dur[k]) / len(dur[k])
print(json.dumps(res, indent=1))
