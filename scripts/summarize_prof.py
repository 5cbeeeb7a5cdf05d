#!/usr/bin/env python3
"""Summarise a scripts/profile.sh output dir: per-kernel mean duration and
mean PMC counter values (one row per kernel)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
keys = sys.argv[2:] or ["pack_kernel", "unpack_kernel"]
stats = os.path.join(d, "trace", "run_kernel_stats.csv")
if os.path.exists(stats):
    for r in csv.DictReader(open(stats)):
        if any(k in r["Name"] for k in keys):
            print(f'{r["Name"][:60]:60s} calls={r["Calls"]} avg_us={float(r["AverageNs"])/1e3:.1f}')
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        for k in keys:
            if k in r["Kernel_Name"]:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, dct in agg.items():
    print(k)
    for c, v in sorted(dct.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.0f}")
