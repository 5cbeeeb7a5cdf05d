#!/usr/bin/env python3
"""Mean counter value per dispatch for each kernel of one rocprofv3 --pmc
output dir (run_counter_collection.csv).  Diagnostic.
    python3 scripts/pmc_table.py DIR [kernel-substring ...]"""
import collections
import csv
import glob
import re
import sys

d, keys = sys.argv[1], sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(anonymous namespace\)::|^void ", "", r["Kernel_Name"]).split("(")[0]
        if keys and not any(k in name for k in keys):
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in sorted(acc.items()):
    print(name)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.0f}   ({len(v)} dispatches)")
