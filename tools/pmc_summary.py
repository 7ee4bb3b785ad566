#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs per kernel (sum over XCD/SE instances,
mean over dispatches).  Usage: pmc_summary.py <dir-with-run_counter_collection.csv> [name-filter]"""
import collections
import csv
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "knnk::"
rows = list(csv.DictReader(open(d + "/run_counter_collection.csv")))
per = collections.defaultdict(float)
for r in rows:
    if flt not in r["Kernel_Name"]:
        continue
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    per[(name, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
agg = collections.defaultdict(list)
for (k, c, _), v in per.items():
    agg[(k, c)].append(v)
for (k, c), v in sorted(agg.items()):
    print("%-45s %-26s %16.0f  (n=%d)" % (k[:45], c, sum(v) / len(v), len(v)))
