#!/usr/bin/env python
"""Per-kernel averages of rocprofv3 counter CSVs: python scripts/pmc_summary.py gpurun_out/pmcab"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    print(k)
    print("   ", {c: f"{sum(v) / len(v):.4g}" for c, v in sorted(d.items())})
