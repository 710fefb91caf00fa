#!/usr/bin/env python3
"""Average per-dispatch PMC values of kernels matching a substring: pmc_summary.py <dir> <kernel substring>."""
import collections
import csv
import glob
import sys

d, pat = sys.argv[1], sys.argv[2]
agg, n = collections.defaultdict(float), collections.Counter()
for f in sorted(glob.glob(f"{d}/*/run_counter_collection.csv") + glob.glob(f"{d}/run_counter_collection.csv") + glob.glob(f"{d}/compact.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
for k in sorted(agg):
    print(f"{k:28s} {agg[k] / n[k]:.4g}")
