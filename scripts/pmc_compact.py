#!/usr/bin/env python3
"""Shrink one rocprofv3 --pmc output directory to per-dispatch sums (dev tool): pmc_compact.py <dir> [kernel substr].

rocprofv3 writes one row per counter INSTANCE (per XCD / SE / TA ...), which for a few passes over a microbenchmark
exceeds gpurun's 64 MiB copy-back; this keeps Dispatch_Id, Kernel_Name, Grid_Size, Counter_Name and the summed value
(in <dir>/compact.csv, kernels matching the substring only) and deletes the raw files."""
import collections
import csv
import glob
import os
import shutil
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.OrderedDict()
files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
for f in files:
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if pat not in name:
            continue
        key = (int(r.get("Dispatch_Id", 0)), name, r.get("Grid_Size", ""), r["Counter_Name"])
        agg[key] = agg.get(key, 0.0) + float(r["Counter_Value"])
for p in os.listdir(d):
    fp = os.path.join(d, p)
    shutil.rmtree(fp) if os.path.isdir(fp) else os.remove(fp)
with open(os.path.join(d, "compact.csv"), "w", newline="") as fo:
    w = csv.writer(fo)
    w.writerow(["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
    for (di, name, g, c), v in sorted(agg.items()):
        w.writerow([di, name, g, c, v])
print(f"{d}: {len(files)} csv -> {len(agg)} rows")
