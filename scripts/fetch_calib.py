#!/usr/bin/env python3
"""Summarise scripts/fetch_calib.sh: counted FETCH_SIZE / WRITE_SIZE (KB units, per rocprofv3) per probe kernel
against the bytes the kernel provably moved (printed by the probe), i.e. the correction factor each access form
needs.  Usage: python3 scripts/fetch_calib.py gpurun_out/fetch_calib"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
known = {}
for line in open(os.path.join(d, "plain.log")):
    m = re.match(r"(\S+)\s+bytes (\d+)\s+([\d.]+) ms\s+([\d.]+) GB/s", line)
    if m:
        known[m.group(1)] = (int(m.group(2)), float(m.group(3)), float(m.group(4)))


def counters(sub):
    out = {}
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            base = re.sub(r"\(.*", "", name).split("::")[-1].strip()
            out[base] = out.get(base, 0.0) + float(r.get("Counter_Value", 0) or 0)
    return out


fe, wr = counters("fetch"), counters("write")
print("| probe kernel | bytes moved | ms | GB/s | FETCH_SIZE x 1024 / bytes | WRITE_SIZE x 1024 / bytes |")
print("|---|---|---|---|---|---|")
for k, (b, ms, gbs) in known.items():
    f = fe.get(k)
    w = wr.get(k)
    print(f"| `{k}` | {b} | {ms:.3f} | {gbs:.0f} | {f * 1024 / b if f else float('nan'):.3f} | "
          f"{w * 1024 / b if w else float('nan'):.3f} |")
