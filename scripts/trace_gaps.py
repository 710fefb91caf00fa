#!/usr/bin/env python3
"""GPU idle time per bench step from a rocprofv3 --kernel-trace CSV (dev tool): steps are delimited by the BigVGAN
output head (post_kernel, once per step); per step: wall between consecutive heads, union of kernel intervals
(any stream), idle = wall - busy, and the largest idle gaps with the kernels on either side.
python scripts/trace_gaps.py <trace dir>"""
import csv
import glob
import sys

f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
rows = []
for r in csv.DictReader(open(f)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
heads = [e for s, e, n in rows if "post_kernel" in n]
print(f"{len(rows)} kernels, {len(heads)} steps")
for a, b in zip(heads[:-1], heads[1:]):
    ks = [(s, e, n) for s, e, n in rows if s >= a and s < b]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    prev = None
    for s, e, n in ks:
        if cur_e is None:
            cur_s, cur_e = s, e
            if s > a:
                gaps.append((s - a, "(step start)", n))
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = n
    busy += min(cur_e, b) - cur_s
    wall = b - a
    print(f"step: wall {wall / 1e6:.3f} ms busy {busy / 1e6:.3f} ms idle {(wall - busy) / 1e6:.3f} ms "
          f"({len(ks)} kernels, {len(gaps)} gaps, >10us: {sum(1 for g in gaps if g[0] > 10000)})")
    for g, p, n in sorted(gaps, reverse=True)[:8]:
        print(f"   {g / 1e3:8.1f} us  after {p[:60] if p else '-'}  before {n[:60]}")
