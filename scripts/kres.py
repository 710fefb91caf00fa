#!/usr/bin/env python3
"""Dev tool: per-kernel VGPR / spill / LDS table of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage).
Usage: python scripts/kres.py audiolcm_amd/csrc/alcm_wconv.hip [name filter]"""
import os
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
d = os.path.dirname(os.path.abspath(src))
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I", d, "-I",
       os.path.join(d, "..", "..", "include"), "-w", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = {}, None
for line in err.splitlines():
    m = re.search(r"remark: +(.*?): (\S+) \[", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for n, r in rows.items():
    if flt in n:
        print(f"{n[:110]:110s} V {r.get('VGPRs')} A {r.get('AGPRs')} spill {r.get('VGPRs Spill')} "
              f"LDS {r.get('LDS Size [bytes/block]')}")
