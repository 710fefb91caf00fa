#!/usr/bin/env python3
"""Per-kernel register / scratch / instruction-count table of one HIP source (dev tool, used for the DESIGN.md
before/after ISA diffs).  python scripts/isa_kres.py audiolcm_amd/csrc/alcm_tconv.hip [substring]"""
import glob
import os
import re
import subprocess
import sys
import tempfile

src = os.path.abspath(sys.argv[1])
sub = sys.argv[2] if len(sys.argv) > 2 else ""
inc = os.path.dirname(src)
root = os.path.dirname(os.path.dirname(inc))
with tempfile.TemporaryDirectory() as d:
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I" + inc,
                        "-I" + os.path.join(root, "include"), "-c", src, "-o", os.path.join(d, "x.o"), "--save-temps",
                        "-Rpass-analysis=kernel-resource-usage"], cwd=d, capture_output=True, text=True)
    rows, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
        m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)", line)
        if m and cur:
            rows[cur][m.group(1).split()[0]] = int(m.group(2))
    asm = open(glob.glob(os.path.join(d, "*gfx950*.s"))[0]).read()
for k, v in sorted(rows.items()):
    m = re.search("^" + re.escape(k) + r":[^\n]*\n(.*?)s_endpgm", asm, re.S | re.M)
    n = len([l for l in m.group(1).splitlines() if l.strip() and not l.strip().startswith((";", "."))]) if m else -1
    dm = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
    if sub in dm:
        print(f"{dm[:120]:120s} V{v.get('VGPRs')} A{v.get('AGPRs')} S{v.get('SGPRs')} scratch{v.get('ScratchSize')} "
              f"occ{v.get('Occupancy')} ins{n}")
