#!/usr/bin/env python3
"""Per-kernel ISA statistics of one HIP source (dev tool): VGPRs, occupancy and counts of selected opcodes.
    python scripts/isa_stats.py audiolcm_amd/csrc/alcm_nconv.hip [kernel-substring ...]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

src = os.path.abspath(sys.argv[1])
pats = sys.argv[2:]
inc = os.path.dirname(src)
root = os.path.dirname(os.path.dirname(inc))
with tempfile.TemporaryDirectory() as d:
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I" + inc,
                        "-I" + os.path.join(root, "include"), "-c", src, "-o", os.path.join(d, "x.o"), "--save-temps",
                        "-Rpass-analysis=kernel-resource-usage"], cwd=d, capture_output=True, text=True)
    res = {}
    cur = None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            res[cur] = {}
        m = re.search(r"(VGPRs|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            res[cur][m.group(1).split()[0]] = int(m.group(2))
    asm = open([os.path.join(d, f) for f in os.listdir(d) if f.endswith("gfx950.s")][0]).read()
for name, info in res.items():
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    if pats and not any(p in dem for p in pats):
        continue
    i = asm.index(name + ":")
    j = asm.index(".Lfunc_end", i)
    ins = [l.split()[0] for l in asm[i:j].splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    c = collections.Counter(ins)
    print(f"{dem[:90]:90s} vgpr {info.get('VGPRs')} occ {info.get('Occupancy')} lds {info.get('LDS')} | "
          f"ins {len(ins)} nop {c['s_nop']} pk_fma {c['v_pk_fma_f32']} cos {c['v_cos_f32_e32']} "
          f"mfma {sum(v for k, v in c.items() if 'mfma' in k)}")
