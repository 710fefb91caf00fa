#!/usr/bin/env python3
"""Per-kernel SQ breakdown from scripts/pmc_bench.sh passes: pmc_table.py gpurun_out/pmc_bench_<tag> [min share]."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(f"{d}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
rows = []
for k, c in tot.items():
    n = max(cnt[k].values())
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    if wc <= 0:
        continue
    g = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0  # per-XCD cycles
    rows.append((g, k, n, dict(
        wait=c.get("SQ_WAIT_ANY", 0) / wc, issue_stall=c.get("SQ_WAIT_INST_ANY", 0) / wc,
        active=c.get("SQ_ACTIVE_INST_ANY", 0) / wc, valu=c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
        lds_stall=c.get("SQ_WAIT_INST_LDS", 0) / wc,
        mfma_busy=c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (g * 1024) if g else 0,
        coexec=c.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / (g * 1024) if g else 0,
        bank_conf=c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_LDS_IDX_ACTIVE", 1), 1),
        waves_per_simd=wc / (g / 4.0 * 1024) if g else 0,  # SQ_WAVE_CYCLES in quad-cycles
        valu_per_wave=c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_WAVES", 1), 1),
        lds_per_wave=c.get("SQ_INSTS_LDS", 0) / max(c.get("SQ_WAVES", 1), 1),
        mfma_per_wave=c.get("SQ_INSTS_MFMA", 0) / max(c.get("SQ_WAVES", 1), 1))))
rows.sort(reverse=True)
g_all = sum(r[0] for r in rows)
print(f"{'kernel':60s} {'share':>6s} " + " ".join(f"{h:>9s}" for h in rows[0][3]))
for g, k, n, v in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{k[:60]:60s} {g / g_all:6.3f} " + " ".join(f"{x:9.3f}" for x in v.values()))
