#!/usr/bin/env python3
"""Summarise one scripts/profile_bench.sh run into profiles/<tag>/: the rocprofv3 --stats table, the
per-kernel HBM traffic from the separate FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE doubled: on gfx950
it reports half the bytes of a wide coalesced read, MI355X_MICROARCH.md §HBM; both counters are KB),
and a JSON the bench reads for roofline.traffic.

usage: python scripts/prof_summary.py gpurun_out/prof_<tag> profiles/<tag>
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    name = name.replace("void ", "")
    return name.split("(")[0] if "<" not in name.split("(")[0] else name[:name.index(">") + 1] if "(" in name else name


def counters(path, counter, scale=1024.0):
    per = collections.defaultdict(list)
    if not os.path.exists(path):  # scripts/pmc_compact.py output (per-dispatch sums) in its place
        path = os.path.join(os.path.dirname(path), "compact.csv")
    if not os.path.exists(path):
        return per
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * scale)
    return per


def mfma_pass(path):
    """Per kernel: MFMA busy fraction = sum(SQ_VALU_MFMA_BUSY_CYCLES) / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
    (rocprofv3's MfmaUtil expression with GRBM_GUI_ACTIVE summed over the 8 XCDs), and the MFMA FLOPs the
    hardware counted (SQ_INSTS_VALU_MFMA_MOPS_{F16,BF16} x 512)."""
    busy = counters(path, "SQ_VALU_MFMA_BUSY_CYCLES", 1.0)
    grbm = counters(path, "GRBM_GUI_ACTIVE", 1.0)
    f16 = counters(path, "SQ_INSTS_VALU_MFMA_MOPS_F16", 512.0)
    bf16 = counters(path, "SQ_INSTS_VALU_MFMA_MOPS_BF16", 512.0)
    out = {}
    for k in busy:
        b, g = sum(busy[k]), sum(grbm.get(k, []))
        n = len(busy[k])
        out[k] = dict(mfma_busy=(b / (g / 8.0 * 1024.0)) if g else None,
                      mfma_flops_per_launch=(sum(f16.get(k, [])) + sum(bf16.get(k, []))) / max(n, 1),
                      clock_ghz_x_us=g / 8.0 / max(n, 1))
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    fetch = counters(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    mf = mfma_pass(os.path.join(src, "pmc_mfma", "run_counter_collection.csv"))
    rows, out = [], {}
    for r in csv.DictReader(open(stats)):
        k = short(r["Name"])
        f, w = fetch.get(k, []), write.get(k, [])
        fb = 2.0 * sum(f) / len(f) if f else None
        wb = sum(w) / len(w) if w else None
        traffic = (fb or 0.0) + (wb or 0.0) if (f or w) else None
        m = mf.get(k, {})
        avg_s = float(r["AverageNs"]) * 1e-9
        tfs = m.get("mfma_flops_per_launch", 0.0) / avg_s / 1e12 if m.get("mfma_flops_per_launch") else 0.0
        out[k] = dict(calls=int(r["Calls"]), avg_us=float(r["AverageNs"]) / 1e3, pct=float(r["Percentage"]),
                      hbm_read_bytes_per_launch=fb, hbm_write_bytes_per_launch=wb,
                      hbm_bytes_per_launch=traffic, mfma_busy=m.get("mfma_busy"),
                      mfma_flops_per_launch=m.get("mfma_flops_per_launch"), mfma_tflops_counted=tfs or None)
        gbs = traffic / avg_s / 1e9 if traffic else None
        busy = m.get("mfma_busy")
        rows.append(f"| `{k}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} | "
                    f"{(fb or 0) / 1e6:.1f} | {(wb or 0) / 1e6:.1f} | {gbs or 0:.0f} | "
                    f"{'' if busy is None else f'{100 * busy:.1f}'} | {tfs:.0f} |")
    json.dump(out, open(os.path.join(dst, "kernels.json"), "w"), indent=1)
    with open(os.path.join(dst, "SUMMARY.md"), "w") as fh:
        fh.write(f"# rocprofv3 summary ({os.path.basename(dst)})\n\n"
                 "Source: `scripts/profile_bench.sh` (rocprofv3 kernel-trace --stats over `bench.py --steps 2 --warmup 1` "
                 "with ALCM_SERIAL_RESBLOCKS=1 — the bench's headline pass plus its roofline pass — then separate "
                 "`--pmc FETCH_SIZE`, `--pmc WRITE_SIZE` and MFMA passes over one step).  HBM read = "
                 "2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE, averaged per launch.  MFMA busy % = "
                 "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) from a third `--pmc` pass (rocprofv3's "
                 "MfmaUtil); MFMA TF/s = (SQ_INSTS_VALU_MFMA_MOPS_F16 + _BF16) x 512 / avg duration (hardware-counted "
                 "MFMA work, including the bf16x3 split's 3 products).\n\n"
                 "| kernel | calls | avg us | % time | HBM read MB/launch | HBM write MB/launch | HBM GB/s | "
                 "MFMA busy % | MFMA TF/s (counted) |\n"
                 "|---|---|---|---|---|---|---|---|---|\n")
        fh.write("\n".join(rows) + "\n")
    print(open(os.path.join(dst, "SUMMARY.md")).read())


if __name__ == "__main__":
    main()
