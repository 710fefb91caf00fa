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


def counters(path, counter):
    per = collections.defaultdict(list)
    if not os.path.exists(path):
        return per
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    fetch = counters(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    rows, out = [], {}
    for r in csv.DictReader(open(stats)):
        k = short(r["Name"])
        f, w = fetch.get(k, []), write.get(k, [])
        fb = 2.0 * sum(f) / len(f) if f else None
        wb = sum(w) / len(w) if w else None
        traffic = (fb or 0.0) + (wb or 0.0) if (f or w) else None
        out[k] = dict(calls=int(r["Calls"]), avg_us=float(r["AverageNs"]) / 1e3, pct=float(r["Percentage"]),
                      hbm_read_bytes_per_launch=fb, hbm_write_bytes_per_launch=wb,
                      hbm_bytes_per_launch=traffic)
        gbs = traffic / (float(r["AverageNs"]) * 1e-9) / 1e9 if traffic else None
        rows.append(f"| `{k}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} | "
                    f"{(fb or 0) / 1e6:.1f} | {(wb or 0) / 1e6:.1f} | {gbs or 0:.0f} |")
    json.dump(out, open(os.path.join(dst, "kernels.json"), "w"), indent=1)
    with open(os.path.join(dst, "SUMMARY.md"), "w") as fh:
        fh.write(f"# rocprofv3 summary ({os.path.basename(dst)})\n\n"
                 "Source: `scripts/gpu_profile.sh` (rocprofv3 kernel-trace --stats over `bench.py --steps 1 --warmup 1` "
                 "with ALCM_SERIAL_RESBLOCKS=1 — the bench's headline pass plus its roofline pass, so every launch "
                 "appears twice per step — then separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes).  HBM read = "
                 "2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE, averaged per launch.\n\n"
                 "| kernel | calls | avg us | % time | HBM read MB/launch | HBM write MB/launch | HBM GB/s |\n"
                 "|---|---|---|---|---|---|---|\n")
        fh.write("\n".join(rows) + "\n")
    print(open(os.path.join(dst, "SUMMARY.md")).read())


if __name__ == "__main__":
    main()
