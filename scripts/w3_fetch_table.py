#!/usr/bin/env python3
"""wconv3 per-launch read attribution from scripts/pmc_w3.sh output: w3_fetch_table.py <dir>.

Per shape (5 launches each, in WSHAPES order) the counted bytes (2 x FETCH_SIZE: the gfx950 FETCH correction for
16-B-per-lane streaming and LDS-DMA reads, profiles/r3z/fetch_calibration.md; WRITE_SIZE as is) beside:
  algorithmic  plane once + weights once + residual / accumulate reads (what bench.py's roofline counts);
  window       the input bytes the kernel actually DMAs: every (tile, N tile, 64-channel chunk) window of 256 +
               (k - 1) d rows x 128 B — the input re-read once per 192-column N tile plus the halo;
  weights      once per XCD that streams an N tile's weight slice (N-major order: each XCD's tiles share one or two
               N tiles; 8 XCDs);
so counted - algorithmic splits into (window - plane) [N-tile re-reads + halo] and weight re-fetch."""
import collections
import csv
import math
import os
import sys

B = 32
SHAPES = [("s0 C768 k11", 2496, 768, 768, 11, 5, True, False), ("s0 C768 k3", 2496, 768, 768, 3, 1, True, True),
          ("s1 C384 k11", 9984, 384, 384, 11, 5, True, False), ("s1 C384 k3", 9984, 384, 384, 3, 1, True, True),
          ("s2 C192 k11", 19968, 192, 192, 11, 5, True, False), ("s2 C192 k3", 19968, 192, 192, 3, 1, True, True)]


def load(path):
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        per[int(r["Dispatch_Id"])] = float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


d = sys.argv[1]
for plane in (0, 1):
    fp, wp = os.path.join(d, f"FETCH_SIZE_{plane}", "compact.csv"), os.path.join(d, f"WRITE_SIZE_{plane}", "compact.csv")
    if not (os.path.exists(fp) and os.path.exists(wp)):
        continue
    fetch, write = load(fp), load(wp)
    print(f"== {'conv1 form (fp16 plane out)' if plane else 'conv2 form (residual; + accumulate at k3)'}: "
          f"MB per launch")
    print(f"{'shape':13s} {'counted rd':>10s} {'algo rd':>8s} {'window':>7s} {'plane':>6s} {'wts':>5s} "
          f"{'res+acc':>7s} {'excess':>7s} {'win-plane':>9s} | {'counted wr':>10s} {'algo wr':>7s}")
    for i, (name, T, C, N, k, dil, res, acc) in enumerate(SHAPES):
        if plane:
            res = acc = False
        f = fetch[5 * i:5 * i + 5]
        w = write[5 * i:5 * i + 5]
        if len(f) < 5:
            break
        rd = 2 * 1024 * sum(f[1:]) / 4 / 1e6   # launches 2..5 (the first runs cold)
        wr = 1024 * sum(w[1:]) / 4 / 1e6
        M = B * T
        kpad = k * C
        tpb = math.ceil(T / 256)
        tn = N // 192
        plane_b = M * C * 2 / 1e6
        wts = N * kpad * 2 / 1e6
        ra = M * N * 4 * (int(res) + int(acc)) / 1e6
        wr_rows = 256 + (k - 1) * dil
        window = B * tpb * tn * (C // 64) * wr_rows * 128 / 1e6
        algo = plane_b + wts + ra
        algo_w = M * N * (2 if plane else 4) / 1e6
        print(f"{name:13s} {rd:10.1f} {algo:8.1f} {window:7.1f} {plane_b:6.1f} {wts:5.1f} {ra:7.1f} {rd - algo:7.1f} "
              f"{window - plane_b:9.1f} | {wr:10.1f} {algo_w:7.1f}")
