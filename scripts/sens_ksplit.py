#!/usr/bin/env python3
"""Sensitivity of the B = 32 mixed-policy pipeline (bench workload) to a summation-order change (dev tool): the DiT FFN
down-projection with and without the K split (ALCM_KSPLIT), and, as a control, the conditioning perturbed by 1e-7
relative with the split off.  Prints per-stage rel-L2 between the runs and each run's clip errors vs the reference
fixtures (tests/golden: e2e_S2_B2 clips 0, 1 and the single-prompt runs 7, 15, 23, 31)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiolcm_amd import _hip, recipe  # noqa: E402
from audiolcm_amd.pipeline import AudioLCMPipeline  # noqa: E402

G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


pipe = AudioLCMPipeline.from_recipe(0, split="mixed")
ids = list(range(32))
cond = torch.cat([recipe.synthetic_context(1, seed0=1000 + i) for i in ids], 0).cuda()
runs = {}
for name, ks, eps in (("ksplit0", "0", 0.0), ("ksplit1", "1", 0.0), ("ctx+1e-7", "0", 1e-7)):
    os.environ["ALCM_KSPLIT"] = ks
    _hip.reload_knobs()
    c = cond * (1.0 + eps) if eps else cond
    out = pipe.generate(c, seeds=ids, steps=2)
    runs[name] = {k: out[k].float().cpu().numpy() for k in ("latent", "mel", "wav")}
    g2 = dict(np.load(os.path.join(G, "e2e_S2_B2.npz")))
    errs = []
    for i, g, j in [(0, g2, 0), (1, g2, 1)] + [(p, dict(np.load(os.path.join(G, f"e2e_S2_prompt{p}.npz"))), 0)
                                              for p in (7, 15, 23, 31)]:
        errs.append(f"clip {i}: lat {rel(runs[name]['latent'][i], g['latent'][j]):.2e} "
                    f"mel {rel(runs[name]['mel'][i], g['mel'][j]):.2e} wav {rel(runs[name]['wav'][i], g['wav'][j].reshape(-1)):.2e}")
    print(f"{name}: " + " | ".join(errs), flush=True)
for a, b in (("ksplit1", "ksplit0"), ("ctx+1e-7", "ksplit0")):
    print(f"{a} vs {b}: " + " ".join(f"{k} {rel(runs[a][k], runs[b][k]):.2e}" for k in ("latent", "mel", "wav")),
          flush=True)
