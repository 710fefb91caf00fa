#!/usr/bin/env python3
"""Diagnostics (dev tool): where the mixed-policy text encode at B = 32 goes non-finite, under kernel-choice knobs."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiolcm_amd import _hip  # noqa: E402
from audiolcm_amd.text_encoder import CLAPT5TextEncoder  # noqa: E402

g = dict(np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "text_B2_L77.npz")))
enc = CLAPT5TextEncoder.from_recipe(0, split="mixed")
for B in (2, 4, 8, 16, 32):
    sel = torch.arange(B) % 2
    a, b = torch.from_numpy(g["clap_ids"])[sel], torch.from_numpy(g["t5_ids"])[sel]
    for knob in ("", "ALCM_WCONV=0", "ALCM_TEXT_GEMM=1"):
        for k in ("ALCM_WCONV", "ALCM_TEXT_GEMM"):
            os.environ.pop(k, None)
        if knob:
            k, v = knob.split("=")
            os.environ[k] = v
        _hip.reload_knobs()
        out = enc.encode_ids(a, b).cpu().numpy()
        bad = ~np.isfinite(out)
        ref = g["out"][sel.numpy()]
        fin = np.where(bad, 0, out)
        err = float(np.linalg.norm(fin - ref) / np.linalg.norm(ref))
        msg = f"B={B:2d} {knob or 'default':22s} nonfinite={int(bad.sum()):8d} relL2(finite)={err:.2e}"
        if bad.any():
            bi, ti, ci = np.nonzero(bad)
            msg += (f" batches {sorted(set(bi.tolist()))[:8]} tokens [{ti.min()},{ti.max()}] (clap half "
                    f"{int((ti < 77).sum())}, t5 half {int((ti >= 77).sum())}) channels [{ci.min()},{ci.max()}]")
        print(msg, flush=True)
