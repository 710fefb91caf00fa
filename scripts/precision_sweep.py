#!/usr/bin/env python3
"""Waveform parity vs the reference golden vectors for every split/bf16 assignment of the three models.

Prints rel-L2 of latent / mel / waveform for the e2e S=2 B=2 fixture (tests/golden/e2e_S2_B2.npz),
which is what decides the per-model precision policy."""
import itertools
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from audiolcm_amd import _hip, recipe  # noqa: E402
from audiolcm_amd.pipeline import AudioLCMPipeline  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def main():
    _hip.require_device(0)
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "e2e_S2_B2.npz")))
    pipe = AudioLCMPipeline.from_recipe(0)
    ctx = recipe.synthetic_context(2).cuda()
    for dit, vae, voc in itertools.product(("split", "mixed", "bf16"), repeat=3):
        pipe.model.unet.diffusion_model.set_split(dit)
        pipe.model.first_stage_model.set_split(vae)
        pipe.vocoder.set_split(voc)
        out = pipe.generate(ctx, seeds=[0, 1], steps=2)
        print(f"dit={dit:5s} vae={vae:5s} voc={voc:5s}"
              f"  latent {rel(out['latent'].cpu(), g['latent']):.2e}  mel {rel(out['mel'].cpu(), g['mel']):.2e}"
              f"  wav {rel(out['wav'].cpu(), g['wav']):.2e}", flush=True)


if __name__ == "__main__":
    main()
