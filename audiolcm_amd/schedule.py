"""Host-side scalar logic of the LCM scheduler (mirrors LCMSampler, scheduling_lcm.py).

Everything here is O(steps) scalar/table work done on the host exactly as the
reference does it (numpy float64 schedule, fp32 casts, torch-CPU fp32
frequency tables); the per-element work (embeddings, the step update, the
denoiser) runs in the HIP kernels.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch


def alphas_cumprod(timesteps: int = 1000, linear_start: float = 0.00085, linear_end: float = 0.012) -> torch.Tensor:
    """DDPM.register_schedule (ddpm.py:116-136) with make_beta_schedule('linear') (util.py:21-24)."""
    betas = np.linspace(linear_start ** 0.5, linear_end ** 0.5, timesteps, dtype=np.float64) ** 2
    return torch.tensor(np.cumprod(1.0 - betas, axis=0), dtype=torch.float32)


def lcm_timesteps(num_inference_steps: Optional[int], original_inference_steps: int = 50,
                  num_train_timesteps: int = 1000, timesteps: Optional[Sequence[int]] = None,
                  strength: float = 1.0) -> List[int]:
    """LCMSampler.set_timesteps (scheduling_lcm.py:119-258), same validation errors."""
    if num_inference_steps is None and timesteps is None:
        raise ValueError("Must pass exactly one of `num_inference_steps` or `custom_timesteps`.")
    if num_inference_steps is not None and timesteps is not None:
        raise ValueError("Can only pass one of `num_inference_steps` or `custom_timesteps`.")
    if original_inference_steps > num_train_timesteps:
        raise ValueError(f"`original_steps`: {original_inference_steps} cannot be larger than "
                         f"`self.config.train_timesteps`: {num_train_timesteps}")
    k = num_train_timesteps // original_inference_steps
    origin = np.asarray(list(range(1, int(original_inference_steps * strength) + 1))) * k - 1
    if timesteps is not None:
        # custom schedule (the reference branch is broken by undefined names; this is its intent)
        ts = list(int(t) for t in timesteps)
        for i in range(1, len(ts)):
            if ts[i] >= ts[i - 1]:
                raise ValueError("`custom_timesteps` must be in descending order.")
        if ts[0] >= num_train_timesteps:
            raise ValueError(f"`timesteps` must start before `self.config.train_timesteps`: {num_train_timesteps}.")
        return ts
    if num_inference_steps > num_train_timesteps:
        raise ValueError(f"`num_inference_steps`: {num_inference_steps} cannot be larger than "
                         f"`self.ddpm_num_timesteps`: {num_train_timesteps}")
    if len(origin) // num_inference_steps < 1:
        raise ValueError(f"The combination of `original_steps x strength`: {original_inference_steps} x {strength} "
                         f"is smaller than `num_inference_steps`: {num_inference_steps}.")
    if num_inference_steps > original_inference_steps:
        raise ValueError(f"`num_inference_steps`: {num_inference_steps} cannot be larger than "
                         f"`original_inference_steps`: {original_inference_steps}")
    origin = origin[::-1].copy()
    idx = np.floor(np.linspace(0, len(origin), num=num_inference_steps, endpoint=False)).astype(np.int64)
    return [int(v) for v in origin[idx]]


def step_coeffs(t: int, prev_t: int, ac: torch.Tensor, timestep_scaling: float = 10.0,
                sigma_data: float = 0.5) -> List[float]:
    """(sqrt_a, sqrt_b, c_out, c_skip, sqrt_a_prev, sqrt_b_prev) of LCMSampler.step, fp32 as the reference."""
    tt = torch.tensor(t, dtype=torch.long)
    a_t = ac[t]
    a_prev = ac[prev_t] if prev_t >= 0 else torch.tensor(1.0)
    scaled = tt * timestep_scaling
    c_skip = sigma_data ** 2 / (scaled ** 2 + sigma_data ** 2)
    c_out = scaled / (scaled ** 2 + sigma_data ** 2) ** 0.5
    vals = [a_t.sqrt(), (1 - a_t).sqrt(), c_out, c_skip, a_prev.sqrt(), (1 - a_prev).sqrt()]
    return [float(torch.as_tensor(v, dtype=torch.float32)) for v in vals]


def _cr_exp(x32: torch.Tensor) -> torch.Tensor:
    """Correctly rounded fp32 exp of an fp32 tensor.  torch's CPU exp is platform dependent in the
    last ulp (AVX2 vs AVX-512 SLEEF paths differ on ~3% of these entries); the correctly rounded value
    makes the tables identical on every host."""
    return torch.from_numpy(np.exp(x32.numpy().astype(np.float64)).astype(np.float32))


def guidance_freqs(embedding_dim: int = 256) -> torch.Tensor:
    """exp(-ln(1e4)/(half-1) * i) (scheduling_lcm.py:103-105): the fp32 exponent exactly as the
    reference computes it, exp correctly rounded."""
    half = embedding_dim // 2
    emb = torch.log(torch.tensor(10000.0)) / (half - 1)
    return _cr_exp(torch.arange(half, dtype=torch.float32) * -emb)


def timestep_freqs(dim: int = 256, max_period: int = 10000) -> torch.Tensor:
    """exp(-ln(max_period) * i / half) (concatDiT.py:60-62): fp32 exponent as the reference, exp
    correctly rounded."""
    half = dim // 2
    return _cr_exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half)


def sample_plan(S: int, original_inference_steps: int = 50, timesteps: Optional[Sequence[int]] = None
                ) -> List[Dict]:
    """Per-step (t, prev_t, coeffs, add_noise) for LCMSampler.lcm_sampling (scheduling_lcm.py:344-382)."""
    ts = lcm_timesteps(None if timesteps is not None else S, original_inference_steps, timesteps=timesteps)
    ac = alphas_cumprod()
    plan = []
    for i, t in enumerate(ts):
        prev_t = ts[i + 1] if i + 1 < len(ts) else t
        plan.append(dict(t=t, prev_t=prev_t, coeffs=step_coeffs(t, prev_t, ac), add_noise=i != len(ts) - 1))
    return plan
