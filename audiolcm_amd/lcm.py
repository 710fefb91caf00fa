"""LCM_audio / LCMSampler mirrors: the sampler hot loop driving the HIP DiT + step kernels.

  LCM_audio    ldm/models/diffusion/lcm_audio.py:46-116 (inference members), apply_model :479-502,
               decode_first_stage :392-406, schedule buffers ddpm.py:116-168
  LCMSampler   ldm/models/diffusion/scheduling_lcm.py:13-496

Differences from the reference that are deliberate and documented in DESIGN.md:
  * RNG: x_T and the per-step noise are drawn per prompt from ``torch.Generator(seed)``
    (SURVEY.md §7 "RNG parity") when ``seeds`` are given, so results do not depend on
    how prompts are sharded over GPUs; without seeds the global device RNG is used as
    in the reference (scheduling_lcm.py:354,485).
  * the condition embedders are step-invariant and run once per ``sample`` call.
  * optional classifier-free guidance (BASELINE config 4): batch-doubled [uc; c] DiT call
    and the combine e_u + s(e_c - e_u) fused into the LCM step kernel.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import torch

from . import _hip, recipe, schedule
from ._hip import check, lib, ptr, stream_handle
from .config import instantiate_from_config
from .models import AutoencoderKL, ConcatDiT2MLP


class DiffusionWrapper:
    """ddpm.py:1397-1437 (crossattn branch): holds ``diffusion_model``."""

    def __init__(self, diffusion_model, conditioning_key="crossattn"):
        self.diffusion_model = diffusion_model
        self.conditioning_key = conditioning_key

    def __call__(self, x, t, c_crossattn=None, w_cond=None, **kw):
        cc = torch.cat(c_crossattn, 1) if isinstance(c_crossattn, (list, tuple)) else c_crossattn
        return self.diffusion_model(x, t, context=cc, w_cond=w_cond)


class LCM_audio:
    """Inference surface of LCM_audio (lcm_audio.py) built from configs/audiolcm.yaml params."""

    def __init__(self, unet_config=None, first_stage_config=None, cond_stage_config=None, timesteps=1000,
                 linear_start=0.00085, linear_end=0.012, mel_dim=20, mel_length=312, conditioning_key="crossattn",
                 scale_factor=1.0, num_ddim_timesteps=50, split: bool = True, **unused):
        self.num_timesteps = int(timesteps)
        self.mel_dim, self.mel_length = mel_dim, mel_length
        self.channels = int(unused.get("channels", 0))
        self.alphas_cumprod = schedule.alphas_cumprod(timesteps, linear_start, linear_end)
        self.scale_factor = float(scale_factor)
        self.num_ddim_timesteps = num_ddim_timesteps
        self.split = split
        dit = instantiate_from_config(unet_config, split=split) if unet_config else ConcatDiT2MLP(split=split)
        self.unet = DiffusionWrapper(dit, conditioning_key)
        self.model = self.unet  # `model`, `unet`, `target_unet` share weights at inference (lcm_audio.py:98-114)
        self.first_stage_model = (instantiate_from_config(first_stage_config, split=split) if first_stage_config
                                  else AutoencoderKL(split=split))
        self.cond_stage_model = (instantiate_from_config(cond_stage_config, split=split) if cond_stage_config
                                 else None)

    # -- weights ---------------------------------------------------------------------------------
    def load_state_dict(self, sd, strict=False):
        """Lightning ``state_dict`` (Appendix A): ``unet.diffusion_model.*`` (the sampler's net; falls back
        to ``model.diffusion_model.*``), ``first_stage_model.*``, ``scale_factor``."""
        def sub(prefix):
            return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}
        dit = sub("unet.diffusion_model.") or sub("model.diffusion_model.")
        if dit:
            self.unet.diffusion_model.load_state_dict(dit)
        fs = sub("first_stage_model.")
        if fs:
            self.first_stage_model.load_state_dict(fs)
        cs = sub("cond_stage_model.")
        if cs and self.cond_stage_model is not None and hasattr(self.cond_stage_model, "load_state_dict"):
            self.cond_stage_model.load_state_dict(cs)
        if "scale_factor" in sd:
            self.scale_factor = float(sd["scale_factor"])
        return self

    def load_recipe(self, seed: int = 0):
        self.unet.diffusion_model.load_state_dict(recipe.dit_state(seed))
        self.first_stage_model.load_state_dict(recipe.vae_state(seed))
        if self.cond_stage_model is not None and hasattr(self.cond_stage_model, "load_state_dict"):
            self.cond_stage_model.load_state_dict(recipe.text_state(seed))
            if hasattr(self.cond_stage_model, "use_synthetic_tokenizer"):  # recipe weights: hash ids are as good
                self.cond_stage_model.use_synthetic_tokenizer()
        return self

    @property
    def betas(self):
        return None

    # -- reference methods -----------------------------------------------------------------------
    def get_learned_conditioning(self, c):
        if self.cond_stage_model is None:
            raise RuntimeError("no cond_stage_model configured")
        return self.cond_stage_model.encode(c) if hasattr(self.cond_stage_model, "encode") else self.cond_stage_model(c)

    def apply_model(self, x_noisy, t, cond, model=None, w_cond=None, return_ids=False):
        model = model or self.unet
        if not isinstance(cond, (list, tuple)):
            cond = [cond]
        return model(x_noisy, t, c_crossattn=cond, w_cond=w_cond)

    def decode_first_stage(self, z):
        return self.first_stage_model.decode(z, self.scale_factor)

    def encode_first_stage(self, x):
        """lcm_audio.py:425-427: mel (B, 80, M) -> DiagonalGaussianDistribution over the latent."""
        return self.first_stage_model.encode(x)

    def get_first_stage_encoding(self, encoder_posterior, generator=None):
        """lcm_audio.py:197-204: scale_factor * posterior.sample() (a tensor passes through)."""
        from .models import DiagonalGaussianDistribution
        if isinstance(encoder_posterior, DiagonalGaussianDistribution):
            z = encoder_posterior.sample(generator)
        elif isinstance(encoder_posterior, torch.Tensor):
            z = encoder_posterior
        else:
            raise NotImplementedError(f"encoder_posterior of type '{type(encoder_posterior)}' not yet implemented")
        return self.scale_factor * z

    def eval(self):
        return self

    def cuda(self):
        return self

    def to(self, *a, **k):
        return self

    class _Null:
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

    def ema_scope(self, context=None):
        return LCM_audio._Null()


def _h2d(t: torch.Tensor, dev) -> torch.Tensor:
    """Host tensor -> device through the pinned caching allocator, asynchronously on the current stream (the pinned
    block stays reserved until the copy has run)."""
    return t.pin_memory().to(dev, non_blocking=True)


class LCMSampler:
    """LCM multistep sampler (scheduling_lcm.py) over the HIP DiT and the fused step kernel."""

    def __init__(self, model: LCM_audio, **kwargs):
        self.model = model
        self.ddpm_num_timesteps = model.num_timesteps
        self.original_inference_steps = 100
        self.num_inference_steps = None
        self.timesteps = torch.arange(self.ddpm_num_timesteps - 1, -1, -1, dtype=torch.long)
        self.timestep_scaling = 10.0
        self.prediction_type = "epsilon"
        self._gfreqs = {}

    def make_schedule(self, ddim_discretize="uniform", verbose=True):
        self.alphas_cumprod = self.model.alphas_cumprod

    def set_timesteps(self, num_inference_steps=None, device=None, original_inference_steps=None, timesteps=None,
                      strength=1.0):
        ts = schedule.lcm_timesteps(num_inference_steps, original_inference_steps or self.original_inference_steps,
                                    self.ddpm_num_timesteps, timesteps, strength)
        self.num_inference_steps = len(ts)
        self.timesteps = torch.tensor(ts, dtype=torch.long)
        self._step_index = None

    def retrieve_timesteps(self, num_inference_steps=None, device=None, timesteps=None, **kwargs):
        if timesteps is not None:
            self.set_timesteps(timesteps=timesteps, device=device, **kwargs)
        else:
            self.set_timesteps(num_inference_steps, device=device, **kwargs)
        return self.timesteps, len(self.timesteps)

    def get_guidance_scale_embedding(self, w: torch.Tensor, embedding_dim: int = 512, dtype=torch.float32):
        """[sin | cos](1000 w f_i) on the device (scheduling_lcm.py:87-113)."""
        assert w.dim() == 1
        dev = torch.device("cuda")
        if embedding_dim not in self._gfreqs:
            self._gfreqs[embedding_dim] = schedule.guidance_freqs(embedding_dim).to(dev)
        f = self._gfreqs[embedding_dim]
        out = torch.empty((w.shape[0], 2 * f.numel()), device=dev, dtype=torch.float32)
        wv = w.to(device=dev, dtype=torch.float32).contiguous()
        check(lib().alcm_sincos_embedding(ptr(wv), 1000.0, ptr(f), w.shape[0], f.numel(), 0, ptr(out),
                                          stream_handle()), "guidance embedding")
        if embedding_dim % 2:
            out = torch.nn.functional.pad(out, (0, 1))
        return out

    @torch.no_grad()
    def sample(self, S, batch_size, shape, conditioning=None, callback=None, normals_sequence=None,
               img_callback=None, verbose=True, x_T=None, guidance_scale=5., original_inference_steps=50,
               timesteps=None, seeds: Optional[Sequence[int]] = None, noise: Optional[torch.Tensor] = None,
               unconditional_conditioning: Optional[torch.Tensor] = None, unconditional_guidance_scale: float = 1.0,
               **kwargs) -> Tuple[torch.Tensor, torch.Tensor]:
        """Returns (denoised, last sample) like the reference (scheduling_lcm.py:298-342)."""
        self.make_schedule(verbose=verbose)
        if len(shape) != 2:
            raise ValueError("audio latents are (C, T)")
        Cc, T = shape
        dev = torch.device("cuda")
        cond = conditioning
        if isinstance(cond, dict):
            cond = cond[list(cond.keys())[0]]
            while isinstance(cond, list):
                cond = cond[0]
        if cond.shape[0] != batch_size:
            print(f"Warning: Got {cond.shape[0]} conditionings but batch-size is {batch_size}")
        plan = schedule.sample_plan(S, original_inference_steps, timesteps)
        self.num_inference_steps = len(plan)
        self.timesteps = torch.tensor([p["t"] for p in plan], dtype=torch.long)
        n_noise = sum(1 for p in plan if p["add_noise"])
        if seeds is not None:
            # host draws (per-prompt generators), copied from pinned memory without blocking the host: a pageable
            # copy waits for everything already queued on the stream, so each call used to start only after the
            # previous call's vocoder had drained, with the GPU idle meanwhile (2.4 ms per bench step, rocprofv3
            # kernel trace of profiles/r4v6)
            xT_h, noise_h = recipe.prompt_noise(seeds, len(plan), Cc, T)
            img = _h2d(xT_h, dev) if x_T is None else x_T.to(dev)
            noise = _h2d(noise_h, dev) if noise is None else noise
        else:
            img = x_T.to(dev).float() if x_T is not None else torch.randn((batch_size, Cc, T), device=dev)
        if noise is None:
            noise = torch.randn((n_noise, batch_size, Cc, T), device=dev) if n_noise else None
        noise = noise.to(dev).float().contiguous() if noise is not None else None
        dit: ConcatDiT2MLP = self.model.unet.diffusion_model
        cfg = unconditional_conditioning is not None and unconditional_guidance_scale != 1.0
        c = cond.to(dev).float()
        if cfg:
            c = torch.cat([unconditional_conditioning.to(dev).float(), c], 0)
        cemb = dit.embed_context(c)
        B2 = c.shape[0]
        w = torch.full((B2,), float(guidance_scale - 1), device=dev, dtype=torch.float32)  # (no host copy)
        w_emb = self.get_guidance_scale_embedding(w, embedding_dim=256)
        img = img.contiguous().float().clone()  # never write into the caller's x_T
        n = img.numel()
        prev = torch.empty_like(img)
        denoised = torch.empty_like(img)
        for i, p in enumerate(plan):
            ts = torch.full((B2,), p["t"], device=dev, dtype=torch.long)
            xin = torch.cat([img, img], 0) if cfg else img
            eps = dit.forward_cached(xin, ts, cemb, w_emb)
            coeffs = (C.c_float * 6)(*p["coeffs"])
            nz = ptr(noise[i]) if p["add_noise"] else None
            if cfg:
                eu, ec = eps[:batch_size], eps[batch_size:]
                check(lib().alcm_lcm_step_cfg(ptr(img), ptr(ec), ptr(eu), float(unconditional_guidance_scale), nz,
                                              coeffs, ptr(prev), ptr(denoised), n, stream_handle()), "lcm_step_cfg")
            else:
                check(lib().alcm_lcm_step(ptr(img), ptr(eps), nz, coeffs, ptr(prev), ptr(denoised), n,
                                          stream_handle()), "lcm_step")
            img, prev = prev, img
        return denoised, img
