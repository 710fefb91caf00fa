"""Host-side mirrors of the reference hot-path modules, backed by libaudiolcm_hip.

Each class keeps the reference constructor signature and forward contract and
owns an ``alcm_model*`` (packed device weights) created from a reference-named
``state_dict``.  All compute runs in the HIP library on the caller's current
stream; these classes only allocate outputs/workspaces with torch.

  ConcatDiT2MLP   ldm/modules/diffusionmodules/concatDiT.py:238-304
  AutoencoderKL   ldm/models/autoencoder1d.py:18-62 (decode path)
  BigVGAN         vocoder/bigvgan/models.py:133-203
  VocoderBigVGAN  vocoder/bigvgan/models.py:393-414
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Iterable, List, Mapping, Optional, Sequence

import numpy as np
import torch

from . import _hip, recipe, schedule
from ._hip import check, lib, ptr, stream_handle


def _state_to_named(state: Mapping[str, torch.Tensor], extra: Optional[Mapping[str, torch.Tensor]] = None):
    keep = []
    items = list(state.items()) + list((extra or {}).items())
    arr = (_hip.NamedTensor * len(items))()
    for i, (k, v) in enumerate(items):
        t = v.detach().to("cpu", torch.float32).contiguous()
        if t.dim() > 4:
            raise ValueError(f"{k}: tensors above 4-D are not on the path")
        kb = k.encode()
        keep.append((t, kb))
        arr[i].name = kb
        arr[i].data = t.data_ptr()
        arr[i].ndim = t.dim()
        for d in range(t.dim()):
            arr[i].shape[d] = t.shape[d]
    return arr, keep


def policy_code(split) -> int:
    """Precision policy from a bool (split / bf16) or a name in _hip.POLICIES."""
    if isinstance(split, str):
        if split not in _hip.POLICIES:
            raise ValueError(f"unknown precision policy {split!r}; expected one of {sorted(_hip.POLICIES)}")
        return _hip.POLICIES[split]
    return _hip.POLICY_SPLIT if split else _hip.POLICY_BF16


class _HipModel:
    KIND = -1

    def __init__(self, split=True):
        self._handle = C.c_void_p(None)
        self.policy = policy_code(split)
        self._ws: Dict[tuple, torch.Tensor] = {}

    @property
    def split(self) -> bool:
        return self.policy != _hip.POLICY_BF16

    # -- weights -----------------------------------------------------------------------------
    def _iconfig(self) -> List[int]:
        raise NotImplementedError

    def _extra_tensors(self) -> Dict[str, torch.Tensor]:
        return {}

    def load_state_dict(self, state: Mapping[str, torch.Tensor], strict: bool = False):
        """Pack reference-named weights into device memory (replaces nn.Module.load_state_dict)."""
        _hip.require_device(torch.cuda.current_device())
        self.release()
        arr, keep = _state_to_named(state, self._extra_tensors())
        ic = self._iconfig()
        icarr = (C.c_int * len(ic))(*ic)
        h = C.c_void_p(None)
        check(lib().alcm_model_create(self.KIND, icarr, len(ic), arr, len(arr), self.policy, C.byref(h)),
              f"{type(self).__name__}.load_state_dict")
        del keep
        self._handle = h
        return self

    def set_split(self, split):
        """True/False (bf16x3 everywhere / bf16 everywhere) or a policy name "bf16" | "split" | "mixed"."""
        self.policy = policy_code(split)
        if self._handle:
            check(lib().alcm_model_set_precision(self._handle, self.policy))

    set_precision = set_split

    def set_resblock_streams(self, concurrent: bool):
        """BigVGAN: resblock chains on auxiliary streams (True) or serially on the caller's stream (False)."""
        self._need()
        check(lib().alcm_model_set_resblock_streams(self._handle, int(bool(concurrent))))

    @property
    def loaded(self) -> bool:
        return bool(self._handle)

    def weight_bytes(self) -> int:
        return int(lib().alcm_model_weight_bytes(self._handle)) if self._handle else 0

    def _need(self):
        if not self._handle:
            raise RuntimeError(f"{type(self).__name__}: weights not loaded (call load_state_dict)")

    def _workspace(self, key: tuple, nbytes: int, device) -> torch.Tensor:
        """Caller-side workspace, one per (call kind, shape, stream): calls issued concurrently on different
        streams never share one (the C-ABI concurrency contract, include/audiolcm_hip.h)."""
        key = key + (stream_handle(),)
        ws = self._ws.get(key)
        if ws is None or ws.numel() < nbytes:
            for k in [k for k in self._ws if k[-1] == key[-1]]:
                del self._ws[k]
            ws = torch.empty(int(nbytes), dtype=torch.uint8, device=device)
            self._ws[key] = ws
        return ws

    def release(self):
        if getattr(self, "_handle", None):
            try:
                lib().alcm_model_destroy(self._handle)
            except Exception:
                pass
            self._handle = C.c_void_p(None)
        self._ws = {}

    def __del__(self):
        self.release()

    def eval(self):
        return self

    def to(self, *a, **k):
        return self

    def cuda(self, *a, **k):
        return self


class ConcatDiT2MLP(_HipModel):
    """DiT denoiser (concatDiT.py:238-304) on the MI355X path."""
    KIND = _hip.ALCM_MODEL_DIT

    def __init__(self, in_channels=20, context_dim=1024, hidden_size=576, depth=4, num_heads=8, max_len=1000,
                 split: bool = True, **unused):
        super().__init__(split)
        self.cfg = recipe.DiTConfig(in_channels=in_channels, context_dim=context_dim, hidden_size=hidden_size,
                                    num_heads=num_heads, depth=depth, max_len=max_len)
        self.in_channels = self.out_channels = in_channels

    def _iconfig(self):
        c = self.cfg
        return [c.in_channels, c.context_dim, c.hidden_size, c.num_heads, c.depth, c.max_len, c.ctx_tokens,
                c.ff_kernel, c.proj_in_kernel]

    def _extra_tensors(self):
        return {"_alcm.t_freqs": schedule.timestep_freqs(256)}

    def workspace_bytes(self, B: int, T: int) -> int:
        self._need()
        return int(lib().alcm_dit_workspace_bytes(self._handle, B, T))

    def embed_context(self, context: torch.Tensor) -> torch.Tensor:
        """Step-invariant part: both ConditionEmbedders + LayerNorm + pos rows 1..154 (hoisted out of the loop)."""
        self._need()
        B, L, D = context.shape
        assert L == self.cfg.ctx_tokens and D == self.cfg.context_dim, context.shape
        context = context.contiguous().float()
        cemb = torch.empty((B, L, self.cfg.hidden_size), device=context.device, dtype=torch.float32)
        nb = self.workspace_bytes(B, 1)
        ws = self._workspace(("ctx", B), nb, context.device)
        check(lib().alcm_dit_embed_context(self._handle, ptr(context), B, ptr(cemb), ptr(ws), ws.numel(),
                                           stream_handle()), "alcm_dit_embed_context")
        return cemb

    def forward_cached(self, x: torch.Tensor, t: torch.Tensor, cemb: torch.Tensor,
                       w_cond: Optional[torch.Tensor]) -> torch.Tensor:
        self._need()
        B, Cc, T = x.shape
        assert Cc == self.cfg.in_channels
        if 1 + self.cfg.ctx_tokens + T > self.cfg.max_len:
            raise ValueError(f"latent length {T} exceeds PositionEmbedding max_len {self.cfg.max_len} "
                             f"(concatDiT.py:261: at most {self.cfg.max_latent_len} frames)")
        x = x.contiguous().float()
        t = t.to(device=x.device, dtype=torch.int64).contiguous()
        if w_cond is not None:
            w_cond = w_cond.contiguous().float()
        eps = torch.empty_like(x)
        nb = self.workspace_bytes(B, T)
        ws = self._workspace(("fwd", B, T), nb, x.device)
        check(lib().alcm_dit_forward(self._handle, ptr(x), ptr(t), ptr(cemb), ptr(w_cond), ptr(eps), B, T, ptr(ws),
                                     ws.numel(), stream_handle()), "alcm_dit_forward")
        return eps

    def forward(self, x, t, context, w_cond=None):
        return self.forward_cached(x, t, self.embed_context(context), w_cond)

    __call__ = forward

    @classmethod
    def from_recipe(cls, seed: int = 0, split: bool = True) -> "ConcatDiT2MLP":
        return cls(split=split).load_state_dict(recipe.dit_state(seed))


class AutoencoderKL(_HipModel):
    """1-D KL autoencoder, decode path (autoencoder1d.py:18-62, Decoder1D 415-517)."""
    KIND = _hip.ALCM_MODEL_VAE

    def __init__(self, embed_dim=20, ddconfig=None, lossconfig=None, ckpt_path=None, ignore_keys=(),
                 image_key="image", monitor=None, split: bool = True, **unused):
        super().__init__(split)
        dd = dict(ddconfig or {})
        self.cfg = recipe.VAEConfig(embed_dim=embed_dim, z_channels=dd.get("z_channels", 20),
                                    out_ch=dd.get("out_ch", 80), kernel_size=dd.get("kernel_size", 5),
                                    ch=dd.get("ch", 384), ch_mult=tuple(dd.get("ch_mult", (1, 2, 4))),
                                    num_res_blocks=dd.get("num_res_blocks", 2),
                                    attn_layers=tuple(dd.get("attn_layers", (3,))),
                                    down_layers=tuple(dd.get("down_layers", (0,))))
        if any(l in range(len(self.cfg.ch_mult)) for l in self.cfg.attn_layers):
            raise NotImplementedError("attention inside decoder up-levels is not on the configured path")
        if ckpt_path is not None and os.path.exists(str(ckpt_path)):
            self.init_from_ckpt(ckpt_path, ignore_keys)

    def _iconfig(self):
        c = self.cfg
        return ([c.z_channels, c.embed_dim, c.out_ch, c.kernel_size, c.ch, c.num_res_blocks, len(c.ch_mult)]
                + list(c.ch_mult) + [len(c.upsample_levels)] + list(c.upsample_levels))

    def init_from_ckpt(self, path, ignore_keys=()):
        """AutoencoderKL.init_from_ckpt (autoencoder1d.py:42-52), safe loader only."""
        from .ckpt import load_checkpoint, state_dict_of
        sd = state_dict_of(load_checkpoint(path))
        sd = {k: v for k, v in sd.items() if not any(k.startswith(ik) for ik in ignore_keys)}
        return self.load_state_dict(sd)

    def load_state_dict(self, state, strict=False):
        keep = {k: v for k, v in state.items() if k.startswith("decoder.") or k.startswith("post_quant_conv.")
                or k.startswith("encoder.") or k.startswith("quant_conv.")}
        return super().load_state_dict(keep, strict)

    def encode(self, x: torch.Tensor) -> "DiagonalGaussianDistribution":
        """AutoencoderKL.encode (autoencoder1d.py:54-58): Encoder1D + quant_conv on (B, 80, M) -> posterior over
        (B, embed_dim, M / 2) latents (needs a checkpoint / recipe with the encoder.* weights)."""
        self._need()
        B, Cm, M = x.shape
        x = x.contiguous().float()
        To = int(lib().alcm_vae_encode_len(self._handle, M))
        moments = torch.empty((B, 2 * self.cfg.embed_dim, To), device=x.device, dtype=torch.float32)
        nb = int(lib().alcm_vae_encode_workspace_bytes(self._handle, B, M))
        ws = self._workspace(("enc", B, M), nb, x.device)
        check(lib().alcm_vae_encode(self._handle, ptr(x), ptr(moments), B, M, ptr(ws), ws.numel(), stream_handle()),
              "alcm_vae_encode")
        return DiagonalGaussianDistribution(moments)

    def forward(self, input: torch.Tensor, sample_posterior: bool = True, generator=None):
        """autoencoder1d.py:64-70: (reconstruction, posterior)."""
        posterior = self.encode(input)
        z = posterior.sample(generator) if sample_posterior else posterior.mode()
        return self.decode(z), posterior

    __call__ = forward

    def decode(self, z: torch.Tensor, scale_factor: float = 1.0) -> torch.Tensor:
        """post_quant_conv + Decoder1D on (B, 20, T) -> mel (B, 80, 2T); z is divided by scale_factor first."""
        self._need()
        B, Cc, T = z.shape
        z = z.contiguous().float()
        mel = torch.empty((B, self.cfg.out_ch, T * self.cfg.time_upsample), device=z.device, dtype=torch.float32)
        nb = int(lib().alcm_vae_workspace_bytes(self._handle, B, T))
        ws = self._workspace(("dec", B, T), nb, z.device)
        check(lib().alcm_vae_decode(self._handle, ptr(z), 1.0 / float(scale_factor), ptr(mel), B, T, ptr(ws),
                                    ws.numel(), stream_handle()), "alcm_vae_decode")
        return mel

    @classmethod
    def from_recipe(cls, seed: int = 0, split: bool = True) -> "AutoencoderKL":
        return cls(split=split).load_state_dict(recipe.vae_state(seed))


class DiagonalGaussianDistribution:
    """ldm/modules/distributions/distributions.py:24-44 over the encoder's (B, 2C, T) moments (device tensors):
    mean | logvar split, logvar clamped to [-30, 20]; sample() draws the noise from `generator` (a torch
    Generator on the device) or the global device RNG."""

    def __init__(self, parameters: torch.Tensor, deterministic: bool = False):
        self.parameters = parameters
        self.mean, self.logvar = torch.chunk(parameters, 2, dim=1)
        self.logvar = torch.clamp(self.logvar, -30.0, 20.0)
        self.deterministic = deterministic
        self.std = torch.exp(0.5 * self.logvar)
        self.var = torch.exp(self.logvar)
        if deterministic:
            self.var = self.std = torch.zeros_like(self.mean)

    def sample(self, generator=None) -> torch.Tensor:
        eps = torch.randn(self.mean.shape, generator=generator, device=self.parameters.device)
        return self.mean + self.std * eps

    def mode(self) -> torch.Tensor:
        return self.mean


class BigVGAN(_HipModel):
    """BigVGAN generator (vocoder/bigvgan/models.py:133-203), weight norm folded at load."""
    KIND = _hip.ALCM_MODEL_BIGVGAN

    def __init__(self, h=None, split: bool = True):
        super().__init__(split)
        c = recipe.BigVGANConfig()
        if h is not None:
            g = (lambda k, d: (h[k] if isinstance(h, Mapping) and k in h else getattr(h, k, d)))
            if str(g("resblock", "1")) != "1":
                raise NotImplementedError("only AMPBlock1 (resblock '1') is on the configured path")
            if g("activation", "snakebeta") != "snakebeta" or not g("snake_logscale", True):
                raise NotImplementedError("only logscale SnakeBeta is on the configured path")
            dil = [tuple(d) for d in g("resblock_dilation_sizes", c.resblock_dilation_sizes)]
            if any(d != dil[0] for d in dil):
                raise NotImplementedError("per-kernel dilation sets must match")
            c = recipe.BigVGANConfig(num_mels=g("num_mels", c.num_mels),
                                     upsample_rates=tuple(g("upsample_rates", c.upsample_rates)),
                                     upsample_kernel_sizes=tuple(g("upsample_kernel_sizes", c.upsample_kernel_sizes)),
                                     upsample_initial_channel=g("upsample_initial_channel",
                                                                c.upsample_initial_channel),
                                     resblock_kernel_sizes=tuple(g("resblock_kernel_sizes", c.resblock_kernel_sizes)),
                                     resblock_dilation_sizes=tuple(dil),
                                     sampling_rate=g("sampling_rate", c.sampling_rate))
        self.cfg = c

    def _iconfig(self):
        c = self.cfg
        return ([c.num_mels, c.upsample_initial_channel, len(c.upsample_rates)] + list(c.upsample_rates)
                + list(c.upsample_kernel_sizes) + [len(c.resblock_kernel_sizes)] + list(c.resblock_kernel_sizes)
                + [len(c.resblock_dilation_sizes[0])] + list(c.resblock_dilation_sizes[0]))

    def forward(self, mel: torch.Tensor) -> torch.Tensor:
        self._need()
        B, Cm, M = mel.shape
        assert Cm == self.cfg.num_mels
        mel = mel.contiguous().float()
        wav = torch.empty((B, 1, M * self.cfg.hop), device=mel.device, dtype=torch.float32)
        nb = int(lib().alcm_bigvgan_workspace_bytes(self._handle, B, M))
        ws = self._workspace(("voc", B, M), nb, mel.device)
        check(lib().alcm_bigvgan_forward(self._handle, ptr(mel), ptr(wav), B, M, ptr(ws), ws.numel(),
                                         stream_handle()), "alcm_bigvgan_forward")
        return wav

    __call__ = forward

    def remove_weight_norm(self):
        """No-op: weight norm is folded when the weights are packed (models.py:205-213)."""

    @classmethod
    def from_recipe(cls, seed: int = 0, split: bool = True) -> "BigVGAN":
        return cls(split=split).load_state_dict(recipe.bigvgan_state(seed))


class VocoderBigVGAN:
    """VocoderBigVGAN (models.py:393-414): loads best_netG.pt['generator'] + args.yml, vocodes mels."""

    def __init__(self, ckpt_vocoder=None, device="cuda", split: bool = True, state=None, h=None):
        import yaml
        if state is None:
            from .ckpt import load_checkpoint, state_dict_of
            state = state_dict_of(load_checkpoint(os.path.join(ckpt_vocoder, "best_netG.pt")), "generator")
            with open(os.path.join(ckpt_vocoder, "args.yml")) as f:
                h = yaml.safe_load(f)
        self.generator = BigVGAN(h, split=split).load_state_dict(state)
        self.device = device

    def vocode(self, spec):
        """(80, M) numpy/tensor or (B, 80, M) tensor -> waveform (numpy for numpy input, as the reference)."""
        as_np = isinstance(spec, np.ndarray)
        t = torch.from_numpy(spec).unsqueeze(0) if as_np else spec
        if t.dim() == 2:
            t = t.unsqueeze(0)
        wav = self.generator(t.to(device="cuda", dtype=torch.float32))
        return wav.squeeze().cpu().numpy() if as_np else wav

    __call__ = vocode
