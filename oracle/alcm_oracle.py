"""CPU restatement of the AudioLCM inference hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity *checker*.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it; the product package
``audiolcm_amd`` never does, and it never runs as part of the measured GPU path.

It restates, in plain fp32 PyTorch-CPU ops, the reference algorithm of each
hot-path function.  Every function cites the
reference file:line it follows.  It is *pinned* against golden vectors that
``tests/golden/make_golden.py`` produced by importing the reference itself in
the build container (``tests/test_oracle_golden.py``): parity is pinned for
every function below except ``pcm16_bytes`` (soundfile/libsndfile is not
installed here, so the PCM16 quantiser is restated from libsndfile's
documented float->short rule and is "parity unpinned").

Weights are dicts keyed by the reference ``state_dict()`` names.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor
W_t = Dict[str, Tensor]


# ---------------------------------------------------------------------------
# diffusion schedule + LCM scheduler  (ddpm.py:116-168, scheduling_lcm.py)
# ---------------------------------------------------------------------------
def alphas_cumprod(timesteps: int = 1000, linear_start: float = 0.00085, linear_end: float = 0.012) -> Tensor:
    """``make_beta_schedule('linear')`` + cumprod in float64, cast to fp32.

    diffusionmodules/util.py:21-24 (linspace of sqrt, squared, float64);
    ddpm.py:121-136 (alphas = 1-betas, cumprod in numpy float64, to_torch fp32)."""
    betas = np.linspace(linear_start ** 0.5, linear_end ** 0.5, timesteps, dtype=np.float64) ** 2
    ac = np.cumprod(1.0 - betas, axis=0)
    return torch.tensor(ac, dtype=torch.float32)


def lcm_timesteps(num_inference_steps: int, original_inference_steps: int = 50,
                  num_train_timesteps: int = 1000) -> List[int]:
    """LCM inference schedule, scheduling_lcm.py:119-258 (standard branch, strength 1)."""
    if original_inference_steps > num_train_timesteps:
        raise ValueError("original_inference_steps larger than train timesteps")
    k = num_train_timesteps // original_inference_steps
    origin = np.asarray(list(range(1, original_inference_steps + 1))) * k - 1
    if num_inference_steps > num_train_timesteps:
        raise ValueError("num_inference_steps larger than train timesteps")
    if len(origin) // num_inference_steps < 1:
        raise ValueError("num_inference_steps larger than original_inference_steps")
    if num_inference_steps > original_inference_steps:
        raise ValueError("num_inference_steps larger than original_inference_steps")
    origin = origin[::-1].copy()
    idx = np.floor(np.linspace(0, len(origin), num=num_inference_steps, endpoint=False)).astype(np.int64)
    return [int(v) for v in origin[idx]]


def guidance_embedding(w: Tensor, embedding_dim: int = 256) -> Tensor:
    """``get_guidance_scale_embedding``, scheduling_lcm.py:87-113: [sin | cos] of 1000*w."""
    w = w * 1000.0
    half = embedding_dim // 2
    emb = torch.log(torch.tensor(10000.0)) / (half - 1)
    emb = torch.exp(torch.arange(half, dtype=torch.float32) * -emb)
    emb = w.to(torch.float32)[:, None] * emb[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=1)
    if embedding_dim % 2 == 1:
        emb = F.pad(emb, (0, 1))
    return emb


def timestep_embedding(t: Tensor, dim: int = 256, max_period: int = 10000) -> Tensor:
    """``TimestepEmbedder.timestep_embedding``, concatDiT.py:49-67: [cos | sin]."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def lcm_step_scalars(t: int, prev_t: int, ac: Tensor, timestep_scaling: float = 10.0,
                     sigma_data: float = 0.5) -> Dict[str, Tensor]:
    """Scalars of ``LCMSampler.step`` (scheduling_lcm.py:402-486) as fp32 tensors."""
    tt = torch.tensor(t, dtype=torch.long)
    a_t = ac[t]
    a_prev = ac[prev_t] if prev_t >= 0 else torch.tensor(1.0)
    scaled = tt * timestep_scaling
    c_skip = sigma_data ** 2 / (scaled ** 2 + sigma_data ** 2)
    c_out = scaled / (scaled ** 2 + sigma_data ** 2) ** 0.5
    return dict(sqrt_a=a_t.sqrt(), sqrt_b=(1 - a_t).sqrt(), c_skip=c_skip, c_out=c_out,
                sqrt_a_prev=a_prev.sqrt(), sqrt_b_prev=(1 - a_prev).sqrt())


def lcm_step(eps: Tensor, x: Tensor, sc: Dict[str, Tensor], noise: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    """``LCMSampler.step`` epsilon branch, scheduling_lcm.py:465-486. Returns (prev, denoised)."""
    x0 = (x - sc["sqrt_b"] * eps) / sc["sqrt_a"]
    denoised = sc["c_out"] * x0 + sc["c_skip"] * x
    if noise is not None:
        prev = sc["sqrt_a_prev"] * denoised + sc["sqrt_b_prev"] * noise
    else:
        prev = denoised
    return prev, denoised


def lcm_sample(eps_fn: Callable[[Tensor, Tensor, Tensor], Tensor], cond: Tensor, x_T: Tensor,
               noise: Tensor, S: int, guidance_scale: float = 5.0,
               original_inference_steps: int = 50) -> Tensor:
    """``LCMSampler.sample``/``lcm_sampling`` (scheduling_lcm.py:298-382) with injected RNG.

    ``eps_fn(x, t_long_B, w_emb)`` is the denoiser; ``noise[i]`` is the step-i noise
    (the reference's second global ``torch.randn``, :485).  Returns ``denoised``."""
    B = x_T.shape[0]
    ts = lcm_timesteps(S, original_inference_steps)
    ac = alphas_cumprod()
    w = torch.tensor(guidance_scale - 1).repeat(B)
    w_emb = guidance_embedding(w, 256)
    img = x_T
    denoised = img
    for i, t in enumerate(ts):
        prev_t = ts[i + 1] if i + 1 < len(ts) else t
        eps = eps_fn(img, torch.full((B,), t, dtype=torch.long), w_emb)
        sc = lcm_step_scalars(t, prev_t, ac)
        img, denoised = lcm_step(eps, img, sc, noise[i] if i != S - 1 else None)
    return denoised


def cfg_combine(e_uncond: Tensor, e_cond: Tensor, scale: float) -> Tensor:
    """Classifier-free guidance combine, plms.py:184-186 / ddim.py:203-205."""
    return e_uncond + scale * (e_cond - e_uncond)


# ---------------------------------------------------------------------------
# ConcatDiT2MLP  (concatDiT.py:34-304, new_attention.py:48-130,212-251)
# ---------------------------------------------------------------------------
def _self_attention(W: W_t, p: str, x: Tensor, heads: int) -> Tensor:
    """``CrossAttention`` with context=None, new_attention.py:89-130."""
    B, L, C = x.shape
    d = C // heads
    q = F.linear(x, W[p + "to_q.weight"])
    k = F.linear(x, W[p + "to_k.weight"])
    v = F.linear(x, W[p + "to_v.weight"])
    q, k, v = (t.reshape(B, L, heads, d).permute(0, 2, 1, 3).reshape(B * heads, L, d) for t in (q, k, v))
    sim = torch.einsum("bid,bjd->bij", q, k) * (d ** -0.5)
    attn = sim.softmax(dim=-1)
    out = torch.einsum("bij,bjd->bid", attn, v)
    out = out.reshape(B, heads, L, d).permute(0, 2, 1, 3).reshape(B, L, C)
    return F.linear(out, W[p + "to_out.0.weight"], W[p + "to_out.0.bias"])


def _conv_ff(W: W_t, p: str, x_bcl: Tensor, k: int = 9) -> Tensor:
    """``Conv1dFeedForward`` with ``Conv1dGEGLU``, new_attention.py:48-74."""
    h = F.conv1d(x_bcl, W[p + "net.0.proj.weight"], W[p + "net.0.proj.bias"], padding=k // 2)
    a, g = h.chunk(2, dim=1)
    h = a * F.gelu(g)
    return F.conv1d(h, W[p + "net.2.weight"], W[p + "net.2.bias"], padding=k // 2)


def _transformer_block(W: W_t, p: str, x: Tensor, heads: int) -> Tensor:
    """``BasicTransformerBlock._forward`` (concatDiT.py:120-125); x is (B,L,C)."""
    C = x.shape[-1]
    ln = lambda n, t: F.layer_norm(t, (C,), W[p + n + ".weight"], W[p + n + ".bias"], 1e-5)
    x = _self_attention(W, p + "attn1.", ln("norm1", x), heads) + x
    x = _self_attention(W, p + "attn2.", ln("norm2", x), heads) + x
    x = _conv_ff(W, p + "ff.", ln("norm3", x).permute(0, 2, 1)).permute(0, 2, 1) + x
    return x


def _temporal_transformer(W: W_t, p: str, x: Tensor, heads: int) -> Tensor:
    """``TemporalTransformer.forward`` (concatDiT.py:159-171); x is (B,C,L)."""
    h = F.group_norm(x, 32, W[p + "norm.weight"], W[p + "norm.bias"], 1e-6)
    h = F.conv1d(h, W[p + "proj_in.weight"], W[p + "proj_in.bias"])
    h = h.permute(0, 2, 1)
    h = _transformer_block(W, p + "transformer_blocks.0.", h, heads)
    h = h.permute(0, 2, 1)
    h = F.conv1d(h, W[p + "proj_out.weight"], W[p + "proj_out.bias"])
    return h + x


def dit_time_embed(W: W_t, t: Tensor, w_cond: Optional[Tensor]) -> Tensor:
    """``TimestepEmbedder.forward`` (concatDiT.py:69-74) -> (B, hidden)."""
    tf = timestep_embedding(t, 256)
    if w_cond is not None:
        tf = tf + F.linear(w_cond, W["t_embedder.proj_w.weight"])
    h = F.silu(F.linear(tf, W["t_embedder.mlp.0.weight"], W["t_embedder.mlp.0.bias"]))
    return F.linear(h, W["t_embedder.mlp.2.weight"], W["t_embedder.mlp.2.bias"])


def dit_context_embed(W: W_t, context: Tensor) -> Tensor:
    """Both ``ConditionEmbedder``s (concatDiT.py:91-102, 288-291) -> (B, 154, hidden)."""
    outs = []
    for e, c in zip(("c1_embedder", "c2_embedder"), context.chunk(2, dim=1)):
        p = e + ".mlp."
        h = F.gelu(F.linear(c, W[p + "0.weight"], W[p + "0.bias"]), approximate="tanh")
        h = F.linear(h, W[p + "2.weight"], W[p + "2.bias"])
        h = F.layer_norm(h, (h.shape[-1],), W[p + "3.weight"], W[p + "3.bias"], 1e-5)
        outs.append(h)
    return torch.cat(outs, dim=1)


def dit_forward(W: W_t, x: Tensor, t: Tensor, context: Tensor, w_cond: Optional[Tensor] = None,
                heads: int = 8, depth: int = 4) -> Tensor:
    """``ConcatDiT2MLP.forward`` (concatDiT.py:282-304). x (B,20,T) -> eps (B,20,T)."""
    temb = dit_time_embed(W, t, w_cond)[:, None, :]
    c = dit_context_embed(W, context)
    extra = c.shape[1] + 1
    h = F.conv1d(x, W["proj_in.weight"], W["proj_in.bias"], padding=W["proj_in.weight"].shape[-1] // 2)
    seq = torch.cat([temb, c, h.permute(0, 2, 1)], dim=1)
    L = seq.shape[1]
    seq = seq + W["pos_emb.weight"][:L].view(1, L, -1)
    h = seq.permute(0, 2, 1)
    for i in range(depth):
        h = _temporal_transformer(W, f"blocks.{i}.", h, heads)
    h = h[..., extra:]
    h = F.group_norm(h, 16, W["final_layer.norm_final.weight"], W["final_layer.norm_final.bias"], 1e-5)
    return F.conv1d(h, W["final_layer.conv1d.weight"], W["final_layer.conv1d.bias"])


# ---------------------------------------------------------------------------
# 1-D VAE decoder  (autoencoder1d.py:59-62,176-295,415-517; lcm_audio.py:392-406)
# ---------------------------------------------------------------------------
def _swish(x: Tensor) -> Tensor:
    return x * torch.sigmoid(x)


def _resnet_block(W: W_t, p: str, x: Tensor) -> Tensor:
    """``ResnetBlock1D.forward`` without temb (autoencoder1d.py:212-235)."""
    h = _swish(F.group_norm(x, 32, W[p + "norm1.weight"], W[p + "norm1.bias"], 1e-6))
    k = W[p + "conv1.weight"].shape[-1]  # 3 in Decoder1D, ddconfig kernel_size (5) in Encoder1D
    h = F.conv1d(h, W[p + "conv1.weight"], W[p + "conv1.bias"], padding=k // 2)
    h = _swish(F.group_norm(h, 32, W[p + "norm2.weight"], W[p + "norm2.bias"], 1e-6))
    h = F.conv1d(h, W[p + "conv2.weight"], W[p + "conv2.bias"], padding=k // 2)
    if (p + "nin_shortcut.weight") in W:
        x = F.conv1d(x, W[p + "nin_shortcut.weight"], W[p + "nin_shortcut.bias"])
    return x + h


def _attn_block(W: W_t, p: str, x: Tensor) -> Tensor:
    """``AttnBlock1D.forward`` (autoencoder1d.py:259-278): logit scale is C^-1/2."""
    h = F.group_norm(x, 32, W[p + "norm.weight"], W[p + "norm.bias"], 1e-6)
    q = F.conv1d(h, W[p + "q.weight"], W[p + "q.bias"])
    k = F.conv1d(h, W[p + "k.weight"], W[p + "k.bias"])
    v = F.conv1d(h, W[p + "v.weight"], W[p + "v.bias"])
    C = q.shape[1]
    w_ = torch.bmm(q.permute(0, 2, 1), k) * (int(C) ** (-0.5))
    w_ = torch.softmax(w_, dim=2)
    h = torch.bmm(v, w_.permute(0, 2, 1))
    h = F.conv1d(h, W[p + "proj_out.weight"], W[p + "proj_out.bias"])
    return x + h


def vae_decode(W: W_t, z: Tensor, scale_factor: float = 1.0, num_levels: int = 3,
               num_res_blocks: int = 2, upsample_levels: Sequence[int] = (1,)) -> Tensor:
    """``decode_first_stage``: z/scale -> post_quant_conv -> ``Decoder1D.forward``. (B,20,T) -> (B,80,2T)."""
    z = 1.0 / scale_factor * z
    z = F.conv1d(z, W["post_quant_conv.weight"], W["post_quant_conv.bias"])
    d = "decoder."
    k = W[d + "conv_in.weight"].shape[-1]
    h = F.conv1d(z, W[d + "conv_in.weight"], W[d + "conv_in.bias"], padding=k // 2)
    h = _resnet_block(W, d + "mid.block_1.", h)
    h = _attn_block(W, d + "mid.attn_1.", h)
    h = _resnet_block(W, d + "mid.block_2.", h)
    for lvl in reversed(range(num_levels)):
        for ib in range(num_res_blocks + 1):
            h = _resnet_block(W, f"{d}up.{lvl}.block.{ib}.", h)
        if lvl in upsample_levels:
            h = F.interpolate(h, scale_factor=2.0, mode="nearest")
            h = F.conv1d(h, W[f"{d}up.{lvl}.upsample.conv.weight"], W[f"{d}up.{lvl}.upsample.conv.bias"], padding=1)
    h = _swish(F.group_norm(h, 32, W[d + "norm_out.weight"], W[d + "norm_out.bias"], 1e-6))
    k = W[d + "conv_out.weight"].shape[-1]
    return F.conv1d(h, W[d + "conv_out.weight"], W[d + "conv_out.bias"], padding=k // 2)


def vae_encode_moments(W: W_t, x: Tensor, num_levels: int = 3, num_res_blocks: int = 2,
                       down_layers: Sequence[int] = (0,)) -> Tensor:
    """``AutoencoderKL.encode`` up to the posterior parameters (autoencoder1d.py:54-58): Encoder1D.forward
    (:388-413: conv_in, per level num_res_blocks ResnetBlock1D (+ Downsample1D: zero pad (0, 1), conv k3
    stride 2), mid block / attn / block, GN + swish + conv_out) -> quant_conv.  (B,80,M) -> (B,40,M/2)."""
    e = "encoder."
    k = W[e + "conv_in.weight"].shape[-1]
    h = F.conv1d(x, W[e + "conv_in.weight"], W[e + "conv_in.bias"], padding=k // 2)
    for lvl in range(num_levels):
        for ib in range(num_res_blocks):
            h = _resnet_block(W, f"{e}down.{lvl}.block.{ib}.", h)
        if lvl in down_layers:
            h = F.conv1d(F.pad(h, (0, 1)), W[f"{e}down.{lvl}.downsample.conv.weight"],
                         W[f"{e}down.{lvl}.downsample.conv.bias"], stride=2)
    h = _resnet_block(W, e + "mid.block_1.", h)
    h = _attn_block(W, e + "mid.attn_1.", h)
    h = _resnet_block(W, e + "mid.block_2.", h)
    h = _swish(F.group_norm(h, 32, W[e + "norm_out.weight"], W[e + "norm_out.bias"], 1e-6))
    h = F.conv1d(h, W[e + "conv_out.weight"], W[e + "conv_out.bias"], padding=k // 2)
    return F.conv1d(h, W["quant_conv.weight"], W["quant_conv.bias"])


def mel_spectrogram(y: Tensor, mel_basis: Tensor, n_fft: int = 1024, hop: int = 256, win: int = 1024) -> Tensor:
    """``MelNet.forward`` (ldm/data/preprocess/NAT_mel.py:66-85, center=False): clamp, reflect pad (n_fft-hop)/2,
    |STFT| (periodic Hann, onesided, sqrt(re^2 + im^2 + 1e-9)), mel_basis @ mag, log10(clamp(1e-5))."""
    y = y.clamp(-1.0, 1.0)
    p = (n_fft - hop) // 2
    y = F.pad(y.unsqueeze(1), [p, p], mode="reflect").squeeze(1)
    spec = torch.stft(y, n_fft, hop_length=hop, win_length=win, window=torch.hann_window(win), center=False,
                      normalized=False, onesided=True, return_complex=True)
    mag = torch.sqrt(spec.real.pow(2) + spec.imag.pow(2) + 1e-9)
    return torch.log10(torch.clamp(torch.matmul(mel_basis, mag), min=1e-5))


# ---------------------------------------------------------------------------
# BigVGAN  (vocoder/bigvgan/models.py, activations.py, alias_free_torch/)
# ---------------------------------------------------------------------------
def weight_norm_fold(g: Tensor, v: Tensor) -> Tensor:
    """``torch.nn.utils.weight_norm`` with dim=0: w = g * v / ||v||_(dims != 0)."""
    norm = v.reshape(v.shape[0], -1).norm(dim=1).reshape((-1,) + (1,) * (v.dim() - 1))
    return v * (g / norm)


def snake_beta(x: Tensor, alpha: Tensor, beta: Tensor, logscale: bool = True) -> Tensor:
    """``SnakeBeta.forward`` (activations.py:107-119): x + 1/(b+1e-9) * sin(x*a)^2."""
    a = alpha.unsqueeze(0).unsqueeze(-1)
    b = beta.unsqueeze(0).unsqueeze(-1)
    if logscale:
        a = torch.exp(a)
        b = torch.exp(b)
    return x + (1.0 / (b + 0.000000001)) * torch.pow(torch.sin(x * a), 2)


def activation1d(x: Tensor, alpha: Tensor, beta: Tensor, up_filter: Tensor, down_filter: Tensor) -> Tensor:
    """``Activation1d`` (act.py:23-27): UpSample1d -> SnakeBeta -> DownSample1d.

    UpSample1d (resample.py:25-33): replicate pad 5, depthwise conv_transpose stride 2,
    x2 gain, crop [15:-15].  DownSample1d/LowPassFilter1d (filter.py:86-94): replicate
    pad (5,6), depthwise conv stride 2."""
    C = x.shape[1]
    ratio, K = 2, up_filter.shape[-1]
    pad = K // ratio - 1
    pad_left = pad * ratio + (K - ratio) // 2
    pad_right = pad * ratio + (K - ratio + 1) // 2
    h = F.pad(x, (pad, pad), mode="replicate")
    h = ratio * F.conv_transpose1d(h, up_filter.expand(C, -1, -1), stride=ratio, groups=C)
    h = h[..., pad_left:-pad_right]
    h = snake_beta(h, alpha, beta)
    Kd = down_filter.shape[-1]
    h = F.pad(h, (Kd // 2 - int(Kd % 2 == 0), Kd // 2), mode="replicate")
    return F.conv1d(h, down_filter.expand(C, -1, -1), stride=2, groups=C)


def _wn(W: W_t, p: str) -> Tuple[Tensor, Tensor]:
    return weight_norm_fold(W[p + "weight_g"], W[p + "weight_v"]), W[p + "bias"]


def _act(W: W_t, p: str, x: Tensor) -> Tensor:
    return activation1d(x, W[p + "act.alpha"], W[p + "act.beta"], W[p + "upsample.filter"],
                        W[p + "downsample.lowpass.filter"])


def amp_block1(W: W_t, p: str, x: Tensor, k: int, dilations: Sequence[int]) -> Tensor:
    """``AMPBlock1.forward`` (models.py:72-81)."""
    n = len(dilations)
    for l, d in enumerate(dilations):
        w1, b1 = _wn(W, f"{p}convs1.{l}.")
        w2, b2 = _wn(W, f"{p}convs2.{l}.")
        xt = _act(W, f"{p}activations.{2 * l}.", x)
        xt = F.conv1d(xt, w1, b1, dilation=d, padding=(k * d - d) // 2)
        xt = _act(W, f"{p}activations.{2 * l + 1}.", xt)
        xt = F.conv1d(xt, w2, b2, dilation=1, padding=(k - 1) // 2)
        x = xt + x
    return x


def bigvgan_forward(W: W_t, mel: Tensor, upsample_rates=(4, 4, 2, 2, 2, 2),
                    upsample_kernel_sizes=(8, 8, 4, 4, 4, 4), resblock_kernel_sizes=(3, 7, 11),
                    resblock_dilation_sizes=((1, 3, 5),) * 3) -> Tensor:
    """``BigVGAN.forward`` (models.py:181-203). mel (B,80,M) -> wav (B,1,256M)."""
    w, b = _wn(W, "conv_pre.")
    x = F.conv1d(mel, w, b, padding=3)
    nk = len(resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(upsample_rates, upsample_kernel_sizes)):
        w, b = _wn(W, f"ups.{i}.0.")
        x = F.conv_transpose1d(x, w, b, stride=u, padding=(k - u) // 2)
        xs = None
        for j, (rk, dil) in enumerate(zip(resblock_kernel_sizes, resblock_dilation_sizes)):
            y = amp_block1(W, f"resblocks.{i * nk + j}.", x, rk, dil)
            xs = y if xs is None else xs + y
        x = xs / nk
    x = _act(W, "activation_post.", x)
    w, b = _wn(W, "conv_post.")
    x = F.conv1d(x, w, b, padding=3)
    return torch.tanh(x)


# ---------------------------------------------------------------------------
# end-to-end + output format
# ---------------------------------------------------------------------------
def generate(Wd: W_t, Wv: W_t, Wg: W_t, context: Tensor, x_T: Tensor, noise: Tensor, S: int = 2,
             guidance_scale: float = 5.0, scale_factor: float = 1.0) -> Dict[str, Tensor]:
    """sampler -> decode_first_stage -> vocoder, as ``GenSamples.gen_test_sample`` (InferAPI.py:63-101)."""
    eps_fn = lambda x, t, w: dit_forward(Wd, x, t, context, w)
    z = lcm_sample(eps_fn, context, x_T, noise, S, guidance_scale)
    mel = vae_decode(Wv, z, scale_factor)
    wav = bigvgan_forward(Wg, mel)
    return dict(latent=z, mel=mel, wav=wav)


def pcm16_bytes(wav: np.ndarray) -> bytes:
    """float -> PCM16 as libsndfile's default ``soundfile.write`` (InferAPI.py:98).

    libsndfile (normalised float -> short) clips to [-1, 1) and rounds
    ``x * 32767`` to nearest (lrintf).  Parity unpinned: libsndfile is absent here."""
    x = np.asarray(wav, dtype=np.float32) * np.float32(32767.0)
    x = np.clip(np.rint(x), -32768, 32767).astype("<i2")
    return x.tobytes()


# ---------------------------------------------------------------------------
# text conditioning  (FrozenCLAPFLANEmbedder.encode, ldm/modules/encoders/modules.py:567-582)
# BERT (transformers BertModel, bert-base-uncased config), CLAP Projection (CLAP/clap.py:8-20) and the
# T5 v1.1 encoder (transformers T5EncoderModel: T5LayerNorm = RMSNorm, unscaled attention + relative position
# bias of block 0, gated-gelu FFN with gelu_new).  Third-party: transformers (5.15 here; the reference pins no
# version, requirements.txt).  Pinned by tests/golden/text_B2_L77.npz from the reference encode() itself.
# ---------------------------------------------------------------------------
def t5_relative_bucket(L: int, num_buckets: int = 32, max_distance: int = 128) -> Tensor:
    """``T5Attention._relative_position_bucket`` (bidirectional) of (j - i) for an L x L self-attention."""
    rel = torch.arange(L)[None, :] - torch.arange(L)[:, None]
    nb = num_buckets // 2
    out = (rel > 0).long() * nb
    rel = rel.abs()
    exact = nb // 2
    large = exact + (torch.log(rel.float() / exact) / math.log(max_distance / exact) * (nb - exact)).long()
    large = torch.clamp(large, max=nb - 1)
    return out + torch.where(rel < exact, rel, large)


def _mha(q: Tensor, k: Tensor, v: Tensor, heads: int, scale: float, bias: Optional[Tensor] = None) -> Tensor:
    B, L, I = q.shape
    d = I // heads
    q, k, v = (t.reshape(B, L, heads, d).permute(0, 2, 1, 3) for t in (q, k, v))
    s = torch.matmul(q, k.transpose(-1, -2)) * scale
    if bias is not None:
        s = s + bias
    p = s.float().softmax(-1)
    return torch.matmul(p, v).permute(0, 2, 1, 3).reshape(B, L, I)


def bert_forward(W: W_t, ids: Tensor, layers: int, heads: int, eps: float = 1e-12,
                 p: str = "caption_encoder.base.") -> Tensor:
    """BertModel(input_ids).last_hidden_state: embeddings (word + position + token_type 0) -> LayerNorm, then
    post-LN layers: x = LN(x + Wo attn(x)); x = LN(x + W2 gelu(W1 x))."""
    B, L = ids.shape
    x = (W[p + "embeddings.word_embeddings.weight"][ids] + W[p + "embeddings.position_embeddings.weight"][:L]
         + W[p + "embeddings.token_type_embeddings.weight"][0])
    H = x.shape[-1]
    x = F.layer_norm(x, (H,), W[p + "embeddings.LayerNorm.weight"], W[p + "embeddings.LayerNorm.bias"], eps)
    for l in range(layers):
        q = f"{p}encoder.layer.{l}."
        lin = lambda t, n: F.linear(t, W[q + n + ".weight"], W[q + n + ".bias"])
        a = _mha(lin(x, "attention.self.query"), lin(x, "attention.self.key"), lin(x, "attention.self.value"),
                 heads, (H // heads) ** -0.5)
        x = F.layer_norm(lin(a, "attention.output.dense") + x, (H,), W[q + "attention.output.LayerNorm.weight"],
                         W[q + "attention.output.LayerNorm.bias"], eps)
        h = F.gelu(lin(x, "intermediate.dense"))
        x = F.layer_norm(lin(h, "output.dense") + x, (H,), W[q + "output.LayerNorm.weight"],
                         W[q + "output.LayerNorm.bias"], eps)
    return x


def clap_projection(W: W_t, x: Tensor, p: str = "caption_encoder.projection.") -> Tensor:
    """CLAP/clap.py:16-20: LayerNorm(e1 + linear2(gelu(e1))), e1 = linear1(x); dropout = identity (eval)."""
    e1 = F.linear(x, W[p + "linear1.weight"])
    e2 = F.linear(F.gelu(e1), W[p + "linear2.weight"])
    return F.layer_norm(e1 + e2, (e1.shape[-1],), W[p + "layer_norm.weight"], W[p + "layer_norm.bias"], 1e-5)


def t5_encoder_forward(W: W_t, ids: Tensor, layers: int, heads: int, eps: float = 1e-6,
                       p: str = "t5_transformer.") -> Tensor:
    """T5EncoderModel(input_ids).last_hidden_state (v1.1): pre-RMSNorm blocks, unscaled attention + the
    relative position bias of block 0, gated-gelu FFN (gelu_new(wi_0 h) * wi_1 h), final RMSNorm."""
    B, L = ids.shape
    x = W[p + "shared.weight"][ids]

    def rms(t, w):
        return w * (t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + eps))
    tab = W[p + "encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]
    bias = tab[t5_relative_bucket(L, tab.shape[0])].permute(2, 0, 1)[None]
    for l in range(layers):
        q = f"{p}encoder.block.{l}.layer."
        h = rms(x, W[q + "0.layer_norm.weight"])
        a = _mha(F.linear(h, W[q + "0.SelfAttention.q.weight"]), F.linear(h, W[q + "0.SelfAttention.k.weight"]),
                 F.linear(h, W[q + "0.SelfAttention.v.weight"]), heads, 1.0, bias)
        x = x + F.linear(a, W[q + "0.SelfAttention.o.weight"])
        h = rms(x, W[q + "1.layer_norm.weight"])
        g = F.gelu(F.linear(h, W[q + "1.DenseReluDense.wi_0.weight"]), approximate="tanh")
        x = x + F.linear(g * F.linear(h, W[q + "1.DenseReluDense.wi_1.weight"]), W[q + "1.DenseReluDense.wo.weight"])
    return rms(x, W[p + "encoder.final_layer_norm.weight"])


def text_encode(W: W_t, clap_ids: Tensor, t5_ids: Tensor, bert_layers: int = 12, bert_heads: int = 12,
                t5_layers: int = 24, t5_heads: int = 16) -> Tensor:
    """FrozenCLAPFLANEmbedder.encode from token ids: concat([Projection(BERT), T5], dim=1) (modules.py:579-582)."""
    z = clap_projection(W, bert_forward(W, clap_ids, bert_layers, bert_heads))
    z2 = t5_encoder_forward(W, t5_ids, t5_layers, t5_heads)
    return torch.cat([z, z2], dim=1)
