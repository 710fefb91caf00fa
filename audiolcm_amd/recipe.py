"""Model hyper-parameters and the seeded synthetic-weight recipe.

Real AudioLCM / BigVGAN checkpoints are not available offline, so every
parity fixture and every benchmark runs on *synthetic* weights drawn from this
recipe.  The recipe is pure host data: a list of ``(state_dict key, shape,
init)`` entries whose keys and shapes are exactly the reference modules'
``state_dict()`` keys, plus a per-tensor seeded
``torch.Generator`` so that the GPU box can regenerate bit-identical weights
without any reference code.

Key layouts followed:
  * ``ConcatDiT2MLP``   ldm/modules/diffusionmodules/concatDiT.py:238-304
  * ``Decoder1D`` + ``post_quant_conv``  ldm/models/autoencoder1d.py:18-62,415-517
  * ``BigVGAN`` (weight-norm ``_g``/``_v`` + filter buffers)
    vocoder/bigvgan/models.py:30-88,133-203, alias_free_torch/*.py

Initialisation deliberately departs from the reference's training init in two
places: the zero-initialised ``proj_out`` convolutions
(concatDiT.py:153-157) get a small non-zero init, otherwise every DiT block is
the identity; and BigVGAN's N(0, 0.01) conv init (models.py:21-24) is replaced
by unit-gain weight norm, otherwise the signal collapses to silence.
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import torch


# ---------------------------------------------------------------------------
# hyper-parameters (configs/audiolcm.yaml:39-72, bigvgan_audioset16khz_80band.json)
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class DiTConfig:
    """``unet_config.params`` of configs/audiolcm.yaml:39-47."""
    in_channels: int = 20
    context_dim: int = 1024
    hidden_size: int = 576
    num_heads: int = 8
    depth: int = 4
    max_len: int = 1000
    ctx_tokens: int = 154          # CLAP(77) + T5(77), modules.py:567-582
    ff_kernel: int = 9             # new_attention.py:57
    proj_in_kernel: int = 5        # concatDiT.py:255

    @property
    def d_head(self) -> int:
        return self.hidden_size // self.num_heads

    @property
    def extra_len(self) -> int:
        return 1 + self.ctx_tokens

    @property
    def max_latent_len(self) -> int:
        return self.max_len - self.extra_len


@dataclass(frozen=True)
class VAEConfig:
    """``first_stage_config.params.ddconfig`` of configs/audiolcm.yaml:48-72."""
    embed_dim: int = 20
    z_channels: int = 20
    out_ch: int = 80
    kernel_size: int = 5
    ch: int = 384
    ch_mult: Tuple[int, ...] = (1, 2, 4)
    num_res_blocks: int = 2
    attn_layers: Tuple[int, ...] = (3,)
    down_layers: Tuple[int, ...] = (0,)

    @property
    def upsample_levels(self) -> Tuple[int, ...]:
        # Decoder1D.down_layers = [i+1 for i in down_layers] (autoencoder1d.py:427)
        return tuple(i + 1 for i in self.down_layers)

    @property
    def time_upsample(self) -> int:
        return 2 ** len(self.down_layers)


@dataclass(frozen=True)
class BigVGANConfig:
    """vocoder/bigvgan/bigvgan_audioset16khz_80band.json."""
    num_mels: int = 80
    upsample_rates: Tuple[int, ...] = (4, 4, 2, 2, 2, 2)
    upsample_kernel_sizes: Tuple[int, ...] = (8, 8, 4, 4, 4, 4)
    upsample_initial_channel: int = 1536
    resblock_kernel_sizes: Tuple[int, ...] = (3, 7, 11)
    resblock_dilation_sizes: Tuple[Tuple[int, ...], ...] = ((1, 3, 5), (1, 3, 5), (1, 3, 5))
    sampling_rate: int = 16000
    hop_size: int = 256
    filter_taps: int = 12

    @property
    def hop(self) -> int:
        return int(math.prod(self.upsample_rates))

    def stage_channels(self, i: int) -> int:
        return self.upsample_initial_channel // (2 ** (i + 1))


# ---------------------------------------------------------------------------
# parameter specs: (key, shape, init-kind, scale)
# ---------------------------------------------------------------------------
Spec = Tuple[str, Tuple[int, ...], str, float]


def _linear(p: str, n_out: int, n_in: int, bias: bool = True, gain: float = 1.0) -> List[Spec]:
    s: List[Spec] = [(p + "weight", (n_out, n_in), "fanin", gain)]
    if bias:
        s.append((p + "bias", (n_out,), "normal", 0.02))
    return s


def _conv(p: str, c_out: int, c_in: int, k: int, bias: bool = True, gain: float = 1.0) -> List[Spec]:
    s: List[Spec] = [(p + "weight", (c_out, c_in, k), "fanin", gain)]
    if bias:
        s.append((p + "bias", (c_out,), "normal", 0.02))
    return s


def _norm(p: str, c: int) -> List[Spec]:
    return [(p + "weight", (c,), "gamma", 0.1), (p + "bias", (c,), "normal", 0.1)]


def dit_specs(cfg: DiTConfig = DiTConfig()) -> List[Spec]:
    """Keys of ``ConcatDiT2MLP.state_dict()`` (concatDiT.py:238-280)."""
    H, C = cfg.hidden_size, cfg.context_dim
    s: List[Spec] = []
    s += _linear("t_embedder.mlp.0.", H, 256)
    s += _linear("t_embedder.mlp.2.", H, H)
    s += [("t_embedder.proj_w.weight", (256, 256), "fanin", 0.5)]
    for e in ("c1_embedder", "c2_embedder"):
        s += _linear(f"{e}.mlp.0.", H, C)
        s += _linear(f"{e}.mlp.2.", H, H)
        s += _norm(f"{e}.mlp.3.", H)
    s += _conv("proj_in.", H, cfg.in_channels, cfg.proj_in_kernel)
    s += [("pos_emb.weight", (cfg.max_len, H), "normal", math.sqrt(2.0 / (cfg.max_len + H)))]
    inner = 4 * H
    for i in range(cfg.depth):
        b = f"blocks.{i}."
        s += _norm(b + "norm.", H)
        s += _conv(b + "proj_in.", H, H, 1)
        tb = b + "transformer_blocks.0."
        for a in ("attn1", "attn2"):
            for q in ("to_q", "to_k", "to_v"):
                s += _linear(f"{tb}{a}.{q}.", H, H, bias=False)
            s += _linear(f"{tb}{a}.to_out.0.", H, H, gain=0.5)
        s += _conv(tb + "ff.net.0.proj.", 2 * inner, H, cfg.ff_kernel)
        s += _conv(tb + "ff.net.2.", H, inner, cfg.ff_kernel, gain=0.5)
        for n in ("norm1", "norm2", "norm3"):
            s += _norm(f"{tb}{n}.", H)
        # reference zero-inits proj_out (concatDiT.py:153); small non-zero here
        s += _conv(b + "proj_out.", H, H, 1, gain=0.5)
    s += _norm("final_layer.norm_final.", H)
    s += _conv("final_layer.conv1d.", cfg.in_channels, H, 1)
    return s


def _resblock_specs(p: str, cin: int, cout: int) -> List[Spec]:
    s: List[Spec] = []
    s += _norm(p + "norm1.", cin)
    s += _conv(p + "conv1.", cout, cin, 3)
    s += _norm(p + "norm2.", cout)
    s += _conv(p + "conv2.", cout, cout, 3, gain=0.5)
    if cin != cout:
        s += _conv(p + "nin_shortcut.", cout, cin, 1)
    return s


def vae_decoder_specs(cfg: VAEConfig = VAEConfig()) -> List[Spec]:
    """Decode-path keys of ``AutoencoderKL.state_dict()`` (autoencoder1d.py:18-62,415-482)."""
    s: List[Spec] = []
    s += _conv("post_quant_conv.", cfg.z_channels, cfg.embed_dim, 1)
    nl = len(cfg.ch_mult)
    block_in = cfg.ch * cfg.ch_mult[-1]
    d = "decoder."
    s += _conv(d + "conv_in.", block_in, cfg.z_channels, cfg.kernel_size)
    s += _resblock_specs(d + "mid.block_1.", block_in, block_in)
    a = d + "mid.attn_1."
    s += _norm(a + "norm.", block_in)
    for q in ("q", "k", "v"):
        s += _conv(f"{a}{q}.", block_in, block_in, 1)
    s += _conv(a + "proj_out.", block_in, block_in, 1, gain=0.5)
    s += _resblock_specs(d + "mid.block_2.", block_in, block_in)
    for lvl in reversed(range(nl)):
        block_out = cfg.ch * cfg.ch_mult[lvl]
        for ib in range(cfg.num_res_blocks + 1):
            s += _resblock_specs(f"{d}up.{lvl}.block.{ib}.", block_in, block_out)
            block_in = block_out
            if lvl in cfg.attn_layers:
                raise NotImplementedError("attention inside up levels is not configured by audiolcm.yaml")
        if lvl in cfg.upsample_levels:
            s += _conv(f"{d}up.{lvl}.upsample.conv.", block_in, block_in, 3)
    s += _norm(d + "norm_out.", block_in)
    s += _conv(d + "conv_out.", cfg.out_ch, block_in, cfg.kernel_size)
    return s


def vae_encoder_specs(cfg: VAEConfig = VAEConfig(), in_channels: int = 80) -> List[Spec]:
    """Encode-path keys of ``AutoencoderKL.state_dict()``: ``encoder.*`` (Encoder1D, autoencoder1d.py:319-413:
    its ResnetBlock1D convs use ddconfig kernel_size) and ``quant_conv`` (2 z -> 2 embed, :31-33)."""
    s: List[Spec] = []
    e, k = "encoder.", cfg.kernel_size
    s += _conv(e + "conv_in.", cfg.ch, in_channels, k)
    block_in = cfg.ch
    for lvl, mult in enumerate(cfg.ch_mult):
        block_out = cfg.ch * mult
        for ib in range(cfg.num_res_blocks):
            p = f"{e}down.{lvl}.block.{ib}."
            s += _norm(p + "norm1.", block_in)
            s += _conv(p + "conv1.", block_out, block_in, k)
            s += _norm(p + "norm2.", block_out)
            s += _conv(p + "conv2.", block_out, block_out, k, gain=0.5)
            if block_in != block_out:
                s += _conv(p + "nin_shortcut.", block_out, block_in, 1)
            block_in = block_out
        if lvl in cfg.down_layers:
            s += _conv(f"{e}down.{lvl}.downsample.conv.", block_in, block_in, 3)
    for b in ("mid.block_1.", "mid.block_2."):
        s += _norm(e + b + "norm1.", block_in)
        s += _conv(e + b + "conv1.", block_in, block_in, k)
        s += _norm(e + b + "norm2.", block_in)
        s += _conv(e + b + "conv2.", block_in, block_in, k, gain=0.5)
    a = e + "mid.attn_1."
    s += _norm(a + "norm.", block_in)
    for q in ("q", "k", "v"):
        s += _conv(f"{a}{q}.", block_in, block_in, 1)
    s += _conv(a + "proj_out.", block_in, block_in, 1, gain=0.5)
    s += _norm(e + "norm_out.", block_in)
    s += _conv(e + "conv_out.", 2 * cfg.z_channels, block_in, k)
    s += _conv("quant_conv.", 2 * cfg.embed_dim, 2 * cfg.z_channels, 1)
    return s


def _wn_conv(p: str, c_out: int, c_in: int, k: int, transposed: bool = False, gain: float = 1.0) -> List[Spec]:
    # weight_norm(dim=0): weight_g has shape (dim0, 1, 1)
    if transposed:
        return [(p + "weight_g", (c_in, 1, 1), "wn_g", gain),
                (p + "weight_v", (c_in, c_out, k), "normal", 1.0),
                (p + "bias", (c_out,), "normal", 0.02)]
    return [(p + "weight_g", (c_out, 1, 1), "wn_g", gain),
            (p + "weight_v", (c_out, c_in, k), "normal", 1.0),
            (p + "bias", (c_out,), "normal", 0.02)]


def _act_specs(p: str, c: int, taps: int) -> List[Spec]:
    return [(p + "act.alpha", (c,), "normal", 0.3),
            (p + "act.beta", (c,), "normal", 0.3),
            (p + "upsample.filter", (1, 1, taps), "kaiser", 0.0),
            (p + "downsample.lowpass.filter", (1, 1, taps), "kaiser", 0.0)]


def bigvgan_specs(cfg: BigVGANConfig = BigVGANConfig()) -> List[Spec]:
    """Keys of ``BigVGAN.state_dict()`` (vocoder/bigvgan/models.py:133-180)."""
    s: List[Spec] = []
    C0 = cfg.upsample_initial_channel
    s += _wn_conv("conv_pre.", C0, cfg.num_mels, 7)
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        s += _wn_conv(f"ups.{i}.0.", C0 // 2 ** (i + 1), C0 // 2 ** i, k, transposed=True)
    nk = len(cfg.resblock_kernel_sizes)
    for i in range(len(cfg.upsample_rates)):
        ch = cfg.stage_channels(i)
        for j, (k, dil) in enumerate(zip(cfg.resblock_kernel_sizes, cfg.resblock_dilation_sizes)):
            p = f"resblocks.{i * nk + j}."
            for l in range(len(dil)):
                s += _wn_conv(f"{p}convs1.{l}.", ch, ch, k)
            for l in range(len(dil)):
                s += _wn_conv(f"{p}convs2.{l}.", ch, ch, k)
            for a in range(2 * len(dil)):
                s += _act_specs(f"{p}activations.{a}.", ch, cfg.filter_taps)
    ch = cfg.stage_channels(len(cfg.upsample_rates) - 1)
    s += _act_specs("activation_post.", ch, cfg.filter_taps)
    s += _wn_conv("conv_post.", 1, ch, 7, gain=6.0)  # audible (~0.25 rms) synthetic waveform
    return s


# ---------------------------------------------------------------------------
# Kaiser-sinc filter (alias_free_torch/filter.py:28-57), restated
# ---------------------------------------------------------------------------
def kaiser_sinc_filter1d(cutoff: float, half_width: float, kernel_size: int) -> torch.Tensor:
    """Windowed-sinc low-pass used by Activation1d up/down sampling.

    Follows alias_free_torch/filter.py:28-57 (Kaiser beta from the stop-band
    attenuation, even-length half-sample time grid, unit DC gain).  That reference
    file is itself adapted from the `julius` package (MIT, Alexandre Défossez,
    ``julius/lowpass.py``) by the alias-free-torch project (Apache-2.0, junjun3518);
    the formula is the standard Kaiser window design (Kaiser & Schafer 1980,
    Oppenheim & Schafer eq. 7.62-7.63) and is restated here with that attribution."""
    even = kernel_size % 2 == 0
    half = kernel_size // 2
    delta_f = 4 * half_width
    A = 2.285 * (half - 1) * math.pi * delta_f + 7.95
    if A > 50.0:
        beta = 0.1102 * (A - 8.7)
    elif A >= 21.0:
        beta = 0.5842 * (A - 21) ** 0.4 + 0.07886 * (A - 21.0)
    else:
        beta = 0.0
    window = torch.kaiser_window(kernel_size, beta=beta, periodic=False)
    if even:
        time = torch.arange(-half, half) + 0.5
    else:
        time = torch.arange(kernel_size) - half
    filt = 2 * cutoff * window * torch.sinc(2 * cutoff * time)
    filt = filt / filt.sum()
    return filt.view(1, 1, kernel_size)


# ---------------------------------------------------------------------------
# materialisation
# ---------------------------------------------------------------------------
def _seed_for(key: str, seed: int) -> int:
    return (zlib.crc32(key.encode()) ^ (seed * 0x9E3779B1)) & 0x7FFFFFFF


def make_state(specs: List[Spec], seed: int = 0) -> Dict[str, torch.Tensor]:
    """Materialise a spec list into fp32 CPU tensors, one seeded generator per key."""
    out: Dict[str, torch.Tensor] = {}
    for key, shape, kind, scale in specs:
        g = torch.Generator().manual_seed(_seed_for(key, seed))
        if kind == "fanin":
            fan_in = int(math.prod(shape[1:]))
            t = torch.randn(shape, generator=g) * (scale / math.sqrt(fan_in))
        elif kind == "normal":
            t = torch.randn(shape, generator=g) * scale
        elif kind == "gamma":
            t = 1.0 + torch.randn(shape, generator=g) * scale
        elif kind == "wn_g":
            # ||w[o]|| = g ; unit-gain conv with a little spread
            t = scale * (0.55 + 0.1 * torch.rand(shape, generator=g))
        elif kind == "kaiser":
            t = kaiser_sinc_filter1d(0.25, 0.3, shape[-1]).reshape(shape).clone()
        else:
            raise ValueError(kind)
        out[key] = t.contiguous()
    return out


def dit_state(seed: int = 0, cfg: DiTConfig = DiTConfig()) -> Dict[str, torch.Tensor]:
    return make_state(dit_specs(cfg), seed)


def vae_state(seed: int = 0, cfg: VAEConfig = VAEConfig()) -> Dict[str, torch.Tensor]:
    return make_state(vae_decoder_specs(cfg), seed + 1)


def vae_encoder_state(seed: int = 0, cfg: VAEConfig = VAEConfig()) -> Dict[str, torch.Tensor]:
    return make_state(vae_encoder_specs(cfg), seed + 1)


def bigvgan_state(seed: int = 0, cfg: BigVGANConfig = BigVGANConfig()) -> Dict[str, torch.Tensor]:
    return make_state(bigvgan_specs(cfg), seed + 2)


@dataclass(frozen=True)
class TextConfig:
    """FrozenCLAPFLANEmbedder (ldm/modules/encoders/modules.py:529-582): CLAP text tower = bert-base-uncased
    (CLAP/config.yaml: transformer_embed_dim 768) + Projection(768 -> d_proj 1024) (CLAP/clap.py:8-20), and
    the t5-v1_1-large encoder (d_model 1024, 16 heads x 64, d_ff 2816 gated-gelu, 24 blocks, 32 relative
    buckets / max distance 128, RMSNorm eps 1e-6); max_length 77 tokens each."""
    b_vocab: int = 30522
    b_hidden: int = 768
    b_layers: int = 12
    b_heads: int = 12
    b_inter: int = 3072
    b_maxpos: int = 512
    p_out: int = 1024
    t_vocab: int = 32128
    t_d: int = 1024
    t_dkv: int = 64
    t_heads: int = 16
    t_ff: int = 2816
    t_layers: int = 24
    t_buckets: int = 32
    t_max_distance: int = 128
    max_len: int = 77

    def iconfig(self) -> List[int]:
        return [self.b_vocab, self.b_hidden, self.b_layers, self.b_heads, self.b_inter, self.b_maxpos, self.p_out,
                self.t_vocab, self.t_d, self.t_dkv, self.t_heads, self.t_ff, self.t_layers, self.max_len]


def text_specs(cfg: TextConfig = TextConfig()) -> List[Spec]:
    """Keys of FrozenCLAPFLANEmbedder's state_dict on the inference path: ``caption_encoder.base.*``
    (transformers BertModel), ``caption_encoder.projection.*`` (CLAP Projection) and ``t5_transformer.*``
    (transformers T5EncoderModel; ``encoder.embed_tokens`` is tied to ``shared``).  Scales keep every
    layer's activations O(1): T5 has no 1/sqrt(d) on its attention logits, so its q projection carries it."""
    s: List[Spec] = []
    H, bp = cfg.b_hidden, "caption_encoder.base."
    s += [(bp + "embeddings.word_embeddings.weight", (cfg.b_vocab, H), "normal", 0.5),
          (bp + "embeddings.position_embeddings.weight", (cfg.b_maxpos, H), "normal", 0.5),
          (bp + "embeddings.token_type_embeddings.weight", (2, H), "normal", 0.5)]
    s += _norm(bp + "embeddings.LayerNorm.", H)
    for l in range(cfg.b_layers):
        p = f"{bp}encoder.layer.{l}."
        for q in ("query", "key", "value"):
            s += _linear(f"{p}attention.self.{q}.", H, H)
        s += _linear(p + "attention.output.dense.", H, H, gain=0.5)
        s += _norm(p + "attention.output.LayerNorm.", H)
        s += _linear(p + "intermediate.dense.", cfg.b_inter, H)
        s += _linear(p + "output.dense.", H, cfg.b_inter, gain=0.5)
        s += _norm(p + "output.LayerNorm.", H)
    s += _linear(bp + "pooler.dense.", H, H)  # in the state_dict, unused by encode()
    pp = "caption_encoder.projection."
    s += _linear(pp + "linear1.", cfg.p_out, H, bias=False)
    s += _linear(pp + "linear2.", cfg.p_out, cfg.p_out, bias=False, gain=0.5)
    s += _norm(pp + "layer_norm.", cfg.p_out)
    D, I, tp = cfg.t_d, cfg.t_heads * cfg.t_dkv, "t5_transformer."
    s += [(tp + "shared.weight", (cfg.t_vocab, D), "normal", 1.0)]
    for l in range(cfg.t_layers):
        p = f"{tp}encoder.block.{l}.layer."
        s += [(p + "0.SelfAttention.q.weight", (I, D), "fanin", cfg.t_dkv ** -0.5),
              (p + "0.SelfAttention.k.weight", (I, D), "fanin", 1.0),
              (p + "0.SelfAttention.v.weight", (I, D), "fanin", 1.0),
              (p + "0.SelfAttention.o.weight", (D, I), "fanin", 0.5)]
        if l == 0:
            s += [(p + "0.SelfAttention.relative_attention_bias.weight", (cfg.t_buckets, cfg.t_heads), "normal", 0.5)]
        s += [(p + "0.layer_norm.weight", (D,), "gamma", 0.1)]
        s += [(p + "1.DenseReluDense.wi_0.weight", (cfg.t_ff, D), "fanin", 1.0),
              (p + "1.DenseReluDense.wi_1.weight", (cfg.t_ff, D), "fanin", 1.0),
              (p + "1.DenseReluDense.wo.weight", (D, cfg.t_ff), "fanin", 0.5),
              (p + "1.layer_norm.weight", (D,), "gamma", 0.1)]
    s += [(tp + "encoder.final_layer_norm.weight", (D,), "gamma", 0.1)]
    return s


def text_state(seed: int = 0, cfg: TextConfig = TextConfig()) -> Dict[str, torch.Tensor]:
    return make_state(text_specs(cfg), seed + 3)


def synthetic_context(batch: int, seed0: int = 1000, tokens: int = 154, dim: int = 1024) -> torch.Tensor:
    """(B, 154, 1024) fp32 conditioning, prompt i seeded with ``seed0 + i``."""
    rows = [torch.randn((tokens, dim), generator=torch.Generator().manual_seed(seed0 + i)) for i in range(batch)]
    return torch.stack(rows, 0)


def prompt_noise(seeds, steps: int, channels: int = 20, length: int = 312):
    """Per-prompt x_T and per-step LCM noise drawn from ``torch.Generator(seed)``.

    The reference draws both from the global RNG over the whole batch
    (scheduling_lcm.py:354,485); per-prompt generators make results
    independent of how prompts are sharded across GPUs (RNG
    parity).  Draw order per prompt: x_T, then one noise tensor per
    non-final step.
    Returns ``x_T`` (B,C,T) and ``noise`` (max(S-1,0),B,C,T)."""
    xs, ns = [], []
    for s in seeds:
        g = torch.Generator().manual_seed(int(s))
        xs.append(torch.randn((channels, length), generator=g))
        ns.append(torch.stack([torch.randn((channels, length), generator=g) for _ in range(max(steps - 1, 0))], 0)
                  if steps > 1 else torch.zeros((0, channels, length)))
    x_T = torch.stack(xs, 0)
    noise = torch.stack(ns, 1) if steps > 1 else torch.zeros((0, len(xs), channels, length))
    return x_T, noise
