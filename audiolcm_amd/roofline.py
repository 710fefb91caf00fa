"""Layer enumeration of the hot path and its MI355X roofline (SURVEY.md §8(d) model).

Model: bf16 activations and weights; the HBM traffic of a layer is its
boundary traffic = weights + layer input + layer output of every conv / linear / attention core (norms,
activations, the Activation1d FIR and the LCM step are fused and cost nothing); per-layer time is
max(F / P_mfma, B / P_hbm) and the path's ideal time is the sum over layers.  ``t_roof`` is the
denominator of ``bench.py``'s ``path_roofline_frac_model`` (ideal / measured wall).

Layer shapes follow the reference modules:
  ConcatDiT2MLP   concatDiT.py:238-304, new_attention.py:48-130
  Decoder1D       autoencoder1d.py:415-517 (ResnetBlock1D :176-235, AttnBlock1D :237-278, Upsample1D :280-295)
  BigVGAN         vocoder/bigvgan/models.py:133-203 (AMPBlock1 :30-88, Activation1d alias_free_torch/act.py)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

PEAK_MFMA = 2.5e15   # dense bf16 / fp16 MFMA FLOP/s (MI355X_MICROARCH.md, spec)
PEAK_HBM = 8.0e12    # HBM3E bytes/s (spec)
ELT = 2              # bf16 bytes per element (the model's boundary format)


@dataclass
class Layer:
    stage: str
    name: str
    flops: float
    bytes: float

    @property
    def t(self) -> float:
        return max(self.flops / PEAK_MFMA, self.bytes / PEAK_HBM)


def _conv(stage, name, rows, cin, cout, k, out_rows=None) -> Layer:
    """conv1d / linear over `rows` input positions (batch folded in), weights cout x cin x k."""
    out_rows = rows if out_rows is None else out_rows
    return Layer(stage, name, 2.0 * out_rows * cout * cin * k, ELT * (cin * cout * k + rows * cin + out_rows * cout))


def dit_layers(B: int, T: int, hidden=576, heads=8, depth=4, ctx_tokens=154, ctx_dim=1024, in_ch=20,
               ff_k=9, pin_k=5, with_context=True) -> List[Layer]:
    H, L = hidden, 1 + ctx_tokens + T
    dh = H // heads
    out: List[Layer] = []
    s = "dit"
    out += [_conv(s, "t.proj_w", B, 256, 256, 1), _conv(s, "t.mlp0", B, 256, H, 1), _conv(s, "t.mlp2", B, H, H, 1)]
    if with_context:  # ConditionEmbedder x2 (the reference runs them in every DiT call)
        n = ctx_tokens // 2
        for e in range(2):
            out += [_conv(s, f"c{e}.mlp0", B * n, ctx_dim, H, 1), _conv(s, f"c{e}.mlp2", B * n, H, H, 1)]
    out.append(_conv(s, "proj_in", B * T, in_ch, H, pin_k))
    for i in range(depth):
        out.append(_conv(s, f"b{i}.proj_in", B * L, H, H, 1))
        for a in range(2):
            out.append(_conv(s, f"b{i}.attn{a}.qkv", B * L, H, 3 * H, 1))
            # attention core: QK^T and PV per head; boundary = q, k, v in, o out
            fl = 2.0 * B * heads * L * L * dh * 2
            out.append(Layer(s, f"b{i}.attn{a}.core", fl, ELT * (4 * B * L * H)))
            out.append(_conv(s, f"b{i}.attn{a}.out", B * L, H, H, 1))
        out.append(_conv(s, f"b{i}.ff0", B * L, H, 8 * H, ff_k))
        out.append(_conv(s, f"b{i}.ff2", B * L, 4 * H, H, ff_k))
        out.append(_conv(s, f"b{i}.proj_out", B * L, H, H, 1))
    out.append(_conv(s, "final", B * T, H, in_ch, 1))
    return out


def vae_layers(B: int, T: int, z=20, ch=384, mult=(1, 2, 4), nrb=2, out_ch=80, ksz=5, up_levels=(1,)) -> List[Layer]:
    s = "vae"
    out: List[Layer] = [_conv(s, "post_quant", B * T, z, z, 1)]
    C = ch * mult[-1]
    out.append(_conv(s, "conv_in", B * T, z, C, ksz))

    def res(name, rows, cin, cout):
        r = [_conv(s, name + ".conv1", rows, cin, cout, 3), _conv(s, name + ".conv2", rows, cout, cout, 3)]
        if cin != cout:
            r.append(_conv(s, name + ".nin", rows, cin, cout, 1))
        return r
    out += res("mid.block_1", B * T, C, C)
    out.append(_conv(s, "mid.attn.qkv", B * T, C, 3 * C, 1))
    out.append(Layer(s, "mid.attn.core", 2.0 * B * T * T * C * 2, ELT * 4 * B * T * C))
    out.append(_conv(s, "mid.attn.proj", B * T, C, C, 1))
    out += res("mid.block_2", B * T, C, C)
    Tc = T
    for lvl in reversed(range(len(mult))):
        co = ch * mult[lvl]
        for ib in range(nrb + 1):
            out += res(f"up{lvl}.block{ib}", B * Tc, C, co)
            C = co
        if lvl in up_levels:
            out.append(_conv(s, f"up{lvl}.upsample", B * 2 * Tc, C, C, 3))
            Tc *= 2
    out.append(_conv(s, "conv_out", B * Tc, C, out_ch, ksz))
    return out


def bigvgan_layers(B: int, M: int, mels=80, c0=1536, rates=(4, 4, 2, 2, 2, 2), kernels=(8, 8, 4, 4, 4, 4),
                   rk=(3, 7, 11), dil=(1, 3, 5), fir_taps=12, with_fir: bool = False) -> List[Layer]:
    """with_fir adds the Activation1d FIR FLOPs (VALU work, ~1.6% of the path's FLOPs); the §8(d) model leaves
    them out of the MFMA roofline (fused, no boundary traffic)."""
    s = "bigvgan"
    out: List[Layer] = [_conv(s, "conv_pre", B * M, mels, c0, 7)]
    T, C = M, c0
    for i, (r, k) in enumerate(zip(rates, kernels)):
        co = C // 2
        # ConvTranspose1d: every input sample feeds k outputs
        out.append(Layer(s, f"ups{i}", 2.0 * B * T * C * co * k, ELT * (C * co * k + B * T * C + B * T * r * co)))
        T, C = T * r, co
        for kk in rk:
            for d in dil:
                out.append(_conv(s, f"s{i}.k{kk}.d{d}.c1", B * T, C, C, kk))
                out.append(_conv(s, f"s{i}.k{kk}.d{d}.c2", B * T, C, C, kk))
        # Activation1d FIR (fused: FLOPs only): up 2T x 6 taps + down T x 12 taps, 2 FLOP per tap
        n_act = 2 * len(dil) * len(rk)
        fir = 2.0 * (2 * fir_taps // 2 + fir_taps)  # FLOP per (channel, sample): 2T x 6 taps up + T x 12 down
        if with_fir:
            out.append(Layer(s, f"s{i}.act_fir", n_act * B * C * T * fir, 0.0))
    if with_fir:
        out.append(Layer(s, "post.act_fir", B * C * T * fir, 0.0))
    out.append(_conv(s, "conv_post", B * T, C, 1, 7))
    return out


def path_layers(B: int, S: int = 2, T: int = 312, cfg: bool = False, decode_only: bool = False) -> List[Layer]:
    """The C2 / C4 / C5 workloads: S DiT calls (batch 2B under CFG) + VAE decode + BigVGAN."""
    out: List[Layer] = []
    if not decode_only:
        for _ in range(S):
            out += dit_layers(2 * B if cfg else B, T)
    out += vae_layers(B, T)
    out += bigvgan_layers(B, 2 * T)
    return out


def summary(layers: List[Layer]) -> dict:
    f = sum(l.flops for l in layers)
    b = sum(l.bytes for l in layers)
    t = sum(l.t for l in layers)
    hb = [l for l in layers if l.bytes / PEAK_HBM > l.flops / PEAK_MFMA]
    return dict(gflop=f / 1e9, gbytes=b / 1e9, t_roof_ms=t * 1e3, mfma_only_ms=f / PEAK_MFMA * 1e3,
                hbm_only_ms=b / PEAK_HBM * 1e3, hbm_bound_layers=len(hb), layers=len(layers),
                hbm_bound_t_ms=sum(l.t for l in hb) * 1e3, hbm_bound_gbytes=sum(l.bytes for l in hb) / 1e9)


CONFIGS = {
    2: dict(B=32, S=2, T=312, cfg=False, decode_only=False),
    4: dict(B=64, S=4, T=312, cfg=True, decode_only=False),
    5: dict(B=16, S=0, T=936, cfg=False, decode_only=True),
}


if __name__ == "__main__":
    for c, kw in CONFIGS.items():
        sm = summary(path_layers(**kw))
        audio = kw["B"] * kw["T"] * 2 * 256 / 16000
        print(f"C{c}: {sm['gflop']:.1f} GFLOP {sm['gbytes']:.2f} GB t_roof {sm['t_roof_ms']:.2f} ms "
              f"-> ideal {audio / sm['t_roof_ms'] * 1e3:.0f} audio-s/s  ({sm['hbm_bound_layers']}/{sm['layers']} "
              f"layers HBM-bound)")
        for st in ("dit", "vae", "bigvgan"):
            ls = [l for l in path_layers(**kw) if l.stage == st]
            if ls:
                s2 = summary(ls)
                print(f"   {st:8s} {s2['gflop']:10.1f} GFLOP {s2['gbytes']:7.2f} GB {s2['t_roof_ms']:7.3f} ms "
                      f"({s2['hbm_bound_layers']}/{s2['layers']} HBM-bound)")
