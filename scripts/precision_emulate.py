#!/usr/bin/env python3
"""CPU emulation of MFMA operand rounding in the BigVGAN vocoder (decides the per-stage precision policy).

Runs the oracle's ``bigvgan_forward`` in float64 with the conv operands (activation and/or weight)
rounded to bf16 / fp16 before each contraction — what an MFMA with fp32 accumulate sees — on the
e2e fixture's mel (tests/golden/e2e_S2_B2.npz, clip 0, first M frames), and prints the waveform
rel-L2 against the unrounded float64 run.  Policies are per layer group:
    pre   conv_pre       ups  ConvTranspose1d      wide  AMP convs of stages 0-2 (C=768/384/192)
    tail  AMP convs of stages 3-5 (C=96/48/24)     post conv_post
usage: python scripts/precision_emulate.py [M]
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiolcm_amd import recipe  # noqa: E402
from oracle import alcm_oracle as O  # noqa: E402

FMT = {"f32": None, "bf16": torch.bfloat16, "f16": torch.float16}


def rnd(t, fmt):
    return t if FMT[fmt] is None else t.to(FMT[fmt]).to(t.dtype)


def scaled_f16(w):
    # per-out-channel power-of-two scale so max|w| lands near 2^14 … exactly undone after the product
    m = w.abs().flatten(1).amax(1).clamp_min(1e-30)
    e = torch.floor(torch.log2(m))
    s = torch.pow(2.0, 10.0 - e).view(-1, *([1] * (w.dim() - 1)))
    return (w * s).to(torch.float16).to(w.dtype) / s


def run(W, mel, policy, wscale=False):
    """policy: dict group -> (act_fmt, w_fmt)."""
    state = {"group": "pre"}
    real_conv, real_convt = F.conv1d, F.conv_transpose1d

    def q(x, w, grp):
        if grp not in policy and grp in ("s3", "s4", "s5"):
            grp = "tail"  # per-stage tail groups fall back to the whole-tail policy
        a_f, w_f = policy.get(grp, ("f32", "f32"))
        w_r = scaled_f16(w) if (w_f == "f16" and wscale) else rnd(w, w_f)
        return rnd(x, a_f), w_r

    def fir(x, w, grp):  # Activation1d FIRs (depthwise): policy "fir" / "fir_<group>" = (input fmt, taps fmt)
        a_f, w_f = policy.get(f"fir_{grp}", policy.get("fir", ("f32", "f32")))
        return rnd(x, a_f), rnd(w, w_f)

    def conv1d(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        if groups == 1:
            x, w = q(x, w, state["group"])
        else:
            x, w = fir(x, w, state["group"])
        return real_conv(x, w, b, stride, padding, dilation, groups)

    def convt(x, w, b=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1):
        if groups != 1:
            x, w = fir(x, w, state["group"])
        if groups == 1:  # per-stage groups ups0 .. ups5 fall back to "ups"
            i = state["ups"] = state.get("ups", -1) + 1
            x, w = q(x, w, f"ups{i}" if f"ups{i}" in policy else "ups")
        return real_convt(x, w, b, stride, padding, output_padding, groups, dilation)

    ns = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith("_")})
    ns.conv1d, ns.conv_transpose1d = conv1d, convt
    real_amp = O.amp_block1

    def amp(Wd, p, x, k, d):
        i = int(p.split(".")[1]) // 3
        state["group"] = "wide" if i < 3 else f"s{i}"
        y = real_amp(Wd, p, x, k, d)
        state["group"] = "post"
        return y

    old_F, O.F, O.amp_block1 = O.F, ns, amp
    try:
        return O.bigvgan_forward(W, mel)
    finally:
        O.F, O.amp_block1 = old_F, real_amp


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    torch.set_num_threads(max(1, min(8, len(os.sched_getaffinity(0)))))
    W = {k: v.double() for k, v in recipe.bigvgan_state(0).items()}
    g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "e2e_S2_B2.npz"))
    mel = torch.from_numpy(g["mel"][:1, :, :M]).double()
    with torch.no_grad():
        ref = run(W, mel, {})
        groups = ("pre", "ups", "wide", "tail", "post")
        cases = {
            "all bf16": {k: ("bf16", "bf16") for k in groups},
            "all f16": {k: ("f16", "f16") for k in groups},
            "all f16, w only": {k: ("f32", "f16") for k in groups},
            "all f16, act only": {k: ("f16", "f32") for k in groups},
            "wide f16": {"wide": ("f16", "f16")},
            "wide f16 w only": {"wide": ("f32", "f16")},
            "wide+tail f16": {"wide": ("f16", "f16"), "tail": ("f16", "f16")},
            "wide+ups f16": {"wide": ("f16", "f16"), "ups": ("f16", "f16")},
            "tail f16": {"tail": ("f16", "f16")},
            "wide bf16": {"wide": ("bf16", "bf16")},
            "tail bf16": {"tail": ("bf16", "bf16")},
            "pre+ups+post bf16": {k: ("bf16", "bf16") for k in ("pre", "ups", "post")},
        }
        if len(sys.argv) > 2 and sys.argv[2] == "fir":  # Activation1d FIRs on fp16 MFMA operands (mixed policy base)
            wide_ups = {f"ups{i}": ("f16", "f16") for i in range(3)}
            base = dict({"wide": ("f16", "f16"), "tail": ("f16", "f32"), "s3": ("f16", "f16")}, **wide_ups)
            cases = {"mixed policy": base,
                     "mixed + FIR inputs f16": dict(base, fir=("f16", "f32")),
                     "mixed + FIR inputs+taps f16": dict(base, fir=("f16", "f16")),
                     "mixed + wide FIR inputs f16": dict(base, fir_wide=("f16", "f32")),
                     "mixed + tail FIR inputs f16": dict(base, **{f"fir_s{i}": ("f16", "f32") for i in (3, 4, 5)}),
                     "mixed + FIR inputs bf16": dict(base, fir=("bf16", "f32"))}
        if len(sys.argv) > 2 and sys.argv[2] == "tail":  # per-stage weight rounding of the tail (mixed policy base)
            base = {"wide": ("f16", "f16"), "tail": ("f16", "f32")}
            cases = {"mixed (tail F16W2)": base}
            for st in ("s3", "s4", "s5"):
                cases[f"mixed + {st} F16"] = dict(base, **{st: ("f16", "f16")})
            cases["mixed + s3,s4 F16"] = dict(base, s3=("f16", "f16"), s4=("f16", "f16"))
            base2 = dict(base, s3=("f16", "f16"))
            cases["mixed(s3 F16) + ups F16W2"] = dict(base2, ups=("f16", "f32"))
            cases["mixed(s3 F16) + ups F16"] = dict(base2, ups=("f16", "f16"))
            cases["mixed(s3 F16) + pre F16W2"] = dict(base2, pre=("f16", "f32"))
            cases["mixed(s3 F16) + ups bf16"] = dict(base2, ups=("bf16", "bf16"))
            wide_ups = {f"ups{i}": ("f16", "f16") for i in range(3)}
            cases["mixed(s3 F16) + ups0-2 F16"] = dict(base2, **wide_ups)
            cases["mixed(s3 F16) + ups0-2 F16, ups3-5 F16W2"] = dict(base2, ups=("f16", "f32"), **wide_ups)
            cases["mixed(s3 F16) + ups0-3 F16"] = dict(base2, ups3=("f16", "f16"), **wide_ups)
        if len(sys.argv) > 2 and sys.argv[2] == "ups45":  # stage 4-5 upsamplers on fp16 activations (current mixed base)
            base = dict({"wide": ("f16", "f16"), "tail": ("f16", "f32"), "s3": ("f16", "f16"), "fir_wide": ("f16", "f32")},
                        **{f"ups{i}": ("f16", "f16") for i in range(4)})
            cases = {"mixed policy (round 4)": base,
                     "mixed + ups4 F16W2": dict(base, ups4=("f16", "f32")),
                     "mixed + ups5 F16W2": dict(base, ups5=("f16", "f32")),
                     "mixed + ups4,5 F16W2": dict(base, ups4=("f16", "f32"), ups5=("f16", "f32")),
                     "mixed + ups4,5 bf16x3-free F16": dict(base, ups4=("f16", "f16"), ups5=("f16", "f16"))}
        for name, pol in cases.items():
            for ws in ((False, True) if any(v[1] == "f16" for v in pol.values()) else (False,)):
                out = run(W, mel, pol, wscale=ws)
                err = float((out - ref).norm() / ref.norm())
                print(f"{name:22s} wscale={int(ws)}  wav rel-L2 {err:.2e}", flush=True)




def run_latent_mel(policy, Wd, Wv, ctx, xT, noise):
    """DiT sampler + VAE decode in float64 with conv/linear operands rounded per policy:
    policy keys: 'dit_ffn' (k=9 GEGLU convs), 'dit_other' (all other DiT convs/linears),
    'vae_conv' (k=3 ResnetBlock/upsample convs), 'vae_other'."""
    state = {"model": "dit"}
    real_conv, real_lin = F.conv1d, F.linear

    def grp(w):
        if state["model"] == "dit":
            return "dit_ffn" if (w.dim() == 3 and w.shape[-1] == 9) else "dit_other"
        return "vae_conv" if (w.dim() == 3 and w.shape[-1] == 3) else "vae_other"

    def conv1d(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        a_f, w_f = policy.get(grp(w), ("f32", "f32"))
        return real_conv(rnd(x.to(w.dtype), a_f), rnd(w, w_f), b, stride, padding, dilation, groups)

    def linear(x, w, b=None):
        a_f, w_f = policy.get(grp(w), ("f32", "f32"))
        return real_lin(rnd(x.to(w.dtype), a_f), rnd(w, w_f), b)

    ns = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith("_")})
    ns.conv1d, ns.linear = conv1d, linear
    old_F, O.F = O.F, ns
    try:
        eps_fn = lambda x, t, w: O.dit_forward(Wd, x, t, ctx, w)
        z = O.lcm_sample(eps_fn, ctx, xT, noise, 2, 5.0)
        state["model"] = "vae"
        mel = O.vae_decode(Wv, z)
    finally:
        O.F = old_F
    return z, mel


def main_dit_vae():
    torch.set_num_threads(max(1, min(8, len(os.sched_getaffinity(0)))))
    Wd = {k: v.double() for k, v in recipe.dit_state(0).items()}
    Wv = {k: v.double() for k, v in recipe.vae_state(0).items()}
    g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "e2e_S2_B2.npz"))
    ctx = recipe.synthetic_context(2).double()
    xT, noise = torch.from_numpy(g["x_T"]).double(), torch.from_numpy(g["noise"]).double()
    with torch.no_grad():
        z0, m0 = run_latent_mel({}, Wd, Wv, ctx, xT, noise)
        print(f"fp64 vs fixture: latent {float((z0.float() - torch.from_numpy(g['latent'])).norm() / z0.norm()):.2e}")
        cases = {
            "dit ffn f16": {"dit_ffn": ("f16", "f16")},
            "dit ffn bf16": {"dit_ffn": ("bf16", "bf16")},
            "dit other f16": {"dit_other": ("f16", "f16")},
            "dit all f16": {"dit_ffn": ("f16", "f16"), "dit_other": ("f16", "f16")},
            "vae conv f16": {"vae_conv": ("f16", "f16")},
            "vae all f16": {"vae_conv": ("f16", "f16"), "vae_other": ("f16", "f16")},
            "dit ffn + vae conv f16": {"dit_ffn": ("f16", "f16"), "vae_conv": ("f16", "f16")},
        }
        for name, pol in cases.items():
            z, m = run_latent_mel(pol, Wd, Wv, ctx, xT, noise)
            print(f"{name:26s} latent {float((z - z0).norm() / z0.norm()):.2e}  mel {float((m - m0).norm() / m0.norm()):.2e}",
                  flush=True)


def run_dit_groups(policy, Wd, ctx, xT, noise):
    """DiT sampler only (float64), operands rounded per group: 'ffn', 'qkv' (to_q/k/v), 'out' (to_out),
    'proj' (TemporalTransformer proj_in/out 1x1), 'emb' (embedders, proj_in k5, final layer),
    'attn' (QK^T and PV products)."""
    real_conv, real_lin, real_einsum = F.conv1d, F.linear, torch.einsum

    def grp_w(w):
        if w.dim() == 3 and w.shape[-1] == 9:
            return "ffn"
        if w.dim() == 3 and w.shape[-1] == 1 and w.shape[0] == w.shape[1] == 576:
            return "proj"
        if w.dim() == 2 and w.shape == (576, 576):
            return "qkv_or_out"
        return "emb"

    def conv1d(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        a_f, w_f = policy.get(grp_w(w), ("f32", "f32"))
        return real_conv(rnd(x.to(w.dtype), a_f), rnd(w, w_f), b, stride, padding, dilation, groups)

    def linear(x, w, b=None):
        g = grp_w(w)
        if g == "qkv_or_out":
            g = "out" if b is not None else "qkv"
        a_f, w_f = policy.get(g, ("f32", "f32"))
        return real_lin(rnd(x.to(w.dtype), a_f), rnd(w, w_f), b)

    def einsum(eq, a, b):
        a_f, b_f = policy.get("attn", ("f32", "f32"))
        return real_einsum(eq, rnd(a, a_f), rnd(b, b_f))

    ns = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith("_")})
    ns.conv1d, ns.linear = conv1d, linear
    tns = types.SimpleNamespace(**{k: getattr(torch, k) for k in dir(torch) if not k.startswith("__")})
    tns.einsum = einsum
    old_F, old_t = O.F, O.torch
    O.F, O.torch = ns, tns
    try:
        eps_fn = lambda x, t, w: O.dit_forward(Wd, x, t, ctx, w)
        return O.lcm_sample(eps_fn, ctx, xT, noise, 2, 5.0)
    finally:
        O.F, O.torch = old_F, old_t


def main_dit_groups():
    torch.set_num_threads(max(1, min(8, len(os.sched_getaffinity(0)))))
    Wd = {k: v.double() for k, v in recipe.dit_state(0).items()}
    g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "e2e_S2_B2.npz"))
    ctx = recipe.synthetic_context(2).double()
    xT, noise = torch.from_numpy(g["x_T"]).double(), torch.from_numpy(g["noise"]).double()
    with torch.no_grad():
        z0 = run_dit_groups({}, Wd, ctx, xT, noise)
        f16, a16 = ("f16", "f16"), ("f16", "f32")
        cases = {"attn f16": {"attn": f16}, "attn bf16": {"attn": ("bf16", "bf16")},
                 "qkv f16": {"qkv": f16}, "qkv act-f16": {"qkv": a16}, "out f16": {"out": f16},
                 "out act-f16": {"out": a16}, "proj f16": {"proj": f16}, "proj act-f16": {"proj": a16},
                 "emb f16": {"emb": f16}, "emb act-f16": {"emb": a16},
                 "ffn+attn f16 + qkv/out/proj act-f16": {"ffn": f16, "attn": f16, "qkv": a16, "out": a16,
                                                         "proj": a16}}
        for name, pol in cases.items():
            z = run_dit_groups(pol, Wd, ctx, xT, noise)
            print(f"{name:40s} latent {float((z - z0).norm() / z0.norm()):.2e}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "ditvae":
        main_dit_vae()
    elif len(sys.argv) > 1 and sys.argv[1] == "dit":
        main_dit_groups()
    else:
        main()

