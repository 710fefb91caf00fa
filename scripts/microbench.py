#!/usr/bin/env python3
"""Per-kernel microbenchmarks on BigVGAN / DiT shapes (B=32), timed with torch CUDA events.

Used to A/B kernel variants in one process and as the target of rocprofv3 PMC passes:
    python scripts/microbench.py op         # Activation1d -> operand planes + plane conv per BigVGAN stage
    python scripts/microbench.py conv       # window conv, BigVGAN stage 0-2 / VAE / DiT FFN shapes
    python scripts/microbench.py act        # standalone Activation1d
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from audiolcm_amd import _hip, kernels as K  # noqa: E402
from audiolcm_amd.recipe import kaiser_sinc_filter1d  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def spin(seconds=3.0):
    """hold the GPU busy until its clocks settle: launches timed right after an idle period run up to 15 % slower
    than the same launches a few seconds later (measured: the first of five identical A/B variants)"""
    a = torch.randn((8192, 8192), device="cuda", dtype=torch.bfloat16)
    t0 = time.time()
    while time.time() - t0 < seconds:
        for _ in range(20):
            a @ a
        torch.cuda.synchronize()


def bench_conv(B=32):
    cases = [("bigvgan s0 k11d5", 2496, 768, 768, 11, 5), ("bigvgan s1 k7d3", 9984, 384, 384, 7, 3),
             ("bigvgan s2 k3d1", 19968, 192, 192, 3, 1), ("dit ffn0 k9", 467, 576, 4608, 9, 1),
             ("dit ffn2 k9", 467, 2304, 576, 9, 1), ("vae k3 1536", 312, 1536, 1536, 3, 1)]
    for name, T, Cin, Cout, k, d in cases:
        x = torch.randn((B, T, Cin), device="cuda")
        w = torch.randn((Cout, Cin, k), device="cuda") * (1 / (Cin * k) ** 0.5)
        pw = K.pack_conv_weight(w)
        for split in (True, False):
            for window, tn in ((True, 0), (True, 64), (True, 128), (False, 0)):
                ms = timeit(lambda: K.conv1d(x, w, None, padding=(k * d - d) // 2, dilation=d, split=split,
                                             channels_last=True, packed=pw, window=window, tile_n=tn), reps=3)
                tf = 2 * B * T * Cin * Cout * k / 1e12
                print(f"conv {name:18s} split={int(split)} window={int(window)} tn={tn:3d}: {ms:8.3f} ms "
                      f"{tf / ms * 1e3:7.1f} TF/s algorithmic ({tf / ms * 1e3 * (3 if split else 1) / 2500:5.1%} "
                      f"of 2.5 PF MFMA)")


def bench_act(B=32):
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    for C, T in ((768, 2496), (384, 9984), (24, 159744)):
        x = torch.randn((B, T, C), device="cuda")
        a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
        ms = timeit(lambda: K.activation1d(x, a, bt, f, f))
        print(f"act1d C={C} T={T}: {ms:.3f} ms {B * T * C * 8 / 1e9 / ms:.2f} TB/s")


def bench_conv_one(B=32, T=9984, C=384, k=7, d=3, split=True):
    """single window-conv configuration (target for rocprofv3 --pmc passes)"""
    x = torch.randn((B, T, C), device="cuda")
    w = torch.randn((C, C, k), device="cuda") * (1 / (C * k) ** 0.5)
    pw = K.pack_conv_weight(w)
    ms = timeit(lambda: K.conv1d(x, w, None, padding=(k * d - d) // 2, dilation=d, split=split, channels_last=True,
                                 packed=pw), reps=3)
    print(f"conv1 C={C} k={k}: {ms:.3f} ms {2 * B * T * C * C * k / 1e9 / ms:.1f} TF/s algorithmic")


def bench_op(B=32):
    """operand-format path: act_op (Activation1d -> planes) and opconv per BigVGAN stage shape"""
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    stages = [(768, 2496, 2), (384, 9984, 2), (192, 19968, 2), (96, 39936, 3), (48, 79872, 3), (24, 159744, 3)]
    for C, T, prec in stages:
        x = torch.randn((B, T, C), device="cuda")
        r = torch.randn((B, T, C), device="cuda")
        a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
        for p in ((prec, 1) if prec != 1 else (1,)):
            npl = 2 if p == 1 else 1
            cp = (C + 31) // 32 * 32
            gb = B * T * (C * 4 + cp * 2 * npl) / 1e9
            ms = timeit(lambda: K.activation1d_op(x, a, bt, f, f, p))
            print(f"act_op C={C:3d} prec={p}: {ms:7.3f} ms {gb / ms:6.2f} TB/s", flush=True)
            pl = K.activation1d_op(x, a, bt, f, f, p)
            for k, d in ((11, 5), (7, 3), (3, 1)):
                w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
                wp = torch.nn.functional.pad(w, (0, 0, 0, cp - C)).contiguous()
                pw = K.pack_conv_weight(wp)
                ms = timeit(lambda: K.opconv(pl, C, w, None, d, p, residual=r, packed=pw))
                tf = 2 * B * T * C * C * k / 1e12
                gb = B * T * (cp * 2 * npl + C * 8) / 1e9
                mf = {1: 3, 3: 2}.get(p, 1)
                print(f"  opconv C={C:3d} k={k:2d} d={d} prec={p}: {ms:7.3f} ms {tf / ms * 1e3:7.1f} TF/s alg "
                      f"({tf * mf / ms * 1e3 / 2500:5.1%} MFMA) {gb / ms:5.2f} TB/s", flush=True)


def bench_wconv(B=32):
    """wide conv (alcm_wconv.hip) vs the 128-row opconv_kernel on the BigVGAN stage 0-2 shapes"""
    for C, T in ((768, 2496), (384, 9984), (192, 19968)):
        x = torch.randn((B, T, C), device="cuda")
        r = torch.randn((B, T, C), device="cuda")
        for p in (2, 0):
            pl = K.operand_planes(x, p)
            for k, d in ((11, 5), (7, 3), (3, 1)):
                w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
                pw = K.pack_conv_weight(w)
                tf = 2 * B * T * C * C * k / 1e12
                outs, line = [], []
                for wc in os.environ.get("WCONV_VARS", "0,1").split(","):
                    os.environ["ALCM_WCONV"] = wc
                    _hip.reload_knobs()
                    ms = timeit(lambda: K.opconv(pl, C, w, None, d, p, residual=r, packed=pw))
                    outs.append(K.opconv(pl, C, w, None, d, p, residual=r, packed=pw))
                    line.append(f"wconv={wc} {ms:7.3f} ms {tf / ms * 1e3:7.1f} TF/s")
                os.environ.pop("ALCM_WCONV")
                _hip.reload_knobs()
                diff = max(float((outs[0] - o).abs().max()) for o in outs[1:])
                print(f"C={C:3d} k={k:2d} d={d} prec={p}: " + " | ".join(line) + f" | max|diff| {diff:.2e}", flush=True)


WIDE_SHAPES = [  # (name, T, Cin, N, k, dil, geglu, residual, accumulate) at B = 32
    ("s0 C768 k11", 2496, 768, 768, 11, 5, False, True, False), ("s0 C768 k3", 2496, 768, 768, 3, 1, False, True, True),
    ("s1 C384 k11", 9984, 384, 384, 11, 5, False, True, False), ("s1 C384 k3", 9984, 384, 384, 3, 1, False, True, True),
    ("s2 C192 k11", 19968, 192, 192, 11, 5, False, True, False), ("s2 C192 k3", 19968, 192, 192, 3, 1, False, True, True),
    ("dit ff0", 467, 576, 4608, 9, 1, True, False, False), ("dit ff2", 467, 2304, 576, 9, 1, False, True, False),
    ("dit qkv", 467, 576, 1728, 1, 1, False, False, False), ("dit out", 467, 576, 576, 1, 1, False, True, False),
    ("vae k3", 312, 1536, 1536, 3, 1, False, True, False)]


def bench_wone(B=32):
    """the WSHAPES wide-layer shapes, 5 launches each with the current ALCM_* settings (target of --pmc passes)"""
    sel = os.environ.get("WSHAPES", "s0 C768 k11")
    for name, T, Cin, N, k, d, gl, res, acc in WIDE_SHAPES:
        if not any(x in name for x in sel.split(",")):
            continue
        x = torch.randn((B, T, Cin), device="cuda")
        w = torch.randn((N, Cin, k), device="cuda") / (Cin * k) ** 0.5
        r = torch.randn((B, T, N), device="cuda") if res else None
        o = torch.zeros((B, T, N), device="cuda") if acc else None
        pw = K.pack_conv_weight(w)
        pl = K.operand_planes(x, 2)
        plane = os.environ.get("WONE_PLANE") == "1"  # the AMPBlock conv1 form: fp16 plane out, no residual
        for _ in range(5):
            if plane:
                K.opconv(pl, Cin, w, None, d, 2, packed=pw, out_plane=True)
            else:
                K.opconv(pl, Cin, w, None, d, 2, residual=r, packed=pw, accumulate_into=o)
        torch.cuda.synchronize()
        print(f"{name}: done", flush=True)


def bench_h16(B=32):
    """the wide stages' conv1 -> Activation1d hand-off: conv1 with an fp32 output + Activation1d of it vs conv1 with
    an fp16 plane output + the fp16-input Activation1d, per stage shape and conv1 kernel size"""
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    for C, T in ((768, 2496), (384, 9984), (192, 19968)):
        x = torch.randn((B, T, C), device="cuda")
        pl = K.operand_planes(x, 2)
        a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
        for k, d in ((11, 5), (7, 3), (3, 1)):
            w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
            b = torch.randn((C,), device="cuda") * 0.05
            pw = K.pack_conv_weight(w)
            t32 = timeit(lambda: K.opconv(pl, C, w, b, d, 2, packed=pw), reps=5)
            t16 = timeit(lambda: K.opconv(pl, C, w, b, d, 2, packed=pw, out_plane=True), reps=5)
            print(f"conv1 C={C:3d} k={k:2d} d={d}: fp32 out {t32:7.3f} ms | fp16 plane out {t16:7.3f} ms", flush=True)
        y32 = K.opconv(pl, C, w, b, 1, 2, packed=pw)
        y16 = K.opconv(pl, C, w, b, 1, 2, packed=pw, out_plane=True)
        ta32 = timeit(lambda: K.activation1d_op(y32, a, bt, f, f, 2), reps=10)
        ta16 = timeit(lambda: K.activation1d_op_f16in(y16, a, bt, f, f, 2), reps=10)
        gb32, gb16 = B * T * C * 6 / 1e9, B * T * C * 4 / 1e9
        print(f"act C={C:3d}: fp32 in {ta32:7.3f} ms ({gb32 / ta32:5.2f} TB/s) | fp16 in {ta16:7.3f} ms "
              f"({gb16 / ta16:5.2f} TB/s)", flush=True)


def bench_xp(B=32):
    """A/B of a scratch switch (XP_NAME=ALCM_XP0 by default, values XP_VALS) on the BigVGAN stage 0-2 AMPBlock conv2
    shapes as the model runs them (residual; the k = 3 resblock's last conv2 also accumulates), alternating, best of 3,
    with the outputs compared bit for bit"""
    name, vals = os.environ.get("XP_NAME", "ALCM_XP0"), os.environ.get("XP_VALS", "0,1").split(",")
    for C, T in ((768, 2496), (384, 9984), (192, 19968)):
        x = torch.randn((B, T, C), device="cuda")
        r = torch.randn((B, T, C), device="cuda")
        acc0 = torch.randn((B, T, C), device="cuda")
        pl = K.operand_planes(x, 2)
        for k, accum in ((11, False), (7, False), (3, False), (3, True)):
            w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
            b = torch.randn((C,), device="cuda") * 0.05
            pw = K.pack_conv_weight(w)
            tf = 2 * B * T * C * C * k / 1e12
            res, outs = {v: [] for v in vals}, {}
            for rep in range(3):
                for v in vals:
                    os.environ[name] = v
                    _hip.reload_knobs()
                    if accum:
                        o = acc0.clone()
                        fn = lambda: K.opconv(pl, C, w, b, 1, 2, residual=r, packed=pw, out_scale=1 / 3, accumulate_into=o)
                    else:
                        fn = lambda: K.opconv(pl, C, w, b, 1, 2, residual=r, packed=pw)
                    res[v].append(timeit(fn, reps=5))
                    if rep == 0:
                        if accum:
                            o = acc0.clone()
                            K.opconv(pl, C, w, b, 1, 2, residual=r, packed=pw, out_scale=1 / 3, accumulate_into=o)
                            outs[v] = o
                        else:
                            outs[v] = K.opconv(pl, C, w, b, 1, 2, residual=r, packed=pw)
            os.environ.pop(name)
            _hip.reload_knobs()
            same = all(torch.equal(outs[vals[0]], outs[v]) for v in vals[1:])
            line = " | ".join(f"{v}: {min(t):7.3f} ms {tf / min(t) * 1e3:6.0f} TF/s" for v, t in res.items())
            print(f"conv2 C={C:3d} k={k:2d}{' acc' if accum else '    '}: {line} | identical {same}", flush=True)


def bench_ffn(B=32):
    """DiT Conv1dFeedForward convs (L = 467 tokens): fp32-operand conv_kernel (LayerNorm prologue path) vs the
    wide-layer kernel on operand planes (GEGLU plane epilogue / residual epilogue)"""
    L, H, inner, k = 467, 576, 2304, 9
    x = torch.randn((B, L, H), device="cuda")
    g = torch.randn((B, L, inner), device="cuda")
    for name, xin, cin, cout, gl in (("ffn0", x, H, 2 * inner, True), ("ffn2", g, inner, H, False)):
        w = torch.randn((cout, cin, k), device="cuda") / (cin * k) ** 0.5
        b = torch.randn(cout, device="cuda") * 0.05
        pw = K.pack_conv_weight(w)
        pl = K.operand_planes(xin, 2)
        tf = 2 * B * L * cin * cout * k / 1e12
        ms0 = timeit(lambda: K.conv1d(xin, w, b, padding=k // 2, channels_last=True, packed=pw, prec=2), reps=3)
        if gl:
            ms1 = timeit(lambda: K.opconv(pl, cin, w, b, 1, 2, packed=pw, geglu=True), reps=3)
        else:
            ms1 = timeit(lambda: K.opconv(pl, cin, w, b, 1, 2, residual=x, packed=pw), reps=3)
        print(f"{name}: conv_kernel {ms0:.3f} ms ({tf / ms0 * 1e3:.0f} TF/s) | planes+wconv {ms1:.3f} ms "
              f"({tf / ms1 * 1e3:.0f} TF/s)", flush=True)


def bench_tail(B=32):
    """BigVGAN tail (C = 96/48/24) conv launches as the model runs them: conv1 (dilated) + fused Activation1d
    epilogue, conv2 + residual (+ fused Activation1d): opconv_kernel (ALCM_NCONV=0) vs nconv_kernel"""
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    for C, T, p in ((96, 39936, 2), (48, 79872, 3), (24, 159744, 3)):  # mixed-policy precisions
        x = torch.randn((B, T, C), device="cuda")
        r = torch.randn((B, T, C), device="cuda")
        a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
        pl = K.operand_planes(x, p)
        cp = (C + 31) // 32 * 32
        for k, d in ((11, 5), (3, 1)):
            w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
            pw = K.pack_conv_weight(torch.nn.functional.pad(w, (0, 0, 0, cp - C)).contiguous())
            line = []
            for v in os.environ.get("NCONV_VARS", "0,1").split(","):
                os.environ["ALCM_NCONV"] = v
                _hip.reload_knobs()
                ms1 = timeit(lambda: K.opconv(pl, C, w, None, d, p, packed=pw, act=(a, bt, f, f), fp32_out=False))
                ms2 = timeit(lambda: K.opconv(pl, C, w, None, d, p, residual=r, packed=pw, act=(a, bt, f, f)))
                ms3 = timeit(lambda: K.opconv(pl, C, w, None, d, p, residual=r, packed=pw))
                line.append(f"nconv{v}: act {ms1:6.3f} res+act {ms2:6.3f} res {ms3:6.3f}")
            os.environ.pop("ALCM_NCONV")
            _hip.reload_knobs()
            print(f"tail C={C:3d} k={k:2d} d={d} prec={p}: " + " | ".join(line), flush=True)


def bench_tconv(B=32):
    """resident-weight narrow conv (alcm_opconv_dense) vs opconv_kernel / nconv on the tail shapes as the model runs
    them (conv1 + fused Activation1d, conv2 + residual + fused Activation1d), with ALCM_TCONV_ABLATE variants
    (1 no epilogue, 2 no MFMA, 4 no window DMA; timing only)"""
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    sel = os.environ.get("TC_SHAPES", "96,48,24")
    for C, T, p in ((96, 39936, 2), (48, 79872, 3), (24, 159744, 3)):  # mixed-policy precisions
        if str(C) not in sel.split(","):
            continue
        x = torch.randn((B, T, C), device="cuda")
        r = torch.randn((B, T, C), device="cuda")
        a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
        pl = K.operand_planes(x, p)
        cp = (C + 31) // 32 * 32
        for k, d in ((11, 5), (3, 1)):
            w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
            pw = K.pack_conv_weight(torch.nn.functional.pad(w, (0, 0, 0, cp - C)).contiguous())
            pd = K.pack_conv_weight(w)
            line = []
            ms1 = timeit(lambda: K.opconv(pl, C, w, None, d, p, packed=pw, act=(a, bt, f, f), fp32_out=False))
            ms2 = timeit(lambda: K.opconv(pl, C, w, None, d, p, residual=r, packed=pw, act=(a, bt, f, f)))
            line.append(f"opconv: conv1+act {ms1:6.3f} conv2+res+act {ms2:6.3f}")
            for var in os.environ.get("VARS", "ALCM_TCONV=3,ALCM_TCONV=2").split(","):
                kv = dict(x.split("=") for x in var.split("+"))
                os.environ.update(kv)
                _hip.reload_knobs()
                ms1 = timeit(lambda: K.opconv(pl, C, w, None, d, p, packed=pd, act=(a, bt, f, f), fp32_out=False,
                                              dense=True))
                ms2 = timeit(lambda: K.opconv(pl, C, w, None, d, p, residual=r, packed=pd, act=(a, bt, f, f),
                                              dense=True))
                line.append(f"{'/'.join(kv.values())}: {ms1:6.3f} {ms2:6.3f}")
                for key in kv:
                    os.environ.pop(key)
            _hip.reload_knobs()
            print(f"tail C={C:3d} k={k:2d} d={d} prec={p}: " + " | ".join(line), flush=True)


def bench_tail1d(B=32):
    """3 launches of one dense narrow conv (alcm_opconv_dense) as the model runs it: TC channels, TK taps (dilation 5
    for k = 11, else 1), TMODE conv1 (fused Activation1d) / conv2 (+ residual, fp32 state, fused Activation1d), with
    the current ALCM_* settings (target of rocprofv3 --pmc passes)"""
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    C, k = int(os.environ.get("TC", "48")), int(os.environ.get("TK", "3"))
    T = {96: 39936, 48: 79872, 24: 159744}[C]
    d, p = (5 if k == 11 else 1), (2 if C == 96 else 3)
    x = torch.randn((B, T, C), device="cuda")
    r = torch.randn((B, T, C), device="cuda")
    a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
    pl = K.operand_planes(x, p)
    w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
    pd = K.pack_conv_weight(w)
    conv2 = os.environ.get("TMODE", "conv1") == "conv2"
    for _ in range(3):
        K.opconv(pl, C, w, None, d, p, residual=r if conv2 else None, packed=pd, act=(a, bt, f, f),
                 fp32_out=conv2, dense=True)
    torch.cuda.synchronize()


def bench_tphase(B=32):
    """per-phase shader-clock breakdown of the tail convs as the model runs them (ALCM_TCONV_TRACE=1, the diagnostics instantiations): cycles per tile
    per wave of [window + first slices, K loop, post-loop barrier, stage v, residual + fp32 out, Activation1d, final
    barrier]; TCONFIGS = C:k:mode,... (mode conv1 / conv2)"""
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    os.environ["ALCM_TCONV_TRACE"] = "1"
    _hip.reload_knobs()
    cfgs = os.environ.get("TCONFIGS", "96:3:conv2,96:11:conv2,96:11:conv1,48:3:conv2,48:11:conv2,24:3:conv2,24:11:conv2")
    for cfg in cfgs.split(","):
        C, k, mode = int(cfg.split(":")[0]), int(cfg.split(":")[1]), cfg.split(":")[2]
        T = {96: 39936, 48: 79872, 24: 159744}[C]
        d, p = (5 if k == 11 else 1), (2 if C == 96 else 3)
        x = torch.randn((B, T, C), device="cuda")
        r = torch.randn((B, T, C), device="cuda")
        a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
        pl = K.operand_planes(x, p)
        w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
        pd = K.pack_conv_weight(w)
        conv2 = mode == "conv2"
        run = lambda: K.opconv(pl, C, w, None, d, p, residual=r if conv2 else None, packed=pd, act=(a, bt, f, f),
                               fp32_out=conv2, dense=True)
        for xv in os.environ.get("XP_VALS", "0").split(","):
            os.environ[os.environ.get("XP_NAME", "ALCM_XP0")] = xv
            _hip.reload_knobs()
            run()
            _hip.debug_tconv_trace()
            ms = timeit(run, reps=5)
            v = _hip.debug_tconv_trace()
            tiles = max(v[7], 1)
            ph = " ".join(f"{x / tiles:7.0f}" for x in v[:7])
            print(f"tphase C={C:3d} k={k:2d} {mode} xp={xv}: {ms:6.3f} ms  cycles/tile/wave [win kloop bar stage res act "
                  f"bar] {ph}  sum {sum(v[:7]) / tiles:7.0f}  wave-tiles {v[7]}", flush=True)
        os.environ.pop(os.environ.get("XP_NAME", "ALCM_XP0"))
    os.environ.pop("ALCM_TCONV_TRACE")
    _hip.reload_knobs()


def bench_tres(B=32):
    """workgroup residency of the resident-weight tail conv (ALCM_TCONV_TRACE=1 records): for TCONFIGS = C:k:mode and
    each ALCM_TCONV in XP_VALS, how many workgroups were resident on one CU at once (max and mean over CUs), the
    spread of entry times and the launch span"""
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    os.environ["ALCM_TCONV_TRACE"] = "1"
    _hip.reload_knobs()
    _hip.debug_tconv_trace()
    for cfg in os.environ.get("TCONFIGS", "48:3:conv2,48:11:conv2").split(","):
        C, k, mode = int(cfg.split(":")[0]), int(cfg.split(":")[1]), cfg.split(":")[2]
        T = {96: 39936, 48: 79872, 24: 159744}[C]
        d, p = (5 if k == 11 else 1), (2 if C == 96 else 3)
        x = torch.randn((B, T, C), device="cuda")
        r = torch.randn((B, T, C), device="cuda")
        a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
        pl = K.operand_planes(x, p)
        w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
        pd = K.pack_conv_weight(w)
        conv2 = mode == "conv2"
        for xv in os.environ.get("XP_VALS", "1").split(","):
            os.environ["ALCM_TCONV"] = xv
            _hip.reload_knobs()
            run = lambda: K.opconv(pl, C, w, None, d, p, residual=r if conv2 else None, packed=pd, act=(a, bt, f, f),
                                   fp32_out=conv2, dense=True)
            _hip.debug_tconv_trace()  # reset: records of earlier (larger) grids cleared
            run()
            torch.cuda.synchronize()
            recs = [x for x in _hip.debug_tconv_wg_times(2048) if x[1] > x[0] > 0]
            if not recs:
                print(f"tres C={C} k={k} {mode} tconv={xv}: no records (streamed kernel?)", flush=True)
                continue
            t0 = min(x[0] for x in recs)
            per = {}
            for s_, e_, hw, xcc in recs:
                per.setdefault((xcc, (hw >> 8) & 0xFF), []).append((s_ - t0, e_ - t0))
            conc = []
            for iv in per.values():
                ev = sorted([(s_, 1) for s_, _ in iv] + [(e_, -1) for _, e_ in iv], key=lambda z: (z[0], z[1]))
                cur = best = 0
                for _, dlt in ev:
                    cur += dlt
                    best = max(best, cur)
                conc.append(best)
            span = max(x[1] for x in recs) - t0
            starts = sorted(x[0] - t0 for x in recs)
            print(f"tres C={C} k={k} {mode} tconv={xv}: {len(recs)} WGs on {len(per)} CUs, resident per CU max "
                  f"{max(conc)} mean {sum(conc) / len(conc):.2f}; entry spread {starts[-1] / 100:.1f} us (median "
                  f"{starts[len(starts) // 2] / 100:.1f}), launch span {span / 100:.1f} us", flush=True)
        os.environ.pop("ALCM_TCONV")
    os.environ.pop("ALCM_TCONV_TRACE")
    _hip.reload_knobs()


def bench_tail1(B=32):
    """3 launches of the stage-4 (C = 48, k = 11, d = 5, F16W2) conv2 + residual + fused Activation1d as the model
    runs it, with the current ALCM_* settings (target of rocprofv3 --pmc passes)"""
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    C, T, p, k, d = int(os.environ.get("TC", "48")), int(os.environ.get("TT", "79872")), 3, 11, 5
    x = torch.randn((B, T, C), device="cuda")
    r = torch.randn((B, T, C), device="cuda")
    a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
    pl = K.operand_planes(x, p)
    cp = (C + 31) // 32 * 32
    w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
    pw = K.pack_conv_weight(torch.nn.functional.pad(w, (0, 0, 0, cp - C)).contiguous())
    for _ in range(3):
        K.opconv(pl, C, w, None, d, p, residual=r, packed=pw, act=(a, bt, f, f))
    torch.cuda.synchronize()


def bench_text(B=32):
    """Text encoders (BERT-base + CLAP Projection + T5-v1.1-large, mixed policy) at the bench batch: per-kernel rows of
    one instrumented call (ALCM_PROF_SHAPES=1 splits them per shape) and the wall time per call."""
    from audiolcm_amd.text_encoder import CLAPT5TextEncoder
    enc = CLAPT5TextEncoder.from_recipe(0, split="mixed")
    g = torch.Generator().manual_seed(7)
    a = torch.randint(1, enc.cfg.b_vocab, (B, enc.cfg.max_len), generator=g)
    b = torch.randint(1, enc.cfg.t_vocab, (B, enc.cfg.max_len), generator=g)
    spin()
    ms = timeit(lambda: enc.encode_ids(a, b), reps=10)
    _hip.profile_begin()
    enc.encode_ids(a, b)
    torch.cuda.synchronize()
    rows = sorted(_hip.profile_end(), key=lambda r: -r["total_ms"])
    print(f"text encode B={B}: {ms:.3f} ms per call", flush=True)
    for r in rows[:40]:
        print(f"  {r['name'][:88]:88s} n={r['launches']:4d} {r['total_ms']:8.3f} ms  roof {r['roof_ms']:7.3f}", flush=True)


def bench_attn(B=32):
    """DiT self-attention at the bench shape (L = 467, 8 heads x 72), fp16 operands"""
    L, H = 467, 576
    qkv = torch.randn((B, L, 3 * H), device="cuda")
    ms = timeit(lambda: K.flash_attention(qkv, 8, 2), reps=20)
    print(f"attn B={B} L={L}: {ms * 1e3:.1f} us ({B * L * 3 * H * 4 / 1e9 / ms:.2f} TB/s of qkv)", flush=True)


def bench_act1(B=32):
    """one standalone Activation1d launch (C = 384 stage-1 shape, fp16 planes) and one fused tail conv (C = 96 k11,
    residual + Activation1d epilogue), 3 launches each (target of rocprofv3 --pmc passes)"""
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    x = torch.randn((B, 9984, 384), device="cuda")
    a, bt = torch.randn(384, device="cuda") * 0.3, torch.randn(384, device="cuda") * 0.3
    for _ in range(3):
        K.activation1d_op(x, a, bt, f, f, 2)
    C, T = 96, 39936
    x = torch.randn((B, T, C), device="cuda")
    r = torch.randn((B, T, C), device="cuda")
    a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
    pl = K.operand_planes(x, 2)
    w = torch.randn((C, C, 11), device="cuda") * (0.5 / (C * 11) ** 0.5)
    pw = K.pack_conv_weight(w)
    for _ in range(3):
        K.opconv(pl, C, w, None, 5, 2, residual=r, packed=pw, act=(a, bt, f, f))
    torch.cuda.synchronize()


def bench_op1(B=32):
    """one act_op + one opconv launch per tail/wide shape (target of rocprofv3 --pmc passes)"""
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    for C, T, prec, k, d in ((768, 2496, 2, 11, 5), (96, 39936, 3, 3, 1), (24, 159744, 3, 3, 1)):
        x = torch.randn((B, T, C), device="cuda")
        r = torch.randn((B, T, C), device="cuda")
        a, bt = torch.randn(C, device="cuda") * 0.3, torch.randn(C, device="cuda") * 0.3
        cp = (C + 31) // 32 * 32
        w = torch.randn((C, C, k), device="cuda") * (0.5 / (C * k) ** 0.5)
        pw = K.pack_conv_weight(torch.nn.functional.pad(w, (0, 0, 0, cp - C)).contiguous())
        for _ in range(2):
            pl = K.activation1d_op(x, a, bt, f, f, prec)
            K.opconv(pl, C, w, None, d, prec, residual=r, packed=pw)
        torch.cuda.synchronize()


if __name__ == "__main__":
    _hip.require_device(0)
    which = sys.argv[1:] or ["op", "conv", "act"]
    spin(float(os.environ.get("SPIN", "3")))
    for w in which:
        {"tres": bench_tres, "tphase": bench_tphase, "xp": bench_xp, "h16": bench_h16, "text": bench_text, "tail1d": bench_tail1d, "tconv": bench_tconv, "tail1": bench_tail1, "attn": bench_attn, "act1": bench_act1, "wone": bench_wone, "op": bench_op, "op1": bench_op1, "conv": bench_conv, "wconv": bench_wconv, "tail": bench_tail, "ffn": bench_ffn, "act": bench_act, "conv1": bench_conv_one}[w]()
