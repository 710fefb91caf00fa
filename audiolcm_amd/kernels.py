"""Thin torch-facing wrappers over the op-level C-ABI entry points.

Each function takes CUDA (HIP) fp32 tensors, allocates its output with torch,
and enqueues one or more libaudiolcm_hip kernels on the current stream.  They
are the per-op drop-ins for the ATen ops the reference path runs
(F.conv1d / conv_transpose1d / linear / group_norm / layer_norm / softmax,
Activation1d, LCMSampler.step) and are what the op-level parity tests call.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from . import _hip
from ._hip import check, lib, ptr, stream_handle

BK = 32


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _prec(split: bool, prec: Optional[int]) -> int:
    """MFMA operand precision code: explicit `prec` (_hip.PREC_*) or split -> PREC_SPLIT / PREC_BF16."""
    if prec is not None:
        assert prec in (_hip.PREC_BF16, _hip.PREC_SPLIT, _hip.PREC_F16, _hip.PREC_F16W2), prec
        return int(prec)
    return _hip.PREC_SPLIT if split else _hip.PREC_BF16


@dataclass
class PackedWeight:
    """[rows][Kpad] GEMM operand planes bf16 hi, bf16 lo, fp16 hi, fp16 lo (K index = tap*cpad + ci)."""
    data: torch.Tensor  # int16 (4, rows, kpad) on device
    rows: int
    cin: int
    cpad: int
    taps: int
    kpad: int

    @property
    def lo_off(self) -> int:
        return self.rows * self.kpad


def pack_conv_weight(w: torch.Tensor, transposed: bool = False, stride: int = 1, phase: int = 0) -> PackedWeight:
    """Pack Conv1d weight (Cout,Cin,K) — or ConvTranspose1d weight (Cin,Cout,K) for one phase."""
    assert w.is_cuda and w.dtype == torch.float32
    w = w.contiguous()
    if w.dim() == 2:
        w = w.unsqueeze(-1)
    if transposed:
        cin, cout, k = w.shape
        taps = k // stride
    else:
        cout, cin, k = w.shape
        taps = k
    cpad = _round_up(cin, 8)
    kpad = _round_up(taps * cpad, BK)
    out = torch.empty((4, cout, kpad), dtype=torch.int16, device=w.device)
    check(lib().alcm_pack_conv_weight(ptr(w), cout, cin, k, cpad, kpad, int(transposed), stride, phase, ptr(out),
                                      stream_handle()), "pack_conv_weight")
    return PackedWeight(out, cout, cin, cpad, taps, kpad)


def _act_operand(x: torch.Tensor, sb: int, st: int, sc: int, T_in: int, C_in: int, cpad: int, ksize: int, dil: int,
                 pad: int, up: int, rows_per_batch: int) -> _hip.Operand:
    o = _hip.Operand()
    o.kind = _hip.ALCM_OPND_ACT
    o.ptr = ptr(x)
    o.sb, o.st, o.sc = sb, st, sc
    o.T_in, o.C_in, o.Cpad, o.ksize, o.dil, o.pad, o.up = T_in, C_in, cpad, ksize, dil, pad, up
    o.rows_per_batch = rows_per_batch
    return o


def gemm(args: _hip.GemmArgs) -> None:
    check(lib().alcm_gemm(C.byref(args), stream_handle()), "alcm_gemm")


def conv1d(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, padding: int = 0,
           dilation: int = 1, upsample: int = 1, split: bool = True, channels_last: bool = False,
           act: int = 0, residual: Optional[torch.Tensor] = None, packed: Optional[PackedWeight] = None,
           prologue: Optional[dict] = None, window: bool = True, tile_n: int = 0,
           prec: Optional[int] = None) -> torch.Tensor:
    """F.conv1d(x, w, bias, padding=padding, dilation=dilation) on the MFMA implicit GEMM.

    x is (B, Cin, T) (reference NCT layout) or, with channels_last, (B, T, Cin); the result
    uses the same layout.  ``upsample=2`` applies nearest x2 to the input first
    (F.interpolate(scale_factor=2, mode='nearest'))."""
    pw = packed or pack_conv_weight(w)
    if channels_last:
        B, T, Cin = x.shape
        sb, st, sc = x.stride()
    else:
        B, Cin, T = x.shape
        sb, sc, st = x.stride()
    K = pw.taps
    Tu = T * upsample
    Tout = Tu + 2 * padding - dilation * (K - 1)
    assert Tout > 0
    g = _hip.GemmArgs()
    g.M, g.N, g.Kpad, g.batch, g.zdiv = B * Tout, pw.rows, pw.kpad, 1, 1
    g.a = _act_operand(x, sb, st, sc, T, Cin, pw.cpad, K, dilation, padding, upsample, Tout)
    if prologue:
        g.a.pro_scale = ptr(prologue.get("scale"))
        g.a.pro_shift = ptr(prologue.get("shift"))
        g.a.pro_sb = prologue.get("sb", 0)
        g.a.pro_mean = ptr(prologue.get("mean"))
        g.a.pro_rstd = ptr(prologue.get("rstd"))
        g.a.pro_act = prologue.get("act", 0)
    b = _hip.Operand()
    b.kind, b.ptr, b.rows, b.w_lo_off = _hip.ALCM_OPND_WEIGHT, ptr(pw.data), pw.rows, pw.lo_off
    g.b = b
    g.bias = ptr(bias)
    g.acc_scale, g.out_scale, g.act = 1.0, 1.0, act
    if channels_last:
        out = torch.empty((B, Tout, pw.rows), device=x.device, dtype=torch.float32)
        g.o_sb, g.o_st, g.o_sc = Tout * pw.rows, pw.rows, 1
    else:
        out = torch.empty((B, pw.rows, Tout), device=x.device, dtype=torch.float32)
        g.o_sb, g.o_st, g.o_sc = pw.rows * Tout, 1, Tout
    if residual is not None:
        assert residual.shape == out.shape
        r = residual
        g.res = ptr(r)
        if channels_last:
            g.r_sb, g.r_st, g.r_sc = r.stride()
        else:
            g.r_sb, g.r_sc, g.r_st = r.stride()
    g.out = ptr(out)
    g.out_rows_per_batch, g.out_step, g.out_off = Tout, 1, 0
    g.prec = _prec(split, prec)
    g.disable_window = int(not window)
    g.tile_n = tile_n
    gemm(g)
    return out


def conv_transpose1d(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], stride: int, padding: int,
                     split: bool = True, prec: Optional[int] = None) -> torch.Tensor:
    """F.conv_transpose1d on NCT input as ``stride`` phase convolutions."""
    B, Cin, T = x.shape
    _, Cout, K = w.shape
    assert K % stride == 0 and (K - stride) == 2 * padding, "polyphase form needs k = s*Q and pad = (k-s)/2"
    Q = K // stride
    Tout = T * stride
    out = torch.empty((B, Cout, Tout), device=x.device, dtype=torch.float32)
    sb, sc, st = x.stride()
    for r in range(stride):
        o = (r - padding) % stride
        c = (o + padding - r) // stride
        pw = pack_conv_weight(w, transposed=True, stride=stride, phase=r)
        g = _hip.GemmArgs()
        g.M, g.N, g.Kpad, g.batch, g.zdiv = B * T, Cout, pw.kpad, 1, 1
        g.a = _act_operand(x, sb, st, sc, T, Cin, pw.cpad, Q, 1, Q - 1 - c, 1, T)
        b = _hip.Operand()
        b.kind, b.ptr, b.rows, b.w_lo_off = _hip.ALCM_OPND_WEIGHT, ptr(pw.data), pw.rows, pw.lo_off
        g.b = b
        g.bias = ptr(bias)
        g.acc_scale, g.out_scale = 1.0, 1.0
        g.out = ptr(out)
        g.o_sb, g.o_st, g.o_sc = Cout * Tout, 1, Tout
        g.out_rows_per_batch, g.out_step, g.out_off = T, stride, o
        g.prec = _prec(split, prec)
        gemm(g)
    return out


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, split: bool = True,
           act: int = 0, prec: Optional[int] = None) -> torch.Tensor:
    """F.linear on (..., K) rows."""
    shp = x.shape
    x2 = x.reshape(-1, shp[-1]).contiguous()
    y = conv1d(x2.unsqueeze(0), w.unsqueeze(-1), bias, split=split, channels_last=True, act=act, prec=prec)
    return y.reshape(*shp[:-1], w.shape[0])


def bmm_nt(a: torch.Tensor, b: torch.Tensor, scale: float = 1.0, split: bool = True,
           prec: Optional[int] = None) -> torch.Tensor:
    """(Z, M, K) x (Z, N, K)^T -> (Z, M, N): the Q K^T product of attention."""
    Z, M, K = a.shape
    N = b.shape[1]
    assert K % 8 == 0 and a.is_contiguous() and b.is_contiguous()
    out = torch.empty((Z, M, N), device=a.device, dtype=torch.float32)
    g = _hip.GemmArgs()
    g.M, g.N, g.Kpad, g.batch, g.zdiv = M, N, _round_up(K, BK), Z, 1
    g.a = _act_operand(a, 0, K, 1, M, K, K, 1, 1, 0, 1, M)
    g.a.zs1 = M * K
    g.b = _act_operand(b, 0, K, 1, N, K, K, 1, 1, 0, 1, N)
    g.b.zs1 = N * K
    g.acc_scale, g.out_scale = scale, 1.0
    g.out = ptr(out)
    g.o_st, g.o_sc, g.o_zs1 = N, 1, M * N
    g.out_rows_per_batch, g.out_step = M, 1
    g.prec = _prec(split, prec)
    gemm(g)
    return out


def bmm_nn(p: torch.Tensor, v: torch.Tensor, split: bool = True, prec: Optional[int] = None) -> torch.Tensor:
    """(Z, M, K) x (Z, K, N) -> (Z, M, N): the P V product (V read N-contiguous)."""
    Z, M, K = p.shape
    N = v.shape[2]
    Kp = _round_up(K, 8)
    if Kp != K:
        p = torch.nn.functional.pad(p, (0, Kp - K))
    p = p.contiguous()
    v = v.contiguous()
    out = torch.empty((Z, M, N), device=p.device, dtype=torch.float32)
    g = _hip.GemmArgs()
    g.M, g.N, g.Kpad, g.batch, g.zdiv = M, N, _round_up(Kp, BK), Z, 1
    g.a = _act_operand(p, 0, Kp, 1, M, Kp, Kp, 1, 1, 0, 1, M)
    g.a.zs1 = M * Kp
    b = _hip.Operand()
    b.kind, b.ptr, b.st, b.sc, b.T_in, b.rows, b.zs1 = _hip.ALCM_OPND_ACT_T, ptr(v), N, 1, K, N, K * N
    g.b = b
    g.acc_scale, g.out_scale = 1.0, 1.0
    g.out = ptr(out)
    g.o_st, g.o_sc, g.o_zs1 = N, 1, M * N
    g.out_rows_per_batch, g.out_step = M, 1
    g.prec = _prec(split, prec)
    gemm(g)
    return out


def group_norm_affine(x_cl: torch.Tensor, groups: int, gamma: torch.Tensor, beta: torch.Tensor,
                      eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-(b, c) scale/shift equal to nn.GroupNorm on a channels-last (B, T, C) tensor."""
    B, T, Cc = x_cl.shape
    sb, st, sc = x_cl.stride()
    assert sc == 1
    scale = torch.empty((B, Cc), device=x_cl.device, dtype=torch.float32)
    shift = torch.empty_like(scale)
    check(lib().alcm_group_norm_affine(ptr(x_cl), B, T, Cc, sb, st, groups, eps, ptr(gamma), ptr(beta), ptr(scale),
                                       ptr(shift), stream_handle()), "group_norm_affine")
    return scale, shift


def row_stats(x: torch.Tensor, eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    rows = x.numel() // x.shape[-1]
    Cc = x.shape[-1]
    x = x.contiguous()
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    check(lib().alcm_row_stats(ptr(x), rows, Cc, Cc, eps, ptr(mean), ptr(rstd), stream_handle()), "row_stats")
    return mean, rstd


def layer_norm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    x = x.contiguous()
    Cc = x.shape[-1]
    rows = x.numel() // Cc
    y = torch.empty_like(x)
    check(lib().alcm_layer_norm(ptr(x), rows, Cc, Cc, eps, ptr(gamma), ptr(beta), None, 0, ptr(y), Cc,
                                stream_handle()), "layer_norm")
    return y


def softmax_(x: torch.Tensor) -> torch.Tensor:
    """In-place softmax over the last dim of a contiguous tensor."""
    n = x.shape[-1]
    rows = x.numel() // n
    check(lib().alcm_softmax_rows(ptr(x), rows, n, n, stream_handle()), "softmax_rows")
    return x


def snake_params(alpha: torch.Tensor, beta: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """SnakeBeta logscale parameters -> (exp(alpha), 1/(exp(beta)+1e-9)) (activations.py:111-119)."""
    return torch.exp(alpha), 1.0 / (torch.exp(beta) + 0.000000001)


def activation1d(x_cl: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor, up_filter: torch.Tensor,
                 down_filter: torch.Tensor) -> torch.Tensor:
    """Fused Activation1d(SnakeBeta) on a channels-last (B, T, C) tensor."""
    B, T, Cc = x_cl.shape
    x_cl = x_cl.contiguous()
    ae, ib = snake_params(alpha, beta)
    y = torch.empty_like(x_cl)
    fu = up_filter.detach().reshape(-1).float().cpu().contiguous()
    fd = down_filter.detach().reshape(-1).float().cpu().contiguous()
    check(lib().alcm_activation1d(ptr(x_cl), ptr(y), B, T, Cc, T * Cc, Cc, ptr(ae.contiguous()),
                                  ptr(ib.contiguous()), fu.data_ptr(), fd.data_ptr(), stream_handle()),
          "activation1d")
    return y


def lcm_step(x: torch.Tensor, eps: torch.Tensor, noise: Optional[torch.Tensor], coeffs) -> Tuple[torch.Tensor,
                                                                                                 torch.Tensor]:
    """LCMSampler.step (eps prediction).  coeffs = (sqrt_a, sqrt_b, c_out, c_skip, sqrt_a_prev, sqrt_b_prev)."""
    prev = torch.empty_like(x)
    den = torch.empty_like(x)
    arr = (C.c_float * 6)(*[float(c) for c in coeffs])
    check(lib().alcm_lcm_step(ptr(x), ptr(eps), ptr(noise), arr, ptr(prev), ptr(den), x.numel(), stream_handle()),
          "lcm_step")
    return prev, den


def sincos_embedding(v: torch.Tensor, freqs: torch.Tensor, scale: float, cos_first: bool) -> torch.Tensor:
    B = v.shape[0]
    half = freqs.numel()
    out = torch.empty((B, 2 * half), device=v.device, dtype=torch.float32)
    check(lib().alcm_sincos_embedding(ptr(v.float().contiguous()), scale, ptr(freqs), B, half, int(cos_first),
                                      ptr(out), stream_handle()), "sincos_embedding")
    return out


def operand_planes(x_cl: torch.Tensor, prec: int, Cp: Optional[int] = None) -> torch.Tensor:
    """(B, T, C) fp32 -> MFMA operand planes int16 (NP, B, T, Cp) as alcm_activation1d_op writes them
    (without the activation): fp16 for PREC_F16/F16W2, bf16 for PREC_BF16, bf16 hi/lo for PREC_SPLIT."""
    B, T, Cc = x_cl.shape
    Cp = Cp or _round_up(Cc, 32)
    x = torch.nn.functional.pad(x_cl.float(), (0, Cp - Cc))
    if prec in (_hip.PREC_F16, _hip.PREC_F16W2):
        return x.half().view(torch.int16).unsqueeze(0).contiguous()
    hi = x.bfloat16()
    if prec == _hip.PREC_BF16:
        return hi.view(torch.int16).unsqueeze(0).contiguous()
    lo = (x - hi.float()).bfloat16()
    return torch.stack([hi.view(torch.int16), lo.view(torch.int16)]).contiguous()


def activation1d_op(x_cl: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor, up_filter: torch.Tensor,
                    down_filter: torch.Tensor, prec: int, Cp: Optional[int] = None) -> torch.Tensor:
    """Activation1d of channels-last (B, T, C) into operand planes int16 (NP, B, T, Cp)."""
    B, T, Cc = x_cl.shape
    Cp = Cp or _round_up(Cc, 32)
    x_cl = x_cl.contiguous()
    ae, ib = snake_params(alpha, beta)
    ae, ib = ae.contiguous(), ib.contiguous()
    fu = up_filter.detach().reshape(-1).float().cpu().contiguous()
    fd = down_filter.detach().reshape(-1).float().cpu().contiguous()
    npl = 2 if prec == _hip.PREC_SPLIT else 1
    y = torch.empty((npl, B, T, Cp), dtype=torch.int16, device=x_cl.device)
    check(lib().alcm_activation1d_op(ptr(x_cl), ptr(y), B, T, Cc, Cp, ptr(ae), ptr(ib), fu.data_ptr(), fd.data_ptr(),
                                     int(prec), stream_handle()), "activation1d_op")
    return y


def activation1d_op_f16in(x16: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor, up_filter: torch.Tensor,
                          down_filter: torch.Tensor, prec: int) -> torch.Tensor:
    """Activation1d of an fp16 operand plane (1, B, T, C) int16 (an `opconv(..., out_plane=True)` result) into
    operand planes (1, B, T, C): alcm_activation1d_op_f16in (the wide-stage conv1 -> Activation1d hand-off)."""
    _, B, T, Cc = x16.shape
    assert x16.dtype == torch.int16 and x16.is_contiguous()
    ae, ib = snake_params(alpha, beta)
    ae, ib = ae.contiguous(), ib.contiguous()
    fu = up_filter.detach().reshape(-1).float().cpu().contiguous()
    fd = down_filter.detach().reshape(-1).float().cpu().contiguous()
    y = torch.empty((1, B, T, Cc), dtype=torch.int16, device=x16.device)
    check(lib().alcm_activation1d_op_f16in(ptr(x16), ptr(y), B, T, Cc, Cc, ptr(ae), ptr(ib), fu.data_ptr(),
                                           fd.data_ptr(), int(prec), stream_handle()), "activation1d_op_f16in")
    return y


def opconv_sum(terms, prec: int, out_scale: float = 1.0, accumulate_into: Optional[torch.Tensor] = None,
               out_plane: bool = False):
    """alcm_opconv_sum: out (B, T, N) = (sum over terms of conv_k(planes) + bias + residual) * out_scale (+ out) — the
    mean over a BigVGAN stage's resblocks at their last conv2 + residual (vocoder/bigvgan/models.py:190-199).
    terms: up to three (planes (1, B, T, Cp), w (N, C, k), bias or None, residual (B, T, N) or None, packed or None),
    same-length dilation-1 convs sharing B, T and N.  out_plane = True: the result as one PREC operand plane
    (1, B, T, N) instead (the one-launch form only, no accumulate)."""
    n = len(terms)
    assert 1 <= n <= 3
    args = (_hip.OpConvArgs * n)()
    keep = []
    out = None
    for i, (planes, w, bias, res, packed) in enumerate(terms):
        npl, B, T, Cp = planes.shape
        assert planes.dtype == torch.int16 and planes.is_contiguous()
        N, cin, k = w.shape
        if packed is None:
            wp = torch.nn.functional.pad(w, (0, 0, 0, Cp - cin)).contiguous() if Cp != cin else w
            packed = pack_conv_weight(wp)
        keep.append(packed)
        if out is None:
            out = accumulate_into if accumulate_into is not None else torch.empty((B, T, N), device=planes.device)
        a = args[i]
        a.a, a.a_lo_off, a.B, a.T, a.C, a.Cp = ptr(planes), B * T * Cp, B, T, cin, Cp
        a.ksize, a.dil, a.pad = k, 1, (k - 1) // 2
        a.w, a.w_lo_off, a.kpad, a.N = ptr(packed.data), packed.lo_off, packed.kpad, N
        a.bias = ptr(bias)
        if res is not None:
            res = res.contiguous()
            keep.append(res)
        a.res = ptr(res)
        a.prec = int(prec)
        if i == 0:
            a.out, a.out_scale, a.accumulate = ptr(out), out_scale, int(accumulate_into is not None)
            if out_plane:
                assert accumulate_into is None
                out = torch.empty((1, B, T, N), dtype=torch.int16, device=planes.device)
                a.out, a.out_plane = None, ptr(out)
    check(lib().alcm_opconv_sum(args, n, stream_handle()), "opconv_sum")
    return out


def opconv(planes: torch.Tensor, C_real: int, w: torch.Tensor, bias: Optional[torch.Tensor], dilation: int,
           prec: int, residual: Optional[torch.Tensor] = None, out_act: int = 0, out_scale: float = 1.0,
           accumulate_into: Optional[torch.Tensor] = None, packed: Optional["PackedWeight"] = None,
           act: Optional[tuple] = None, fp32_out: bool = True, geglu: bool = False,
           strided: Optional[tuple] = None, dense: bool = False, out_plane: bool = False,
           ksplit_ws: Optional[torch.Tensor] = None):
    """Same-length conv1d (B, T, N) = conv_{k,dilation}(operand planes (NP, B, T, Cp)) + bias (+res ...).

    act = (alpha, beta, up_filter, down_filter): also return Activation1d(conv + bias (+res)) as operand
    planes (NP, B, T, round_up(N, 32)) from the fused epilogue -> (out or None, planes).
    strided = (out, stride, offset, pad): one ConvTranspose1d phase, row t -> row t*stride + offset of the
    fp32 (B, R, N) tensor `out` (written in place and returned), input rows t - pad + tap*dilation.
    dense = True: the narrow-stage resident-weight kernel (alcm_opconv_dense): weights packed with cpad = C_real
    (pack_conv_weight(w)), planes channels >= C_real ignored, the fused Activation1d writes channels < N only.
    out_plane = True: conv + bias as one PREC operand plane (1, B, T, N) instead of the fp32 output (no residual /
    activation / accumulate; the DiT q,k,v projection).
    ksplit_ws: fp32 device workspace the library may use for K-split partial sums (alcm_opconv_args.ksplit_ws)."""
    npl, B, T, Cp = planes.shape
    assert planes.dtype == torch.int16 and planes.is_contiguous()
    N, cin, k = w.shape
    assert cin == C_real <= Cp
    if dense and packed is None:
        packed = pack_conv_weight(w)
    if packed is None:
        wp = torch.nn.functional.pad(w, (0, 0, 0, Cp - cin)).contiguous() if Cp != cin else w
        packed = pack_conv_weight(wp)
    a = _hip.OpConvArgs()
    a.a, a.a_lo_off, a.B, a.T, a.C, a.Cp = ptr(planes), B * T * Cp, B, T, C_real, Cp
    a.ksize, a.dil, a.pad = k, dilation, (k - 1) * dilation // 2
    a.w, a.w_lo_off, a.kpad, a.N = ptr(packed.data), packed.lo_off, packed.kpad, N
    a.bias = ptr(bias)
    if ksplit_ws is not None:
        assert ksplit_ws.dtype == torch.float32 and ksplit_ws.is_contiguous()
        a.ksplit_ws, a.ksplit_ws_floats = ptr(ksplit_ws), ksplit_ws.numel()
    if strided is not None:
        out, a.out_stride, a.out_offset, a.pad = strided
        assert out.is_contiguous() and out.shape[0] == B and out.shape[2] == N
        a.out, a.out_rows, a.out_scale, a.prec = ptr(out), out.shape[1], 1.0, int(prec)
        check(lib().alcm_opconv(C.byref(a), stream_handle()), "opconv")
        return out
    a.res = ptr(residual.contiguous()) if residual is not None else None
    if accumulate_into is not None:
        out = accumulate_into
    else:
        out = torch.empty((B, T, N), device=planes.device) if (fp32_out or act is None) else None
    a.out, a.out_act, a.accumulate, a.out_scale, a.prec = ptr(out), out_act, int(accumulate_into is not None), \
        out_scale, int(prec)
    keep = []
    if out_plane:
        op = torch.empty((1, B, T, N), dtype=torch.int16, device=planes.device)
        a.out, a.out_plane = None, ptr(op)
        check(lib().alcm_opconv(C.byref(a), stream_handle()), "opconv")
        return op
    if geglu:  # GEGLU epilogue (interleaved value/gate output columns) -> operand plane (1, B, T, N/2)
        gp = torch.empty((1, B, T, N // 2), dtype=torch.int16, device=planes.device)
        a.out, a.geglu_plane = None, ptr(gp)
        check(lib().alcm_opconv(C.byref(a), stream_handle()), "opconv")
        return gp
    if act is not None:
        alpha, beta, fu, fd = act
        ae, ib = snake_params(alpha, beta)
        ae, ib = ae.contiguous(), ib.contiguous()
        fu = fu.detach().reshape(-1).float().cpu().contiguous()
        fd = fd.detach().reshape(-1).float().cpu().contiguous()
        cpo = _round_up(N, 32)
        nplo = 2 if prec == _hip.PREC_SPLIT else 1
        # (dense=True writes channels < N only: zero planes keep the operand padding safe for any consumer)
        y = (torch.zeros if dense else torch.empty)((nplo, B, T, cpo), dtype=torch.int16, device=planes.device)
        keep = [ae, ib, fu, fd]
        a.act_plane, a.act_plane_lo_off = ptr(y), B * T * cpo
        a.act_alpha_exp, a.act_inv_beta = ptr(ae), ptr(ib)
        a.act_up_filter = fu.data_ptr()
        a.act_down_filter = fd.data_ptr()
    if dense:
        check(lib().alcm_opconv_dense(C.byref(a), stream_handle()), "opconv_dense")
    else:
        check(lib().alcm_opconv(C.byref(a), stream_handle()), "opconv")
    del keep
    if act is not None:
        return out, y
    return out


def flash_attention(qkv: torch.Tensor, heads: int, prec: int) -> torch.Tensor:
    """(B, L, 3H) fp32 [q | k | v] rows -> (B, L, H) multi-head softmax(q k^T / sqrt(dh)) v (fused kernel)."""
    B, L, H3 = qkv.shape
    H = H3 // 3
    qkv = qkv.contiguous()
    out = torch.empty((B, L, H), device=qkv.device)
    check(lib().alcm_flash_attention(ptr(qkv), ptr(out), B, L, H, heads, int(prec), stream_handle()),
          "flash_attention")
    return out


def layer_norm_plane(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, prec: int, eps: float = 1e-5):
    """LayerNorm over the last dim of (B, T, C) fp32 -> operand plane int16 (1, B, T, C) (fp16 or bf16 bits)."""
    B, T, Cc = x.shape
    x = x.contiguous()
    y = torch.empty((1, B, T, Cc), dtype=torch.int16, device=x.device)
    check(lib().alcm_layer_norm_plane(ptr(x), B * T, Cc, Cc, eps, ptr(gamma.contiguous()), ptr(beta.contiguous()),
                                      ptr(y), int(prec), stream_handle()), "layer_norm_plane")
    return y
