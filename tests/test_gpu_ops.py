"""Op-level parity of the HIP kernels (through the C-ABI) against plain fp32 PyTorch on CPU.

Tolerances: split (bf16x3) MFMA mode is fp32-accurate -> relative L2 <= 2e-5;
plain bf16 MFMA mode -> relative L2 <= 1.5e-2; fp16 MFMA mode (prec=2) -> relative L2 <= 2e-3.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden, rel_l2

pytestmark = pytest.mark.gpu

SPLIT_TOL = 2e-5
BF16_TOL = 1.5e-2
F16_TOL = 2e-3
PRECS = [1, 0, 2]                     # _hip.PREC_SPLIT, PREC_BF16, PREC_F16
TOL = {1: SPLIT_TOL, 0: BF16_TOL, 2: F16_TOL, 3: F16_TOL}


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from audiolcm_amd import _hip, kernels
    _hip.require_device(0)
    return kernels


def _r(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g) * scale


def dev(t):
    return t.cuda()


@pytest.mark.parametrize("B,Cin,T,Cout,k,pad,dil,cl", [
    (2, 24, 50, 40, 3, 1, 1, False),     # NCT (scalar loader), generic N tile
    (2, 64, 37, 130, 9, 4, 1, True),     # vector loader, ragged M/N tiles, FFN-like k9
    (1, 24, 300, 24, 11, 25, 5, True),   # BigVGAN tail: N=24 (256x32 tile), dilation 5
    (3, 48, 129, 48, 7, 9, 3, True),     # N=48 (256x64 tile), dilation 3
    (2, 20, 33, 576, 5, 2, 1, False),    # DiT proj_in: 20 channels (padded K)
    (1, 24, 64, 1, 7, 3, 1, True),       # conv_post: N=1
    (2, 80, 16, 1536, 7, 3, 1, False),   # conv_pre from NCT mel
    (2, 96, 300, 130, 11, 25, 5, True),  # window-conv: k11 d5, 3 row tiles per batch, ragged N
    (3, 64, 129, 48, 7, 9, 3, True),     # window-conv, BN=64 tile, T not a tile multiple
    (1, 32, 5, 64, 3, 1, 1, True),       # window-conv, T shorter than the halo
])
@pytest.mark.parametrize("prec", PRECS)
def test_conv1d(K, B, Cin, T, Cout, k, pad, dil, cl, prec):
    x = _r((B, Cin, T), 1)
    w = _r((Cout, Cin, k), 2, 1.0 / np.sqrt(Cin * k))
    b = _r((Cout,), 3, 0.1)
    ref = F.conv1d(x, w, b, padding=pad, dilation=dil)
    xin = x.permute(0, 2, 1).contiguous() if cl else x
    y = K.conv1d(dev(xin), dev(w), dev(b), padding=pad, dilation=dil, prec=prec, channels_last=cl).cpu()
    if cl:
        y = y.permute(0, 2, 1)
    assert y.shape == ref.shape
    assert rel_l2(y.numpy(), ref.numpy()) < TOL[prec]


@pytest.mark.parametrize("prec", PRECS)
def test_window_conv_matches_tap_loader(K, prec):
    """The window-conv kernel and the tap-by-tap implicit GEMM give the same result (same bf16 operands)."""
    x = _r((2, 300, 128), 40)
    w = _r((192, 128, 7), 41, 0.03)
    b = _r((192,), 42, 0.1)
    y1 = K.conv1d(dev(x), dev(w), dev(b), padding=9, dilation=3, prec=prec, channels_last=True)
    y2 = K.conv1d(dev(x), dev(w), dev(b), padding=9, dilation=3, prec=prec, channels_last=True, window=False)
    assert rel_l2(y1.cpu().numpy(), y2.cpu().numpy()) < (1e-6 if prec == 1 else 1e-5)


def test_conv1d_upsample_nearest(K):
    x = _r((2, 768 // 8, 20), 4)
    w = _r((64, 96, 3), 5, 0.1)
    b = _r((64,), 6, 0.1)
    ref = F.conv1d(F.interpolate(x, scale_factor=2.0, mode="nearest"), w, b, padding=1)
    y = K.conv1d(dev(x.permute(0, 2, 1).contiguous()), dev(w), dev(b), padding=1, upsample=2,
                 channels_last=True).cpu().permute(0, 2, 1)
    assert rel_l2(y.numpy(), ref.numpy()) < SPLIT_TOL


def test_conv1d_groupnorm_swish_prologue_and_residual(K):
    B, T, Cc, Co = 2, 45, 64, 96
    x = _r((B, Cc, T), 7, 2.0) + 0.5
    gam, bet = 1 + _r((Cc,), 8, 0.1), _r((Cc,), 9, 0.1)
    w, b = _r((Co, Cc, 3), 10, 0.08), _r((Co,), 11, 0.1)
    res = _r((B, Co, T), 12)
    h = F.group_norm(x, 32, gam, bet, 1e-6)
    ref = F.conv1d(h * torch.sigmoid(h), w, b, padding=1) + res
    xc = dev(x.permute(0, 2, 1).contiguous())
    sc, sh = K.group_norm_affine(xc, 32, dev(gam), dev(bet), 1e-6)
    y = K.conv1d(xc, dev(w), dev(b), padding=1, channels_last=True,
                 residual=dev(res.permute(0, 2, 1).contiguous()),
                 prologue=dict(scale=sc, shift=sh, sb=Cc, act=1)).cpu().permute(0, 2, 1)
    assert rel_l2(y.numpy(), ref.numpy()) < SPLIT_TOL


def test_conv1d_layernorm_prologue(K):
    B, T, Cc = 2, 31, 64
    x = _r((B, T, Cc), 13, 3.0) + 1.0
    gam, bet = 1 + _r((Cc,), 14, 0.1), _r((Cc,), 15, 0.1)
    w, b = _r((128, Cc, 9), 16, 0.05), _r((128,), 17, 0.1)
    ln = F.layer_norm(x, (Cc,), gam, bet, 1e-5)
    ref = F.conv1d(ln.permute(0, 2, 1), w, b, padding=4)
    xd = dev(x)
    mean, rstd = K.row_stats(xd, 1e-5)
    y = K.conv1d(xd, dev(w), dev(b), padding=4, channels_last=True,
                 prologue=dict(scale=dev(gam), shift=dev(bet), sb=0, mean=mean, rstd=rstd)).cpu().permute(0, 2, 1)
    assert rel_l2(y.numpy(), ref.numpy()) < SPLIT_TOL


@pytest.mark.parametrize("Cin,Cout,k,s", [(64, 32, 8, 4), (48, 24, 4, 2), (1536 // 16, 768 // 16, 8, 4)])
def test_conv_transpose1d(K, Cin, Cout, k, s):
    x = _r((2, Cin, 19), 18)
    w = _r((Cin, Cout, k), 19, 1.0 / np.sqrt(Cin * k / s))
    b = _r((Cout,), 20, 0.1)
    ref = F.conv_transpose1d(x, w, b, stride=s, padding=(k - s) // 2)
    y = K.conv_transpose1d(dev(x), dev(w), dev(b), s, (k - s) // 2).cpu()
    assert y.shape == ref.shape
    assert rel_l2(y.numpy(), ref.numpy()) < SPLIT_TOL


@pytest.mark.parametrize("Z,L,d", [(4, 467, 72), (2, 40, 1536)])
def test_attention_products(K, Z, L, d):
    q, k, v = _r((Z, L, d), 21), _r((Z, L, d), 22), _r((Z, L, d), 23)
    sim = torch.einsum("bid,bjd->bij", q, k) * d ** -0.5
    s = K.bmm_nt(dev(q), dev(k), d ** -0.5).cpu()
    assert rel_l2(s.numpy(), sim.numpy()) < SPLIT_TOL
    p = sim.softmax(-1)
    pd = K.softmax_(dev(sim.clone())).cpu()
    np.testing.assert_allclose(pd.numpy(), p.numpy(), rtol=1e-5, atol=1e-7)
    o = K.bmm_nn(dev(p), dev(v)).cpu()
    assert rel_l2(o.numpy(), torch.einsum("bij,bjd->bid", p, v).numpy()) < SPLIT_TOL


@pytest.mark.parametrize("B,L,heads,dh", [(2, 467, 8, 72), (1, 40, 8, 72), (3, 130, 4, 64), (1, 1, 2, 36), (2, 512, 8, 72),
                                          (1, 700, 8, 72)])
@pytest.mark.parametrize("prec", [2, 0])
def test_flash_attention(K, B, L, heads, dh, prec):
    """Fused attention (online softmax, scores on chip) vs fp32 softmax(q k^T / sqrt(dh)) v: the resident-K/V kernel
    (L <= 512) and the 64-query tiled kernel (L = 700)."""
    H = heads * dh
    qkv = _r((B, L, 3 * H), 100, 1.5)
    q, k, v = qkv.split(H, dim=-1)
    sh = lambda t: t.reshape(B, L, heads, dh).permute(0, 2, 1, 3)
    att = torch.softmax(sh(q) @ sh(k).transpose(-1, -2) / dh ** 0.5, dim=-1) @ sh(v)
    ref = att.permute(0, 2, 1, 3).reshape(B, L, H)
    y = K.flash_attention(dev(qkv), heads, prec).cpu()
    assert rel_l2(y.numpy(), ref.numpy()) < TOL[prec]


@pytest.mark.parametrize("prec", [2, 0])
@pytest.mark.parametrize("L", [300, 700])
def test_feedforward_on_planes(K, prec, L):
    """DiT Conv1dFeedForward on operand planes: LayerNorm -> plane, conv k9 with the GEGLU plane epilogue
    (interleaved value/gate columns), conv k9 + residual — vs fp32 F.conv1d / F.gelu.  L = 700 (1400 rows)
    puts the 2304 -> 576 conv on the wide-layer kernel, as at the bench's B = 32 (alcm_wconv.hip)."""
    B, H, inner, k = 2, 576, 2304, 9
    x = _r((B, L, H), 110)
    gam, bet = 1 + _r((H,), 111, 0.1), _r((H,), 112, 0.1)
    w0, b0 = _r((2 * inner, H, k), 113, 1 / np.sqrt(H * k)), _r((2 * inner,), 114, 0.05)
    w2, b2 = _r((H, inner, k), 115, 1 / np.sqrt(inner * k)), _r((H,), 116, 0.05)
    h = F.layer_norm(x, (H,), gam, bet, 1e-5)
    y0 = F.conv1d(h.permute(0, 2, 1), w0, b0, padding=k // 2)
    val, gate = y0.chunk(2, dim=1)
    gg = val * F.gelu(gate)
    ref = (F.conv1d(gg, w2, b2, padding=k // 2) + x.permute(0, 2, 1)).permute(0, 2, 1)
    p1 = K.layer_norm_plane(dev(x), dev(gam), dev(bet), prec)
    dec = (lambda p: p.view(torch.float16).float()) if prec == 2 else (lambda p: p.view(torch.bfloat16).float())
    assert rel_l2(dec(p1[0].cpu()).numpy(), h.numpy()) < (1e-3 if prec == 2 else 6e-3)
    wi = torch.stack([w0[:inner], w0[inner:]], 1).reshape(2 * inner, H, k)   # rows (value j, gate j)
    bi = torch.stack([b0[:inner], b0[inner:]], 1).reshape(2 * inner)
    p2 = K.opconv(p1, H, dev(wi), dev(bi), 1, prec, geglu=True)
    assert rel_l2(dec(p2[0].cpu()).numpy(), gg.permute(0, 2, 1).numpy()) < TOL[prec]
    y = K.opconv(p2, inner, dev(w2), dev(b2), 1, prec, residual=dev(x)).cpu()
    assert rel_l2(y.numpy(), ref.numpy()) < TOL[prec]


@pytest.mark.parametrize("N,rows", [(1728, 600), (1728, 1400), (576, 600), (576, 1400), (576, 2 * 4 * 467)])
@pytest.mark.parametrize("prec", [0, 2])
def test_opconv_dit_projection_shapes(K, N, rows, prec):
    """The DiT attention projections on operand planes: fused q/k/v (576 -> 1728, k = 1) and to_out (576 -> 576,
    + bias + residual) at row counts below (opconv_kernel) and above (wide-layer kernel) the 1024-row switch,
    up to the bench's B = 32 x 467 rows divided over several launches' worth (3736 rows)."""
    B, H = 2, 576
    L = rows // B
    x = _r((B, L, H), 130)
    w, bias = _r((N, H, 1), 131, 1 / np.sqrt(H)), _r((N,), 132, 0.05)
    r = _r((B, L, N), 133)
    ref = F.conv1d(x.permute(0, 2, 1), w, bias).permute(0, 2, 1) + r
    pl = K.operand_planes(dev(x), prec)
    y = K.opconv(pl, H, dev(w), dev(bias), 1, prec, residual=dev(r)).cpu()
    assert rel_l2(y.numpy(), ref.numpy()) < TOL[prec]


def test_group_norm_stats_large_mean(K):
    """One-pass (fp64 sum / sum of squares) GroupNorm statistics on data whose mean is 1e4 x its standard
    deviation (the cancellation case of E[x^2] - mean^2): the normalised output matches F.group_norm."""
    B, C, T = 2, 32, 3200   # 1e5 elements per (b, group) with 2 groups
    xf = (_r((B, C, T), 140, 0.1).double() + 1e3).float()
    g, b = 1 + _r((C,), 141, 0.1), _r((C,), 142, 0.1)
    ref = F.group_norm(xf.double(), 2, g.double(), b.double(), 1e-6)
    sc, sh = K.group_norm_affine(dev(xf.permute(0, 2, 1).contiguous()), 2, dev(g), dev(b), 1e-6)
    y = xf.double() * sc.cpu().double()[:, :, None] + sh.cpu().double()[:, :, None]
    # the fp32 scale (~10) and shift (~-1e4) carry ~1e-3 absolute rounding on y = x*scale + shift; an fp32
    # one-pass variance would be off by ~0.06 against the true 0.01 (y wrong by O(1))
    assert (y - ref).abs().max().item() < 3e-3


def test_linear_and_layer_norm(K):
    x = _r((3, 77, 1024), 24)
    w, b = _r((576, 1024), 25, 1 / 32.0), _r((576,), 26, 0.1)
    y = K.linear(dev(x), dev(w), dev(b), act=3).cpu()
    assert rel_l2(y.numpy(), F.gelu(F.linear(x, w, b), approximate="tanh").numpy()) < SPLIT_TOL
    g, be = 1 + _r((576,), 27, 0.1), _r((576,), 28, 0.1)
    ln = K.layer_norm(dev(y), dev(g), dev(be), 1e-5).cpu()
    ref = F.layer_norm(F.gelu(F.linear(x, w, b), approximate="tanh"), (576,), g, be, 1e-5)
    assert rel_l2(ln.numpy(), ref.numpy()) < SPLIT_TOL


def test_group_norm_stats(K):
    x = _r((2, 36, 467), 29, 3.0) + 2.0
    g, b = 1 + _r((36,), 30, 0.1), _r((36,), 31, 0.1)
    ref = F.group_norm(x, 6, g, b, 1e-6)
    sc, sh = K.group_norm_affine(dev(x.permute(0, 2, 1).contiguous()), 6, dev(g), dev(b), 1e-6)
    y = x * sc.cpu()[:, :, None] + sh.cpu()[:, :, None]
    assert rel_l2(y.numpy(), ref.numpy()) < 1e-6


@pytest.mark.parametrize("name", ["act1d_T50.npz", "act1d_T3.npz"])
def test_activation1d_golden(K, name):
    g = golden(name)
    x = torch.from_numpy(g["x"])
    y = K.activation1d(dev(x.permute(0, 2, 1).contiguous()), *(dev(torch.from_numpy(g[k])) for k in
                       ("alpha", "beta", "up_filter", "down_filter"))).cpu().permute(0, 2, 1)
    np.testing.assert_allclose(y.numpy(), g["y"], rtol=2e-5, atol=2e-6)


def test_activation1d_long(K):
    from oracle import alcm_oracle as O
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    C, T = 96, 1000
    x = _r((2, C, T), 32, 1.5)
    a, b = _r((C,), 33, 0.3), _r((C,), 34, 0.3)
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    ref = O.activation1d(x, a, b, f, f)
    y = K.activation1d(dev(x.permute(0, 2, 1).contiguous()), dev(a), dev(b), dev(f), dev(f)).cpu().permute(0, 2, 1)
    np.testing.assert_allclose(y.numpy(), ref.numpy(), rtol=2e-5, atol=5e-6)





def test_lcm_step_golden(K):
    from oracle import alcm_oracle as O
    g = golden("lcm_step.npz")
    ac = O.alphas_cumprod()
    x, eps, nz = (dev(torch.from_numpy(g[k])) for k in ("x", "eps", "noise"))
    for t, pt, xin, noise, kp, kd in ((999, 499, x, nz, "prev0", "den0"), (499, 499, None, None, "prev1", "den1")):
        sc = O.lcm_step_scalars(t, pt, ac)
        coeffs = [sc[k].item() for k in ("sqrt_a", "sqrt_b", "c_out", "c_skip", "sqrt_a_prev", "sqrt_b_prev")]
        xx = xin if xin is not None else dev(torch.from_numpy(g["prev0"]))
        prev, den = K.lcm_step(xx, eps, noise, coeffs)
        np.testing.assert_allclose(prev.cpu().numpy(), g[kp], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(den.cpu().numpy(), g[kd], rtol=1e-6, atol=1e-6)


def test_embeddings_golden(K):
    from audiolcm_amd import schedule
    g = golden("schedule.npz")
    t = torch.from_numpy(g["t"])
    f = schedule.timestep_freqs()
    te = K.sincos_embedding(dev(t.float()), dev(f), 1.0, True).cpu()
    # exact check against the same frequency table (fp64 reference of the fp32 arguments)
    args = (t[:, None].float() * f[None]).double()
    np.testing.assert_allclose(te.numpy(), torch.cat([torch.cos(args), torch.sin(args)], 1).numpy(), atol=2e-7)
    # against the reference's own vectors: its CPU exp differs from ours by <= 1 ulp (<= 3e-5 here)
    np.testing.assert_allclose(te.numpy(), g["timestep_emb"], atol=5e-5)
    w = torch.full((3,), 4.0)
    gf = schedule.guidance_freqs()
    ge = K.sincos_embedding(dev(w), dev(gf), 1000.0, False).cpu()
    a = (w[:, None] * 1000.0 * gf[None]).double()
    np.testing.assert_allclose(ge.numpy(), torch.cat([torch.sin(a), torch.cos(a)], 1).numpy(), atol=2e-7)
    np.testing.assert_allclose(ge.numpy(), g["guidance_w4"], atol=3e-4)


@pytest.mark.parametrize("C,T,k,dil", [(24, 300, 11, 5), (48, 200, 7, 3), (96, 257, 3, 1), (96, 130, 11, 5),
                                       (192, 100, 3, 5), (384, 77, 7, 1), (768, 40, 11, 3), (64, 5, 3, 1)])
@pytest.mark.parametrize("prec", [1, 0, 2, 3])
def test_opconv(K, C, T, k, dil, prec):
    """Implicit-GEMM conv on operand planes vs F.conv1d (planes built on the host from the same fp32 input)."""
    B = 2
    x = _r((B, T, C), 70)
    w, bias = _r((C, C, k), 71, 0.7 / np.sqrt(C * k)), _r((C,), 72, 0.05)
    r = _r((B, T, C), 73)
    ref = F.conv1d(x.permute(0, 2, 1), w, bias, dilation=dil, padding=(k - 1) * dil // 2).permute(0, 2, 1) + r
    y = K.opconv(K.operand_planes(dev(x), prec), C, dev(w), dev(bias), dil, prec, residual=dev(r)).cpu()
    assert y.shape == ref.shape
    assert rel_l2(y.numpy(), ref.numpy()) < (3e-5 if prec == 1 else TOL[prec])


@pytest.mark.parametrize("prec", [1, 2, 0])
def test_opconv_underfilled_wide_n(K, prec, monkeypatch):
    """N % 128 == 0 problems with fewer 128 x 128 tiles than CUs (the text encoders' N = 1024 projections) take the
    96-column tiles by default (a partial last column tile at N = 1024): vs F.conv1d, and vs the 128 x 128 tiles
    (ALCM_OPCONV_TILE=-1) on the same planes (same products and K order: bit-identical)."""
    from audiolcm_amd import _hip
    B, T, C, N = 1, 300, 256, 1024
    x = _r((B, T, C), 120)
    w, bias = _r((N, C, 1), 121, 1.0 / np.sqrt(C)), _r((N,), 122, 0.05)
    r = _r((B, T, N), 123)
    ref = F.conv1d(x.permute(0, 2, 1), w, bias).permute(0, 2, 1) + r
    pl = K.operand_planes(dev(x), prec)
    y = K.opconv(pl, C, dev(w), dev(bias), 1, prec, residual=dev(r)).cpu()
    monkeypatch.setenv("ALCM_OPCONV_TILE", "-1")
    _hip.reload_knobs()
    try:
        y0 = K.opconv(pl, C, dev(w), dev(bias), 1, prec, residual=dev(r)).cpu()
    finally:
        monkeypatch.delenv("ALCM_OPCONV_TILE")
        _hip.reload_knobs()
    assert rel_l2(y.numpy(), ref.numpy()) < (3e-5 if prec == 1 else TOL[prec])
    assert torch.equal(y, y0)


@pytest.mark.parametrize("C,T,k,dil", [(768, 600, 11, 5), (384, 1100, 7, 3), (192, 1500, 3, 1), (256, 700, 5, 2),
                                       (384, 520, 11, 1)])
@pytest.mark.parametrize("prec", [0, 2])
def test_opconv_wide(K, C, T, k, dil, prec, monkeypatch):
    """Wide-layer kernel (alcm_wconv.hip: 256-row tiles, LDS-DMA staging) vs F.conv1d and vs the 128-row
    opconv_kernel on the same operand planes (identical products, only the fp32 summation order differs)."""
    B = 2
    x = _r((B, T, C), 80)
    w, bias = _r((C, C, k), 81, 0.7 / np.sqrt(C * k)), _r((C,), 82, 0.05)
    r = _r((B, T, C), 83)
    ref = (F.conv1d(x.permute(0, 2, 1), w, bias, dilation=dil, padding=(k - 1) * dil // 2).permute(0, 2, 1) + r) * 0.5
    pl = K.operand_planes(dev(x), prec)
    acc = dev(torch.ones((B, T, C)))
    y = K.opconv(pl, C, dev(w), dev(bias), dil, prec, residual=dev(r), out_scale=0.5, accumulate_into=acc).cpu() - 1
    assert rel_l2(y.numpy(), ref.numpy()) < TOL[prec]
    from audiolcm_amd import _hip
    # the default (wconv3 where its tiles are full, else the two-workgroup kernel) vs each wide kernel forced
    # (ALCM_WCONV3=1 / 0) and vs opconv_kernel (ALCM_WCONV=0: no wide kernel at all)
    for knob, var in (("ALCM_WCONV3", "1"), ("ALCM_WCONV3", "0"), ("ALCM_WCONV", "0")):
        monkeypatch.setenv(knob, var)
        _hip.reload_knobs()
        try:
            acc0 = dev(torch.ones((B, T, C)))
            y0 = K.opconv(pl, C, dev(w), dev(bias), dil, prec, residual=dev(r), out_scale=0.5,
                          accumulate_into=acc0).cpu() - 1
        finally:
            monkeypatch.delenv(knob)
            _hip.reload_knobs()
        assert rel_l2(y.numpy(), y0.numpy()) < 1e-5, (knob, var)


@pytest.mark.parametrize("prec", [0, 2])
def test_wconv2_tile160(K, prec, monkeypatch):
    """160-row wconv2 tiles (chosen where they take fewer rounds of the chip's workgroup slots: T = 312 as two tiles
    instead of three, 24 x 2 x 8 = 384 tiles instead of 576): vs F.conv1d (fp32, on the GPU) and vs the 128-row
    opconv_kernel on the same operand planes (ALCM_WCONV=0)."""
    B, T, C, N, k = 24, 312, 256, 1536, 3
    x = _r((B, T, C), 90)
    w, bias = _r((N, C, k), 91, 0.7 / np.sqrt(C * k)), _r((N,), 92, 0.05)
    r = _r((B, T, N), 93)
    ref = (F.conv1d(dev(x).permute(0, 2, 1), dev(w), dev(bias), padding=1).permute(0, 2, 1) + dev(r)).cpu()
    pl = K.operand_planes(dev(x), prec)
    y = K.opconv(pl, C, dev(w), dev(bias), 1, prec, residual=dev(r)).cpu()
    assert rel_l2(y.numpy(), ref.numpy()) < TOL[prec]
    from audiolcm_amd import _hip
    monkeypatch.setenv("ALCM_WCONV", "0")
    _hip.reload_knobs()
    try:
        y0 = K.opconv(pl, C, dev(w), dev(bias), 1, prec, residual=dev(r)).cpu()
    finally:
        monkeypatch.delenv("ALCM_WCONV")
        _hip.reload_knobs()
    assert rel_l2(y.numpy(), y0.numpy()) < 1e-5


@pytest.mark.parametrize("C,N,T,k,act", [(256, 200, 700, 1, 2), (256, 200, 700, 3, 0), (768, 1000, 300, 1, 2),
                                          (192, 388, 1300, 3, 1)])
@pytest.mark.parametrize("prec", [0, 2])
def test_wconv2_ragged_n_out_act(K, C, N, T, k, act, prec, monkeypatch):
    """Two-workgroup wide conv with N not a multiple of 96 (a partial last 192-column tile: weight rows clamped, its
    columns masked; the T5 wi at N = 5632) and an output activation (act(acc + bias), the BERT intermediate GELU) vs
    F.conv1d and vs opconv_kernel (ALCM_WCONV=0) on the same planes."""
    from audiolcm_amd import _hip
    B = 2
    x = _r((B, T, C), 170)
    w, bias = _r((N, C, k), 171, 0.7 / np.sqrt(C * k)), _r((N,), 172, 0.05)
    ref = F.conv1d(x.permute(0, 2, 1), w, bias, padding=(k - 1) // 2).permute(0, 2, 1)
    ref = {0: ref, 1: F.silu(ref), 2: F.gelu(ref)}[act]
    pl = K.operand_planes(dev(x), prec)
    y = K.opconv(pl, C, dev(w), dev(bias), 1, prec, out_act=act).cpu()
    assert rel_l2(y.numpy(), ref.numpy()) < TOL[prec]
    monkeypatch.setenv("ALCM_WCONV", "0")
    _hip.reload_knobs()
    try:
        y0 = K.opconv(pl, C, dev(w), dev(bias), 1, prec, out_act=act).cpu()
    finally:
        monkeypatch.delenv("ALCM_WCONV")
        _hip.reload_knobs()
    assert rel_l2(y.numpy(), y0.numpy()) < 1e-5


@pytest.mark.parametrize("C,T,k,dil,grid", [(384, 1100, 7, 3, 0), (384, 1100, 7, 3, 8), (192, 1500, 3, 1, 16),
                                            (768, 600, 11, 5, 8), (576, 467, 9, 1, 0)])
@pytest.mark.parametrize("prec", [0, 2])
def test_wconv3_persistent(K, C, T, k, dil, grid, prec, monkeypatch):
    """Persistent 8-wave wide conv (ALCM_WCONV3: one flat (tile, chunk, tap) pipeline per workgroup, epilogue from
    the accumulators) vs F.conv1d and vs the two-workgroup kernel on the same planes (same per-element product order:
    bit-identical); ALCM_WCONV3_GRID caps the workgroups so each walks several tiles (cross-tile prefetch)."""
    from audiolcm_amd import _hip
    B = 2
    x = _r((B, T, C), 90)
    w, bias = _r((C, C, k), 91, 0.7 / np.sqrt(C * k)), _r((C,), 92, 0.05)
    r = _r((B, T, C), 93)
    ref = (F.conv1d(x.permute(0, 2, 1), w, bias, dilation=dil, padding=(k - 1) * dil // 2).permute(0, 2, 1) + r) * 0.5
    pl = K.operand_planes(dev(x), prec)

    def run():
        acc = dev(torch.ones((B, T, C)))
        return K.opconv(pl, C, dev(w), dev(bias), dil, prec, residual=dev(r), out_scale=0.5,
                        accumulate_into=acc).cpu() - 1
    monkeypatch.setenv("ALCM_WCONV3", "0")
    _hip.reload_knobs()
    try:
        y2 = run()
    finally:
        monkeypatch.delenv("ALCM_WCONV3")
    monkeypatch.setenv("ALCM_WCONV3", "1")
    monkeypatch.setenv("ALCM_WCONV3_GRID", str(grid))
    _hip.reload_knobs()
    try:
        y3 = run()
    finally:
        monkeypatch.delenv("ALCM_WCONV3")
        monkeypatch.delenv("ALCM_WCONV3_GRID")
        _hip.reload_knobs()
    assert rel_l2(y3.numpy(), ref.numpy()) < TOL[prec]
    assert rel_l2(y3.numpy(), y2.numpy()) < 1e-6


@pytest.mark.parametrize("C,T,k,res,grid", [(384, 1100, 3, True, 0), (192, 1500, 3, False, 16),
                                            (768, 600, 11, True, 8), (192, 257, 7, False, 0)])
def test_wconv3_partial_tile_epilogue(K, C, T, k, res, grid, monkeypatch):
    """wconv3's fp32 epilogue straight from the accumulators ((acc + bias + res) * scale + out, 4-B column accesses)
    on the masked rows of a partial last tile (T % 256 != 0) and in the residual-free form, vs the two-workgroup
    kernel on the same planes (same products and order) and vs F.conv1d."""
    from audiolcm_amd import _hip
    B, prec = 2, 2
    x = _r((B, T, C), 110)
    w, bias = _r((C, C, k), 111, 0.7 / np.sqrt(C * k)), _r((C,), 112, 0.05)
    r = dev(_r((B, T, C), 113)) if res else None
    pl = K.operand_planes(dev(x), prec)
    outs = []
    for env in ({"ALCM_WCONV3": "1", "ALCM_WCONV3_GRID": str(grid)}, {"ALCM_WCONV3": "0"}):
        for kk, v in env.items():
            monkeypatch.setenv(kk, v)
        _hip.reload_knobs()
        try:
            acc = dev(_r((B, T, C), 114))
            outs.append(K.opconv(pl, C, dev(w), dev(bias), 1, prec, residual=r, out_scale=0.5,
                                 accumulate_into=acc).cpu())
        finally:
            for kk in env:
                monkeypatch.delenv(kk)
            _hip.reload_knobs()
    assert rel_l2(outs[0].numpy(), outs[1].numpy()) < 1e-6
    ref = F.conv1d(x.permute(0, 2, 1), w, bias, padding=(k - 1) // 2).permute(0, 2, 1)
    if res:
        ref = ref + r.cpu()
    ref = ref * 0.5 + _r((B, T, C), 114)
    assert rel_l2(outs[0].numpy(), ref.numpy()) < TOL[prec]


@pytest.mark.parametrize("T,prec", [(467, 2), (467, 0), (300, 2)])
def test_wconv2_geglu_plane(K, T, prec):
    """DiT Conv1dFeedForward up-projection (k9, GEGLU, new_attention.py:48-55) on the two-workgroup wide conv: the
    GEGLU plane (value * gelu_erf(gate) from interleaved columns, LDS-staged epilogue) vs the fp32 reference within
    the plane tolerance."""
    B, C, N, k = 2, 576, 4608, 9
    x = _r((B, T, C), 95)
    w, bias = _r((N, C, k), 96, 1.0 / np.sqrt(C * k)), _r((N,), 97, 0.05)
    pl = K.operand_planes(dev(x), prec)
    y = K.opconv(pl, C, dev(w), dev(bias), 1, prec, geglu=True)
    got = (y.view(torch.float16) if prec == 2 else y.view(torch.bfloat16)).float().cpu()[0]
    h = F.conv1d(x.permute(0, 2, 1), w, bias, padding=(k - 1) // 2).permute(0, 2, 1)
    ref = h[..., 0::2] * F.gelu(h[..., 1::2])
    assert rel_l2(got.numpy(), ref.numpy()) < TOL[prec] * 4


@pytest.mark.parametrize("C,N,T,mode", [(576, 1728, 467, "plane"), (576, 576, 467, "res"), (768, 384, 1000, "plain"),
                                         (256, 192, 700, "plane"), (1536, 768, 520, "res")])
@pytest.mark.parametrize("prec", [0, 2])
def test_lin_plane_k1(K, C, N, T, mode, prec, monkeypatch):
    """1x1 convs on one operand plane (alcm_sgemm.hip lin_plane_kernel: the DiT q,k,v projection with its plane
    output, to_out with residual + scale) vs F.conv1d, and vs the two-workgroup wide conv (ALCM_LIN1=0) bit for bit
    (same 32-deep slice order), in both ring builds (ALCM_LIN1=1 / 2); B * T is not a multiple of the 128-row tile."""
    from audiolcm_amd import _hip
    B = 2
    x = _r((B, T, C), 180)
    w, bias = _r((N, C, 1), 181, 1.0 / np.sqrt(C)), _r((N,), 182, 0.05)
    r = _r((B, T, N), 183)
    pl = K.operand_planes(dev(x), prec)
    ref = F.conv1d(x.permute(0, 2, 1), w, bias).permute(0, 2, 1)

    def run():
        if mode == "plane":
            y = K.opconv(pl, C, dev(w), dev(bias), 1, prec, out_plane=True)
            return (y.view(torch.float16) if prec == 2 else y.view(torch.bfloat16)).float().cpu()[0]
        if mode == "res":
            return K.opconv(pl, C, dev(w), dev(bias), 1, prec, residual=dev(r), out_scale=0.5).cpu()
        return K.opconv(pl, C, dev(w), dev(bias), 1, prec).cpu()
    outs = {}
    for v in ("1", "2", "0", "-1"):
        monkeypatch.setenv("ALCM_LIN1", v)
        _hip.reload_knobs()
        try:
            outs[v] = run()
        finally:
            monkeypatch.delenv("ALCM_LIN1")
            _hip.reload_knobs()
    want = (ref + r) * 0.5 if mode == "res" else ref
    assert rel_l2(outs["1"].numpy(), want.numpy()) < TOL[prec] * (4 if mode == "plane" else 1)
    assert all(torch.equal(outs[v], outs["0"]) for v in ("1", "2", "-1"))


@pytest.mark.parametrize("C,N,mode", [(1024, 1024, "res"), (1024, 5632, "plain"), (768, 3072, "gelu"),
                                      (576, 576, "res")])
@pytest.mark.parametrize("lin1", ["0", "-1"])
def test_k1_text_shapes_concurrent_streams(K, C, N, mode, lin1, monkeypatch):
    """The k = 1 convs at the benchmarked text-encoder batch (B = 32 x 77 tokens = 2464 rows; T5 o / wi with ragged
    N = 1024 / 5632, the BERT intermediate with its GELU epilogue, the DiT to_out shape), on the two-workgroup wide conv
    (ALCM_LIN1=0: its single-buffered window is re-staged at every step behind a vmcnt(0) + barrier) and on the default
    routing (lin_plane_kernel where eligible).  The round-1 wconv_kernel raced here: its K = 1 chunks read a window
    whose DMA the step's counted wait left in flight.  Two launches on concurrent streams, repeated,
    must equal the single-stream result bit for bit and match F.conv1d."""
    from audiolcm_amd import _hip
    B, T, prec = 32, 77, 2
    xs = [_r((B, T, C), 190 + i) for i in range(2)]
    w, bias = _r((N, C, 1), 192, 1.0 / np.sqrt(C)), _r((N,), 193, 0.05)
    r = dev(_r((B, T, N), 194))
    pls = [K.operand_planes(dev(x), prec) for x in xs]
    wd, bd = dev(w), dev(bias)
    pw = K.pack_conv_weight(wd)

    def run(pl):
        if mode == "res":
            return K.opconv(pl, C, wd, bd, 1, prec, residual=r, out_scale=0.5, packed=pw)
        return K.opconv(pl, C, wd, bd, 1, prec, packed=pw, out_act=2 if mode == "gelu" else 0)
    monkeypatch.setenv("ALCM_LIN1", lin1)
    _hip.reload_knobs()
    try:
        single = [run(pl).cpu() for pl in pls]
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for _ in range(4):
            torch.cuda.synchronize()
            with torch.cuda.stream(s1):
                y1 = run(pls[0])
            with torch.cuda.stream(s2):
                y2 = run(pls[1])
            torch.cuda.synchronize()
            assert torch.equal(y1.cpu(), single[0]) and torch.equal(y2.cpu(), single[1])
    finally:
        monkeypatch.delenv("ALCM_LIN1")
        _hip.reload_knobs()
    for x, y in zip(xs, single):
        ref = F.conv1d(x.permute(0, 2, 1), w, bias).permute(0, 2, 1)
        if mode == "gelu":
            ref = F.gelu(ref)
        if mode == "res":
            ref = (ref + r.cpu()) * 0.5
        assert torch.isfinite(y).all()
        assert rel_l2(y.numpy(), ref.numpy()) < TOL[prec]


@pytest.mark.parametrize("Cin,N,T,rate,prec", [(768, 384, 300, 4, 2), (384, 192, 700, 2, 0), (1536, 768, 40, 4, 2),
                                                 (192, 96, 900, 2, 2), (96, 48, 333, 2, 0)])
def test_opconv_strided_convtranspose(K, Cin, N, T, rate, prec):
    """ConvTranspose1d(Cin, N, 2*rate, rate, padding=rate/2) (BigVGAN upsampler, models.py:160-165) as `rate`
    phase convs on operand planes with the strided epilogue (wide-layer kernel; opconv_kernel for N <= 96), vs torch's fp32
    conv_transpose1d on the same plane-rounded input and weight."""
    B, k = 2, 2 * rate
    x = _r((B, T, Cin), 30)
    w, bias = _r((Cin, N, k), 31, 1.0 / np.sqrt(Cin * 2)), _r((N,), 32, 0.05)
    pl = K.operand_planes(dev(x), prec)
    rd = (lambda t: t.half().float()) if prec == 2 else (lambda t: t.bfloat16().float())
    ref = torch.nn.functional.conv_transpose1d(rd(x).transpose(1, 2), rd(w), bias, stride=rate, padding=rate // 2)
    out = dev(torch.full((B, T * rate, N), float("nan")))
    pad, Q = rate // 2, 2
    shape_only = dev(torch.zeros((N, Cin, Q)))
    for r in range(rate):  # phase r writes outputs t = rate*v + o from inputs v - pad_r .. v - pad_r + Q - 1
        o = (r - pad) % rate
        c = (o + pad - r) // rate
        pw = K.pack_conv_weight(dev(w), transposed=True, stride=rate, phase=r)
        K.opconv(pl, Cin, shape_only, dev(bias), 1, prec, packed=pw, strided=(out, rate, o, Q - 1 - c))
    got = out.cpu().transpose(1, 2).numpy()
    assert np.isfinite(got).all()
    assert rel_l2(got, ref.numpy()) < 2e-6


@pytest.mark.parametrize("C,T,k,dil,prec", [(24, 1000, 11, 5, 3), (48, 700, 7, 3, 3), (96, 500, 3, 1, 3),
                                            (96, 333, 11, 5, 1), (24, 250, 3, 1, 2), (48, 37, 7, 1, 0)])
@pytest.mark.parametrize("res", [False, True])
def test_opconv_fused_activation(K, C, T, k, dil, prec, res):
    """Fused Activation1d epilogue (overlapping tiles, 8 halo rows) == fp32 conv output followed by the
    standalone act_op kernel: the same fp32 values go through the same activation code, so the planes match
    bit for bit, and the fp32 output (owned rows only) matches the unfused conv."""
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    B = 2
    x = _r((B, T, C), 90)
    w, bias = _r((C, C, k), 91, 0.7 / np.sqrt(C * k)), _r((C,), 92, 0.05)
    r = dev(_r((B, T, C), 93)) if res else None
    a, bt = dev(_r((C,), 94, 0.3)), dev(_r((C,), 95, 0.3))
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    pl = K.operand_planes(dev(x), prec)
    y_ref = K.opconv(pl, C, dev(w), dev(bias), dil, prec, residual=r)
    pl_ref = K.activation1d_op(y_ref, a, bt, f, f, prec)
    y, pl2 = K.opconv(pl, C, dev(w), dev(bias), dil, prec, residual=r, act=(a, bt, f, f))
    assert pl2.shape == pl_ref.shape

    def dec(p):  # operand planes -> fp32 values
        p = p.cpu()
        if prec in (2, 3):
            return p[0].view(torch.float16).float()
        v = p[0].view(torch.bfloat16).float()
        return v + p[1].view(torch.bfloat16).float() if prec == 1 else v

    # (the unfused call may take a kernel with another K order for small B*T: fp32 rounding only)
    assert rel_l2(y.cpu().numpy(), y_ref.cpu().numpy()) < 1e-6
    assert rel_l2(dec(pl2).numpy(), dec(pl_ref).numpy()) < 1e-5
    assert torch.all(pl2.cpu()[..., C:] == 0)
    _, pl3 = K.opconv(pl, C, dev(w), dev(bias), dil, prec, residual=r, act=(a, bt, f, f), fp32_out=False)
    assert torch.equal(pl3.cpu(), pl2.cpu())


@pytest.mark.parametrize("prec", [1, 2, 3])
def test_opconv_post_tanh_accumulate(K, prec):
    """conv_post shape (N = 1, k7) with tanh, and the accumulate/out_scale epilogue (resblock mean)."""
    x = _r((2, 333, 24), 74)
    w, bias = _r((1, 24, 7), 75, 0.2), _r((1,), 76, 0.05)
    ref = torch.tanh(F.conv1d(x.permute(0, 2, 1), w, bias, padding=3)).permute(0, 2, 1)
    pl = K.operand_planes(dev(x), prec)
    y = K.opconv(pl, 24, dev(w), dev(bias), 1, prec, out_act=4).cpu()
    tol = 3e-5 if prec == 1 else TOL[prec]
    assert rel_l2(y.numpy(), ref.numpy()) < tol
    acc = dev(torch.ones((2, 333, 1)))
    K.opconv(pl, 24, dev(w), dev(bias), 1, prec, out_act=4, out_scale=0.5, accumulate_into=acc)
    assert rel_l2(acc.cpu().numpy(), (1 + 0.5 * ref).numpy()) < tol


@pytest.mark.parametrize("C,T", [(24, 700), (96, 50), (768, 37), (48, 3), (192, 300), (24, 5000)])
@pytest.mark.parametrize("prec", [1, 2])
def test_activation1d_op(K, C, T, prec):
    """Activation1d into operand planes == oracle Activation1d rounded to the operand format."""
    from oracle import alcm_oracle as O
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    x = _r((2, C, T), 77, 1.2)
    a, bt = _r((C,), 78, 0.3), _r((C,), 79, 0.3)
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    ref = O.activation1d(x, a, bt, f, f).permute(0, 2, 1).contiguous()
    pl = K.activation1d_op(dev(x.permute(0, 2, 1).contiguous()), dev(a), dev(bt), f, f, prec).cpu()
    Cp = pl.shape[-1]
    assert Cp % 32 == 0 and torch.all(pl[..., C:] == 0)
    if prec == 2:
        got = pl[0, ..., :C].view(torch.float16).float()
        assert rel_l2(got.numpy(), ref.numpy()) < 1e-3
    else:
        got = pl[0, ..., :C].view(torch.bfloat16).float() + pl[1, ..., :C].view(torch.bfloat16).float()
        assert rel_l2(got.numpy(), ref.numpy()) < 2e-5


@pytest.mark.parametrize("C,T,k,dil,prec", [(24, 1000, 11, 5, 3), (48, 700, 7, 3, 3), (96, 500, 3, 1, 2),
                                            (96, 333, 11, 5, 2), (24, 250, 3, 1, 2), (48, 2000, 11, 5, 2),
                                            (48, 37, 3, 1, 3),
                                            # > 256 tiles: persistent workgroups walk several, the loader wave
                                            # prefetching the next tile's window (k <= 7) or refilling after the
                                            # epilogue (k = 11); C = 24 at four workgroups per CU
                                            (48, 70000, 3, 1, 3), (48, 70000, 7, 3, 3), (48, 70000, 11, 5, 3),
                                            (24, 70000, 3, 1, 3)])
@pytest.mark.parametrize("mode", ["conv1", "conv2", "last"])
def test_opconv_dense_resident_weights(K, C, T, k, dil, prec, mode):
    """alcm_opconv_dense (BigVGAN stages 3-5: dense K = tap*C + c, weights resident in LDS, persistent tiles) == the
    Cp-padded opconv path on the same planes: conv1 (+ fused Activation1d), conv2 (+ residual, fp32 state, fused
    Activation1d), a resblock's last conv2 (+ residual, out_scale, accumulate).  fp32 outputs differ by the K order
    only (rel-L2 1e-5); the planes by fp16 rounding flips of those values (channels < N compared: the dense kernel
    leaves the operand padding alone)."""
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    B = 2
    x = _r((B, T, C), 60)
    w, bias = _r((C, C, k), 61, 0.7 / np.sqrt(C * k)), _r((C,), 62, 0.05)
    r = dev(_r((B, T, C), 63))
    a, bt = dev(_r((C,), 64, 0.3)), dev(_r((C,), 65, 0.3))
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    pl = K.operand_planes(dev(x), prec)
    dw = dev(w)

    def dec(p):
        return p[0, ..., :C].cpu().view(torch.float16).float().numpy()
    if mode == "conv1":
        _, pl_ref = K.opconv(pl, C, dw, dev(bias), dil, prec, act=(a, bt, f, f), fp32_out=False)
        _, pl_d = K.opconv(pl, C, dw, dev(bias), dil, prec, act=(a, bt, f, f), fp32_out=False, dense=True)
        assert np.isfinite(dec(pl_d)).all()
        assert rel_l2(dec(pl_d), dec(pl_ref)) < 5e-4
    elif mode == "conv2":
        y_ref, pl_ref = K.opconv(pl, C, dw, dev(bias), dil, prec, residual=r, act=(a, bt, f, f))
        y_d, pl_d = K.opconv(pl, C, dw, dev(bias), dil, prec, residual=r, act=(a, bt, f, f), dense=True)
        assert rel_l2(y_d.cpu().numpy(), y_ref.cpu().numpy()) < 1e-5
        assert rel_l2(dec(pl_d), dec(pl_ref)) < 5e-4
    else:
        o0 = _r((B, T, C), 66)
        o_ref, o_d = dev(o0.clone()), dev(o0.clone())
        K.opconv(pl, C, dw, dev(bias), dil, prec, residual=r, out_scale=1 / 3, accumulate_into=o_ref)
        K.opconv(pl, C, dw, dev(bias), dil, prec, residual=r, out_scale=1 / 3, accumulate_into=o_d, dense=True)
        assert rel_l2(o_d.cpu().numpy(), o_ref.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("C,k,dil,mode,tk", [(48, 11, 5, "conv2", "1"), (48, 7, 3, "conv2", "1"), (48, 3, 1, "conv1", "1"),
                                             (24, 3, 1, "conv2", "1"), (24, 11, 5, "conv1", "1"), (96, 11, 5, "conv2", "1"),
                                             (48, 11, 5, "last", "1"),
                                             # C = 48 column halves on 128-row tiles, two / three workgroups per CU
                                             (48, 11, 5, "conv2", "4"), (48, 7, 3, "conv1", "4"), (48, 3, 1, "conv2", "4"),
                                             (48, 3, 1, "conv2", "5"), (48, 3, 1, "conv1", "5"), (48, 11, 5, "last", "4"),
                                             (48, 3, 1, "last", "5")])
def test_tail_conv_multitile_vs_oracle(K, C, k, dil, mode, tk, monkeypatch):
    """The narrow AMPBlock convs (vocoder/bigvgan/models.py:72-81, stages 3-5) on > 256 tiles — persistent resident
    workgroups walking several tiles with the loader wave's next-window prefetch (C = 48), four streamed workgroups
    per CU (C = 24), the C = 96 persistent streamed grid — against the fp32 ORACLE, not another HIP kernel:
    F.conv1d on the fp16 operand values the kernel reads (weights in fp32; F16W2 carries them as hi + lo fp16) +
    bias (+ residual), then oracle Activation1d (alias_free_torch/act.py:23-27).  fp32 state within accumulation-order
    rounding (rel-L2 2e-5); the Activation1d plane within its fp16 rounding (rel-L2 1e-3, measured ~3e-4)."""
    from oracle import alcm_oracle as O
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    B, T = 2, 70000
    prec = 2 if C == 96 else 3
    x = _r((B, T, C), 160)
    w, bias = _r((C, C, k), 161, 0.7 / np.sqrt(C * k)), _r((C,), 162, 0.05)
    r = _r((B, T, C), 163)
    a, bt = _r((C,), 164, 0.3), _r((C,), 165, 0.3)
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    pl = K.operand_planes(dev(x), prec)
    w_k = w.half().float() if prec == 2 else w   # F16: fp16 weights; F16W2: hi + lo fp16 (~fp32)
    ref = F.conv1d(x.half().float().permute(0, 2, 1), w_k, bias, padding=(k - 1) * dil // 2, dilation=dil)
    if mode != "conv1":
        ref = ref + r.permute(0, 2, 1)
    act = (dev(a), dev(bt), f, f)
    from audiolcm_amd import _hip
    monkeypatch.setenv("ALCM_TCONV", tk)
    _hip.reload_knobs()
    try:
        _tail_run_and_check(K, C, k, dil, mode, prec, pl, w, bias, r, a, bt, f, act, ref, B, T)
    finally:
        monkeypatch.delenv("ALCM_TCONV")
        _hip.reload_knobs()


def _tail_run_and_check(K, C, k, dil, mode, prec, pl, w, bias, r, a, bt, f, act, ref, B, T):
    from oracle import alcm_oracle as O
    if mode == "conv1":
        _, pl_d = K.opconv(pl, C, dev(w), dev(bias), dil, prec, act=act, fp32_out=False, dense=True)
    elif mode == "conv2":
        y_d, pl_d = K.opconv(pl, C, dev(w), dev(bias), dil, prec, residual=dev(r), act=act, dense=True)
        e_y = rel_l2(y_d.cpu().permute(0, 2, 1).numpy(), ref.numpy())
        print(f"tail {mode} C{C} k{k}: state rel-L2 {e_y:.2e}")
        assert e_y < 2e-5
    else:
        o0 = _r((B, T, C), 166)
        o_d = dev(o0.clone())
        K.opconv(pl, C, dev(w), dev(bias), dil, prec, residual=dev(r), out_scale=1 / 3, accumulate_into=o_d,
                 dense=True)
        e_o = rel_l2(o_d.cpu().numpy(), (o0 + ref.permute(0, 2, 1) / 3).numpy())
        print(f"tail last C{C} k{k}: accumulated rel-L2 {e_o:.2e}")
        assert e_o < 2e-5
        return
    ref_act = O.activation1d(ref, a, bt, f, f).permute(0, 2, 1)
    got = pl_d[0, ..., :C].cpu().view(torch.float16).float()
    e_a = rel_l2(got.numpy(), ref_act.numpy())
    print(f"tail {mode} C{C} k{k}: Activation1d plane rel-L2 {e_a:.2e}")
    assert torch.isfinite(got).all() and e_a < 1e-3


@pytest.mark.parametrize("C,T", [(192, 37), (384, 300), (768, 2496), (192, 1000)])
def test_activation1d_mfma(K, C, T, monkeypatch):
    """Activation1d with both FIRs on MFMA (act_mfma_kernel: the wide stages under the mixed policy; fp16 FIR inputs,
    taps split hi/lo) vs the fp32 oracle and vs the VALU kernel (ALCM_ACT_MFMA=0), on fp16 planes: within the fp16
    rounding of the inputs (alias_free_torch/act.py:23-27).  T = 37 is one partial tile with both sequence ends."""
    from audiolcm_amd import _hip
    from oracle import alcm_oracle as O
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    x = _r((2, C, T), 140, 1.5)
    a, bt = _r((C,), 141, 0.3), _r((C,), 142, 0.3)
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    ref = O.activation1d(x, a, bt, f, f).permute(0, 2, 1).contiguous()
    xd = dev(x.permute(0, 2, 1).contiguous())
    got = K.activation1d_op(xd, dev(a), dev(bt), f, f, 2).cpu()[0].view(torch.float16).float()
    monkeypatch.setenv("ALCM_ACT_MFMA", "0")
    _hip.reload_knobs()
    try:
        valu = K.activation1d_op(xd, dev(a), dev(bt), f, f, 2).cpu()[0].view(torch.float16).float()
    finally:
        monkeypatch.delenv("ALCM_ACT_MFMA")
        _hip.reload_knobs()
    e_mfma, e_valu = rel_l2(got.numpy(), ref.numpy()), rel_l2(valu.numpy(), ref.numpy())
    print(f"act C{C} T{T}: mfma {e_mfma:.2e} valu {e_valu:.2e} mfma-vs-valu {rel_l2(got.numpy(), valu.numpy()):.2e}")
    assert torch.isfinite(got).all()
    assert e_mfma < 1e-3 and e_mfma < 2.5 * e_valu
    # the stores at the end of their own tile (ALCM_ACT_DEFER=0) instead of one tile late: the same values
    monkeypatch.setenv("ALCM_ACT_DEFER", "0")
    _hip.reload_knobs()
    try:
        inl = K.activation1d_op(xd, dev(a), dev(bt), f, f, 2).cpu()[0].view(torch.float16).float()
    finally:
        monkeypatch.delenv("ALCM_ACT_DEFER")
        _hip.reload_knobs()
    assert torch.equal(got, inl)


@pytest.mark.parametrize("C,T,k,dil,grid", [(768, 600, 11, 5, 8), (384, 1100, 7, 3, 0), (192, 1500, 3, 1, 16),
                                            (192, 257, 11, 5, 0), (192, 37, 3, 1, 0)])
def test_conv1_fp16_handoff(K, C, T, k, dil, grid, monkeypatch):
    """The wide-stage AMPBlock conv1 -> Activation1d hand-off (vocoder/bigvgan/models.py:74-79) as an fp16 plane:
    conv1's out_plane epilogue (wconv3 where its tiles are full, else wconv2) writes fp16(acc + bias) and
    alcm_activation1d_op_f16in reads it.  Both halves are bit-identical to the fp32 path they replace: the plane equals
    the fp32 output rounded to fp16, and the activation equals alcm_activation1d_op on the fp32 output (its MFMA FIRs
    round their input to that same fp16 value)."""
    from audiolcm_amd import _hip
    from audiolcm_amd.recipe import kaiser_sinc_filter1d
    B, prec = 2, 2
    x = _r((B, T, C), 150)
    w, bias = _r((C, C, k), 151, 0.7 / np.sqrt(C * k)), _r((C,), 152, 0.05)
    a, bt = _r((C,), 153, 0.3), _r((C,), 154, 0.3)
    f = kaiser_sinc_filter1d(0.25, 0.3, 12)
    pl = K.operand_planes(dev(x), prec)
    for w3 in ("1", "0"):  # persistent kernel (grid-capped: several tiles per workgroup), two-workgroup kernel
        monkeypatch.setenv("ALCM_WCONV3", w3)
        monkeypatch.setenv("ALCM_WCONV3_GRID", str(grid))
        _hip.reload_knobs()
        try:
            y32 = K.opconv(pl, C, dev(w), dev(bias), dil, prec)
            y16 = K.opconv(pl, C, dev(w), dev(bias), dil, prec, out_plane=True)
            act32 = K.activation1d_op(y16[0].view(torch.float16).float(), dev(a), dev(bt), f, f, prec).cpu()
            act16 = K.activation1d_op_f16in(y16, dev(a), dev(bt), f, f, prec).cpu()
        finally:
            monkeypatch.delenv("ALCM_WCONV3")
            monkeypatch.delenv("ALCM_WCONV3_GRID")
            _hip.reload_knobs()
        if w3 == "1" or B * T >= 1024:  # the same kernel (below 1024 rows the fp32 output takes opconv_kernel)
            assert torch.equal(y16.cpu()[0], y32.cpu().half().view(torch.int16)), f"plane != fp16(fp32), wconv3={w3}"
        else:
            assert rel_l2(y16.cpu()[0].view(torch.float16).float().numpy(), y32.cpu().numpy()) < 1e-3
        assert torch.equal(act16, act32), f"activation on the fp16 plane differs, wconv3={w3}"


@pytest.mark.parametrize("B,acc", [(4, False), (8, True)])
def test_wconv3_ksplit_underfilled(K, B, acc, monkeypatch):
    """K-split persistent wide conv on a grid that does not fill the chip (the DiT FFN down-projection shape, k9
    2304 -> 576 at L = 467: 6 B tiles of 256 x 192; new_attention.py:48-55 / concatDiT.py FeedForward): partial sums
    per K part + the ordered reduction with bias / residual / scale (/ accumulate).  vs the unsplit launch (fp32
    summation order only: rel-L2 1e-6), vs F.conv1d on the fp16 operands, and bit-stable across runs."""
    from audiolcm_amd import _hip
    T, C, N, k = 467, 2304, 576, 9
    x = _r((B, T, C), 170, 0.5)
    w, bias = _r((N, C, k), 171, 1.0 / np.sqrt(C * k)), _r((N,), 172, 0.05)
    r = _r((B, T, N), 173)
    o0 = _r((B, T, N), 174)
    pl = K.operand_planes(dev(x), 2)
    pw = K.pack_conv_weight(dev(w))
    ws = torch.empty(8 * B * T * N, device="cuda")

    def run(split):
        o = dev(o0.clone()) if acc else None
        y = K.opconv(pl, C, dev(w), dev(bias), 1, 2, residual=dev(r), packed=pw, out_scale=0.5,
                     accumulate_into=o, ksplit_ws=ws if split else None)
        return y.cpu()
    monkeypatch.setenv("ALCM_PROF_SHAPES", "1")
    _hip.reload_knobs()
    _hip.profile_begin()
    ys = run(True)
    torch.cuda.synchronize()
    prof = _hip.profile_end()
    monkeypatch.delenv("ALCM_PROF_SHAPES")
    _hip.reload_knobs()
    assert any("ksplit_reduce" in p["name"] for p in prof), [p["name"] for p in prof]
    y1 = run(False)
    assert torch.equal(ys, run(True)), "K-split result not bit-stable"
    ref = (F.conv1d(x.half().float().permute(0, 2, 1), w.half().float(), bias, padding=k // 2).permute(0, 2, 1) + r) * 0.5
    if acc:
        ref = ref + o0
    e_s, e_1 = rel_l2(ys.numpy(), y1.numpy()), rel_l2(ys.numpy(), ref.numpy())
    print(f"ksplit B{B}: split vs unsplit {e_s:.2e}, vs F.conv1d {e_1:.2e}")
    assert e_s < 1e-6 and e_1 < 1e-5


@pytest.mark.parametrize("C,N", [(1024, 1024), (3072, 768), (768, 768)])
def test_wconv2_ksplit_text_linears(K, C, N):
    """K-split two-workgroup wide conv on the text towers' under-filled linears (2464 rows = 32 prompts x 77 tokens:
    the T5 attention out-projection 1024 -> 1024 with its ragged last N tile, the BERT output 3072 -> 768 and
    attention output 768 -> 768, each + bias + residual; modules.py:567-582 via HF T5 / BERT): vs the unsplit launch
    (summation order only) and vs F.linear on the fp16 operands, bit-stable."""
    from audiolcm_amd import _hip
    R = 2464
    x = _r((1, R, C), 190, 0.5)
    w, bias = _r((N, C, 1), 191, 1.0 / np.sqrt(C)), _r((N,), 192, 0.05)
    r = _r((1, R, N), 193)
    pl = K.operand_planes(dev(x), 2)
    pw = K.pack_conv_weight(dev(w))
    ws = torch.empty(8 * R * N, device="cuda")
    run = lambda split: K.opconv(pl, C, dev(w), dev(bias), 1, 2, residual=dev(r), packed=pw,
                                 ksplit_ws=ws if split else None).cpu()
    _hip.profile_begin()
    ys = run(True)
    torch.cuda.synchronize()
    names = [p["name"] for p in _hip.profile_end()]
    assert any("wconv2_kernel" in n and "ksplit_reduce" in n for n in names), names
    y1 = run(False)
    assert torch.equal(ys, run(True))
    ref = F.linear(x.half().float()[0], w.half().float()[..., 0], bias) + r[0]
    e_s, e_r = rel_l2(ys.numpy(), y1.numpy()), rel_l2(ys[0].numpy(), ref.numpy())
    print(f"wconv2 ksplit C{C} N{N}: split vs unsplit {e_s:.2e}, vs F.linear {e_r:.2e}")
    assert e_s < 1e-6 and e_r < 1e-5


@pytest.mark.parametrize("C,T,grid,acc", [(384, 1100, 0, False), (192, 1500, 16, True), (768, 600, 8, False)])
def test_opconv_sum_three_chains(K, C, T, grid, acc, monkeypatch):
    """alcm_opconv_sum: a BigVGAN stage's mean over its three resblocks taken at the chains' last conv2 + residual
    (vocoder/bigvgan/models.py:190-199 with AMPBlock1's conv2 + x, models.py:76-80): k = 3 / 7 / 11 terms with their
    own planes, weights, biases and residuals summed in one persistent launch (ALCM_WCONV3_GRID caps the workgroups
    so each walks several tiles across the terms' window / weight switches) vs F.conv1d on the fp16 operands and vs
    the three accumulating launches (ALCM_WCONV_SUM=0: fp32 rounding order only)."""
    from audiolcm_amd import _hip
    B, inv = 2, 1.0 / 3
    ks = (3, 7, 11)
    xs = [_r((B, T, C), 210 + i, 0.5) for i in range(3)]
    ws = [_r((C, C, k), 213 + i, 1.0 / np.sqrt(C * k)) for i, k in enumerate(ks)]
    bs = [_r((C,), 216 + i, 0.05) for i in range(3)]
    rs = [_r((B, T, C), 219 + i) for i in range(3)]
    o0 = _r((B, T, C), 222)
    pls = [K.operand_planes(dev(x), 2) for x in xs]
    pws = [K.pack_conv_weight(dev(w)) for w in ws]
    terms = [(pls[i], dev(ws[i]), dev(bs[i]), dev(rs[i]), pws[i]) for i in range(3)]
    outs, names = [], []
    for sm in ("1", "0"):
        env = {"ALCM_WCONV_SUM": sm, "ALCM_WCONV3": "1", "ALCM_WCONV3_GRID": str(grid), "ALCM_PROF_SHAPES": "1"}
        for kk, v in env.items():
            monkeypatch.setenv(kk, v)
        _hip.reload_knobs()
        try:
            _hip.profile_begin()
            y = K.opconv_sum(terms, 2, out_scale=inv, accumulate_into=dev(o0.clone()) if acc else None)
            torch.cuda.synchronize()
            names.append([p["name"] for p in _hip.profile_end()])
            outs.append(y.cpu())
        finally:
            for kk in env:
                monkeypatch.delenv(kk)
            _hip.reload_knobs()
    assert any("wconv3_kernel<2, 3, false>" in n for n in names[0]), names[0]
    assert not any("wconv3_kernel<2, 3, false>" in n for n in names[1]), names[1]
    ref = sum(F.conv1d(xs[i].half().float().permute(0, 2, 1), ws[i].half().float(), bs[i],
                       padding=(ks[i] - 1) // 2).permute(0, 2, 1) + rs[i] for i in range(3)) * inv
    if acc:
        ref = ref + o0
    e_ref, e_seq = rel_l2(outs[0].numpy(), ref.numpy()), rel_l2(outs[0].numpy(), outs[1].numpy())
    print(f"opconv_sum C{C} T{T}: vs F.conv1d {e_ref:.2e}, vs three launches {e_seq:.2e}")
    assert e_ref < 1e-5 and e_seq < 1e-6


@pytest.mark.parametrize("C,T,grid", [(384, 1100, 0), (768, 600, 8)])
def test_opconv_sum_plane_output(K, C, T, grid, monkeypatch):
    """alcm_opconv_sum writing the stage output as the next stage's fp16 operand plane (its only consumer, the
    upsampler's phase convs, vocoder/bigvgan/models.py:187-188, reads that format): bit for bit the fp16 rounding
    (operand_planes) of the same launch's fp32 output, on the multi-tile walk too."""
    from audiolcm_amd import _hip
    B, inv = 2, 1.0 / 3
    ks = (3, 7, 11)
    terms = []
    for i, k in enumerate(ks):
        pl = K.operand_planes(dev(_r((B, T, C), 230 + i, 0.5)), 2)
        w = dev(_r((C, C, k), 233 + i, 1.0 / np.sqrt(C * k)))
        terms.append((pl, w, dev(_r((C,), 236 + i, 0.05)), dev(_r((B, T, C), 239 + i)), K.pack_conv_weight(w)))
    monkeypatch.setenv("ALCM_WCONV3", "1")
    monkeypatch.setenv("ALCM_WCONV3_GRID", str(grid))
    _hip.reload_knobs()
    try:
        y32 = K.opconv_sum(terms, 2, out_scale=inv)
        y16 = K.opconv_sum(terms, 2, out_scale=inv, out_plane=True)
        ref16 = K.operand_planes(y32, 2)
        torch.cuda.synchronize()
    finally:
        monkeypatch.delenv("ALCM_WCONV3")
        monkeypatch.delenv("ALCM_WCONV3_GRID")
        _hip.reload_knobs()
    assert torch.equal(y16.cpu(), ref16.cpu()), "sum-form plane != fp16(fp32 sum output)"


@pytest.mark.parametrize("M,K_,N,act,res,split", [(32, 256, 576, 1, False, True), (32, 576, 576, 0, True, True),
                                                (20, 96, 200, 0, True, True), (64, 256, 256, 1, False, False)])
def test_gemm_skinny_rows(K, M, K_, N, act, res, split, monkeypatch):
    """gemm_skinny_kernel: the DiT embedder MLPs at M = B rows (concatDiT.py TimestepEmbedder: Linear -> SiLU ->
    Linear, + residual) on fp32 FMAs of the operand-format values vs F.linear (fp32) and vs the MFMA tiles
    (ALCM_GEMM_SKINNY=0); the split form uses the weight's hi + lo value and the fp32 activation."""
    from audiolcm_amd import _hip
    x = _r((1, M, K_), 240, 0.5)
    w, b = _r((N, K_, 1), 241, 1.0 / np.sqrt(K_)), _r((N,), 242, 0.05)
    r = _r((1, M, N), 243) if res else None
    ref = F.linear(x, w[..., 0], b)
    if act:
        ref = F.silu(ref)
    if res:
        ref = ref + r
    outs, names = [], []
    for sk in ("1", "0"):
        monkeypatch.setenv("ALCM_GEMM_SKINNY", sk)
        _hip.reload_knobs()
        try:
            _hip.profile_begin()
            y = K.conv1d(dev(x), dev(w), dev(b), channels_last=True, act=act,
                         residual=dev(r) if res else None, split=split)
            torch.cuda.synchronize()
            names.append([p["name"] for p in _hip.profile_end()])
            outs.append(y.cpu())
        finally:
            monkeypatch.delenv("ALCM_GEMM_SKINNY")
            _hip.reload_knobs()
    assert any("skinny" in n for n in names[0]) and not any("skinny" in n for n in names[1]), names
    # (split: the weight's hi + lo value carries ~2^-17 relative error per weight, on both paths)
    tol = 1e-5 if split else 1e-2
    e_ref, e_mfma = rel_l2(outs[0].numpy(), ref.numpy()), rel_l2(outs[0].numpy(), outs[1].numpy())
    print(f"skinny M{M} K{K_} N{N}: vs F.linear {e_ref:.2e}, vs MFMA tiles {e_mfma:.2e}")
    assert e_ref < tol and e_mfma < 2 * tol


def test_gemm_narrow_n_small_tiles(K, monkeypatch):
    """The DiT final layer shape class (N = 20 output channels over B T rows, concatDiT.py FinalLayer linear) on
    64-row MFMA tiles (4x the workgroups of the 256-row tiles): the same K order per output, so bit-identical to the
    256-row tiles (ALCM_GEMM_SKINNY=0), and vs F.linear within the split bound."""
    from audiolcm_amd import _hip
    M, K_, N = 2000, 576, 20
    x = _r((1, M, K_), 250, 0.5)
    w, b = _r((N, K_, 1), 251, 1.0 / np.sqrt(K_)), _r((N,), 252, 0.05)
    outs = []
    for sk in ("1", "0"):
        monkeypatch.setenv("ALCM_GEMM_SKINNY", sk)
        monkeypatch.setenv("ALCM_PROF_SHAPES", "1")
        _hip.reload_knobs()
        try:
            _hip.profile_begin()
            outs.append(K.conv1d(dev(x), dev(w), dev(b), channels_last=True).cpu())
            torch.cuda.synchronize()
            names = [p["name"] for p in _hip.profile_end()]
        finally:
            monkeypatch.delenv("ALCM_GEMM_SKINNY")
            monkeypatch.delenv("ALCM_PROF_SHAPES")
            _hip.reload_knobs()
        assert any(("gemm_kernel<64, 32" if sk == "1" else "gemm_kernel<256, 32") in n for n in names), names
    assert torch.equal(outs[0], outs[1])
    assert rel_l2(outs[0].numpy(), F.linear(x, w[..., 0], b).numpy()) < 1e-5


@pytest.mark.parametrize("Cin,N,T,rate", [(1536, 768, 624, 4), (768, 384, 2496, 4)])
def test_strided_upsampler_160_row_tiles(K, Cin, N, T, rate, monkeypatch):
    """The BigVGAN stage 0 / 1 upsampler phases at the bench batch (B = 32; models.py:160-165 ConvTranspose1d as
    phase convs with the strided epilogue) on 160-row wconv2 tiles: the same K order per output as the 128-row
    tiles (ALCM_UPS_T160=0, checked against torch's conv_transpose1d in test_opconv_strided_convtranspose), so
    bit-identical; the profile shows the 160-row instantiation ran."""
    from audiolcm_amd import _hip
    B, k, prec = 32, 2 * rate, 2
    x = _r((B, T, Cin), 260, 0.5)
    w, bias = _r((Cin, N, k), 261, 1.0 / np.sqrt(Cin * 2)), _r((N,), 262, 0.05)
    pl = K.operand_planes(dev(x), prec)
    pad, Q = rate // 2, 2
    shape_only = dev(torch.zeros((N, Cin, Q)))
    pws = [K.pack_conv_weight(dev(w), transposed=True, stride=rate, phase=r) for r in range(rate)]
    outs = []
    for t160 in ("1", "0"):
        monkeypatch.setenv("ALCM_UPS_T160", t160)
        _hip.reload_knobs()
        try:
            _hip.profile_begin()
            out = dev(torch.full((B, T * rate, N), float("nan")))
            for r in range(rate):
                o = (r - pad) % rate
                c = (o + pad - r) // rate
                K.opconv(pl, Cin, shape_only, dev(bias), 1, prec, packed=pws[r], strided=(out, rate, o, Q - 1 - c))
            torch.cuda.synchronize()
            names = [p["name"] for p in _hip.profile_end()]
            outs.append(out.cpu())
        finally:
            monkeypatch.delenv("ALCM_UPS_T160")
            _hip.reload_knobs()
        assert any(("160, 192" if t160 == "1" else "128, 192") in n for n in names), names
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])


def test_gemm_skinny_batch_split_invariant(K):
    """The skinny-row GEMM's rows are computed in fixed 32-row blocks and its eligibility does not depend on M (up to
    1024 rows), so a batch split into shards gives bit-identical rows (bench.py's world-2 vs world-1 waveforms,
    test_gpu_dist): 96 rows in one call == the same rows as 32 + 64."""
    x = _r((1, 96, 576), 270, 0.5)
    w, b = _r((576, 576, 1), 271, 1.0 / np.sqrt(576)), _r((576,), 272, 0.05)
    full = K.conv1d(dev(x), dev(w), dev(b), channels_last=True, act=1).cpu()
    a = K.conv1d(dev(x[:, :32].contiguous()), dev(w), dev(b), channels_last=True, act=1).cpu()
    c = K.conv1d(dev(x[:, 32:].contiguous()), dev(w), dev(b), channels_last=True, act=1).cpu()
    assert torch.equal(full, torch.cat([a, c], 1))


def test_opconv_sum_fallback_and_errors(K):
    """alcm_opconv_sum outside the one-launch form: two terms (or shapes the persistent kernel does not take) run as
    accumulating launches with the same result up to fp32 order (vs F.conv1d); a plane output there is an error, not a
    silent fp32 write (include/audiolcm_hip.h)."""
    from audiolcm_amd import _hip
    B, T, C, inv = 2, 300, 192, 0.5
    ks = (3, 5)
    xs = [_r((B, T, C), 280 + i, 0.5) for i in range(2)]
    ws = [_r((C, C, k), 282 + i, 1.0 / np.sqrt(C * k)) for i, k in enumerate(ks)]
    bs = [_r((C,), 284 + i, 0.05) for i in range(2)]
    rs = [_r((B, T, C), 286 + i) for i in range(2)]
    terms = [(K.operand_planes(dev(xs[i]), 2), dev(ws[i]), dev(bs[i]), dev(rs[i]), None) for i in range(2)]
    y = K.opconv_sum(terms, 2, out_scale=inv).cpu()
    ref = sum(F.conv1d(xs[i].half().float().permute(0, 2, 1), ws[i].half().float(), bs[i],
                       padding=(ks[i] - 1) // 2).permute(0, 2, 1) + rs[i] for i in range(2)) * inv
    e = rel_l2(y.numpy(), ref.numpy())
    print(f"opconv_sum two terms (accumulating launches): vs F.conv1d {e:.2e}")
    assert e < 1e-5
    with pytest.raises(RuntimeError):
        K.opconv_sum(terms, 2, out_scale=inv, out_plane=True)
