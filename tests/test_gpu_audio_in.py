"""Audio -> latent direction on the HIP path: the NAT_mel log-mel front-end and the 1-D VAE
Encoder1D (+ quant_conv), through the C-ABI, vs fixtures of the reference itself (tests/golden/make_golden.py
group "enc": AutoencoderKL.encode and NAT_mel.MelNet run by the reference code).
Tolerances (relative L2): moments split <= 1e-4, mixed <= 2e-3; log-mel <= 1e-5 (bf16x3 STFT / projection)."""
import numpy as np
import pytest
import torch

from conftest import golden, rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vae():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from audiolcm_amd import _hip, recipe
    from audiolcm_amd.models import AutoencoderKL
    _hip.require_device(0)
    st = dict(recipe.vae_state(0))
    st.update(recipe.vae_encoder_state(0))
    return AutoencoderKL(split=True).load_state_dict(st)


@pytest.mark.parametrize("M", [40, 624])
def test_vae_encode_split(vae, M):
    g = golden(f"vae_enc_M{M}.npz")
    post = vae.encode(torch.from_numpy(g["mel"]).cuda())
    mom = post.parameters.cpu().numpy()
    assert mom.shape == g["moments"].shape
    err = rel_l2(mom, g["moments"])
    print(f"encode M={M} split: {err:.2e}")
    assert err < 1e-4
    assert torch.equal(post.mode(), post.mean) and post.mean.shape == (1, 20, M // 2)


def test_vae_encode_mixed_and_batched(vae):
    """mixed policy (fp16 operand planes on the k5 ResnetBlock convs) with B = 4 rows of 624 frames: the k5 convs
    reach the wide-layer kernel; every clip within the mixed bound."""
    g = golden("vae_enc_M624.npz")
    vae.set_split("mixed")
    try:
        mom = vae.encode(torch.from_numpy(g["mel"]).repeat(4, 1, 1).cuda()).parameters.cpu().numpy()
    finally:
        vae.set_split(True)
    for i in range(4):
        err = rel_l2(mom[i:i + 1], g["moments"])
        assert err < 2e-3, err
    print(f"encode mixed: {rel_l2(mom[:1], g['moments']):.2e}")


def test_reconstruct_forward_matches_oracle(vae):
    """AutoencoderKL.forward(mel, sample_posterior=False) = decode(mode(encode(mel))) vs the oracle composition."""
    from audiolcm_amd import recipe
    from oracle import alcm_oracle as O
    g = golden("vae_enc_M40.npz")
    rec, post = vae(torch.from_numpy(g["mel"]).cuda(), sample_posterior=False)
    W = dict(recipe.vae_state(0))
    W.update(recipe.vae_encoder_state(0))
    with torch.no_grad():
        mean = O.vae_encode_moments(W, torch.from_numpy(g["mel"]))[:, :20]
        ref = O.vae_decode(W, mean)
    assert rec.shape == ref.shape == (1, 80, 40)
    assert rel_l2(rec.cpu().numpy(), ref.numpy()) < 1e-4
    gen = torch.Generator(device="cuda").manual_seed(3)
    s1 = post.sample(gen)
    gen.manual_seed(3)
    assert torch.equal(s1, post.sample(gen))


def test_mel_front_end(vae):
    from audiolcm_amd.mel import MelNet, NAT_MEL_16K
    g = golden("mel_B2.npz")
    net = MelNet(NAT_MEL_16K)
    assert np.array_equal(net.mel_basis.numpy(), g["mel_basis"])
    mel = net(torch.from_numpy(g["wav"])).cpu().numpy()
    assert mel.shape == g["mel"].shape
    err = rel_l2(mel, g["mel"])
    print(f"log-mel: {err:.2e}")
    assert err < 1e-5
    one = net(g["wav"][1]).cpu().numpy()  # numpy 1-D input, as MelNet accepts
    assert rel_l2(one, g["mel"][1:2]) < 1e-5


def test_wav_to_wav_round_trip(vae):
    """wav -> MelNet -> encode_first_stage -> get_first_stage_encoding -> decode_first_stage -> BigVGAN: the
    reconstruct path (scripts/reconstruct_audio.py) end to end on the HIP kernels, finite and shape-consistent."""
    from audiolcm_amd import recipe
    from audiolcm_amd.lcm import LCM_audio
    from audiolcm_amd.mel import MelNet
    from audiolcm_amd.models import BigVGAN
    lcm = LCM_audio(split="mixed")
    lcm.first_stage_model = vae
    net = MelNet()
    voc = BigVGAN.from_recipe(0, split="mixed")
    wav = torch.from_numpy(golden("mel_B2.npz")["wav"])
    mel = net(wav)
    z = lcm.get_first_stage_encoding(lcm.encode_first_stage(mel), torch.Generator(device="cuda").manual_seed(0))
    assert z.shape == (2, 20, 48)
    out = voc(lcm.decode_first_stage(z))
    assert out.shape == (2, 1, 96 * 256) and torch.isfinite(out).all()
