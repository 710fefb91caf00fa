"""Pin the CPU oracle (oracle/alcm_oracle.py) to the reference's own outputs.

The fixtures under tests/golden/ were produced by tests/golden/make_golden.py,
which runs the reference AudioLCM modules (with import-only stubs) on the
recipe's synthetic weights.  Passing here means the oracle restates the
reference algorithm to fp32 rounding; the HIP path is then checked against
the oracle (and the same fixtures) in the gpu-marked tests.
"""
import json

import numpy as np
import torch

from conftest import golden, rel_l2
from oracle import alcm_oracle as O
from audiolcm_amd import recipe


def test_recipe_digest_matches_fixtures(states):
    import hashlib
    meta = json.loads(str(golden("schedule.npz")["meta"]))

    def digest(state):
        h = hashlib.sha256()
        for k in sorted(state):
            h.update(k.encode())
            h.update(state[k].numpy().astype(np.float32).tobytes())
        return h.hexdigest()[:16]
    assert digest(states["dit"]) == meta["dit"]
    assert digest(states["vae"]) == meta["vae"]
    assert digest(states["bigvgan"]) == meta["bigvgan"]


def test_schedule_and_embeddings():
    g = golden("schedule.npz")
    np.testing.assert_array_equal(O.alphas_cumprod().numpy(), g["alphas_cumprod"])
    for S in (1, 2, 4, 8):
        assert O.lcm_timesteps(S, 50) == list(g[f"timesteps_S{S}"])
    assert O.lcm_timesteps(2) == [999, 499]
    assert O.lcm_timesteps(4) == [999, 759, 499, 259]
    w = torch.tensor(5 - 1).repeat(3)
    np.testing.assert_array_equal(O.guidance_embedding(w, 256).numpy(), g["guidance_w4"])
    np.testing.assert_array_equal(O.timestep_embedding(torch.from_numpy(g["t"]), 256).numpy(), g["timestep_emb"])


def test_schedule_errors():
    import pytest
    with pytest.raises(ValueError):
        O.lcm_timesteps(51, 50)
    with pytest.raises(ValueError):
        O.lcm_timesteps(2, 2000)


def test_lcm_step():
    g = golden("lcm_step.npz")
    ac = O.alphas_cumprod()
    x, eps, nz = (torch.from_numpy(g[k]) for k in ("x", "eps", "noise"))
    p0, d0 = O.lcm_step(eps, x, O.lcm_step_scalars(999, 499, ac), nz)
    p1, d1 = O.lcm_step(eps, p0, O.lcm_step_scalars(499, 499, ac), None)
    for a, k in ((p0, "prev0"), (d0, "den0"), (p1, "prev1"), (d1, "den1")):
        np.testing.assert_allclose(a.numpy(), g[k], rtol=1e-6, atol=1e-6)


def test_activation1d():
    for T in (50, 3):
        g = golden(f"act1d_T{T}.npz")
        y = O.activation1d(*(torch.from_numpy(g[k]) for k in ("x", "alpha", "beta", "up_filter", "down_filter")))
        np.testing.assert_allclose(y.numpy(), g["y"], rtol=1e-6, atol=1e-6)


def test_kaiser_filter_matches_buffers():
    g = golden("act1d_T50.npz")
    np.testing.assert_allclose(recipe.kaiser_sinc_filter1d(0.25, 0.3, 12).numpy(), g["up_filter"], atol=1e-7)


def test_dit_forward(states):
    for T in (40, 312):
        g = golden(f"dit_T{T}.npz")
        ctx = torch.from_numpy(golden("dit_T312.npz")["context"])
        eps = O.dit_forward(states["dit"], torch.from_numpy(g["x"]), torch.from_numpy(g["t"]), ctx,
                            torch.from_numpy(g["w_emb"]))
        assert rel_l2(eps.numpy(), g["eps"]) < 1e-5


def test_vae_decode(states):
    for T in (24, 312):
        g = golden(f"vae_T{T}.npz")
        mel = O.vae_decode(states["vae"], torch.from_numpy(g["z"]), float(g["scale_factor"]))
        assert rel_l2(mel.numpy(), g["mel"]) < 1e-5


def test_bigvgan(states):
    g = golden("bigvgan_M20.npz")
    wav = O.bigvgan_forward(states["bigvgan"], torch.from_numpy(g["mel"]))
    assert rel_l2(wav.numpy(), g["wav"]) < 1e-5


def test_end_to_end_small(states):
    g = golden("e2e_S1_B1_T40.npz")
    ctx = recipe.synthetic_context(1)
    out = O.generate(states["dit"], states["vae"], states["bigvgan"], ctx, torch.from_numpy(g["x_T"]),
                     torch.from_numpy(g["noise"]), S=1)
    assert rel_l2(out["latent"].numpy(), g["latent"]) < 1e-5
    assert rel_l2(out["mel"].numpy(), g["mel"]) < 1e-5
    assert rel_l2(out["wav"].numpy().reshape(g["wav"].shape), g["wav"]) < 1e-5


def test_end_to_end_sampler_S4(states):
    g = golden("e2e_S4_B1.npz")
    ctx = recipe.synthetic_context(1)
    eps_fn = lambda x, t, w: O.dit_forward(states["dit"], x, t, ctx, w)
    z = O.lcm_sample(eps_fn, ctx, torch.from_numpy(g["x_T"]), torch.from_numpy(g["noise"]), 4)
    assert rel_l2(z.numpy(), g["latent"]) < 1e-5


def test_prompt_noise_is_shard_invariant():
    a, na = recipe.prompt_noise(range(4), 2, 20, 16)
    b, nb = recipe.prompt_noise([2, 3], 2, 20, 16)
    assert torch.equal(a[2:], b) and torch.equal(na[:, 2:], nb)


def test_pcm16_quantiser():
    b = O.pcm16_bytes(np.array([0.0, 1.0, -1.0, 0.5, 2.0], dtype=np.float32))
    v = np.frombuffer(b, dtype="<i2")
    assert list(v) == [0, 32767, -32767, 16384, 32767]


def test_cfg_composition_config4(states):
    """Config 4 (S=4, batch-doubled CFG, T=312, B=2): the oracle composition vs the reference pieces."""
    g = golden("e2e_cfg_S4_B2_T312.npz")
    ctx = recipe.synthetic_context(2, seed0=int(g["context_seed0"]))
    uc = recipe.synthetic_context(2, seed0=int(g["uncond_seed0"]))
    scale = float(g["cfg_scale"])

    def eps_fn(x, t, w):
        e = O.dit_forward(states["dit"], torch.cat([x, x]), torch.cat([t, t]), torch.cat([uc, ctx]),
                          torch.cat([w, w]))
        e_u, e_c = e.chunk(2)
        return O.cfg_combine(e_u, e_c, scale)
    z = O.lcm_sample(eps_fn, ctx, torch.from_numpy(g["x_T"]), torch.from_numpy(g["noise"]), 4)
    assert rel_l2(z.numpy(), g["latent"]) < 1e-5


def test_bigvgan_long_form_config5(states):
    """Config 5 vocoder leg: 1872 mel frames (30 s) -> 479,232 samples."""
    g = golden("bigvgan_M1872.npz")
    wav = O.bigvgan_forward(states["bigvgan"], torch.from_numpy(g["mel"]))
    assert wav.shape == g["wav"].shape
    assert rel_l2(wav.numpy(), g["wav"]) < 1e-5


def test_text_encoder_oracle():
    """Text conditioning (FrozenCLAPFLANEmbedder.encode from token ids: BERT-base + CLAP Projection + T5-v1.1-large
    encoder, no attention mask) restated in the oracle vs the reference encode() run on transformers' models."""
    g = golden("text_B2_L77.npz")
    W = recipe.text_state(0)
    import hashlib
    h = hashlib.sha256()
    for k in sorted(W):
        h.update(k.encode())
        h.update(W[k].numpy().astype(np.float32).tobytes())
    assert h.hexdigest()[:16] == str(g["digest"])
    with torch.no_grad():
        out = O.text_encode(W, torch.from_numpy(g["clap_ids"]), torch.from_numpy(g["t5_ids"]))
    assert out.shape == (2, 154, 1024)
    assert rel_l2(out.numpy(), g["out"]) < 1e-5


def test_t5_relative_bucket_matches_product_restatement():
    from audiolcm_amd.text_encoder import relative_position_bucket
    for L in (1, 5, 77, 200):
        assert torch.equal(relative_position_bucket(L), O.t5_relative_bucket(L))


def test_vae_encoder_oracle():
    """Encoder1D + quant_conv (audiolcm.yaml ddconfig) restated vs the reference AutoencoderKL.encode moments."""
    W = recipe.vae_encoder_state(0)
    for M in (40, 624):
        g = golden(f"vae_enc_M{M}.npz")
        with torch.no_grad():
            mom = O.vae_encode_moments(W, torch.from_numpy(g["mel"]))
        assert mom.shape == g["moments"].shape == (1, 40, M // 2)
        assert rel_l2(mom.numpy(), g["moments"]) < 1e-5


def test_mel_front_end_oracle():
    """NAT_mel.MelNet (reflect pad, |STFT|, mel projection, log10) restated vs the reference run on the restated
    librosa slaney filterbank (the filterbank itself is parity unpinned: librosa is absent)."""
    from audiolcm_amd.mel import mel_filterbank
    g = golden("mel_B2.npz")
    np.testing.assert_array_equal(mel_filterbank(16000, 1024, 80, 0, 8000), g["mel_basis"])
    mel = O.mel_spectrogram(torch.from_numpy(g["wav"]), torch.from_numpy(g["mel_basis"]))
    assert mel.shape == g["mel"].shape == (2, 80, 96)
    assert rel_l2(mel.numpy(), g["mel"]) < 1e-5


def test_mel_filterbank_properties():
    """Slaney filterbank sanity (the values are unpinned): 80 triangles over 0..8 kHz, non-negative, each filter
    non-zero on a contiguous band, peaks ordered, area-normalised (sum * bin width ~ 2 / bandwidth scale)."""
    from audiolcm_amd.mel import mel_filterbank
    fb = mel_filterbank(16000, 1024, 80, 0, 8000)
    assert fb.shape == (80, 513) and (fb >= 0).all()
    peaks = fb.argmax(1)
    assert (np.diff(peaks) >= 0).all() and peaks[-1] > peaks[0]
    for row in fb:
        nz = np.nonzero(row)[0]
        assert len(nz) > 0 and (np.diff(nz) == 1).all()
