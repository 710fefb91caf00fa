"""Generate the golden parity fixtures by running the *reference* AudioLCM code.

Runs ONLY in the build container, where the read-only reference checkout is
mounted at /root/reference (never on the GPU box).  It imports the reference
hot-path modules with in-process ``sys.modules`` stubs for import-only,
non-arithmetic packages that are absent here (pytorch_lightning, omegaconf,
pytorch_memlab, torchvision, taming, icecream), loads the
build's seeded synthetic weights (``audiolcm_amd.recipe``) into the reference
modules, and writes input/output vectors as ``.npz`` files next to this script.

The fixtures pin ``oracle/alcm_oracle.py`` (tests/test_oracle_golden.py) and the
HIP path's model-level outputs (tests/test_gpu_models.py).

Usage:  python tests/golden/make_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import hashlib
import math
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from audiolcm_amd import recipe  # noqa: E402


def install_stubs():
    class LM(nn.Module):
        @property
        def device(self):
            return next(self.parameters()).device

    def mod(name, **attrs):
        m = types.ModuleType(name)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    di = mod("pytorch_lightning.utilities.distributed", rank_zero_only=lambda f: f)
    ut = mod("pytorch_lightning.utilities", distributed=di)
    mod("pytorch_lightning", LightningModule=LM, utilities=ut)
    mod("pytorch_memlab", LineProfiler=object, profile=lambda f: f)
    tvu = mod("torchvision.utils", make_grid=None)
    mod("torchvision", utils=tvu)
    q = mod("taming.modules.vqvae.quantize", VectorQuantizer2=object)
    v = mod("taming.modules.vqvae", quantize=q)
    m = mod("taming.modules", vqvae=v)
    mod("taming", modules=m)
    mod("icecream", ic=print)
    mod("omegaconf", OmegaConf=object, ListConfig=list)
    # the CLAP package imports its (unused) audio encoder's torchlibrosa front-end; modules.py imports
    # importlib_resources.files (used only to read the CLAP config in __init__)
    st = mod("torchlibrosa.stft", Spectrogram=object, LogmelFilterBank=object)
    mod("torchlibrosa", stft=st)
    import importlib.resources
    mod("importlib_resources", files=importlib.resources.files)


def digest(state):
    h = hashlib.sha256()
    for k in sorted(state):
        h.update(k.encode())
        h.update(state[k].detach().cpu().numpy().astype(np.float32).tobytes())
    return h.hexdigest()[:16]


def load_exact(module, state, prefix=""):
    """Load recipe weights; assert every recipe key exists with the reference shape."""
    ref = module.state_dict()
    for k, t in state.items():
        rk = prefix + k
        assert rk in ref, f"recipe key {rk} missing from reference module"
        assert tuple(ref[rk].shape) == tuple(t.shape), (rk, ref[rk].shape, t.shape)
    missing = module.load_state_dict({prefix + k: v for k, v in state.items()}, strict=False)
    return missing


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in arrays.items()})
    print(f"wrote {name}: {os.path.getsize(path) / 1e6:.2f} MB")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="", help="comma-separated fixture groups to (re)generate: base, c2, c4, c5, text, enc "
                                               "(default: all)")
    args = ap.parse_args()
    groups = set(filter(None, args.only.split(","))) or {"base", "c2", "c4", "c5", "text", "enc"}
    if "text" in groups:  # load transformers' model modules before the stubs shadow torchvision
        from transformers import BertConfig, BertModel, T5Config, T5EncoderModel  # noqa: F401
    install_stubs()
    sys.path.insert(0, args.ref)
    torch.set_num_threads(max(1, len(os.sched_getaffinity(0))))

    from ldm.modules.diffusionmodules.concatDiT import ConcatDiT2MLP
    from ldm.models.autoencoder1d import AutoencoderKL
    from ldm.models.diffusion.lcm_audio import LCM_audio
    from ldm.models.diffusion import scheduling_lcm
    from ldm.models.diffusion.scheduling_lcm import LCMSampler
    from vocoder.bigvgan.models import BigVGAN
    from vocoder.bigvgan.alias_free_torch import Activation1d
    from vocoder.bigvgan.activations import SnakeBeta

    LCMSampler.register_buffer = lambda self, n, a: setattr(self, n, a)  # reference forces .to('cuda')

    dcfg, vcfg, gcfg = recipe.DiTConfig(), recipe.VAEConfig(), recipe.BigVGANConfig()
    Sd, Sv, Sg = recipe.dit_state(0), recipe.vae_state(0), recipe.bigvgan_state(0)
    meta = dict(dit=digest(Sd), vae=digest(Sv), bigvgan=digest(Sg), torch=torch.__version__)

    dd = dict(double_z=True, in_channels=80, out_ch=80, z_channels=20, kernel_size=5, ch=384,
              ch_mult=[1, 2, 4], num_res_blocks=2, attn_layers=[3], down_layers=[0], dropout=0.0)
    lcm = LCM_audio(
        first_stage_config={"target": "ldm.models.autoencoder1d.AutoencoderKL",
                            "params": {"embed_dim": 20, "ddconfig": dd, "lossconfig": {"target": "torch.nn.Identity"}}},
        cond_stage_config={"target": "torch.nn.Identity"}, linear_start=0.00085, linear_end=0.012,
        num_timesteps_cond=1, log_every_t=200, timesteps=1000, first_stage_key="image",
        cond_stage_key="caption", mel_dim=20, mel_length=312, channels=0, cond_stage_trainable=False,
        conditioning_key="crossattn", monitor="val/loss_simple_ema", scale_by_std=True, use_lcm=True,
        num_ddim_timesteps=50, w_min=4, w_max=12, use_ema=False,
        unet_config={"target": "ldm.modules.diffusionmodules.concatDiT.ConcatDiT2MLP",
                     "params": dict(in_channels=20, context_dim=1024, hidden_size=576, num_heads=8, depth=4,
                                    max_len=1000)}).eval()
    load_exact(lcm.unet.diffusion_model, Sd)
    load_exact(lcm.model.diffusion_model, Sd)
    load_exact(lcm.first_stage_model, Sv)

    class A(dict):
        __getattr__ = dict.__getitem__
    hjson = json.load(open(os.path.join(args.ref, "vocoder/bigvgan/bigvgan_audioset16khz_80band.json")))
    voc = BigVGAN(A(hjson)).eval()
    ref_keys = set(voc.state_dict().keys())
    assert ref_keys == set(Sg.keys()), sorted(ref_keys ^ set(Sg.keys()))[:10]
    load_exact(voc, Sg)
    dit_keys = set(lcm.unet.diffusion_model.state_dict().keys())
    assert dit_keys == set(Sd.keys()), sorted(dit_keys ^ set(Sd.keys()))[:10]

    if "text" in groups:
        with torch.no_grad():
            text_fixture()
    with torch.no_grad():
        smp = LCMSampler(lcm)
        smp.make_schedule(verbose=False)
        orig = scheduling_lcm.torch.randn
        if "base" in groups:
            base_fixtures(lcm, smp, voc, scheduling_lcm, orig, meta, Activation1d, SnakeBeta)
        if "c2" in groups:
            # ---- config 2, single prompts spread over the bench batch: prompt id p has seed p and context seed
            # 1000 + p (bench.py ids 0..31); 31 is the last one, 7 / 15 / 23 the interior ones ----
            for pid in (7, 15, 23, 31):
                xT, noise = recipe.prompt_noise([pid], 2, 20, 312)
                c = recipe.synthetic_context(1, seed0=1000 + pid)
                calls = {"i": 0}

                def fake_randn_p(*a, **k):
                    calls["i"] += 1
                    return noise[calls["i"] - 1].clone()
                scheduling_lcm.torch.randn = fake_randn_p
                try:
                    z, _ = smp.sample(S=2, conditioning=c, batch_size=1, shape=[20, 312], verbose=False,
                                      guidance_scale=5, original_inference_steps=50, x_T=xT.clone())
                finally:
                    scheduling_lcm.torch.randn = orig
                mel = lcm.decode_first_stage(z)
                save(f"e2e_S2_prompt{pid}.npz", x_T=xT, noise=noise, latent=z, mel=mel, wav=voc(mel).squeeze(1))
        if "enc" in groups:
            # ---- audio -> latent direction: Encoder1D + quant_conv of the reference
            # AutoencoderKL, and the reference MelNet (NAT_mel.py) with librosa's filterbank restated
            # (audiolcm_amd/mel.py; librosa is absent, so the filterbank values are parity unpinned)
            load_exact(lcm.first_stage_model, recipe.vae_encoder_state(0))
            for M in (624, 40):
                gx = torch.Generator().manual_seed(400 + M)
                mel = torch.randn((1, 80, M), generator=gx) * 1.5 - 4.0
                post = lcm.first_stage_model.encode(mel)
                save(f"vae_enc_M{M}.npz", mel=mel, moments=post.parameters)
            from audiolcm_amd.mel import NAT_MEL_16K, mel_filterbank
            fb = types.ModuleType("librosa.filters")
            fb.mel = lambda sr, n_fft, n_mels=128, fmin=0.0, fmax=None, **kw: mel_filterbank(sr, n_fft, n_mels, fmin,
                                                                                            fmax)
            sys.modules["librosa"] = types.ModuleType("librosa")
            sys.modules["librosa"].filters = fb
            sys.modules["librosa.filters"] = fb
            from ldm.data.preprocess.NAT_mel import MelNet as RefMelNet
            net = RefMelNet(dict(NAT_MEL_16K))
            gw = torch.Generator().manual_seed(500)
            t = torch.arange(256 * 96, dtype=torch.float64) / 16000.0
            wav = torch.stack([(0.6 * torch.sin(2 * math.pi * 440.0 * t) + 0.3 * torch.sin(2 * math.pi * 3100.0 * t)
                                ).float() + 0.05 * torch.randn(t.shape, generator=gw),
                               1.3 * torch.randn(t.shape, generator=gw).clamp(-2, 2)], 0)  # second row clips
            save("mel_B2.npz", wav=wav, mel_basis=net.mel_basis, mel=net(wav))
        if "c5" in groups:
            # ---- config 5: 30-s long-form vocoder leg (M = 1872 mel frames -> 479,232 samples) ---------
            gm = torch.Generator().manual_seed(300 + 1872)
            mel = torch.randn((1, 80, 1872), generator=gm) * 1.5 - 4.0
            save("bigvgan_M1872.npz", mel=mel, wav=voc(mel))
        if "c4" in groups:
            # ---- config 4: 4 LCM steps with batch-doubled classifier-free guidance at T = 312 ---------
            # The reference LCMSampler has no CFG (scheduling_lcm.py:359-377); config 4 composes the reference
            # pieces: the [uc; c] batch-doubled DiT call and combine of ddim.py:203-205 / plms.py:184-186, then
            # the reference LCMSampler.step (scheduling_lcm.py:410-496) with the recorded step noise.
            S, B, T, scale = 4, 2, 312, 5.0
            xT, noise = recipe.prompt_noise([5, 6], S, 20, T)
            c = recipe.synthetic_context(B)
            uc = recipe.synthetic_context(B, seed0=900)
            smp.set_timesteps(S, original_inference_steps=50)
            smp._step_index = None
            w = torch.tensor(5 - 1).repeat(2 * B)
            wemb = smp.get_guidance_scale_embedding(w, embedding_dim=256)
            img = xT.clone()
            calls = {"i": 0}

            def fake_randn(*a, **k):
                i = calls["i"]
                calls["i"] += 1
                return noise[i].clone()
            scheduling_lcm.torch.randn = fake_randn
            try:
                for t in smp.timesteps:
                    ts = torch.full((2 * B,), int(t), dtype=torch.long)
                    e = lcm.apply_model(torch.cat([img, img]), ts, torch.cat([uc, c]), lcm.unet, w_cond=wemb)
                    e_u, e_c = e.chunk(2)
                    img, den = smp.step(e_u + scale * (e_c - e_u), t, img, return_dict=False)
            finally:
                scheduling_lcm.torch.randn = orig
            assert calls["i"] == S - 1
            save("e2e_cfg_S4_B2_T312.npz", x_T=xT, noise=noise, context_seed0=1000, uncond_seed0=900, cfg_scale=scale, latent=den,
                 mel=lcm.decode_first_stage(den))


def text_fixture():
    """FrozenCLAPFLANEmbedder.encode (ldm/modules/encoders/modules.py:567-582) run as the reference code itself on
    transformers BertModel / T5EncoderModel built from the bert-base-uncased / t5-v1_1-large configs and the
    reference CLAP Projection, all loaded with the recipe's text weights; the tokenizers (vocab files absent
    offline) are replaced by fixed token ids, which encode() receives through stub tokenizer objects."""
    from transformers import BertConfig, BertModel, T5Config, T5EncoderModel
    from ldm.modules.encoders import modules
    from ldm.modules.encoders.CLAP.clap import Projection
    from audiolcm_amd.text_encoder import SyntheticTokenizer
    cfg = recipe.TextConfig()
    W = recipe.text_state(0, cfg)
    bert = BertModel(BertConfig(vocab_size=cfg.b_vocab, hidden_size=cfg.b_hidden, num_hidden_layers=cfg.b_layers,
                                num_attention_heads=cfg.b_heads, intermediate_size=cfg.b_inter,
                                max_position_embeddings=cfg.b_maxpos, attn_implementation="eager")).eval()
    t5 = T5EncoderModel(T5Config(vocab_size=cfg.t_vocab, d_model=cfg.t_d, d_kv=cfg.t_dkv, d_ff=cfg.t_ff,
                                 num_layers=cfg.t_layers, num_heads=cfg.t_heads, feed_forward_proj="gated-gelu",
                                 relative_attention_num_buckets=cfg.t_buckets,
                                 relative_attention_max_distance=cfg.t_max_distance, layer_norm_epsilon=1e-6,
                                 is_encoder_decoder=False, attn_implementation="eager")).eval()
    proj = Projection(cfg.b_hidden, cfg.p_out).eval()
    sub = lambda pre: {k[len(pre):]: v for k, v in W.items() if k.startswith(pre)}
    for m, pre in ((bert, "caption_encoder.base."), (proj, "caption_encoder.projection."), (t5, "t5_transformer.")):
        sd = sub(pre)
        if m is t5:
            sd["encoder.embed_tokens.weight"] = sd["shared.weight"]
        missing, unexpected = m.load_state_dict(sd, strict=False)
        assert not unexpected and not [k for k in missing if "position_ids" not in k], (missing, unexpected)
    caps = ["A man is speaking while birds chirp in the background",
            "Rain falls on a tin roof as thunder rumbles far away, and a dog barks twice near the door"]
    struct = [f"<{c}& all>" for c in caps]
    clap_ids = SyntheticTokenizer("bert", cfg.b_vocab)(caps, max_length=77)["input_ids"]
    t5_ids = SyntheticTokenizer("t5", cfg.t_vocab)(struct, max_length=77)["input_ids"]

    class Tok:
        def __init__(self, ids):
            self.ids = ids

        def __call__(self, texts, **kw):
            return {"input_ids": self.ids}

    class Enc(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.base, self.projection = bert, proj

    stub = types.SimpleNamespace(clap_tokenizer=Tok(clap_ids), t5_tokenizer=Tok(t5_ids), caption_encoder=Enc(),
                                 t5_transformer=t5, max_length=77, device="cpu")
    out = modules.FrozenCLAPFLANEmbedder.encode(stub, {"ori_caption": caps, "struct_caption": struct})
    save("text_B2_L77.npz", clap_ids=clap_ids, t5_ids=t5_ids, out=out, digest=digest(W))


def base_fixtures(lcm, smp, voc, scheduling_lcm, orig, meta, Activation1d, SnakeBeta):
    if True:
        # ---- schedule / embeddings / step -------------------------------------------------
        sched = {}
        for S in (1, 2, 4, 8):
            smp.set_timesteps(S, original_inference_steps=50)
            sched[f"timesteps_S{S}"] = smp.timesteps.numpy()
        w = torch.tensor(5 - 1).repeat(3)
        t = torch.tensor([999, 759, 499, 259, 0], dtype=torch.long)
        te = lcm.unet.diffusion_model.t_embedder.timestep_embedding(t, 256)
        save("schedule.npz", alphas_cumprod=lcm.alphas_cumprod.float(), guidance_w4=smp.get_guidance_scale_embedding(w, 256),
             t=t, timestep_emb=te, **sched, meta=json.dumps(meta))

        g = torch.Generator().manual_seed(7)
        x = torch.randn((2, 20, 16), generator=g)
        eps = torch.randn((2, 20, 16), generator=g)
        nz = torch.randn((2, 20, 16), generator=g)
        smp.set_timesteps(2, original_inference_steps=50)
        smp.num_inference_steps = 2
        smp._step_index = None
        scheduling_lcm.torch.randn = lambda *a, **k: nz.clone()
        try:
            prev0, den0 = smp.step(eps, 999, x, return_dict=False)
            prev1, den1 = smp.step(eps, 499, prev0, return_dict=False)
        finally:
            scheduling_lcm.torch.randn = orig
        save("lcm_step.npz", x=x, eps=eps, noise=nz, prev0=prev0, den0=den0, prev1=prev1, den1=den1)

        # ---- Activation1d / SnakeBeta ------------------------------------------------------
        for T in (50, 3):
            a1 = Activation1d(activation=SnakeBeta(24, alpha_logscale=True)).eval()
            ga = torch.Generator().manual_seed(11 + T)
            a1.act.alpha.copy_(torch.randn(24, generator=ga) * 0.3)
            a1.act.beta.copy_(torch.randn(24, generator=ga) * 0.3)
            xa = torch.randn((2, 24, T), generator=ga) * 1.5
            save(f"act1d_T{T}.npz", x=xa, alpha=a1.act.alpha, beta=a1.act.beta, up_filter=a1.upsample.filter,
                 down_filter=a1.downsample.lowpass.filter, y=a1(xa))

        # ---- DiT ---------------------------------------------------------------------------
        dit = lcm.unet.diffusion_model
        ctx = recipe.synthetic_context(2)
        wemb = smp.get_guidance_scale_embedding(torch.tensor(5 - 1).repeat(2), 256)
        for T in (312, 40):
            gx = torch.Generator().manual_seed(100 + T)
            xd = torch.randn((2, 20, T), generator=gx)
            td = torch.tensor([999, 499], dtype=torch.long)
            out = lcm.apply_model(xd, td, ctx, lcm.unet, w_cond=wemb)
            save(f"dit_T{T}.npz", x=xd, t=td, w_emb=wemb, eps=out, **({"context": ctx} if T == 312 else {}))

        # ---- VAE decode --------------------------------------------------------------------
        for T in (312, 936, 24):
            gz = torch.Generator().manual_seed(200 + T)
            z = torch.randn((1, 20, T), generator=gz)
            save(f"vae_T{T}.npz", z=z, scale_factor=float(lcm.scale_factor), mel=lcm.decode_first_stage(z))

        # ---- BigVGAN -----------------------------------------------------------------------
        for M in (624, 20):
            gm = torch.Generator().manual_seed(300 + M)
            mel = torch.randn((1, 80, M), generator=gm) * 1.5 - 4.0
            save(f"bigvgan_M{M}.npz", mel=mel, wav=voc(mel))

        # ---- end-to-end: sampler (injected RNG) -> decode -> vocode per clip ---------------
        def run_e2e(S, B, T, vocode):
            xT, noise = recipe.prompt_noise(range(B), S, 20, T)
            c = recipe.synthetic_context(B)
            calls = {"i": 0}

            def fake_randn(*a, **k):
                i = calls["i"]
                calls["i"] += 1
                return noise[i].clone()
            scheduling_lcm.torch.randn = fake_randn
            try:
                z, _ = smp.sample(S=S, conditioning=c, batch_size=B, shape=[20, T], verbose=False,
                                  guidance_scale=5, original_inference_steps=50, x_T=xT.clone())
            finally:
                scheduling_lcm.torch.randn = orig
            assert calls["i"] == max(S - 1, 0)
            mel = lcm.decode_first_stage(z)
            out = dict(x_T=xT, noise=noise, latent=z, mel=mel)
            if vocode:
                out["wav"] = torch.stack([torch.from_numpy(np.asarray(voc(m.unsqueeze(0)).squeeze().numpy()))
                                          for m in mel], 0)
            return out

        save("e2e_S2_B2.npz", **run_e2e(2, 2, 312, True))
        save("e2e_S4_B1.npz", **run_e2e(4, 1, 312, False))
        save("e2e_S1_B1_T40.npz", **run_e2e(1, 1, 40, True))


if __name__ == "__main__":
    main()
