"""Public inference API with the reference signatures (pythonscripts/InferAPI.py:26-166).

``AudioLCMInfer`` / ``AudioLCMBatchInfer`` build the model from the YAML config surface,
generate 2-step LCM samples, vocode them and write PCM16 16 kHz WAVs to
``results/test/<prompt-with-dashes>_0.wav``, returning the (last) path like the reference.
Prompts are batched (the reference loops at batch 1); everything on the path runs in the HIP
library.  Checkpoints are read with safe loaders only (audiolcm_amd/ckpt.py: ``weights_only=True`` with inert
placeholders for a Lightning checkpoint's non-tensor objects; yaml.safe_load).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import torch

from . import recipe
from .ckpt import load_checkpoint, state_dict_of
from .config import instantiate_from_config, load_config
from .lcm import LCM_audio, LCMSampler
from .models import BigVGAN, VocoderBigVGAN
from .wavio import write_pcm16


def load_model_from_config(config, ckpt: Optional[str] = None, verbose: bool = True, split: bool = True,
                           synthetic_seed: Optional[int] = None) -> LCM_audio:
    """InferAPI.py:26-45: instantiate LCM_audio and load the Lightning ``state_dict``."""
    model = instantiate_from_config(config.model, split=split)
    if ckpt:
        print(f"Loading model from {ckpt}")
        model.load_state_dict(state_dict_of(load_checkpoint(ckpt)), strict=False)
    elif synthetic_seed is not None:
        model.load_recipe(synthetic_seed)
    else:
        print("Note chat no ckpt is loaded !!!")
    return model


def struct_caption(p: str) -> str:
    return f"<{p}& all>"


def wav_name_for(prompt: str) -> str:
    return prompt.strip().replace(" ", "-")


class GenSamples:
    """InferAPI.py:49-101, batched."""

    def __init__(self, sampler: LCMSampler, model: LCM_audio, outpath: str, vocoder=None, save_mel=True,
                 save_wav=True, original_inference_steps=None, steps: int = 2, guidance_scale: float = 5.0):
        self.sampler, self.model, self.outpath = sampler, model, outpath
        if save_wav:
            assert vocoder is not None
        self.vocoder = vocoder
        self.save_mel, self.save_wav = save_mel, save_wav
        self.channel_dim = model.channels
        self.original_inference_steps = original_inference_steps or 50
        self.steps, self.guidance_scale = steps, guidance_scale

    def gen_batch(self, prompts: List[Dict[str, str]], names: List[str], seeds=None) -> List[Dict[str, str]]:
        c = self.model.get_learned_conditioning({"ori_caption": [p["ori_caption"] for p in prompts],
                                                 "struct_caption": [p["struct_caption"] for p in prompts]})
        shape = [self.model.mel_dim, self.model.mel_length]
        z, _ = self.sampler.sample(S=self.steps, conditioning=c, batch_size=len(prompts), shape=shape,
                                   verbose=False, guidance_scale=self.guidance_scale,
                                   original_inference_steps=self.original_inference_steps, seeds=seeds)
        mel = self.model.decode_first_stage(z)
        wav = self.vocoder.vocode(mel).squeeze(1).cpu().numpy() if self.save_wav else None
        mel_np = mel.cpu().numpy()
        records = []
        for i, p in enumerate(prompts):
            rec = {"caption": p["ori_caption"]}
            if self.save_mel:
                mp = os.path.join(self.outpath, names[i] + "_0.npy")
                np.save(mp, mel_np[i])
                rec["mel_path"] = mp
            if self.save_wav:
                wp = os.path.join(self.outpath, names[i] + "_0.wav")
                write_pcm16(wp, wav[i], 16000)
                rec["audio_path"] = wp
            records.append(rec)
        return records

    def gen_test_sample(self, prompt: Dict[str, str], mel_name=None, wav_name=None):
        name = wav_name or mel_name or wav_name_for(prompt["ori_caption"])
        return self.gen_batch([prompt], [name])


def _build(config_path, model_path, vocoder_path, synthetic_seed, split, synthetic_tokenizer=False):
    config = load_config(config_path)
    if synthetic_seed is None:
        if not model_path or not os.path.exists(model_path):
            raise FileNotFoundError(f"model checkpoint {model_path!r} not found (pass synthetic_seed=... to run "
                                    "on the seeded synthetic weights)")
        if not vocoder_path or not os.path.exists(os.path.join(vocoder_path, "best_netG.pt")):
            raise FileNotFoundError(f"vocoder checkpoint dir {vocoder_path!r} not found")
        model = load_model_from_config(config, model_path, split=split)
        if synthetic_tokenizer and model.cond_stage_model is not None:
            model.cond_stage_model.use_synthetic_tokenizer()
        vocoder = VocoderBigVGAN(vocoder_path, split=split)
    else:
        model = load_model_from_config(config, None, split=split, synthetic_seed=synthetic_seed)
        vocoder = VocoderBigVGAN(state=recipe.bigvgan_state(synthetic_seed), h=None, split=split)
    sampler = LCMSampler(model)
    steps_cfg = config.model.params.get("num_ddim_timesteps", 50)
    return model, sampler, vocoder, steps_cfg


def AudioLCMBatchInfer(ori_prompts: List[str], config_path: str = "configs/audiolcm.yaml",
                       model_path: str = "./model/000184.ckpt", vocoder_path: str = "./model/vocoder",
                       batch_size: int = 32, synthetic_seed: Optional[int] = None, split: bool = True,
                       outpath: str = "results/test", seed: Optional[int] = None,
                       synthetic_tokenizer: bool = False) -> str:
    """InferAPI.py:135-166. Returns the path of the last prompt's WAV.  ``seed``: per-prompt RNG seeds
    seed + i (default None: the global device RNG, as the reference).  ``synthetic_tokenizer``: run checkpoint
    weights on the hash-id tokenizer stand-in when the tokenizer directories are absent (tests only)."""
    prompts = [dict(ori_caption=p, struct_caption=struct_caption(p)) for p in ori_prompts]
    model, sampler, vocoder, orig_steps = _build(config_path, model_path, vocoder_path, synthetic_seed, split,
                                                 synthetic_tokenizer)
    os.makedirs(outpath, exist_ok=True)
    gen = GenSamples(sampler, model, outpath, vocoder, save_mel=False, save_wav=True,
                     original_inference_steps=orig_steps)
    names = [wav_name_for(p["ori_caption"]) for p in prompts]
    with torch.no_grad():
        for lo in range(0, len(prompts), batch_size):
            n = len(prompts[lo:lo + batch_size])
            gen.gen_batch(prompts[lo:lo + batch_size], names[lo:lo + batch_size],
                          seeds=None if seed is None else list(range(seed + lo, seed + lo + n)))
    print(f"Your samples are ready and waiting four you here: \n{outpath} \nEnjoy.")
    return os.path.join(outpath, names[-1] + "_0.wav")


def AudioLCMInfer(ori_prompt: str, config_path: str = "configs/audiolcm.yaml",
                  model_path: str = "./model/000184.ckpt", vocoder_path: str = "./model/vocoder",
                  synthetic_seed: Optional[int] = None, split: bool = True, outpath: str = "results/test",
                  seed: Optional[int] = None) -> str:
    """InferAPI.py:103-133."""
    return AudioLCMBatchInfer([ori_prompt], config_path, model_path, vocoder_path, 1, synthetic_seed, split, outpath,
                              seed)
