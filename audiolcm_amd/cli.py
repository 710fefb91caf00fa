"""Config-1 command line: ``scripts/txt2audio_for_lcm.py`` on the MI355X path.

Mirrors the reference CLI (scripts/txt2audio_for_lcm.py:48-152 arguments, :209-270 main) — the same flags,
output names and ``result.csv`` — with every model stage in libaudiolcm_hip.  Differences, all deliberate:
  * prompts are generated in batches (``--batch-size``, the reference loops at batch 1) with per-clip RNG
    seeds derived from the global prompt index, the iteration and the sample
    (``--seed + (prompt * n_iter + iteration) * n_samples + sample``; the reference draws from the global RNG),
    so outputs do not depend on the batching;
  * ``--prompt_txt`` lines become ``{'ori_caption': p, 'struct_caption': '<p& all>'}`` as InferAPI.py:137 builds
    them (the reference passes the raw string to ``gen_test_sample``, which fails on ``prompt.items()``);
  * the unused unconditional embedding (``uc``, computed when ``--scale != 1`` and never passed to the LCM
    sampler, :90-92) is skipped;
  * ``--plms`` (teacher sampler, out of the hot-path scope and broken for LCM_audio, plms.py:185) and
    ``--inpaint`` raise;
  * ``--synthetic-seed N`` runs on the seeded recipe weights (no checkpoints offline).
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .config import instantiate_from_config, load_config
from .infer_api import load_model_from_config, struct_caption
from .lcm import LCMSampler
from .models import VocoderBigVGAN
from .wavio import write_pcm16


def parse_args(argv: Optional[Sequence[str]] = None):
    p = argparse.ArgumentParser(description="AudioLCM text-to-audio on MI355X (scripts/txt2audio_for_lcm.py)")
    p.add_argument("--prompt_txt", type=str, nargs="?", default="prompt.txt", help="txt file with prompts in it")
    p.add_argument("--sample_rate", type=int, default=22050, help="sample rate of wav")
    p.add_argument("--inpaint", action="store_true", help="if test txt guided inpaint task")
    p.add_argument("--test-dataset", default="none", help="test which dataset: audiocaps/clotho/fsd50k")
    p.add_argument("--outdir", type=str, nargs="?", default="outputs/txt2audio-samples", help="dir to write results to")
    p.add_argument("--ddim_steps", type=int, default=100, help="number of ddim sampling steps")
    p.add_argument("--plms", action="store_true", help="use plms sampling")
    p.add_argument("--n_iter", type=int, default=1, help="sample this often")
    p.add_argument("--H", type=int, default=20, help="image height, in pixel space")
    p.add_argument("--W", type=int, default=312, help="image width, in pixel space")
    p.add_argument("--n_samples", type=int, default=1, help="how many samples to produce for the given prompt")
    p.add_argument("--scale", type=float, default=5.0, help="guidance scale (LCM w-embedding: w = scale - 1)")
    p.add_argument("-r", "--resume", type=str, const=True, default="", nargs="?", help="checkpoint to load")
    p.add_argument("-b", "--base", type=str, default="configs/audiolcm.yaml", help="path to the base config")
    p.add_argument("--vocoder-ckpt", type=str, default="vocoder/logs/audioset", help="path to vocoder checkpoint")
    # MI355X build options
    p.add_argument("--synthetic-seed", type=int, default=None, help="run on the seeded synthetic recipe weights")
    p.add_argument("--synthetic-tokenizer", action="store_true",
                   help="with -r: use the hash-id tokenizer stand-in when the tokenizer directories are absent")
    p.add_argument("--batch-size", type=int, default=32, help="prompts per batched generation")
    p.add_argument("--seed", type=int, default=0, help="per-clip RNG seeds: seed + (prompt * n_iter + iteration) * n_samples + sample")
    p.add_argument("--precision", choices=["split", "mixed", "bf16"], default="mixed",
                   help="MFMA precision policy (DESIGN.md §3)")
    p.add_argument("--test-dataset-tsv", type=str, default=None, help="override the config's test_dataset tsv_path")
    return p.parse_args(argv)


class GenSamples:
    """scripts/txt2audio_for_lcm.py:96-147 (GenSamples.gen_test_sample), batched over prompts."""

    def __init__(self, opt, sampler: LCMSampler, model, outpath: str, vocoder, save_mel: bool = True,
                 save_wav: bool = True, original_inference_steps: Optional[int] = None):
        self.opt, self.sampler, self.model, self.outpath = opt, sampler, model, outpath
        self.vocoder = vocoder
        self.save_mel, self.save_wav = save_mel, save_wav
        self.channel_dim = model.channels
        self.original_inference_steps = original_inference_steps

    def clip_seed(self, prompt_index: int, it: int, j: int) -> int:
        """RNG seed of sample j of iteration `it` of the prompt at global index `prompt_index` (batch-invariant)."""
        return self.opt.seed + (prompt_index * self.opt.n_iter + it) * self.opt.n_samples + j

    def gen_batch(self, prompts: List[Dict[str, str]], names: List[str], first_index: int = 0) -> List[Dict[str, str]]:
        """prompts[i] (global prompt index first_index + i) -> n_iter x n_samples clips named <names[i]>_<idx>;
        returns the records in the reference's order (per prompt, per iteration, per sample)."""
        n = self.opt.n_samples
        records: List[List[Dict[str, str]]] = [[] for _ in prompts]
        for it in range(self.opt.n_iter):
            text = {"ori_caption": [p["ori_caption"] for p in prompts for _ in range(n)],
                    "struct_caption": [p["struct_caption"] for p in prompts for _ in range(n)]}
            c = self.model.get_learned_conditioning(text)
            B = c.shape[0]
            seeds = [self.clip_seed(first_index + i, it, j) for i in range(len(prompts)) for j in range(n)]
            shape = [self.channel_dim, self.opt.H, self.opt.W] if self.channel_dim > 0 else [self.opt.H, self.opt.W]
            z, _ = self.sampler.sample(S=self.opt.ddim_steps, conditioning=c, batch_size=B, shape=shape,
                                       verbose=False, guidance_scale=self.opt.scale,
                                       original_inference_steps=self.original_inference_steps, seeds=seeds)
            mel = self.model.decode_first_stage(z)
            wav = self.vocoder.vocode(mel).squeeze(1).cpu().numpy() if self.save_wav else None
            mel_np = mel.cpu().numpy()
            for i in range(len(prompts)):
                for j in range(n):
                    idx = it * n + j  # the reference restarts idx per iteration (overwriting files); keep them apart
                    k = i * n + j
                    rec = {"caption": prompts[i]["ori_caption"]}
                    if self.save_mel:
                        mp = os.path.join(self.outpath, f"{names[i]}_{idx}.npy")
                        np.save(mp, mel_np[k])
                        rec["mel_path"] = mp
                    if self.save_wav:
                        wp = os.path.join(self.outpath, f"{names[i]}_{idx}.wav")
                        write_pcm16(wp, wav[k], self.opt.sample_rate)
                        rec["audio_path"] = wp
                    records[i].append(rec)
        return [r for rs in records for r in rs]


def build(opt):
    if opt.plms:
        raise NotImplementedError("--plms: the teacher PLMS sampler is outside the LCM hot path (and calls the 3-arg "
                                  "apply_model, plms.py:185, which LCM_audio does not have)")
    if opt.inpaint:
        raise NotImplementedError("--inpaint is not part of the text-to-audio path")
    config = load_config(opt.base)
    split = {"split": True, "bf16": "bf16", "mixed": "mixed"}[opt.precision]
    if opt.synthetic_seed is not None:
        model = load_model_from_config(config, None, split=split, synthetic_seed=opt.synthetic_seed)
        from . import recipe
        vocoder = VocoderBigVGAN(state=recipe.bigvgan_state(opt.synthetic_seed), split=split)
    else:
        if not opt.resume or not os.path.exists(str(opt.resume)):
            raise FileNotFoundError(f"checkpoint {opt.resume!r} not found (pass --synthetic-seed N to run on the "
                                    "seeded synthetic weights)")
        model = load_model_from_config(config, opt.resume, split=split)
        if opt.synthetic_tokenizer and model.cond_stage_model is not None:
            model.cond_stage_model.use_synthetic_tokenizer()
        if "bigv" not in opt.vocoder_ckpt:
            raise NotImplementedError(f"vocoder {opt.vocoder_ckpt!r}: only BigVGAN checkpoints are on the path")
        vocoder = VocoderBigVGAN(opt.vocoder_ckpt, split=split)
    return config, model, LCMSampler(model), vocoder


def main(argv: Optional[Sequence[str]] = None) -> List[Dict[str, str]]:
    opt = parse_args(argv)
    config, model, sampler, vocoder = build(opt)
    os.makedirs(opt.outdir, exist_ok=True)
    gen = GenSamples(opt, sampler, model, opt.outdir, vocoder, save_mel=False, save_wav=True,
                     original_inference_steps=config.model.params.num_ddim_timesteps)
    csv_dicts: List[Dict[str, str]] = []
    bs = max(1, opt.batch_size // max(1, opt.n_samples))
    with torch.no_grad():
        if opt.test_dataset != "none":
            if opt.test_dataset not in ("audiocaps", "clotho", "fsd50k"):
                raise ValueError(f"unknown test dataset {opt.test_dataset!r}")
            key = "test_dataset3" if opt.test_dataset == "fsd50k" else "test_dataset"
            dcfg = dict(config[key])
            if opt.test_dataset_tsv:
                dcfg["params"] = dict(dcfg.get("params", {}), tsv_path=opt.test_dataset_tsv)
            test_dataset = instantiate_from_config(dcfg)
            test_dataset.load_mel = False  # ground-truth mels are for evaluation only
            print(f"Dataset: {type(test_dataset)} LEN: {len(test_dataset)}")
            for lo in range(0, len(test_dataset), bs):
                prompts, names = [], []
                for item in (test_dataset[i] for i in range(lo, min(lo + bs, len(test_dataset)))):
                    f_name = item["f_name"]
                    cut = f_name.rfind("_")  # file name = video_name + '_' + num
                    v_n, num = f_name[:cut], f_name[cut + 1:]
                    prompts.append(dict(item["caption"]))
                    names.append(f"{v_n}_sample_{num}")
                csv_dicts.extend(gen.gen_batch(prompts, names, lo))
            import pandas as pd
            pd.DataFrame.from_dict(csv_dicts).to_csv(os.path.join(opt.outdir, "result.csv"), sep="\t", index=False)
        else:
            with open(opt.prompt_txt) as f:
                lines = [l.strip() for l in f.readlines() if l.strip()]
            for lo in range(0, len(lines), bs):
                chunk = lines[lo:lo + bs]
                csv_dicts.extend(gen.gen_batch([dict(ori_caption=p, struct_caption=struct_caption(p)) for p in chunk],
                                               [p.replace(" ", "-") for p in chunk], lo))
    print(f"Your samples are ready and waiting four you here: \n{opt.outdir} \nEnjoy.")
    return csv_dicts


if __name__ == "__main__":
    main(sys.argv[1:])
