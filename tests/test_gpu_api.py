"""Public surface on the GPU: checkpoint ingestion and the config-1 CLI / dataset mode (§8f-3).

* A Lightning-shaped ``.ckpt`` (``state_dict`` with ``model.`` / ``unet.`` / ``target_unet.`` / ``first_stage_model.``
  / ``cond_stage_model.`` keys plus non-tensor ``hyper_parameters`` / callbacks / optimizer state) and a BigVGAN
  ``best_netG.pt['generator']`` (weight_g / weight_v) + ``args.yml`` directory load through
  ``AudioLCMBatchInfer(model_path=..., vocoder_path=...)`` and give the same PCM16 files, byte for byte, as the
  recipe-loaded pipeline (InferAPI.py:26-45, vocoder/bigvgan/models.py:393-404).
* ``scripts/txt2audio_for_lcm.py`` (audiolcm_amd/cli.py) in ``--prompt_txt`` mode and ``--test-dataset audiocaps``
  mode: WAV names ``<prompt-dashes>_<idx>.wav`` / ``<name>_sample_<num>_<idx>.wav`` and ``result.csv``
  (scripts/txt2audio_for_lcm.py:236-268).
"""
import os

import numpy as np
import pytest
import torch

from conftest import REPO

pytestmark = pytest.mark.gpu

CFG = os.path.join(REPO, "configs", "audiolcm.yaml")
BIGVGAN_ARGS = {"resblock": "1", "upsample_rates": [4, 4, 2, 2, 2, 2], "upsample_kernel_sizes": [8, 8, 4, 4, 4, 4],
                "upsample_initial_channel": 1536, "resblock_kernel_sizes": [3, 7, 11],
                "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5], [1, 3, 5]], "activation": "snakebeta",
                "snake_logscale": True, "num_mels": 80, "hop_size": 256, "sampling_rate": 16000}


class _HParams:  # a Lightning checkpoint pickles objects like this (OmegaConf configs, Namespaces)
    def __init__(self, **kw):
        self.__dict__.update(kw)


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from audiolcm_amd import _hip
    _hip.require_device(0)


def test_checkpoint_ingestion_matches_recipe(gpu, tmp_path):
    import yaml
    from audiolcm_amd import recipe
    from audiolcm_amd.infer_api import AudioLCMBatchInfer
    sd = {}
    dit = recipe.dit_state(0)
    for pre in ("model.diffusion_model.", "unet.diffusion_model.", "target_unet.diffusion_model."):
        sd.update({pre + k: v for k, v in dit.items()})
    sd.update({"first_stage_model." + k: v for k, v in recipe.vae_state(0).items()})
    sd.update({"first_stage_model." + k: v for k, v in recipe.vae_encoder_state(0).items()})
    sd["first_stage_model.loss.discriminator.main.0.weight"] = torch.zeros(64, 1, 4, 4)  # training-only: ignored
    sd.update({"cond_stage_model." + k: v for k, v in recipe.text_state(0).items()})
    sd["scale_factor"] = torch.tensor(1.0)
    sd["alphas_cumprod"] = torch.ones(1000)
    ckpt = {"state_dict": sd, "hyper_parameters": _HParams(base_learning_rate=3e-6), "epoch": 184,
            "callbacks": {_HParams: {"best_model_score": None}}, "optimizer_states": [{"state": {}}]}
    mp = str(tmp_path / "000184.ckpt")
    torch.save(ckpt, mp)
    del ckpt, sd
    vd = tmp_path / "vocoder"
    vd.mkdir()
    torch.save({"generator": recipe.bigvgan_state(0), "steps": 935000}, str(vd / "best_netG.pt"))
    (vd / "args.yml").write_text(yaml.safe_dump(BIGVGAN_ARGS))
    prompts = ["a dog barks", "rain falls on a tin roof"]
    out_ck, out_rc = tmp_path / "ck", tmp_path / "rc"
    with pytest.raises(RuntimeError, match="tokenizer"):  # real-layout weights, no vocabulary: refuse, don't guess
        AudioLCMBatchInfer(prompts, config_path=CFG, model_path=mp, vocoder_path=str(vd), outpath=str(out_ck), seed=7)
    p1 = AudioLCMBatchInfer(prompts, config_path=CFG, model_path=mp, vocoder_path=str(vd), outpath=str(out_ck),
                            seed=7, synthetic_tokenizer=True)
    p2 = AudioLCMBatchInfer(prompts, config_path=CFG, synthetic_seed=0, outpath=str(out_rc), seed=7)
    assert os.path.basename(p1) == os.path.basename(p2) == "rain-falls-on-a-tin-roof_0.wav"
    for p in prompts:
        name = p.replace(" ", "-") + "_0.wav"
        a, b = (open(os.path.join(d, name), "rb").read() for d in (out_ck, out_rc))
        assert a == b and len(a) > 159744 * 2


def test_cli_prompt_txt_and_audiocaps_dataset(gpu, tmp_path):
    import pandas as pd
    from audiolcm_amd.cli import main
    from audiolcm_amd.wavio import read_pcm16
    from test_host import AUDIOCAPS_ROWS
    txt = tmp_path / "prompts.txt"
    txt.write_text("a dog barks\nbirds chirping in a forest\n")
    out1 = tmp_path / "txt"
    main(["--prompt_txt", str(txt), "--outdir", str(out1), "--ddim_steps", "2", "--sample_rate", "16000",
          "-b", CFG, "--synthetic-seed", "0"])
    assert sorted(os.listdir(out1)) == ["a-dog-barks_0.wav", "birds-chirping-in-a-forest_0.wav"]
    data, sr = read_pcm16(str(out1 / "a-dog-barks_0.wav"))
    assert sr == 16000 and data.shape == (159744,) and np.abs(data).max() > 0
    tsv = tmp_path / "caps.tsv"
    tsv.write_text(AUDIOCAPS_ROWS)
    out2 = tmp_path / "ds"
    recs = main(["--test-dataset", "audiocaps", "--test-dataset-tsv", str(tsv), "--outdir", str(out2),
                 "--ddim_steps", "2", "--sample_rate", "16000", "-b", CFG, "--synthetic-seed", "0",
                 "--n_samples", "2", "--batch-size", "4"])
    df = pd.read_csv(out2 / "result.csv", sep="\t")
    assert list(df.columns) == ["caption", "audio_path"] and len(df) == 6 == len(recs)
    names = [os.path.basename(p) for p in df["audio_path"]]
    assert names == ["Y7fmOlUlwoNg_sample_0_0.wav", "Y7fmOlUlwoNg_sample_0_1.wav", "Y6BJ455B1aAs_sample_0_0.wav",
                     "Y6BJ455B1aAs_sample_0_1.wav", "Y7fmOlUlwoNg_sample_1_0.wav", "Y7fmOlUlwoNg_sample_1_1.wav"]
    assert df["caption"][2].startswith("A rocket flies by")
    assert all(os.path.exists(p) for p in df["audio_path"])


def test_vocoder_numpy_vocode_branch(gpu, tmp_path):
    """VocoderBigVGAN.vocode (vocoder/bigvgan/models.py:406-411) with a numpy (80, M) mel returns a numpy waveform equal
    to the tensor path; loaded from best_netG.pt + args.yml."""
    import yaml
    from audiolcm_amd import recipe
    from audiolcm_amd.models import VocoderBigVGAN
    from conftest import golden
    vd = tmp_path / "voc"
    vd.mkdir()
    torch.save({"generator": recipe.bigvgan_state(0)}, str(vd / "best_netG.pt"))
    (vd / "args.yml").write_text(yaml.safe_dump(BIGVGAN_ARGS))
    voc = VocoderBigVGAN(str(vd))
    g = golden("bigvgan_M20.npz")
    w_np = voc.vocode(g["mel"][0])
    assert isinstance(w_np, np.ndarray) and w_np.shape == (20 * 256,)
    w_t = voc.vocode(torch.from_numpy(g["mel"]).cuda()).reshape(-1).cpu().numpy()
    assert np.array_equal(w_np, w_t)
    assert np.linalg.norm(w_np - g["wav"].reshape(-1)) / np.linalg.norm(g["wav"]) < 1e-3
