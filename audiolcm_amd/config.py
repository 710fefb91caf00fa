"""Config surface: YAML loading and the ``target:`` plugin mechanism.

The reference resolves every component of ``configs/audiolcm.yaml`` with
``instantiate_from_config`` / ``get_obj_from_str`` (ldm/util.py:111-126).  Here
the same mechanism runs over an alias table that maps the reference's dotted
``target`` strings onto the MI355X classes, so an unchanged audiolcm.yaml builds
the HIP path.  OmegaConf is not available offline; ``load_config`` returns an
attribute-access dict built with ``yaml.safe_load``.
"""
from __future__ import annotations

import importlib
from typing import Any, Dict

import yaml

# reference target -> build class
TARGET_ALIASES: Dict[str, str] = {
    "ldm.models.diffusion.lcm_audio.LCM_audio": "audiolcm_amd.lcm.LCM_audio",
    "ldm.modules.diffusionmodules.concatDiT.ConcatDiT2MLP": "audiolcm_amd.models.ConcatDiT2MLP",
    "ldm.models.autoencoder1d.AutoencoderKL": "audiolcm_amd.models.AutoencoderKL",
    "vocoder.bigvgan.models.VocoderBigVGAN": "audiolcm_amd.models.VocoderBigVGAN",
    "vocoder.bigvgan.models.BigVGAN": "audiolcm_amd.models.BigVGAN",
    "ldm.modules.encoders.modules.FrozenCLAPFLANEmbedder": "audiolcm_amd.text_encoder.FrozenCLAPFLANEmbedder",
    "ldm.models.diffusion.scheduling_lcm.LCMSampler": "audiolcm_amd.lcm.LCMSampler",
    "ldm.data.tsvdataset.TSVDatasetStruct": "audiolcm_amd.data.TSVDatasetStruct",
    "ldm.data.tsvdataset.TSVDataset": "audiolcm_amd.data.TSVDataset",
}
# accepted but inert at inference (training-only components named by the YAML)
INERT_TARGETS = {"torch.nn.Identity", "ldm.lr_scheduler.LambdaLinearScheduler"}


class Cfg(dict):
    """Minimal OmegaConf stand-in: nested dicts with attribute access."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def _wrap(x):
    if isinstance(x, dict):
        return Cfg({k: _wrap(v) for k, v in x.items()})
    if isinstance(x, list):
        return [_wrap(v) for v in x]
    return x


def load_config(path: str) -> Cfg:
    with open(path) as f:
        return _wrap(yaml.safe_load(f))


def get_obj_from_str(string: str, reload: bool = False):
    """ldm/util.py:121-126, with the alias table in front."""
    string = TARGET_ALIASES.get(string, string)
    module, cls = string.rsplit(".", 1)
    if module.startswith("ldm.") or module.startswith("vocoder."):
        raise ImportError(f"target '{string}' has no MI355X implementation (out of the hot-path scope)")
    mod = importlib.import_module(module)
    if reload:
        importlib.reload(mod)
    return getattr(mod, cls)


def instantiate_from_config(config: Any, **extra):
    """ldm/util.py:111-118: ``{"target": dotted.path, "params": {...}}`` -> object."""
    if "target" not in config:
        if config in ("__is_first_stage__", "__is_unconditional__"):
            return None
        raise KeyError("Expected key `target` to instantiate.")
    target = config["target"]
    params = dict(config.get("params", dict()) or {})
    if target in INERT_TARGETS:
        import torch
        return torch.nn.Identity() if target == "torch.nn.Identity" else None
    cls = get_obj_from_str(target)
    import inspect
    try:
        sig = inspect.signature(cls)
        accepts_kw = any(p.kind == p.VAR_KEYWORD for p in sig.parameters.values())
        extra = {k: v for k, v in extra.items() if accepts_kw or k in sig.parameters}
    except (TypeError, ValueError):
        pass
    return cls(**params, **extra)
