"""Checkpoint ingestion without executing anything from the file.

The reference loads its checkpoints with a plain ``torch.load`` (pythonscripts/InferAPI.py:30,
vocoder/bigvgan/models.py:394-400), i.e. a full unpickler.  Here every checkpoint goes through
``torch.load(weights_only=True)``: tensors, containers and primitive values only.  A Lightning ``.ckpt`` also
pickles non-tensor objects (``hyper_parameters`` as OmegaConf / argparse objects, callback classes as dict keys,
optimizer state); their global names are read from the archive without unpickling
(``torch.serialization.get_unsafe_globals_in_checkpoint``) and mapped to inert placeholder classes, so the load
succeeds while none of the checkpoint's own classes or callables is imported or run.  Only the tensors
(``state_dict`` / ``generator``) are used.
"""
from __future__ import annotations

from typing import Any, Dict, List

import torch


class OpaqueObject:
    """Placeholder for a pickled object of a class the loader does not import; keeps its raw state."""

    def __init__(self, *args, **kwargs):
        self._args, self._kwargs = args, kwargs

    def __setstate__(self, state):
        self._state = state

    def __repr__(self):
        return f"<opaque {type(self).__module__}.{type(self).__qualname__}>"


def _placeholder(name: str):
    mod, _, qual = name.rpartition(".")
    return type(qual or name, (OpaqueObject,), {"__module__": mod or "opaque"})


def load_checkpoint(path: str) -> Dict[str, Any]:
    """torch.load(path, weights_only=True) with inert placeholders for the file's non-tensor classes."""
    names: List[str] = torch.serialization.get_unsafe_globals_in_checkpoint(path)
    if not names:
        return torch.load(path, map_location="cpu", weights_only=True)
    with torch.serialization.safe_globals([(_placeholder(n), n) for n in names]):
        return torch.load(path, map_location="cpu", weights_only=True)


def state_dict_of(ckpt: Dict[str, Any], key: str = "state_dict") -> Dict[str, torch.Tensor]:
    """The tensor entries of ckpt[key] (a Lightning checkpoint's ``state_dict``, BigVGAN's ``generator``)."""
    if key not in ckpt:
        raise KeyError(f"checkpoint has no '{key}' entry (keys: {sorted(map(str, ckpt))[:10]})")
    return {k: v for k, v in ckpt[key].items() if torch.is_tensor(v)}
