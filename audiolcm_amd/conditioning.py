"""Text conditioning stand-in for ``FrozenCLAPFLANEmbedder`` (ldm/modules/encoders/modules.py:529-582).

The synthetic mode keeps the reference interface (``encode(dict of caption lists) -> (B, 154, 1024)``) and
returns a deterministic N(0, 1) embedding per caption (seeded by a stable hash of the struct caption), so the
public API runs end to end on the seeded synthetic weights.  Asking for real weights (``synthetic=False`` or a
``weights_path`` that exists) raises NotImplementedError instead of silently returning noise; a configured but
absent ``weights_path`` (the reference YAML's relative path) prints that the synthetic embedding is used.
"""
from __future__ import annotations

import zlib
from typing import Dict, List

import torch


class FrozenCLAPFLANEmbedder:
    def __init__(self, weights_path=None, t5version=None, max_length=77, device="cuda", synthetic: bool = True,
                 **unused):
        import os
        if not synthetic or (weights_path is not None and os.path.exists(str(weights_path))):
            raise NotImplementedError("FrozenCLAPFLANEmbedder with real weights is not available in the synthetic "
                                      "stand-in")
        if weights_path is not None:
            print(f"FrozenCLAPFLANEmbedder: {weights_path!r} not found; using the synthetic caption embedding")
        self.max_length = max_length

    @staticmethod
    def caption_seed(caption: str) -> int:
        return zlib.crc32(caption.encode("utf-8")) & 0x7FFFFFFF

    def encode(self, text: Dict[str, List[str]]) -> torch.Tensor:
        caps = text["struct_caption"] if isinstance(text, dict) else list(text)
        rows = [torch.randn((2 * self.max_length, 1024), generator=torch.Generator().manual_seed(self.caption_seed(c)))
                for c in caps]
        return torch.stack(rows, 0).to("cuda")

    __call__ = encode
