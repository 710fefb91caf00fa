"""Text conditioning stand-in for ``FrozenCLAPFLANEmbedder`` (ldm/modules/encoders/modules.py:529-582).

The real encoder (BERT-base + CLAP projection + T5-v1.1-large, 77 tokens each)
is SURVEY.md §8f "next" row 1 and its weights/tokenizers are not available
offline.  This class keeps the reference interface (``encode(dict of caption
lists) -> (B, 154, 1024)``) and returns a deterministic synthetic embedding
per caption (seeded by a stable hash of the struct caption), so the public
API runs end to end; it raises if real weights are requested.
"""
from __future__ import annotations

import zlib
from typing import Dict, List

import torch


class FrozenCLAPFLANEmbedder:
    def __init__(self, weights_path=None, t5version=None, max_length=77, device="cuda", synthetic: bool = True,
                 **unused):
        self.max_length = max_length
        self.synthetic = synthetic
        self.weights_path = weights_path

    @staticmethod
    def caption_seed(caption: str) -> int:
        return zlib.crc32(caption.encode("utf-8")) & 0x7FFFFFFF

    def encode(self, text: Dict[str, List[str]]) -> torch.Tensor:
        caps = text["struct_caption"] if isinstance(text, dict) else list(text)
        rows = [torch.randn((2 * self.max_length, 1024), generator=torch.Generator().manual_seed(self.caption_seed(c)))
                for c in caps]
        return torch.stack(rows, 0).to("cuda")

    __call__ = encode
