"""Text conditioning on the MI355X path: ``FrozenCLAPFLANEmbedder`` (ldm/modules/encoders/modules.py:529-582).

``encode({"ori_caption": [...], "struct_caption": [...]})`` tokenizes the captions (CLAP-BERT tokenizer for the
original captions, T5 tokenizer for the struct captions, both padded / truncated to max_length = 77) and runs
    z  = Projection(BertModel(clap_ids).last_hidden_state)      CLAP/clap.py:8-20 (linear1, gelu, linear2, LN)
    z2 = T5EncoderModel(t5_ids).last_hidden_state               t5-v1_1-large encoder
    c  = concat([z, z2], dim=1)                                  (B, 154, 1024)
as one C call (``alcm_text_encode``): every linear, attention and norm in libaudiolcm_hip.  As in the reference
no attention mask is passed, so the padding tokens take part in attention.

Weights: the reference's checkpoint layout (``cond_stage_model.caption_encoder.base.*`` / ``.projection.*`` /
``cond_stage_model.t5_transformer.*``, loaded by LCM_audio.load_state_dict), local HuggingFace model
directories with ``model.safetensors`` (the reference's ``from_pretrained`` paths), or the seeded recipe.
Tokenizers: local HuggingFace tokenizer directories (the reference's ``bert-base-uncased`` / ``t5-v1_1-large``
paths).  A deterministic stand-in (``SyntheticTokenizer``, words -> ids by a stable hash) is used only on
request — with the seeded recipe weights (``synthetic_seed`` / ``load_recipe``) or ``synthetic_tokenizer=True`` —
because real encoder weights fed made-up ids would give silently wrong conditioning; without a loadable tokenizer
directory and without that opt-in, ``encode`` raises.  The real vocabularies are not available offline, so
token ids are parity-unpinned, while the encoders themselves are pinned from ids (tests/golden/text_B2_L77.npz).
"""
from __future__ import annotations

import math
import os
import zlib
from typing import Dict, List, Mapping, Optional, Sequence

import torch

from . import _hip, recipe
from ._hip import check, lib, ptr, stream_handle
from .models import _HipModel


def relative_position_bucket(L: int, num_buckets: int = 32, max_distance: int = 128) -> torch.Tensor:
    """Bidirectional T5 relative-position bucket of (key j - query i), (L, L) int64: the rule of
    transformers' ``T5Attention._relative_position_bucket`` (bidirectional=True), restated with the same
    fp32 torch ops so the bucket boundaries round identically."""
    ctx = torch.arange(L, dtype=torch.long)[:, None]
    mem = torch.arange(L, dtype=torch.long)[None, :]
    rel = mem - ctx
    nb = num_buckets // 2
    buckets = (rel > 0).to(torch.long) * nb
    rel = torch.abs(rel)
    max_exact = nb // 2
    is_small = rel < max_exact
    large = max_exact + (torch.log(rel.float() / max_exact) / math.log(max_distance / max_exact)
                         * (nb - max_exact)).to(torch.long)
    large = torch.min(large, torch.full_like(large, nb - 1))
    return buckets + torch.where(is_small, rel, large)


class SyntheticTokenizer:
    """Deterministic stand-in for a HuggingFace tokenizer (vocab files are absent offline): lower-cased
    whitespace/punctuation words -> ids by crc32, with the model's special-token layout
    (BERT: [CLS] w... [SEP] [PAD]...; T5: w... </s> <pad>...), padded / truncated to max_length."""

    def __init__(self, kind: str, vocab: int):
        self.kind, self.vocab = kind, vocab

    def ids(self, text: str, max_length: int) -> List[int]:
        import re
        words = re.findall(r"\w+|[^\w\s]", text.lower())
        if self.kind == "bert":
            body = [1000 + zlib.crc32(w.encode()) % (self.vocab - 1000) for w in words]
            seq = [101] + body[:max_length - 2] + [102]
        else:
            body = [100 + zlib.crc32(w.encode()) % (self.vocab - 228) for w in words]
            seq = body[:max_length - 1] + [1]
        return seq + [0] * (max_length - len(seq))

    def __call__(self, texts, truncation=True, max_length=77, padding="max_length", return_tensors="pt", **kw):
        texts = [texts] if isinstance(texts, str) else list(texts)
        return {"input_ids": torch.tensor([self.ids(t, max_length) for t in texts], dtype=torch.long)}


def _hf_tokenizer(path: Optional[str], kind: str):
    if path and os.path.isdir(path):
        try:
            if kind == "t5":
                from transformers import T5Tokenizer
                return T5Tokenizer.from_pretrained(path)
            from transformers import AutoTokenizer
            return AutoTokenizer.from_pretrained(path)
        except Exception as e:  # pragma: no cover - depends on local files
            print(f"tokenizer at {path!r} not loadable ({e})")
    return None


class CLAPT5TextEncoder(_HipModel):
    """The two text towers + projection as one packed model (C-ABI kind ALCM_MODEL_TEXT)."""
    KIND = _hip.ALCM_MODEL_TEXT

    def __init__(self, cfg: recipe.TextConfig = recipe.TextConfig(), split=True):
        super().__init__(split)
        self.cfg = cfg

    def _iconfig(self):
        return self.cfg.iconfig()

    def _extra_tensors(self):
        return {"_alcm.t5_rel_buckets": relative_position_bucket(self.cfg.max_len, self.cfg.t_buckets,
                                                                 self.cfg.t_max_distance).float()}

    def load_state_dict(self, state: Mapping[str, torch.Tensor], strict: bool = False):
        keep = {k: v for k, v in state.items()
                if k.startswith("caption_encoder.base.") or k.startswith("caption_encoder.projection.")
                or k.startswith("t5_transformer.")}
        # pooler (unused by encode) and the tied copy of the T5 token embedding stay on the host
        keep = {k: v for k, v in keep.items() if ".pooler." not in k and not
                (k == "t5_transformer.encoder.embed_tokens.weight" and "t5_transformer.shared.weight" in keep)}
        return super().load_state_dict(keep, strict)

    def encode_ids(self, clap_ids: torch.Tensor, t5_ids: torch.Tensor) -> torch.Tensor:
        """(B, L) int64 token ids of each tokenizer -> (B, 2L, d_proj) conditioning on the current stream."""
        self._need()
        if clap_ids.shape != t5_ids.shape or clap_ids.dim() != 2:
            raise ValueError("clap_ids and t5_ids must both be (B, L)")
        B, L = clap_ids.shape
        if L > self.cfg.max_len:
            raise ValueError(f"sequence length {L} exceeds max_length {self.cfg.max_len}")
        for ids, v, name in ((clap_ids, self.cfg.b_vocab, "clap"), (t5_ids, self.cfg.t_vocab, "t5")):
            lo, hi = int(ids.min()), int(ids.max())
            if lo < 0 or hi >= v:  # nn.Embedding raises on out-of-range ids
                raise IndexError(f"{name} token id out of range [0, {v}): {lo}..{hi}")
        dev = torch.device("cuda")
        a = clap_ids.to(dev, torch.int64).contiguous()
        b = t5_ids.to(dev, torch.int64).contiguous()
        out = torch.empty((B, 2 * L, self.cfg.p_out), device=dev, dtype=torch.float32)
        nb = int(lib().alcm_text_workspace_bytes(self._handle, B, L))
        ws = self._workspace(("text", B, L), nb, dev)
        check(lib().alcm_text_encode(self._handle, ptr(a), ptr(b), ptr(out), B, L, ptr(ws), ws.numel(),
                                     stream_handle()), "alcm_text_encode")
        return out

    @classmethod
    def from_recipe(cls, seed: int = 0, split=True, cfg: recipe.TextConfig = recipe.TextConfig()):
        return cls(cfg, split=split).load_state_dict(recipe.text_state(seed, cfg))


def _safetensors_state(path: str, prefix: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file
    f = os.path.join(path, "model.safetensors")
    return {prefix + k: v for k, v in load_file(f).items()} if os.path.exists(f) else {}


class FrozenCLAPFLANEmbedder:
    """ldm/modules/encoders/modules.py:529-582 on the MI355X path (same constructor and ``encode`` contract).

    ``weights_path`` (CLAP_weights_2022.pth) is accepted like the reference, which reads it but never applies
    its tensors (``match_params`` is unused at modules.py:535-540); the caption encoder weights come from the
    LCM checkpoint's ``cond_stage_model.*`` keys (``load_state_dict``), from local HF model directories, or from
    the recipe (``synthetic_seed``)."""

    def __init__(self, weights_path=None, t5version="../ldm/modules/encoders/CLAP/t5-v1_1-large", freeze=True,
                 device="cuda", max_length=77, text_model="../ldm/modules/encoders/CLAP/bert-base-uncased",
                 synthetic_seed: Optional[int] = None, split=True, cfg: Optional[recipe.TextConfig] = None,
                 synthetic_tokenizer: bool = False, **unused):
        self.max_length = max_length
        self.device = device
        self.cfg = cfg or recipe.TextConfig(max_len=max_length)
        self.tokenizer_paths = (text_model, t5version)
        self.clap_tokenizer = _hf_tokenizer(text_model, "bert")
        self.t5_tokenizer = _hf_tokenizer(t5version, "t5")
        if synthetic_tokenizer or synthetic_seed is not None:
            self.use_synthetic_tokenizer()
        self.model = CLAPT5TextEncoder(self.cfg, split=split)
        state = {}
        if text_model and os.path.isdir(text_model):
            state.update(_safetensors_state(text_model, "caption_encoder.base."))
        if t5version and os.path.isdir(t5version):
            state.update(_safetensors_state(t5version, "t5_transformer."))
        if synthetic_seed is not None:
            self.model.load_state_dict(recipe.text_state(synthetic_seed, self.cfg))
        elif state and any(k.startswith("caption_encoder.projection.") for k in state):
            self.model.load_state_dict(state)
        self._pending = state  # completed by load_state_dict(cond_stage_model.*) when the projection is missing

    def load_state_dict(self, state: Mapping[str, torch.Tensor], strict: bool = False):
        merged = dict(self._pending)
        merged.update(state)
        self.model.load_state_dict(merged, strict)
        self._pending = {}
        return self

    def use_synthetic_tokenizer(self):
        """Opt in to the hash stand-in for whichever tokenizer directory is missing (recipe weights / tests)."""
        self.clap_tokenizer = self.clap_tokenizer or SyntheticTokenizer("bert", self.cfg.b_vocab)
        self.t5_tokenizer = self.t5_tokenizer or SyntheticTokenizer("t5", self.cfg.t_vocab)
        return self

    def set_split(self, split):
        self.model.set_split(split)

    def tokenize(self, ori_caption: Sequence[str], struct_caption: Sequence[str]):
        if self.clap_tokenizer is None or self.t5_tokenizer is None:
            missing = [p for p, t in zip(self.tokenizer_paths, (self.clap_tokenizer, self.t5_tokenizer)) if t is None]
            raise RuntimeError(f"FrozenCLAPFLANEmbedder: no loadable HuggingFace tokenizer at {missing!r}; real "
                               "encoder weights need the real vocabularies (pass text_model= / t5version= tokenizer "
                               "directories, or synthetic_tokenizer=True to run the hash stand-in deliberately)")
        kw = dict(truncation=True, max_length=self.max_length, return_length=True, return_overflowing_tokens=False,
                  padding="max_length", return_tensors="pt")
        return self.clap_tokenizer(list(ori_caption), **kw)["input_ids"], \
            self.t5_tokenizer(list(struct_caption), **kw)["input_ids"]

    def encode(self, text: Dict[str, List[str]]) -> torch.Tensor:
        """modules.py:567-582: captions -> (B, 2 * max_length, 1024) on the device."""
        if not self.model.loaded:
            raise RuntimeError("FrozenCLAPFLANEmbedder: text-encoder weights not loaded (checkpoint cond_stage_model.* "
                               "keys, local HF model directories, or synthetic_seed)")
        ori, struct = text["ori_caption"], text["struct_caption"]
        a, b = self.tokenize(ori, struct)
        return self.model.encode_ids(a, b)

    __call__ = encode

    def to(self, device):
        return self

    def freeze(self):
        return self

    def eval(self):
        return self
