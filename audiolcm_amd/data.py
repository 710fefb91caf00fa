"""Prompt datasets of the config-1 CLI's dataset mode (scripts/txt2audio_for_lcm.py --test-dataset).

``TSVDatasetStruct`` restates ldm/data/tsvdataset.py:6-58 (TSVDataset.add_name_num + TSVDatasetStruct.__getitem__):
rows of a tab-separated file with columns ``name, dataset, ori_cap, mel_path, caption, audio_path``
(audiocaps_test_16000_struct.tsv); each repeated ``name`` gets a running ``_<num>`` suffix so every
(audio, caption) pair has its own file name, and an item is
``{"caption": {"ori_caption": ori_cap, "struct_caption": caption}, "f_name": name_num, "image": mel}``.
The ground-truth mel (``mel_path`` .npy) is only needed for evaluation, not for generation: it is loaded
when the file exists (padded / cropped to ``spec_crop_len`` as the reference) and is ``None`` otherwise
(the AudioCaps mels are not in this container).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np


class TSVDataset:
    def __init__(self, tsv_path: str, spec_crop_len: Optional[int] = None, load_mel: bool = True):
        import pandas as pd
        self.batch_max_length = spec_crop_len
        self.load_mel = load_mel  # generation (the CLI's dataset mode) never reads the ground-truth mel
        df = pd.read_csv(tsv_path, sep="\t")
        self.dataset = self.add_name_num(df)
        self.root = os.path.dirname(os.path.abspath(tsv_path))
        print("dataset len:", len(self.dataset))

    @staticmethod
    def add_name_num(df):
        """tsvdataset.py:16-29: the i-th occurrence of a name becomes name_i."""
        seen: Dict[str, int] = {}
        names: List[str] = []
        for name in df["name"].tolist():
            seen[name] = seen.get(name, -1) + 1
            names.append(f"{name}_{seen[name]}")
        df = df.copy()
        df["name"] = names
        return df

    def _mel(self, path) -> Optional[np.ndarray]:
        if not self.load_mel or not isinstance(path, str):
            return None
        p = path if os.path.isabs(path) or os.path.exists(path) else os.path.join(self.root, path)
        if not os.path.exists(p):
            return None
        spec = np.load(p, allow_pickle=False)
        L = self.batch_max_length
        if L is not None and spec.shape[1] <= L:
            spec = np.pad(spec, ((0, 0), (0, L - spec.shape[1])))
        return spec[:, :L] if L is not None else spec

    def __getitem__(self, idx: int):
        data = self.dataset.iloc[idx]
        return {"image": self._mel(data["mel_path"]), "caption": data["caption"], "f_name": data["name"]}

    def __len__(self) -> int:
        return len(self.dataset)

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


class TSVDatasetStruct(TSVDataset):
    """tsvdataset.py:47-58: the caption is the {ori_caption, struct_caption} dict the embedder encodes."""

    def __getitem__(self, idx: int):
        data = self.dataset.iloc[idx]
        return {"image": self._mel(data["mel_path"]),
                "caption": {"ori_caption": data["ori_cap"], "struct_caption": data["caption"]},
                "f_name": data["name"]}
