"""PCM16 WAV output, as ``soundfile.write(path, wav, 16000)`` does by default (InferAPI.py:98).

libsndfile's normalised float->short conversion rounds ``x * 32767`` to nearest
(lrintf, ties to even) and clips; soundfile is not installed offline, so the
writer is restated here (parity of the bytes is unpinned, the float waveform is
the parity target).
"""
from __future__ import annotations

import struct

import numpy as np


def pcm16(wav) -> np.ndarray:
    x = np.asarray(wav, dtype=np.float32).reshape(-1) * np.float32(32767.0)
    return np.clip(np.rint(x), -32768, 32767).astype("<i2")


def write_pcm16(path: str, wav, sample_rate: int = 16000) -> None:
    data = pcm16(wav).tobytes()
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, sample_rate, sample_rate * 2, 2, 16))
        f.write(b"data" + struct.pack("<I", len(data)) + data)


def read_pcm16(path: str):
    with open(path, "rb") as f:
        raw = f.read()
    assert raw[:4] == b"RIFF" and raw[8:12] == b"WAVE"
    sr = struct.unpack("<I", raw[24:28])[0]
    n = struct.unpack("<I", raw[40:44])[0]
    return np.frombuffer(raw[44:44 + n], dtype="<i2"), sr
