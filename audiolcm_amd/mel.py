"""Log-mel front-end on the MI355X path: ``MelNet`` of ldm/data/preprocess/NAT_mel.py:42-85.

``MelNet(hparams)(y)``: clamp to [-1, 1], reflect-pad (n_fft - hop) / 2 on both sides, |STFT| with a periodic Hann
window (center=False, onesided; magnitude sqrt(re^2 + im^2 + 1e-9)), mel projection, log10(clamp(x, 1e-5)) —
one C call (``alcm_mel_spectrogram``): the STFT is an MFMA GEMM over the frames (a conv over hop-sized rows of the
padded waveform with the windowed DFT as its weight), the mel projection a second GEMM.

The mel filterbank is librosa's ``filters.mel`` (librosa 0.9.2 in the reference's requirements.txt; slaney mel
scale and slaney area normalisation, the defaults the reference uses), restated in ``mel_filterbank`` below because
librosa is not installed here: the filterbank values are *parity unpinned*; everything after it (STFT, magnitude,
projection, log) is pinned to the reference MelNet run on this filterbank (tests/golden/mel_B2.npz).
"""
from __future__ import annotations

from typing import Mapping, Optional

import numpy as np
import torch

from . import _hip
from ._hip import check, lib, ptr, stream_handle
from .models import _HipModel

NAT_MEL_16K = {"audio_sample_rate": 16000, "audio_num_mel_bins": 80, "fft_size": 1024, "win_size": 1024,
               "hop_size": 256, "fmin": 0, "fmax": 8000}  # ldm/data/preprocess/mel_spec.py:196-203


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, logstep = 1000.0, np.log(6.4) / 27.0
    min_log_mel = min_log_hz / f_sp
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    min_log_hz, logstep = 1000.0, np.log(6.4) / 27.0
    min_log_mel = min_log_hz / f_sp
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filterbank(sr: int, n_fft: int, n_mels: int = 128, fmin: float = 0.0, fmax: Optional[float] = None) -> np.ndarray:
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) with htk=False, norm='slaney' (its defaults):
    triangular filters between consecutive slaney-mel points, area-normalised by 2 / (f[i+2] - f[i])."""
    fmax = sr / 2.0 if fmax is None else fmax
    fftfreqs = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float64)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    weights *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return weights.astype(np.float32)


class MelNet(_HipModel):
    """NAT_mel.MelNet on the HIP path (model kind ALCM_MODEL_MEL)."""
    KIND = _hip.ALCM_MODEL_MEL

    def __init__(self, hparams: Mapping = NAT_MEL_16K, device="cuda", mel_basis: Optional[np.ndarray] = None):
        super().__init__(True)
        self.n_fft, self.num_mels = int(hparams["fft_size"]), int(hparams["audio_num_mel_bins"])
        self.sampling_rate, self.hop_size = int(hparams["audio_sample_rate"]), int(hparams["hop_size"])
        self.win_size, self.fmin, self.fmax = int(hparams["win_size"]), hparams["fmin"], hparams["fmax"]
        basis = mel_basis if mel_basis is not None else mel_filterbank(self.sampling_rate, self.n_fft, self.num_mels,
                                                                       self.fmin, self.fmax)
        self.mel_basis = torch.from_numpy(np.asarray(basis, dtype=np.float32))
        self.hann_window = torch.hann_window(self.win_size)
        self.load_state_dict({"mel_basis": self.mel_basis, "window": self.hann_window})

    def _iconfig(self):
        return [self.n_fft, self.hop_size, self.win_size, self.num_mels]

    def forward(self, y, center: bool = False, complex: bool = False) -> torch.Tensor:
        """y: (B, L) or (L,) waveform (np or tensor), L % hop == 0 -> (B, num_mels, L / hop) log10 mel."""
        if center or complex:
            raise NotImplementedError("MelNet: only the center=False magnitude path is used (NAT_mel.py:66-85)")
        self._need()
        if isinstance(y, np.ndarray):
            y = torch.from_numpy(y.astype(np.float32))
        if y.dim() == 1:
            y = y.unsqueeze(0)
        y = y.to("cuda", torch.float32).contiguous()
        B, L = y.shape
        out = torch.empty((B, self.num_mels, L // self.hop_size), device=y.device, dtype=torch.float32)
        nb = int(lib().alcm_mel_workspace_bytes(self._handle, B, L))
        ws = self._workspace(("mel", B, L), nb, y.device)
        check(lib().alcm_mel_spectrogram(self._handle, ptr(y), ptr(out), B, L, ptr(ws), ws.numel(), stream_handle()),
              "alcm_mel_spectrogram")
        return out

    __call__ = forward
