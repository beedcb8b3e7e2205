"""Front-end constant tables for zs_logmel (built once on the host, uploaded to HBM).

torchlibrosa 0.0.9 / librosa 0.9.2 (pinned by retrieval/work.yaml) are not installed, so the
tables follow their published definitions: periodic Hann window (scipy get_window 'hann',
fftbins=True), librosa ``filters.mel(sr=32000, n_fft=1024, n_mels=64, fmin=50, fmax=14000,
htk=False, norm='slaney')``.  When a real CLAP checkpoint is loaded, its
``audio_feats_extractor.log_trans.melW`` [513, 64] replaces the computed filterbank verbatim
(:func:`tables_from_state_dict`), removing any restatement ambiguity.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

SR, N_FFT, HOP, N_MELS, FMIN, FMAX = 32000, 1024, 320, 64, 50.0, 14000.0


def _hz_to_mel(f):
    f = np.atleast_1d(np.asarray(f, dtype=np.float64)).copy()
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    m = f / f_sp
    hi = f >= min_log_hz
    m[hi] = min_log_mel + np.log(f[hi] / min_log_hz) / logstep
    return m


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    f = f_sp * m
    hi = m >= min_log_mel
    f[hi] = min_log_hz * np.exp(logstep * (m[hi] - min_log_mel))
    return f


def slaney_mel(sr=SR, n_fft=N_FFT, n_mels=N_MELS, fmin=FMIN, fmax=FMAX) -> np.ndarray:
    """[n_mels, n_fft//2+1] float32 Slaney-scale, Slaney-normalised triangular filters."""
    w = np.zeros((n_mels, n_fft // 2 + 1), dtype=np.float32)
    freqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin)[0], _hz_to_mel(fmax)[0], n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, freqs)
    for i in range(n_mels):
        w[i] = np.maximum(0, np.minimum(-ramps[i] / fdiff[i], ramps[i + 2] / fdiff[i + 1]))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w


def hann_periodic(n=N_FFT) -> np.ndarray:
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def dft_conv_weights(n_fft=N_FFT):
    """torchlibrosa STFT ``conv_real`` / ``conv_imag`` weights [n_fft//2+1, 1, n_fft] (the
    windowed DFT rows), kept only so reference checkpoints load into the drop-in AudioFeature;
    the kernel computes the same transform as an FFT."""
    n = np.arange(n_fft)
    W = np.exp(-2j * np.pi * np.outer(n, n[: n_fft // 2 + 1]) / n_fft) * hann_periodic(n_fft)[:, None]
    return (torch.from_numpy(np.real(W).T.astype(np.float32))[:, None, :],
            torch.from_numpy(np.imag(W).T.astype(np.float32))[:, None, :])


def make_tables(device, melW: Optional[np.ndarray] = None) -> Dict[str, torch.Tensor]:
    """Device tables for zs_logmel.  ``melW`` [64, 513] overrides the computed filterbank."""
    mel = slaney_mel() if melW is None else np.asarray(melW, dtype=np.float32)
    assert mel.shape == (N_MELS, N_FFT // 2 + 1), mel.shape
    nz = mel != 0
    lo = np.array([int(np.argmax(r)) if r.any() else 0 for r in nz], dtype=np.int32)
    hi = np.array([int(len(r) - np.argmax(r[::-1])) if r.any() else 0 for r in nz], dtype=np.int32)
    k = np.arange(N_FFT // 2, dtype=np.float64)
    tw = np.stack([np.cos(-2 * np.pi * k / N_FFT), np.sin(-2 * np.pi * k / N_FFT)], 1)
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dt)
    return {
        "window": t(hann_periodic().astype(np.float32)),
        "twiddle": t(tw.astype(np.float32).reshape(-1)),
        "melW": t(mel),
        "mel_lo": t(lo, torch.int32),
        "mel_hi": t(hi, torch.int32),
    }


def tables_from_state_dict(sd, device, prefix="audio_encoder.audio_enc.audio_feats_extractor."):
    key = prefix + "log_trans.melW"
    melW = sd[key].detach().cpu().numpy().T if key in sd else None
    return make_tables(device, melW)
