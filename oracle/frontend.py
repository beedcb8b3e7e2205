"""Oracle for the audio front end: torchlibrosa 0.0.9 ``Spectrogram`` + ``LogmelFilterBank`` with
the CLAP arguments of retrieval/models/feature_extractor.py:16-32 (n_fft 1024, hop 320, hann,
center, reflect, 64 mels, fmin 50, fmax 14000, ref 1.0, amin 1e-10, top_db None) and the
``librosa.filters.mel`` (0.9.2, Slaney scale + Slaney norm) matrix it builds.

PARITY UNPINNED: torchlibrosa/librosa are not in /root/reference and not installed; these are
restatements of their published algorithms (see module docstrings of each function), checked
against an independent numpy.fft formulation in tests/test_oracle_frontend.py.
"""
from __future__ import annotations

import numpy as np
import torch

SR, N_FFT, HOP, N_MELS, FMIN, FMAX = 32000, 1024, 320, 64, 50.0, 14000.0
AMIN, REF = 1e-10, 1.0


def hann_periodic(n: int = N_FFT) -> np.ndarray:
    """scipy.signal.get_window('hann', n, fftbins=True) (torchlibrosa STFT ``fft_window``)."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def dft_weights(n_fft: int = N_FFT):
    """torchlibrosa STFT conv weights: real/imag of ``W[:, :n_fft//2+1] * window[:, None]`` with
    ``W = omega ** (x*y)``, omega = exp(-2*pi*i/n) (complex128), stored as float32
    [n_fft//2+1, n_fft]."""
    n = np.arange(n_fft)
    x, y = np.meshgrid(n, n)
    omega = np.exp(-2 * np.pi * 1j / n_fft)
    W = np.power(omega, x * y)
    out = n_fft // 2 + 1
    win = hann_periodic(n_fft)
    Wc = W[:, :out] * win[:, None]
    return (np.real(Wc).T.astype(np.float32), np.imag(Wc).T.astype(np.float32))


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    if f.ndim:
        log_t = f >= min_log_hz
        mels[log_t] = min_log_mel + np.log(f[log_t] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    log_t = m >= min_log_mel
    freqs[log_t] = min_log_hz * np.exp(logstep * (m[log_t] - min_log_mel))
    return freqs


def mel_filterbank(sr=SR, n_fft=N_FFT, n_mels=N_MELS, fmin=FMIN, fmax=FMAX) -> np.ndarray:
    """librosa 0.9.2 ``filters.mel(htk=False, norm='slaney', dtype=float32)`` -> [n_mels, 1+n_fft//2].
    torchlibrosa stores its transpose as ``melW`` [513, 64]."""
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


def logmel(wav: torch.Tensor) -> torch.Tensor:
    """``AudioFeature.forward`` (feature_extractor.py:34-38): wav [B, T] f32 -> [B, 1, frames, 64].

    Spectrogram: reflect-pad n_fft//2 each side, conv1d with the DFT weights (stride hop),
    power = re^2 + im^2.  LogmelFilterBank: ``power @ melW``, ``10*log10(clamp(., amin))``
    minus ``10*log10(max(amin, ref))`` (= 0)."""
    wr, wi = dft_weights()
    x = torch.nn.functional.pad(wav[:, None, :].float(), (N_FFT // 2, N_FFT // 2), mode="reflect")
    real = torch.nn.functional.conv1d(x, torch.from_numpy(wr)[:, None, :], stride=HOP)
    imag = torch.nn.functional.conv1d(x, torch.from_numpy(wi)[:, None, :], stride=HOP)
    power = (real ** 2 + imag ** 2)[:, None].transpose(2, 3)          # [B,1,frames,513]
    mel = torch.matmul(power, torch.from_numpy(mel_filterbank().T.copy()))
    db = 10.0 * torch.log10(torch.clamp(mel, min=AMIN))
    db = db - 10.0 * np.log10(np.maximum(AMIN, REF))
    return db


def logmel_numpy_fft(wav: np.ndarray) -> np.ndarray:
    """Independent float64 formulation with numpy.fft.rfft (cross-check of :func:`logmel`)."""
    x = np.pad(wav.astype(np.float64), ((0, 0), (N_FFT // 2, N_FFT // 2)), mode="reflect")
    n_frames = 1 + (x.shape[1] - N_FFT) // HOP
    idx = np.arange(N_FFT)[None, :] + HOP * np.arange(n_frames)[:, None]
    frames = x[:, idx] * hann_periodic()[None, None, :]
    spec = np.abs(np.fft.rfft(frames, axis=-1)) ** 2
    mel = spec @ mel_filterbank().T.astype(np.float64)
    return 10.0 * np.log10(np.maximum(mel, AMIN))[:, None]
