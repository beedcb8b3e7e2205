"""CPU: the front-end restatement (torchlibrosa 0.0.9 / librosa 0.9.2 semantics; PARITY UNPINNED
against the reference, whose third-party front end is not installable here) cross-checked
against an independent float64 numpy.fft formulation, and the product's tables against it."""
import numpy as np
import torch

from zsaac import synthetic as S


def test_logmel_conv_dft_vs_numpy_fft():
    from oracle import frontend as OF
    wav = S.synthetic_waveforms(1, seed=5, length=32000)
    a = OF.logmel(wav)[:, 0].numpy()
    b = OF.logmel_numpy_fft(wav.numpy())[:, 0]
    assert a.shape == (1, 101, 64)
    assert np.abs(a - b).max() < 2e-3          # dB; f32 conv-DFT vs f64 FFT


def test_mel_filterbank_properties():
    from oracle import frontend as OF
    m = OF.mel_filterbank()
    assert m.shape == (64, 513) and m.dtype == np.float32
    assert (m >= 0).all() and (m.sum(1) > 0).all()
    # Slaney normalisation: each triangle has unit area in Hz (2/(f_hi - f_lo) * peak 1 * base/2)
    freqs = np.fft.rfftfreq(1024, 1 / 32000)
    area = (m * (freqs[1] - freqs[0])).sum(1)
    assert np.allclose(area, 1.0, rtol=0.12)
    # band centres increase monotonically and stay in [fmin, fmax]
    centres = (m * freqs).sum(1) / m.sum(1)
    assert (np.diff(centres) > 0).all() and centres[0] > 50 and centres[-1] < 14000


def test_product_tables_match_oracle():
    from oracle import frontend as OF
    from zsaac.frontend import hann_periodic, make_tables, slaney_mel
    assert np.array_equal(slaney_mel(), OF.mel_filterbank())
    assert np.allclose(hann_periodic(), OF.hann_periodic())
    t = make_tables("cpu")
    mel = t["melW"].numpy()
    lo, hi = t["mel_lo"].numpy(), t["mel_hi"].numpy()
    for i in range(64):
        nz = np.nonzero(mel[i])[0]
        assert lo[i] == nz[0] and hi[i] == nz[-1] + 1
    tw = t["twiddle"].numpy().reshape(-1, 2)
    k = np.arange(512)
    assert np.allclose(tw[:, 0], np.cos(-2 * np.pi * k / 1024), atol=1e-7)


def test_bicubic_fold_oracle_is_torch_interpolate():
    from oracle import audio as A
    lm = torch.randn(1, 1, 1001, 64)
    img = A.reshape_wav2img(lm)
    assert img.shape == (1, 1, 256, 256)
    up = torch.nn.functional.interpolate(lm, (1024, 64), mode="bicubic", align_corners=True)
    # image row r = chunk*64 + mel, column c -> time chunk*256 + c
    assert torch.equal(img[0, 0, 64 + 5, 10], up[0, 0, 256 + 10, 5])
