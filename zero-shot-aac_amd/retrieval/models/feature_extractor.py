"""Drop-in for retrieval/models/feature_extractor.py:12-38 ``AudioFeature`` (torchlibrosa
Spectrogram + LogmelFilterBank).  Holds the same parameters as the reference
(``mel_trans.stft.conv_{real,imag}.weight``, ``log_trans.melW``) so checkpoints load; the forward
is the fused zs_logmel kernel (FFT instead of conv-DFT, same transform)."""
import torch
import torch.nn as nn

from zsaac import ops
from zsaac.frontend import dft_conv_weights, make_tables, slaney_mel
from zsaac.modules import require_device


class _Stft(nn.Module):
    def __init__(self):
        super().__init__()
        re, im = dft_conv_weights()
        self.conv_real = nn.Conv1d(1, re.shape[0], re.shape[2], bias=False)
        self.conv_imag = nn.Conv1d(1, im.shape[0], im.shape[2], bias=False)
        self.conv_real.weight.data.copy_(re)
        self.conv_imag.weight.data.copy_(im)
        for p in self.parameters():
            p.requires_grad = False


class _Spectrogram(nn.Module):
    def __init__(self):
        super().__init__()
        self.stft = _Stft()


class _LogMel(nn.Module):
    def __init__(self):
        super().__init__()
        self.melW = nn.Parameter(torch.from_numpy(slaney_mel().T.copy()), requires_grad=False)


class AudioFeature(nn.Module):

    def __init__(self, audio_config):
        super().__init__()
        assert (audio_config["n_fft"], audio_config["hop_length"], audio_config["n_mels"]) == (1024, 320, 64)
        self.mel_trans = _Spectrogram()
        self.log_trans = _LogMel()
        self._tables = None

    def tables(self, device):
        if self._tables is None or self._tables["melW"].device != device:
            self._tables = make_tables(device, self.log_trans.melW.detach().cpu().numpy().T)
        return self._tables

    def forward(self, input):
        """waveform [bs, wav_length] -> log-mel [bs, 1, frames, 64]."""
        require_device(input, "AudioFeature.forward")
        return ops.logmel(input.float().contiguous(), self.tables(input.device)).unsqueeze(1)
