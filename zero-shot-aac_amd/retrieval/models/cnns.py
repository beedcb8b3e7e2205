"""Drop-in for retrieval/models/cnns.py:137-201 ``Cnn14`` (inference): bn0 + 6 ConvBlocks
(conv3x3-BN-ReLU x2, avgpool 2x2) + mean over mel + (max + mean) over time -> [B, 2048], on the
zsaac implicit-GEMM conv kernels.  Same state-dict keys as the reference.

Cnn10 / ResNet38 are not provided: in the reference they read a missing ``self.dropout``
(cnns.py:121, 388) and cannot run.
"""
import torch
import torch.nn as nn

from zsaac.modules import (EngineCache, cnn14_reference_spec, register_tree, require_device,
                           zs_dtype_of)

from .feature_extractor import AudioFeature


class Cnn14(nn.Module):

    def __init__(self, config):
        super(Cnn14, self).__init__()
        self.audio_feats_extractor = AudioFeature(config["audio_args"])
        register_tree(self, cnn14_reference_spec())
        self._cache = EngineCache()

    def forward(self, input):
        from zsaac.encoder import AudioEncoder
        require_device(input, "Cnn14.forward")
        B, dt = input.shape[0], zs_dtype_of(self)

        def build():
            sd = {"audio_encoder.audio_enc." + k: v for k, v in self.state_dict().items()}
            return AudioEncoder(sd, "cnn14", dt, B, input.device, n_samples=input.shape[1])
        eng = self._cache.get(self, build, (dt, B, str(input.device), input.shape[1]))
        return eng.encode(input.float().contiguous()).clone()
