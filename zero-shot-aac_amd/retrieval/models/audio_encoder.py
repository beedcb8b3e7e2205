"""Drop-in for retrieval/models/audio_encoder.py:16-79 ``AudioEncoder`` (inference only; the
``pretrained`` branch that loads pretrained_models/*.pth is the training-time path)."""
import torch.nn as nn

from .cnns import Cnn14
from .htsat import HTSAT_Swin_Transformer


class AudioEncoder(nn.Module):

    def __init__(self, config):
        super().__init__()
        args = config["audio_encoder_args"]
        if args["type"] == "cnn":
            if args.get("model") != "Cnn14":
                raise NotImplementedError("only Cnn14 (Cnn10/ResNet38 cannot run in the reference)")
            self.audio_enc = Cnn14(config)
            self.audio_width = 2048
        elif args["type"] == "transformer":
            self.audio_enc = HTSAT_Swin_Transformer(spec_size=256, patch_size=4, patch_stride=(4, 4),
                                                    num_classes=527, embed_dim=96, depths=[2, 2, 6, 2],
                                                    num_heads=[4, 8, 16, 32], window_size=8,
                                                    config=config)
            self.audio_width = 768
        else:
            raise NotImplementedError('No such audio encoder network.')

    def forward(self, inputs):
        return self.audio_enc(inputs)
