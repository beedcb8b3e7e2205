"""Drop-in for retrieval/models/htsat.py:588-958 ``HTSAT_Swin_Transformer`` (inference).

Same constructor, same state-dict keys (parameters + relative_position_index / attn_mask
buffers + audio_feats_extractor), ``forward(waveform) -> embedding [B, 768]`` like the reference
(htsat.py:941-958 returns output_dict["embedding"]).  The forward is the zsaac HTSAT engine: fused
log-mel+bn0, bicubic fold, patch-embed+LN, 12 Swin blocks (MFMA GEMMs, fused window attention),
patch merging, final LN + mean-pool.  The dead tscam_conv / head branch is kept as parameters (so
checkpoints load) but not computed: it does not feed ``embedding``.

Only the CLAP configuration of retrieval/models/audio_encoder.py:41-51 is supported.
"""
import torch
import torch.nn as nn

from zsaac.modules import EngineCache, htsat_reference_spec, register_tree, require_device, zs_dtype_of

from .feature_extractor import AudioFeature


class HTSAT_Swin_Transformer(nn.Module):

    def __init__(self, spec_size=256, patch_size=4, patch_stride=(4, 4), in_chans=1, num_classes=527,
                 embed_dim=96, depths=[2, 2, 6, 2], num_heads=[4, 8, 16, 32], window_size=8,
                 mlp_ratio=4., qkv_bias=True, qk_scale=None, drop_rate=0., attn_drop_rate=0.,
                 drop_path_rate=0.1, norm_layer=nn.LayerNorm, ape=False, patch_norm=True,
                 use_checkpoint=False, norm_before_mlp='ln', config=None, **kwargs):
        super().__init__()
        clap = (spec_size, patch_size, tuple(patch_stride), in_chans, num_classes, embed_dim,
                list(depths), list(num_heads), window_size, mlp_ratio, qkv_bias, ape, patch_norm)
        if clap != (256, 4, (4, 4), 1, 527, 96, [2, 2, 6, 2], [4, 8, 16, 32], 8, 4., True, False, True):
            raise NotImplementedError("only the CLAP HTSAT configuration (audio_encoder.py:41-51)")
        self.config = config
        self.audio_feats_extractor = AudioFeature(config["audio_args"])
        register_tree(self, htsat_reference_spec(), buffers=("relative_position_index", "attn_mask"))
        self._cache = EngineCache()

    def _engine(self, B, T, device):
        from zsaac.encoder import AudioEncoder
        dt = zs_dtype_of(self)

        def build():
            sd = {"audio_encoder.audio_enc." + k: v for k, v in self.state_dict().items()}
            return AudioEncoder(sd, "htsat", dt, B, device, n_samples=T)
        return self._cache.get(self, build, (dt, B, T, str(device)))

    def forward(self, input: torch.Tensor, infer_mode=False):
        require_device(input, "HTSAT_Swin_Transformer.forward")
        eng = self._engine(input.shape[0], input.shape[1], input.device)
        return eng.encode(input.float().contiguous()).clone()
