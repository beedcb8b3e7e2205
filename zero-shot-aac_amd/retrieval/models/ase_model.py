"""Drop-in for retrieval/models/ase_model.py:21-78 ``ASE`` — the audio side only:
``encode_audio(audio[B, T]) -> F.normalize(audio_proj(audio_encoder(audio)), dim=-1)`` [B, 1024]
(ase_model.py:52-55) runs as one zsaac.encoder.AudioEncoder engine (front end + encoder +
projection + L2 norm on the HIP kernels).

OUT OF SCOPE: the BERT text encoder / ``encode_text`` / contrastive ``forward`` (they only produce
training data and the precomputed label table).  ``load_state_dict`` therefore ignores the
``text_encoder.*``, ``text_proj.*`` and ``temp`` entries of a full CLAP checkpoint.
"""
import torch
import torch.nn as nn

from zsaac.modules import EngineCache, require_device, zs_dtype_of

from .audio_encoder import AudioEncoder


class ASE(nn.Module):

    def __init__(self, config):
        super().__init__()
        self.audio_encoder = AudioEncoder(config)
        embed_size = config["embed_size"]
        audio_width = self.audio_encoder.audio_width
        self.audio_proj = nn.Sequential(
            nn.Linear(audio_width, embed_size),
            nn.ReLU(),
            nn.Linear(embed_size, embed_size),
        )
        self.kind = "htsat" if audio_width == 768 else "cnn14"
        self._cache = EngineCache()

    def load_state_dict(self, state_dict, strict: bool = True):
        keep = {k: v for k, v in state_dict.items()
                if not (k.startswith("text_encoder.") or k.startswith("text_proj.") or k == "temp")}
        return super().load_state_dict(keep, strict=strict)

    def encode_audio(self, audio):
        from zsaac.encoder import AudioEncoder as Engine
        require_device(audio, "ASE.encode_audio")
        B, dt = audio.shape[0], zs_dtype_of(self)

        def build():
            return Engine(self.state_dict(), self.kind, dt, B, audio.device, n_samples=audio.shape[1])
        eng = self._cache.get(self, build, (dt, B, str(audio.device), audio.shape[1]))
        return eng.encode(audio.float().contiguous()).clone()

    def encode_text(self, text):
        raise NotImplementedError("the BERT text encoder is out of scope for the captioning path")

    def forward(self, audio, text, idx):
        raise NotImplementedError("contrastive training is out of scope")
