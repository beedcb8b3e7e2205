"""Drop-in for retrieval/models/ase_model.py:21-78 ``ASE`` on the HIP kernels:

* ``encode_audio(audio[B, T]) -> F.normalize(audio_proj(audio_encoder(audio)), dim=-1)`` [B, 1024]
  (ase_model.py:52-55): one zsaac.encoder.AudioEncoder engine (front end + encoder + projection
  + L2 norm);
* ``encode_text(texts) -> F.normalize(text_proj(text_encoder(texts)[:, 0, :]), dim=-1)``
  (ase_model.py:57-60): the tokenizer call on the host, then one zsaac.bert.BertTextEngine
  (BERT + text_proj + L2 norm).  CLAP-guided decoding (gpt2_prefix_eval.py:549-551) is its
  caller on the captioning path.

The text tower exists when the config names one (``text_encoder_args``, as every reference
config does).  OUT OF SCOPE: the contrastive training ``forward``.
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
        self.has_text = "text_encoder_args" in config
        if self.has_text:
            from .text_encoder import TextEncoder
            self.text_encoder = TextEncoder(config)
            text_width = self.text_encoder.text_width
            self.text_proj = nn.Sequential(
                nn.Linear(text_width, embed_size),
                nn.ReLU(),
                nn.Linear(embed_size, embed_size),
            )
            self.temp = nn.Parameter(torch.ones([]) * config.get("temp", 0.07), requires_grad=False)
        self.kind = "htsat" if audio_width == 768 else "cnn14"
        self._cache = EngineCache()

    def load_state_dict(self, state_dict, strict: bool = True):
        keep = {k: v for k, v in state_dict.items() if not k.endswith("embeddings.position_ids")}
        if not self.has_text:
            keep = {k: v for k, v in keep.items()
                    if not (k.startswith("text_encoder.") or k.startswith("text_proj.") or k == "temp")}
        return super().load_state_dict(keep, strict=strict)

    def encode_audio(self, audio):
        from zsaac.encoder import AudioEncoder as Engine
        require_device(audio, "ASE.encode_audio")
        B, dt = audio.shape[0], zs_dtype_of(self)

        def build():
            sd = {k: v for k, v in self.state_dict().items()
                  if k.startswith("audio_encoder.") or k.startswith("audio_proj.")}
            return Engine(sd, self.kind, dt, B, audio.device, n_samples=audio.shape[1])
        eng = self._cache.get(self, build, (dt, B, str(audio.device), audio.shape[1]))
        return eng.encode(audio.float().contiguous()).clone()

    def text_engine(self):
        """The BertTextEngine of the text tower + text_proj (+ temp)."""
        if not self.has_text:
            raise RuntimeError("ASE built without text_encoder_args: no text tower")
        self.text_encoder.zs_dtype = zs_dtype_of(self)
        proj = {k: v for k, v in self.state_dict(keep_vars=True).items()
                if k.startswith("text_proj.") or k == "temp"}
        return self.text_encoder.engine(proj)

    def encode_text(self, text):
        tok = self.text_encoder.tokenizer if self.has_text else None
        if tok is None:
            raise RuntimeError("ASE.encode_text: text_encoder.tokenizer is not set")
        require_device(self.temp, "ASE.encode_text")
        return self.text_engine().encode_texts(tok, list(text)).clone()

    def forward(self, audio, text, idx):
        raise NotImplementedError("contrastive training is out of scope")
