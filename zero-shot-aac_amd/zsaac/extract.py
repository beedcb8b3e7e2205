"""Batched embedding extraction: the reference's ``Extract_embeddings``
(data_handing/embeddings_generator.py:34-75) on the HIP encoder.

Per clip the reference decodes the audio file (librosa, 32 kHz mono — file decoding is out of
scope here: clips arrive as sample arrays), skips empty clips, crops to the first
``max_length * sr`` samples or zero-pads to that length (lines 53-59), runs
``ASE.encode_audio`` on a batch of ONE and appends the record
``{"audio_embedding": [1, 1024] cpu tensor, "caption": captions, "text_embedding": 0,
"audio_id": id}`` (lines 70-71; the ``text_or_not`` branch also encodes every caption with the
BERT text encoder, which is not part of this path).  The split's records are pickled to
``<out>/<split>/clap_embedding/ZS/data.pkl`` (lines 100-101).

Here the clips of a chunk are packed on the device (zs_pack_clips: the same crop / pad) and
encoded ``batch`` at a time; the records and the pickle have the reference's format, so
predict_prompt.py / zsaac.predict read them unchanged.
"""
from __future__ import annotations

import os
import pickle
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import ops
from .encoder import AudioEncoder


def fit_plan(lengths: Sequence[int], max_samples: int):
    """Which clips are encoded (the reference skips empty ones) and how many samples of each
    are kept (crop to max_samples, the rest zero-padded)."""
    keep = [i for i, n in enumerate(lengths) if n > 0]
    return keep, [min(int(lengths[i]), max_samples) for i in keep]


def make_record(emb_row: torch.Tensor, caption, audio_id) -> dict:
    """One entry of the reference's data.pkl (embeddings_generator.py:70-71, text_or_not False)."""
    return {"audio_embedding": emb_row.detach().reshape(1, -1).float().cpu(), "caption": caption,
            "text_embedding": 0, "audio_id": audio_id}


class EmbeddingExtractor:
    """``Extract_embeddings`` for in-memory clips.  ``audio_sd``: the ASE audio-side state dict
    (``audio_encoder.*`` + ``audio_proj.*``), ``kind`` "htsat" | "cnn14"."""

    def __init__(self, audio_sd, kind="htsat", dtype=torch.bfloat16, batch=64, device="cuda",
                 sr=32000, max_length=10):
        self.sr, self.max_length = sr, max_length
        self.T = max_length * sr if max_length else 320000
        self.device = torch.device(device)
        self.enc = AudioEncoder(audio_sd, kind, dtype, batch, self.device, n_samples=self.T)
        self.B = batch
        self.wav = torch.empty(batch, self.T, device=self.device)

    def encode_clips(self, clips: Sequence) -> torch.Tensor:
        """Ragged 1-D clips (numpy / torch, any length >= 1) -> [n, 1024] device embeddings, in
        order."""
        n = len(clips)
        out = torch.empty(n, 1024, device=self.device)
        for c0 in range(0, n, self.B):
            chunk = clips[c0:c0 + self.B]
            lens = [int(np.asarray(c).shape[-1]) if not torch.is_tensor(c) else int(c.shape[-1])
                    for c in chunk]
            flat = torch.cat([torch.as_tensor(c, dtype=torch.float32).reshape(-1) for c in chunk])
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            dflat = flat.to(self.device, non_blocking=True)
            b = len(chunk)
            ops.pack_clips(dflat, torch.from_numpy(offs).to(self.device),
                           torch.tensor(lens, dtype=torch.int32, device=self.device), self.T,
                           self.wav)
            out[c0:c0 + b].copy_(self.enc.encode(self.wav[:b]))
        return out

    def extract(self, clips: Sequence, audio_ids: Sequence, captions: Sequence,
                text_or_not: bool = False) -> List[dict]:
        """The records of ``Extract_embeddings`` (empty clips skipped, like the reference)."""
        if text_or_not:
            raise NotImplementedError("text embeddings need the BERT text encoder "
                                      "(retrieval/models/text_encoder.py), not part of this path")
        lengths = [int(torch.as_tensor(c).shape[-1]) for c in clips]
        keep, _ = fit_plan(lengths, self.T)
        emb = self.encode_clips([clips[i] for i in keep]).cpu()
        return [make_record(emb[j], captions[i], audio_ids[i]) for j, i in enumerate(keep)]


def save_records(records: List[dict], out_path: str, split: Optional[str] = None) -> str:
    """Pickle the records where the reference writes them
    (``<out_path>/<split>/clap_embedding/ZS/data.pkl``, embeddings_generator.py:100-101); with
    ``split=None`` ``out_path`` is the file itself."""
    path = out_path if split is None else os.path.join(out_path, split, "clap_embedding", "ZS",
                                                        "data.pkl")
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as f:
        pickle.dump(records, f)
    return path
