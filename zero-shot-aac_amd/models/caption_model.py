"""Drop-in for the reference's ``models/caption_model.py`` caption classes on the hot path:
``ClapCaptionModel`` (caption_model.py:13-89) and ``ClapCaption_prompt`` (291-338).

Same constructor arguments and state-dict keys (``gpt.*`` = HF GPT2LMHeadModel layout, 149 keys,
plus ``clap_project.*``), so ``load_state_dict(torch.load(best.pth))`` works unchanged.  The only
construction difference: the reference fetches ``GPT2LMHeadModel.from_pretrained('gpt2')`` by name
(caption_model.py:52); here ``gpt`` is built at the GPT-2-small architecture and its weights come
from the checkpoint (``best.pth`` holds all of them).  Forward math runs on the HIP kernels.

OUT OF SCOPE (not on the captioning hot path): training forward with labels, the sound-effect
cross-attention variants (ClapCaptionCrossattention*) and the Mistral classes.
"""
from enum import Enum
from typing import Optional

import torch
import torch.nn as nn

from zsaac.modules import ZsGPT2LMHeadModel

from .mapper import MLP, TransformerMapper


class MappingType(Enum):
    MLP = 'mlp'
    Transformer = 'transformer'


class ClapCaptionModel(nn.Module):

    def get_dummy_token(self, batch_size: int, device: torch.device) -> torch.Tensor:
        return torch.zeros(batch_size, self.prefix_length, dtype=torch.int64, device=device)

    def forward(self, *args, **kwargs):
        raise NotImplementedError("training forward is out of scope; use clap_to_gpt + "
                                  "gpt2_prefix_eval.generate2/generate_beam")

    def __init__(self, prefix_length: int, clip_length: Optional[int] = None, prefix_size: int = 512,
                 num_layers: int = 8, mapping_type='mlp', sound_effect_embeddings: torch.Tensor = None,
                 sound_effect_num: Optional[int] = 0, only_prefix: Optional[bool] = False,
                 mask_probability: Optional[float] = 0):
        super(ClapCaptionModel, self).__init__()
        if sound_effect_embeddings is not None:
            raise NotImplementedError("sound-effect projection variant is out of scope")
        self.prefix_length = prefix_length
        self.sound_effect_embeddings = None
        self.sound_effect_num = sound_effect_num
        self.only_prefix = only_prefix
        self.mask_probability = mask_probability
        self.gpt = ZsGPT2LMHeadModel()
        self.gpt_embedding_size = self.gpt.transformer.wte.weight.shape[1]
        if mapping_type in ('mlp', MappingType.MLP):
            self.clap_project = MLP((prefix_size, (self.gpt_embedding_size * prefix_length) // 2,
                                     self.gpt_embedding_size * prefix_length))
        else:
            self.clap_project = TransformerMapper(prefix_size, self.gpt_embedding_size, prefix_length,
                                                  clip_length, num_layers)

    def clap_to_gpt(self, prefix: torch.Tensor, embedding_text: Optional[torch.Tensor] = None,
                    mask: Optional[torch.Tensor] = None):
        """caption_model.py:66-82 (without the sound-effect branch)."""
        proj = self.clap_project(prefix).view(-1, self.prefix_length, self.gpt_embedding_size)
        emb = proj if embedding_text is None else torch.cat((proj, embedding_text), dim=1)
        return emb, mask

    def set_dtype(self, dtype: torch.dtype):
        """float32 = parity mode (default), bfloat16 = perf mode, for every kernel engine."""
        for m in (self, self.gpt, self.clap_project):
            m.zs_dtype = dtype
        return self


class ClapCaption_prompt(ClapCaptionModel):

    def __init__(self, prefix_length: int, clip_length: Optional[int] = None, prefix_size: int = 512,
                 num_layers: int = 8, mapping_type='mlp', only_prefix: Optional[bool] = False,
                 only_soft_prompt: Optional[bool] = False):
        super(ClapCaption_prompt, self).__init__(prefix_length, clip_length, prefix_size, num_layers,
                                                 mapping_type, only_prefix=only_prefix)
        self.only_soft_prompt = only_soft_prompt

    def clap_to_gpt(self, prefix: torch.Tensor, embedding_hard_prompt: torch.Tensor,
                    embedding_text: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None,
                    hard_prompts_masks: Optional[torch.Tensor] = None):
        """caption_model.py:315-329: [wte(hard prompt) ; mapper(prefix)] (+ text embeddings)."""
        prefix_projections = self.clap_project(prefix).view(-1, self.prefix_length, self.gpt_embedding_size)
        if not self.only_soft_prompt:
            prefix_projections = torch.cat((embedding_hard_prompt, prefix_projections), dim=1)
        if embedding_text is not None:
            embedding_cat = torch.cat((prefix_projections, embedding_text), dim=1)
            if not self.only_soft_prompt:
                mask = torch.cat((hard_prompts_masks, mask), dim=1)
        else:
            embedding_cat = prefix_projections
        return embedding_cat, mask
