"""Drop-in for the reference's ``models/caption_model.py`` caption classes:
``ClapCaptionModel`` (caption_model.py:13-89) with and without the sound-effect projection,
``ClapCaptionPrefix`` (90-98), ``ClapCaptionCrossattention`` (100-149),
``ClapCaptionCrossattention_v2`` (151-206) and ``ClapCaption_prompt`` (291-338).

Same constructor arguments and state-dict keys (``gpt.*`` = HF GPT2LMHeadModel layout, 149 keys,
plus ``clap_project.*`` and ``sound_effect_project.*``), so ``load_state_dict(torch.load(...))``
works unchanged.  The only construction difference: the reference fetches
``GPT2LMHeadModel.from_pretrained('gpt2')`` by name (caption_model.py:52); here ``gpt`` is built at
the GPT-2-small architecture and its weights come from the checkpoint.  Every forward runs on the
HIP kernels: the mappers' GEMMs, sound_effect_choice (zs_label_topk), the cross-attention
(in_proj / out_proj GEMMs + zs_cross_attention) and GPT-2.

Inference only: ``forward`` (the training forward, with labels and attention masks) serves
labels=None / mask=None; ClapCaptionCrossattention_v2's training-time random key mask is not
provided (eval uses no mask, caption_model.py:182-183).

``ClapCaption_Mistralai_prompt`` (caption_model.py:340-413, BASELINE config C5) holds the
MistralForCausalLM parameter tree under ``LMmodel.base_model.model`` (the peft path its callers
use: ``LMmodel.base_model.model.model.embed_tokens``, predict_mistralai_multilingual.py:95-101)
and ``LMmodel.generate`` runs zsaac.mistral on the HIP kernels (fp8 e4m3 weights by default;
``zs_dtype = torch.float32`` selects the f32 parity mode).  A peft checkpoint's LoRA factors are
merged into the base weights at load; the reference's NF4 storage (bitsandbytes) is replaced by
fp8 (zsaac/mistral.py).
"""
from enum import Enum
from typing import Optional

import torch
import torch.nn as nn

from zsaac import ops
from zsaac.modules import EngineCache, ZsGPT2LMHeadModel, require_device, zs_dtype_of

from .mapper import MLP, TransformerMapper


class MappingType(Enum):
    MLP = 'mlp'
    Transformer = 'transformer'


class ZsMultiheadAttention(nn.Module):
    """``nn.MultiheadAttention(embed_dim, num_heads, batch_first=True)`` (the sound-effect
    cross-attention, caption_model.py:109, 160) with its parameter names (in_proj_weight,
    in_proj_bias, out_proj.weight / .bias) and torch's initialisation; inference forward on the
    HIP kernels: in_proj GEMMs -> zs_cross_attention -> out_proj GEMM (+ ``residual`` fused into
    its epilogue).  Returns (attn_output, None): the averaged attention weights are not
    computed (no caller reads them)."""

    def __init__(self, embed_dim: int, num_heads: int, batch_first: bool = True, bias: bool = True):
        super().__init__()
        if not batch_first:
            raise NotImplementedError("batch_first=False")
        self.embed_dim, self.num_heads, self.batch_first = embed_dim, num_heads, batch_first
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * embed_dim)) if bias else None
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=bias)
        nn.init.xavier_uniform_(self.in_proj_weight)
        if bias:
            nn.init.zeros_(self.out_proj.bias)
        self._cache = EngineCache()

    def forward(self, query, key, value, attn_mask=None, need_weights=True, residual=None):
        require_device(query, "MultiheadAttention.forward")
        if attn_mask is not None:
            raise NotImplementedError("attention masks (training-time) are not provided")
        dt = zs_dtype_of(self)
        E, H = self.embed_dim, self.num_heads
        B, Lq, _ = query.shape
        Lk = key.shape[1]
        w = self._cache.get(self, lambda: (
            self.in_proj_weight.detach().to(dt).contiguous(),
            None if self.in_proj_bias is None else self.in_proj_bias.detach().float().contiguous(),
            self.out_proj.weight.detach().to(dt).contiguous(),
            None if self.out_proj.bias is None else self.out_proj.bias.detach().float().contiguous()),
            (dt,))
        wi, bi, wo, bo = w
        dev = query.device

        def rows(t, n):
            r = torch.empty(n, E, device=dev, dtype=dt)
            ops.cast(t.reshape(n, E).float().contiguous(), r)
            return r
        qa = rows(query, B * Lq)
        q = torch.empty(B * Lq, E, device=dev, dtype=dt)
        ops.gemm(qa, wi[:E], q, bias=None if bi is None else bi[:E])
        kv = torch.empty(B * Lk, 2 * E, device=dev, dtype=dt)
        if key is value:
            ops.gemm(rows(key, B * Lk), wi[E:], kv, bias=None if bi is None else bi[E:])
        else:
            ops.gemm(rows(key, B * Lk), wi[E:2 * E], kv[:, :E], bias=None if bi is None else bi[E:2 * E])
            ops.gemm(rows(value, B * Lk), wi[2 * E:], kv[:, E:], bias=None if bi is None else bi[2 * E:])
        att = torch.empty(B * Lq, E, device=dev, dtype=dt)
        ops.cross_attention(q, kv[:, :E], kv[:, E:], B, Lq, Lk, H, att)
        out = torch.empty(B * Lq, E, device=dev)
        res = None if residual is None else residual.reshape(B * Lq, E).float().contiguous()
        if res is not None:
            out.copy_(res)
        ops.gemm(att, wo, out, bias=bo, residual=None if res is None else out)
        return out.view(B, Lq, E), None


class ClapCaptionModel(nn.Module):

    def sound_effect_choice(self, prefix, sound_effect_embeddings, choice_num):
        """caption_model.py:15-20: the choice_num label embeddings most similar to the prefix
        (softmax is monotone: top-k of the similarities), [B, choice_num, D]; zs_label_topk."""
        require_device(prefix, "sound_effect_choice")
        D = prefix.shape[-1]
        e = prefix.reshape(-1, D).float().contiguous()
        rows = torch.empty(e.shape[0], choice_num, D, device=e.device)
        ops.label_topk(e, sound_effect_embeddings.float().contiguous(), choice_num, rows)
        return rows

    def get_dummy_token(self, batch_size: int, device: torch.device) -> torch.Tensor:
        return torch.zeros(batch_size, self.prefix_length, dtype=torch.int64, device=device)

    def _check_inference(self, mask, labels):
        if labels is not None or mask is not None:
            raise NotImplementedError("the training forward (labels / attention masks) is out of "
                                      "scope; inference: forward(tokens, prefix)")

    def forward(self, tokens: torch.Tensor, prefix: torch.Tensor, mask: Optional[torch.Tensor] = None,
                labels: Optional[torch.Tensor] = None):
        """caption_model.py:25-37 at inference (labels=None, mask=None): (gpt output, logits of
        the positions after the sound-effect and prefix tokens)."""
        self._check_inference(mask, labels)
        embedding_text = self.gpt.transformer.wte(tokens)
        embedding_cat, mask = self.clap_to_gpt(prefix, embedding_text, mask)
        out = self.gpt(inputs_embeds=embedding_cat)
        n = self.prefix_length + (self.sound_effect_num if self.sound_effect_embeddings is not None else 0)
        return out, out.logits[:, n - 1: -1]

    def __init__(self, prefix_length: int, clip_length: Optional[int] = None, prefix_size: int = 512,
                 num_layers: int = 8, mapping_type='mlp', sound_effect_embeddings: torch.Tensor = None,
                 sound_effect_num: Optional[int] = 0, only_prefix: Optional[bool] = False,
                 mask_probability: Optional[float] = 0):
        super(ClapCaptionModel, self).__init__()
        self.prefix_length = prefix_length
        self.sound_effect_embeddings = sound_effect_embeddings
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
        if self.sound_effect_embeddings is not None:
            self.sound_effect_project = MLP((prefix_size, self.gpt_embedding_size // 2,
                                             self.gpt_embedding_size))

    def clap_to_gpt(self, prefix: torch.Tensor, embedding_text: Optional[torch.Tensor] = None,
                    mask: Optional[torch.Tensor] = None):
        """caption_model.py:66-82: [sound-effect projections (k) ; mapper(prefix) ; text]."""
        proj = self.clap_project(prefix).view(-1, self.prefix_length, self.gpt_embedding_size)
        emb = proj if embedding_text is None else torch.cat((proj, embedding_text), dim=1)
        if self.sound_effect_embeddings is not None:
            se = self.sound_effect_choice(prefix, self.sound_effect_embeddings, self.sound_effect_num)
            se_proj = self.sound_effect_project(se).view(-1, self.sound_effect_num, self.gpt_embedding_size)
            emb = torch.cat((se_proj, emb), dim=1)
            if mask is not None:
                mask = torch.cat((torch.ones((prefix.shape[0], self.sound_effect_num), device=prefix.device),
                                  mask), dim=-1)
        return emb, mask

    def set_dtype(self, dtype: torch.dtype):
        """float32 = parity mode (default), bfloat16 = perf mode, for every kernel engine."""
        mods = [self, self.gpt, self.clap_project]
        if hasattr(self, "sound_effect_project"):
            mods.append(self.sound_effect_project)
        for m in mods:
            m.zs_dtype = dtype
        return self


class ClapCaptionPrefix(ClapCaptionModel):
    """caption_model.py:90-98: only the mapper's parameters are trained; GPT-2 stays in eval."""

    def parameters(self, recurse: bool = True):
        return self.clap_project.parameters()

    def train(self, mode: bool = True):
        super(ClapCaptionPrefix, self).train(mode)
        self.gpt.eval()
        return self


class ClapCaptionCrossattention(ClapCaptionModel):
    """caption_model.py:100-149: the prefix attends over its k chosen sound-effect label
    embeddings (nn.MultiheadAttention, 4 heads) and the attention output replaces it before the
    mapper; no sound-effect tokens in the GPT-2 sequence."""

    RESIDUAL = False

    def __init__(self, prefix_length: int, clip_length: Optional[int] = None, prefix_size: int = 512,
                 num_layers: int = 8, mapping_type='mlp', sound_effect_embeddings: torch.Tensor = None,
                 sound_effect_num: Optional[int] = 0, only_prefix: Optional[bool] = False,
                 mask_probability: Optional[float] = 0):
        super(ClapCaptionCrossattention, self).__init__(prefix_length, clip_length, prefix_size,
                                                        num_layers, mapping_type,
                                                        sound_effect_embeddings, sound_effect_num,
                                                        only_prefix, mask_probability)
        if self.sound_effect_embeddings is not None:
            self.sound_effect_project = ZsMultiheadAttention(prefix_size, 4, batch_first=True)

    def forward(self, tokens: torch.Tensor, prefix: torch.Tensor, mask: Optional[torch.Tensor] = None,
                labels: Optional[torch.Tensor] = None):
        self._check_inference(mask, labels)
        embedding_text = self.gpt.transformer.wte(tokens)
        embedding_cat, mask = self.clap_to_gpt(prefix, embedding_text, mask)
        out = self.gpt(inputs_embeds=embedding_cat)
        return out, out.logits[:, self.prefix_length - 1: -1]

    def clap_to_gpt(self, prefix: torch.Tensor, embedding_text: Optional[torch.Tensor] = None,
                    mask: Optional[torch.Tensor] = None):
        """caption_model.py:122-138 (v2, 170-196: the attention output is added to the prefix)."""
        if self.sound_effect_embeddings is not None:
            se = self.sound_effect_choice(prefix, self.sound_effect_embeddings, self.sound_effect_num)
            prefix, _ = self.sound_effect_project(prefix, se, se,
                                                  residual=prefix if self.RESIDUAL else None)
        proj = self.clap_project(prefix).view(-1, self.prefix_length, self.gpt_embedding_size)
        emb = proj if embedding_text is None else torch.cat((proj, embedding_text), dim=1)
        return emb, mask


class ClapCaptionCrossattention_v2(ClapCaptionCrossattention):
    """caption_model.py:151-206 at inference: prefix = MHA(prefix, sound effects) + prefix."""

    RESIDUAL = True

    def __init__(self, prefix_length: int, clip_length: Optional[int] = None, prefix_size: int = 512,
                 num_layers: int = 8, mapping_type='mlp', sound_effect_embeddings: torch.Tensor = None,
                 sound_effect_num: Optional[int] = 0, only_prefix: Optional[bool] = False,
                 mask_probability: Optional[float] = 0.25):
        super(ClapCaptionCrossattention_v2, self).__init__(prefix_length, clip_length, prefix_size,
                                                           num_layers, mapping_type,
                                                           sound_effect_embeddings,
                                                           sound_effect_num, only_prefix,
                                                           mask_probability)


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


# ----------------------------------------------------------------------------- Mistral (C5)
MISTRAL_7B_CONFIG = dict(vocab_size=32000, hidden_size=4096, intermediate_size=14336,
                         num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8,
                         rms_norm_eps=1e-5, rope_theta=10000.0)


class _ZsMistralModel(nn.Module):
    def __init__(self, c):
        super().__init__()
        D, F = c["hidden_size"], c["intermediate_size"]
        hd = D // c["num_attention_heads"]
        kv = c["num_key_value_heads"] * hd
        self.embed_tokens = nn.Embedding(c["vocab_size"], D)
        self.layers = nn.ModuleList()
        for _ in range(c["num_hidden_layers"]):
            ly = nn.Module()
            ly.self_attn = nn.Module()
            for n, o in (("q_proj", D), ("k_proj", kv), ("v_proj", kv), ("o_proj", D)):
                setattr(ly.self_attn, n, nn.Linear(D, o, bias=False))
            ly.mlp = nn.Module()
            ly.mlp.gate_proj = nn.Linear(D, F, bias=False)
            ly.mlp.up_proj = nn.Linear(D, F, bias=False)
            ly.mlp.down_proj = nn.Linear(F, D, bias=False)
            ly.input_layernorm = nn.Module()
            ly.input_layernorm.weight = nn.Parameter(torch.ones(D))
            ly.post_attention_layernorm = nn.Module()
            ly.post_attention_layernorm.weight = nn.Parameter(torch.ones(D))
            self.layers.append(ly)
        self.norm = nn.Module()
        self.norm.weight = nn.Parameter(torch.ones(D))


class ZsMistralForCausalLM(nn.Module):
    """MistralForCausalLM's module tree / keys (``model.*``, ``lm_head``); ``generate`` with
    inputs_embeds runs the HIP decoder (greedy only, as the reference calls it)."""

    def __init__(self, config: dict):
        super().__init__()
        with torch.device("meta"):
            self.model = _ZsMistralModel(config)
            self.lm_head = nn.Linear(config["hidden_size"], config["vocab_size"], bias=False)
        self.config = dict(config)
        self._cache = EngineCache()

    def engine(self, device, max_batch, max_prompt, max_new):
        from zsaac.mistral import MistralDecoder, MistralWeights
        # fp8 weights unless set_mode() / zs_mistral_mode picks "bf16" or the "f32" parity mode
        mode = getattr(self, "zs_mistral_mode", "fp8")
        c = self.config
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:        # "cuda" and "cuda:0" are one key
            device = torch.device("cuda", torch.cuda.current_device())

        def build():
            return MistralWeights(self.state_dict(), device, mode, c["num_attention_heads"],
                                  c["num_key_value_heads"], c.get("rms_norm_eps", 1e-5),
                                  c.get("rope_theta", 10000.0))
        w = self._cache.get(self, build, (mode, str(device)))
        # one decoder per weights, reused while its capacity covers the call (the reference pads
        # each batch's hard prompt to its longest and appends a per-language tag, so P changes
        # from call to call; rebuilding per (B, P, new) re-allocated the KV caches and slabs and
        # re-captured the decode graph every time); grown to the max of old and new bounds
        dec = w.__dict__.get("_decoder")
        if dec is None or dec.B < max_batch or dec.Pmax < max_prompt or dec.max_new < max_new:
            if dec is not None:
                max_batch, max_prompt = max(max_batch, dec.B), max(max_prompt, dec.Pmax)
                max_new = max(max_new, dec.max_new)
            w.__dict__["_decoder"] = None
            dec = w.__dict__["_decoder"] = MistralDecoder(w, max_batch, max_prompt, max_new)
        return dec

    def generate(self, inputs_embeds=None, attention_mask=None, do_sample=False, max_length=60,
                 eos_token_id=2, pad_token_id=2, **kw):
        """Greedy generate over inputs_embeds with an all-ones mask (the only call the reference
        makes, predict_mistralai_multilingual.py:105-111): [B, max_length - P] ids, rows that
        finished padded with ``pad_token_id`` (HF's output)."""
        if do_sample or kw.get("num_beams", 1) != 1:
            raise NotImplementedError("only greedy generate (do_sample=False) is provided")
        if attention_mask is not None and not bool((attention_mask == 1).all()):
            raise NotImplementedError("attention_mask must be all ones (as the reference passes)")
        require_device(inputs_embeds, "MistralForCausalLM.generate")
        B, P, _ = inputs_embeds.shape
        new = max(max_length - P, 0)
        # capacity by the call's upper bounds: any prompt up to 64 rows (or P), any new <= max_length
        dec = self.engine(inputs_embeds.device, max(B, 32), max(P, 64), max(max_length, 1))
        rows = dec.generate_embeds(inputs_embeds, max_length=max_length, eos=eos_token_id)
        # HF generate returns only as many columns as were generated: until every row emitted eos
        # (finished rows padded with pad_token_id) or max_length - P
        width = min(new, max([len(r) for r in rows] + [0]))
        out = torch.full((B, width), pad_token_id, dtype=torch.long)
        for b, r in enumerate(rows):
            out[b, :len(r)] = torch.tensor(r, dtype=torch.long)
        return out.to(inputs_embeds.device)


class _LoraModel(nn.Module):
    def __init__(self, lm):
        super().__init__()
        self.model = lm


class _PeftModel(nn.Module):
    """The attribute path of peft's PeftModelForCausalLM that the reference's callers use."""

    def __init__(self, lm):
        super().__init__()
        self.base_model = _LoraModel(lm)

    def generate(self, *a, **k):
        return self.base_model.model.generate(*a, **k)


class ClapCaption_Mistralai_prompt(nn.Module):

    def __init__(self, prefix_length: int, clip_length: Optional[int] = None, prefix_size: int = 512,
                 num_layers: int = 8, mapping_type: MappingType = 'mlp',
                 only_prefix: Optional[bool] = False, only_soft_prompt: Optional[bool] = False,
                 islang: Optional[int] = 0, mistral_config: Optional[dict] = None):
        super().__init__()
        self.prefix_length = prefix_length
        self.only_soft_prompt = only_soft_prompt
        self.only_prefix = only_prefix
        self.islang = islang
        self.LMmodel = _PeftModel(ZsMistralForCausalLM(mistral_config or MISTRAL_7B_CONFIG))
        self.lm_embedding_size = (mistral_config or MISTRAL_7B_CONFIG)["hidden_size"]
        if mapping_type in ('mlp', MappingType.MLP):
            self.clap_project = MLP((prefix_size, (self.lm_embedding_size * prefix_length) // 2,
                                     self.lm_embedding_size * prefix_length))
        else:
            self.clap_project = TransformerMapper(prefix_size, self.lm_embedding_size, prefix_length,
                                                  clip_length, num_layers)

    def set_mode(self, mode: str):
        """Decoder weight storage: "fp8" (default), "bf16" or "f32" (parity mode)."""
        self.LMmodel.base_model.model.zs_mistral_mode = mode
        return self

    def load_state_dict(self, state_dict, strict: bool = True):
        """Reference checkpoints hold the peft tree (``LMmodel.base_model.model.*`` with
        ``base_layer`` / ``lora_A`` / ``lora_B``, 4-bit bitsandbytes base weights): NF4 dequantized,
        LoRA merged, the rest loaded as is."""
        from zsaac.mistral import merge_peft_state_dict
        lm = {k: v for k, v in state_dict.items() if k.startswith("LMmodel.")}
        rest = {k: v for k, v in state_dict.items() if not k.startswith("LMmodel.")}
        if any(".lora_A." in k or ".quant_state.bitsandbytes__" in k for k in lm):
            merged = merge_peft_state_dict(lm, prefix="LMmodel.")
        else:
            merged = {k[len("LMmodel.base_model.model."):]: v for k, v in lm.items()
                      if k.startswith("LMmodel.base_model.model.")}
        self.LMmodel.base_model.model.load_state_dict(merged, strict=strict, assign=True)
        return self.clap_project.load_state_dict(
            {k[len("clap_project."):]: v for k, v in rest.items() if k.startswith("clap_project.")},
            strict=strict)

    def clap_to_gpt(self, prefix: torch.Tensor, embedding_hard_prompt: torch.Tensor,
                    embedding_text: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None,
                    hard_prompts_masks: Optional[torch.Tensor] = None):
        """caption_model.py:392-413: [hard ; clap_project(prefix) ; text]."""
        prefix_projections = self.clap_project(prefix).view(-1, self.prefix_length, self.lm_embedding_size)
        if not self.only_soft_prompt:
            prefix_projections = torch.cat((embedding_hard_prompt.float(), prefix_projections), dim=1)
            if hard_prompts_masks is not None:
                mask = torch.cat((hard_prompts_masks, mask), dim=1)
        if embedding_text is not None:
            return torch.cat((prefix_projections, embedding_text.float()), dim=1), mask
        return prefix_projections, mask

    def forward(self, *a, **k):
        raise NotImplementedError("the training forward is out of scope (inference drop-in)")
