"""Oracle for the C5 Mistral caption path.  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

References (/root/reference): predict_mistralai_multilingual.py:97-111 (clap_to_gpt with the
language tag, then ``LMmodel.generate(inputs_embeds, attention_mask=ones, do_sample=False,
max_length=60, eos_token_id=2, pad_token_id=2)``), models/caption_model.py:340-413
(ClapCaption_Mistralai_prompt; MLP mapper 1024 -> 5*D -> 10*D).  Decoder arithmetic restated from
HF MistralForCausalLM (the reference's transformers dependency, not vendored): RMSNorm
x * rsqrt(mean(x^2) + eps) * w; rotary embedding with rotate_half, inv_freq = theta^(-2i/128);
grouped-query attention (kv head = q head // (H / KVH)), causal, softmax((q k^T) / sqrt(128));
MLP down(silu(gate(x)) * up(x)); untied lm_head.  generate with only inputs_embeds (transformers
5.x, this container): at most max_length - P new tokens, greedy, a finished row emits pad.
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.nn.functional as F


def rms(x, w, eps):
    return w * (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps))


def rope_tables(L, hd=128, theta=10000.0):
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, dtype=torch.int64).float() / hd))
    fr = torch.arange(L, dtype=torch.float32)[:, None] * inv[None]
    emb = torch.cat((fr, fr), dim=-1)
    return emb.cos(), emb.sin()


def _rot(x):
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


def forward(x, sd, H, KVH, eps, past=None, pos0=0, theta=10000.0):
    """MistralModel over inputs_embeds x [B, L, D] (+ per-layer (k, v) caches): returns
    (final-norm hidden [B, L, D], new caches)."""
    B, L, D = x.shape
    hd = D // H
    cos, sin = rope_tables(pos0 + L, hd, theta)
    cos, sin = cos[pos0:pos0 + L], sin[pos0:pos0 + L]
    new = []
    i = 0
    while f"model.layers.{i}.self_attn.q_proj.weight" in sd:
        p = f"model.layers.{i}."
        a = rms(x, sd[p + "input_layernorm.weight"], eps)
        q = (a @ sd[p + "self_attn.q_proj.weight"].t()).view(B, L, H, hd).transpose(1, 2)
        k = (a @ sd[p + "self_attn.k_proj.weight"].t()).view(B, L, KVH, hd).transpose(1, 2)
        v = (a @ sd[p + "self_attn.v_proj.weight"].t()).view(B, L, KVH, hd).transpose(1, 2)
        q = q * cos + _rot(q) * sin
        k = k * cos + _rot(k) * sin
        if past is not None:
            k = torch.cat((past[i][0], k), dim=2)
            v = torch.cat((past[i][1], v), dim=2)
        new.append((k, v))
        kk = k.repeat_interleave(H // KVH, dim=1)
        vv = v.repeat_interleave(H // KVH, dim=1)
        S = kk.shape[2]
        att = (q @ kk.transpose(-1, -2)) * (hd ** -0.5)
        causal = torch.ones(L, S, dtype=torch.bool).tril(S - L)
        att = att.masked_fill(~causal, torch.finfo(att.dtype).min).softmax(-1)
        o = (att @ vv).transpose(1, 2).reshape(B, L, D)
        x = x + o @ sd[p + "self_attn.o_proj.weight"].t()
        a = rms(x, sd[p + "post_attention_layernorm.weight"], eps)
        m = F.silu(a @ sd[p + "mlp.gate_proj.weight"].t()) * (a @ sd[p + "mlp.up_proj.weight"].t())
        x = x + m @ sd[p + "mlp.down_proj.weight"].t()
        i += 1
    return rms(x, sd["model.norm.weight"], eps), new


def clap_to_gpt(prefix, hard_ids, tag_ids, sd, mlp_sd, prefix_length=10):
    """caption_model.py:392-413 with the caller's embed_tokens lookups
    (predict_mistralai_multilingual.py:95-101): [embed(hard) ; MLP(prefix) ; embed(tag)]."""
    emb = sd["model.embed_tokens.weight"]
    D = emb.shape[1]
    h = torch.tanh(F.linear(prefix, mlp_sd["clap_project.model.0.weight"], mlp_sd["clap_project.model.0.bias"]))
    soft = F.linear(h, mlp_sd["clap_project.model.2.weight"], mlp_sd["clap_project.model.2.bias"])
    soft = soft.view(-1, prefix_length, D)
    B = soft.shape[0]
    return torch.cat((emb[hard_ids], soft, emb[tag_ids][None].expand(B, -1, -1)), dim=1), soft


def generate(embeds, sd, H, KVH, eps, max_length=60, eos=2, pad=2, margins=None) -> List[List[int]]:
    """Batched greedy generate over inputs_embeds (KV cache): per row the ids up to and
    including eos (pads after it dropped); ``margins`` (a list) receives per row the top-1 minus
    top-2 logit at every emitted step."""
    B, P, _ = embeds.shape
    lm = sd["lm_head.weight"]
    wemb = sd["model.embed_tokens.weight"]
    out = [[] for _ in range(B)]
    mg = [[] for _ in range(B)]
    done = torch.zeros(B, dtype=torch.bool)
    with torch.no_grad():
        h, past = forward(embeds, sd, H, KVH, eps)
        logits = h[:, -1] @ lm.t()
        for step in range(max_length - P):
            nxt = logits.argmax(-1)
            top2 = logits.topk(2, dim=-1).values
            nxt = torch.where(done, torch.full_like(nxt, pad), nxt)
            for b in range(B):
                if not done[b]:
                    out[b].append(int(nxt[b]))
                    mg[b].append(float(top2[b, 0] - top2[b, 1]))
            done = done | (nxt == eos)
            if bool(done.all()) or step + 1 == max_length - P:
                break
            h, past = forward(wemb[nxt][:, None], sd, H, KVH, eps, past, P + step)
            logits = h[:, -1] @ lm.t()
    if margins is not None:
        margins.extend(mg)
    return out
