"""Oracle for the caption side: prompt assembly, mappers, clap_to_gpt, GPT-2 and decoding.
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

References:
  sound_effect_choice       utils.py:131-137 (called from dataset/dataset.py:445)
  compose_discrete_prompts  utils.py:158-176;  padding_captions utils.py:190-208
  MLP / TransformerMapper   models/mapper.py:6-18, 20-139
  clap_to_gpt               models/caption_model.py:315-329 (hard prompt first, then soft prefix)
  GPT-2 small forward       HF GPT2LMHeadModel (transformers 4.24 pin), eager attention
  generate2 (greedy)        gpt2_prefix_eval.py:161-222
  generate_beam             gpt2_prefix_eval.py:99-158
  get_prefix_tokens         gpt2_prefix_eval.py:271-278 (+ normalize(wte) predict_prompt.py:117-118)
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

D, NH, HD, NL, V = 768, 12, 64, 12, 50257
STOP_GREEDY = (13, 764)
STOP_BEAM = 13


# ------------------------------------------------------------------ prompt

def sound_effect_choice(prefix: torch.Tensor, labels: torch.Tensor, k: int) -> torch.Tensor:
    """utils.py:131-137: topk(softmax(prefix @ labels^T)) -> label indices [.., k]."""
    sim = prefix @ labels.t()
    return torch.topk(F.softmax(sim, dim=-1), k, dim=-1)[1]


def prompt_ids(label_idx: Sequence[int], label_tokens: Sequence[Sequence[int]]) -> List[int]:
    """Ids of compose_discrete_prompts (utils.py:158-176) built from per-piece BPE ids (the GPT-2
    pre-tokenizer splits the prompt at exactly these piece boundaries; zsaac/tokenizer.py)."""
    if len(label_idx) == 0:
        return [1858, 389, 1223, 287, 428, 6597, 13]
    out = [1858, 389]
    for n, li in enumerate(label_idx):
        out += list(label_tokens[int(li)])
        if n + 1 < len(label_idx):
            out.append(11)
    return out + [287, 428, 6597, 13]


# ------------------------------------------------------------------ mappers

def mlp_mapper(x, sd, prefix="clap_project.model."):
    """MLP((1024, 3840, 7680)) with Tanh between the two Linears (mapper.py:6-18)."""
    h = torch.tanh(F.linear(x, sd[prefix + "0.weight"], sd[prefix + "0.bias"]))
    return F.linear(h, sd[prefix + "2.weight"], sd[prefix + "2.bias"])


def transformer_mapper(x, sd, prefix="clap_project.", clip_length=10, num_layers=8, heads=8):
    """TransformerMapper.forward (mapper.py:127-131) -> Transformer (enc_dec False: self-attn,
    mapper.py:99-107) -> TransformerLayer pre-LN (mapper.py:77-80) -> MultiHeadAttention
    (mapper.py:49-66, softmax over keys, scale head_dim^-0.5) -> MlpTransformer ReLU (20-35)."""
    B = x.shape[0]
    h = F.linear(x, sd[prefix + "linear.weight"], sd[prefix + "linear.bias"]).view(B, clip_length, -1)
    pc = sd[prefix + "prefix_const"]
    h = torch.cat((h, pc.unsqueeze(0).expand(B, *pc.shape)), dim=1)
    for i in range(num_layers):
        L = prefix + f"transformer.layers.{i}."
        a = F.layer_norm(h, (h.shape[-1],), sd[L + "norm1.weight"], sd[L + "norm1.bias"])
        b, n, c = a.shape
        q = F.linear(a, sd[L + "attn.to_queries.weight"]).reshape(b, n, heads, c // heads)
        kv = F.linear(a, sd[L + "attn.to_keys_values.weight"]).reshape(b, n, 2, heads, c // heads)
        k, v = kv[:, :, 0], kv[:, :, 1]
        att = torch.einsum("bnhd,bmhd->bnmh", q, k) * (c // heads) ** -0.5
        att = att.softmax(dim=2)
        o = torch.einsum("bnmh,bmhd->bnhd", att, v).reshape(b, n, c)
        h = h + F.linear(o, sd[L + "attn.project.weight"], sd[L + "attn.project.bias"])
        a = F.layer_norm(h, (c,), sd[L + "norm2.weight"], sd[L + "norm2.bias"])
        m = F.linear(F.relu(F.linear(a, sd[L + "mlp.fc1.weight"], sd[L + "mlp.fc1.bias"])),
                     sd[L + "mlp.fc2.weight"], sd[L + "mlp.fc2.bias"])
        h = h + m
    return h[:, clip_length:]


def clap_to_gpt(prefix, hard_ids, sd, mapping_type="mlp", prefix_length=10):
    """ClapCaption_prompt.clap_to_gpt (caption_model.py:315-329) with the caller's wte lookup of
    the hard prompt (predict_prompt.py:133): [wte(hard) ; mapper(prefix).view(-1,10,768)]."""
    proj = mlp_mapper(prefix, sd) if mapping_type == "mlp" else transformer_mapper(prefix, sd)
    proj = proj.reshape(-1, prefix_length, D)
    emb_h = sd["gpt.transformer.wte.weight"][hard_ids]
    return torch.cat((emb_h, proj), dim=1)


# ------------------------------------------------------------------ GPT-2

def gelu_new(x):
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


def _ln(x, sd, name):
    return F.layer_norm(x, (D,), sd[name + ".weight"], sd[name + ".bias"], 1e-5)


def gpt2_hidden(embeds: torch.Tensor, sd, past: Optional[list] = None, pos0: int = 0):
    """GPT-2 transformer over ``inputs_embeds`` [B,L,768]; ``past`` = per-layer (k, v) caches
    (None = full recompute as the reference does).  Returns (ln_f hidden [B,L,768], new past)."""
    p = "gpt.transformer."
    B, L, _ = embeds.shape
    h = embeds + sd[p + "wpe.weight"][pos0:pos0 + L]
    new_past = []
    for i in range(NL):
        n = p + f"h.{i}."
        a = _ln(h, sd, n + "ln_1")
        qkv = a @ sd[n + "attn.c_attn.weight"] + sd[n + "attn.c_attn.bias"]
        q, k, v = qkv.split(D, dim=2)
        q, k, v = (t.view(B, L, NH, HD).transpose(1, 2) for t in (q, k, v))
        if past is not None and past[i] is not None:
            k = torch.cat((past[i][0], k), dim=2)
            v = torch.cat((past[i][1], v), dim=2)
        new_past.append((k, v))
        S = k.shape[2]
        att = (q @ k.transpose(-1, -2)) * (HD ** -0.5)
        causal = torch.ones(L, S, dtype=torch.bool).tril(S - L)
        att = att.masked_fill(~causal, torch.finfo(att.dtype).min).softmax(-1)
        o = (att @ v).transpose(1, 2).reshape(B, L, D)
        h = h + (o @ sd[n + "attn.c_proj.weight"] + sd[n + "attn.c_proj.bias"])
        a = _ln(h, sd, n + "ln_2")
        m = gelu_new(a @ sd[n + "mlp.c_fc.weight"] + sd[n + "mlp.c_fc.bias"])
        h = h + (m @ sd[n + "mlp.c_proj.weight"] + sd[n + "mlp.c_proj.bias"])
    return _ln(h, sd, p + "ln_f"), new_past


def gpt2_logits(embeds, sd, past=None, pos0=0):
    h, new_past = gpt2_hidden(embeds, sd, past, pos0)
    return h @ sd["gpt.transformer.wte.weight"].t(), new_past


def generate2(embed: torch.Tensor, sd, entry_length=67, use_cache=False,
              margins: Optional[list] = None, temperature=1.0) -> List[int]:
    """generate2 (gpt2_prefix_eval.py:161-222), batch 1.  Logits are divided by ``temperature``
    (line 196: ``temperature if temperature > 0 else 1.0``); the top-p filter never removes the
    sorted-first token (lines 197-206), so the pick is the argmax of the scaled logits.
    Stops after appending 13 ('.') or 764 (' .').  ``use_cache`` swaps the reference's full
    recompute for a KV cache (same math, ~1e-6 different rounding)."""
    generated = embed
    tokens: List[int] = []
    wte = sd["gpt.transformer.wte.weight"]
    past, pos = None, 0
    with torch.no_grad():
        for _ in range(entry_length):
            if use_cache:
                logits, past = gpt2_logits(generated if past is None else generated[:, -1:], sd,
                                           past, pos)
                pos = generated.shape[1]
            else:
                logits, _ = gpt2_logits(generated, sd)
            last = logits[0, -1] / (temperature if temperature > 0 else 1.0)
            nxt = int(torch.argmax(last))
            if margins is not None:
                top2 = last.topk(2).values
                margins.append(float(top2[0] - top2[1]))
            tokens.append(nxt)
            generated = torch.cat((generated, wte[nxt].view(1, 1, -1)), dim=1)
            if nxt in STOP_GREEDY:
                break
    return tokens


def generate_beam(embed: torch.Tensor, sd, beam_size=5, entry_length=67,
                  use_cache=False, temperature=1.0,
                  gaps: Optional[List[float]] = None) -> Tuple[List[List[int]], List[float]]:
    """generate_beam (gpt2_prefix_eval.py:99-158): logits / temperature (line 121, ``temperature
    if temperature > 0 else 1.0``), log(softmax) scores, stopped
    beams only extend with id 0 at zero cost, length-normalised top-k over beam x vocab, stop when
    every beam has emitted 13.  Returns (token lists ordered best-first, their final scores).

    ``gaps`` (test instrumentation, not in the reference): when a list is given, every selection
    appends the score gap between the last kept and the first dropped candidate (step 0: log-probs;
    later steps: the length-normalised sums the top-k ranks), and the end appends the gap between
    the best and second-best final scores -- the margins a perturbed search must clear to make the
    same choices."""
    wte = sd["gpt.transformer.wte.weight"]
    tokens = None
    scores = None
    seq_lengths = torch.ones(beam_size)
    is_stopped = torch.zeros(beam_size, dtype=torch.bool)
    generated = embed
    past, pos = None, 0
    with torch.no_grad():
        for _ in range(entry_length):
            if use_cache:
                logits, past = gpt2_logits(generated if past is None else generated[:, -1:], sd,
                                           past, pos)
                pos = generated.shape[1]
            else:
                logits, _ = gpt2_logits(generated, sd)
            logits = (logits[:, -1, :] / (temperature if temperature > 0 else 1.0)).softmax(-1).log()
            if scores is None:
                if gaps is not None:
                    v = logits[0].topk(beam_size + 1).values
                    gaps.append(float(v[beam_size - 1] - v[beam_size]))
                scores, next_tokens = logits.topk(beam_size, -1)
                generated = generated.expand(beam_size, *generated.shape[1:])
                if past is not None:
                    past = [(k.expand(beam_size, *k.shape[1:]), v.expand(beam_size, *v.shape[1:]))
                            for k, v in past]
                next_tokens, scores = next_tokens.permute(1, 0), scores.squeeze(0)
                tokens = next_tokens
            else:
                logits[is_stopped] = -float("inf")
                logits[is_stopped, 0] = 0
                scores_sum = scores[:, None] + logits
                seq_lengths[~is_stopped] += 1
                avg = scores_sum / seq_lengths[:, None]
                if gaps is not None:
                    v = avg.view(-1).topk(beam_size + 1).values
                    gaps.append(float(v[beam_size - 1] - v[beam_size]))
                avg, next_tokens = avg.view(-1).topk(beam_size, -1)
                src = next_tokens // scores_sum.shape[1]
                seq_lengths = seq_lengths[src]
                next_tokens = (next_tokens % scores_sum.shape[1]).unsqueeze(1)
                tokens = torch.cat((tokens[src], next_tokens), dim=1)
                generated = generated[src]
                if past is not None:
                    past = [(k[src], v[src]) for k, v in past]
                scores = avg * seq_lengths
                is_stopped = is_stopped[src]
            nxt = wte[next_tokens.squeeze()].view(generated.shape[0], 1, -1)
            generated = torch.cat((generated, nxt), dim=1)
            is_stopped = is_stopped + next_tokens.eq(STOP_BEAM).squeeze()
            if is_stopped.all():
                break
    scores = scores / seq_lengths
    outs = [tokens[i, :int(seq_lengths[i])].tolist() for i in range(beam_size)]
    order = scores.argsort(descending=True)
    if gaps is not None:
        gaps.append(float(scores[order[0]] - scores[order[1]]))
    return [outs[i] for i in order], [float(scores[i]) for i in order]


def prefix_tokens(prefix_embed: torch.Tensor, sd) -> List[int]:
    """get_prefix_tokens (gpt2_prefix_eval.py:271-278): argmax_n cos(prefix_embed[0,p], wte[n])."""
    emb = F.normalize(sd["gpt.transformer.wte.weight"], 2, 1)
    sim = torch.einsum("pd,nd->pn", F.normalize(prefix_embed[0], 2, 1), emb)
    return sim.argmax(-1).tolist()
