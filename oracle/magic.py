"""Oracle for CLAP-guided ("magic") decoding and the CLAP text tower it calls every step.
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): imported by tests/ only, never by the package.

References (/root/reference):
  TextEncoder.forward          retrieval/models/text_encoder.py:58-68 (HF BertModel,
                               add_pooling_layer=False; tokenizer padding='longest',
                               truncation=True, max_length=30)
  ASE.encode_text              retrieval/models/ase_model.py:57-60 (CLS row -> text_proj -> L2)
  compute_audio_text_similarity_via_embeddings / _via_raw_text   gpt2_prefix_eval.py:536-551
  plug_and_play_fast_ranking   gpt2_prefix_eval.py:497-534
  ComputeMagicScore            gpt2_prefix_eval.py:553-599
  generate_beam_magic          gpt2_prefix_eval.py:602-689
  magic_search + PlugAndPlayContrastiveDecodingOneStepFast + enlarge/select_past_key_values
                               gpt2_prefix_eval.py:341-494
BERT arithmetic follows HF BertModel (eager attention): embeddings word + position + token type
0 -> LayerNorm(eps 1e-12); per layer post-LN self-attention (scale 1/sqrt(64), additive
finfo.min key mask) and GELU(erf) feed-forward.  The GPT-2 side reuses oracle.caption.gpt2_hidden
(ln_f hidden states, as HF's ``hidden_states[-1]``), with the reference's full recompute in
generate_beam_magic and its KV-cached steps in magic_search.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from .caption import D, gpt2_hidden

BERT_EPS = 1e-12


def bert_hidden(ids: torch.Tensor, mask: torch.Tensor, sd, layers: int,
                prefix: str = "text_encoder.text_encoder.") -> torch.Tensor:
    """BertModel(input_ids, attention_mask)[0]: last hidden state [T, L, 768]."""
    e = prefix + "embeddings."
    T, L = ids.shape
    x = (sd[e + "word_embeddings.weight"][ids] + sd[e + "position_embeddings.weight"][:L][None]
         + sd[e + "token_type_embeddings.weight"][0][None, None])
    x = F.layer_norm(x, (D,), sd[e + "LayerNorm.weight"], sd[e + "LayerNorm.bias"], BERT_EPS)
    ext = (1.0 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    for i in range(layers):
        p = prefix + f"encoder.layer.{i}."

        def lin(name, t):
            return F.linear(t, sd[p + name + ".weight"], sd[p + name + ".bias"])
        q, k, v = (lin(f"attention.self.{n}", x).view(T, L, 12, 64).transpose(1, 2)
                   for n in ("query", "key", "value"))
        att = (q @ k.transpose(-1, -2)) / 8.0 + ext
        ctx = (att.softmax(-1) @ v).transpose(1, 2).reshape(T, L, D)
        a = F.layer_norm(lin("attention.output.dense", ctx) + x, (D,),
                         sd[p + "attention.output.LayerNorm.weight"],
                         sd[p + "attention.output.LayerNorm.bias"], BERT_EPS)
        h = F.gelu(lin("intermediate.dense", a))
        x = F.layer_norm(lin("output.dense", h) + a, (D,), sd[p + "output.LayerNorm.weight"],
                         sd[p + "output.LayerNorm.bias"], BERT_EPS)
    return x


def encode_text_ids(ids: torch.Tensor, mask: torch.Tensor, sd, layers: int) -> torch.Tensor:
    """ASE.encode_text from tokenised text: normalize(text_proj(BERT(...)[:, 0, :]))."""
    h = bert_hidden(ids, mask, sd, layers)[:, 0, :]
    t = F.linear(F.relu(F.linear(h, sd["text_proj.0.weight"], sd["text_proj.0.bias"])),
                 sd["text_proj.2.weight"], sd["text_proj.2.bias"])
    return F.normalize(t, dim=-1)


def text_encoder(bert_tokenizer, sd, layers: int) -> Callable[[List[str]], torch.Tensor]:
    """clap.encode_text(text_list) (text_encoder.py:58-68 tokenizer call + encode_text)."""
    def enc(texts: List[str]) -> torch.Tensor:
        t = bert_tokenizer(texts, padding="longest", truncation=True, max_length=30,
                           return_tensors="pt")
        return encode_text_ids(t["input_ids"], t["attention_mask"], sd, layers)
    return enc


def clap_log_softmax(audio_embeds: torch.Tensor, text_embeds: torch.Tensor, temp: float):
    """gpt2_prefix_eval.py:541-547: both re-normalised, text @ audio^T / temp, transposed,
    log(softmax(dim=1)) -> [1, T].  ``audio_embeds`` is [1, 1024] (the reference's ``.t()``
    needs a 2-D tensor)."""
    a = audio_embeds / audio_embeds.norm(dim=-1, keepdim=True)
    t = text_embeds / text_embeds.norm(dim=-1, keepdim=True)
    return (torch.matmul(t, a.t()) / temp).T.softmax(dim=1).log()


def ranking(context_hidden, next_hidden, next_top_k_probs, alpha, beta, clap_score, width,
            prefix_length=1):
    """plug_and_play_fast_ranking (gpt2_prefix_eval.py:497-534): returns (selected_idx, scores
    [bsz, width])."""
    c = context_hidden[:, prefix_length - 1:, :]
    nc = c / c.norm(dim=2, keepdim=True)
    nn_ = next_hidden / next_hidden.norm(dim=2, keepdim=True)
    cos = torch.matmul(nc, nn_.transpose(1, 2)).squeeze(-1)
    s, _ = torch.max(cos, dim=-1)
    s = (1.0 - alpha) * next_top_k_probs.view(-1) - alpha * s + beta * clap_score.view(-1)
    s = torch.stack(torch.split(s, width))
    return s.max(dim=-1)[1], s


def _expand(past, w):
    return [(k.repeat_interleave(w, 0), v.repeat_interleave(w, 0)) for k, v in past]


def compute_magic_score(generated, sd, width, input_token, decode, text_encode, audio_embeds,
                        temp, alpha, beta, prefix_length=1):
    """ComputeMagicScore (gpt2_prefix_eval.py:553-599): full GPT-2 recompute over ``generated``,
    top-``width`` candidates of the last position, their next hidden states through the KV
    cache, CLAP text scores of (tokens so far + candidate).  Returns (scores [bsz, 1, width],
    candidate ids [bsz, width])."""
    wte = sd["gpt.transformer.wte.weight"]
    hid, past = gpt2_hidden(generated, sd)
    bsz, seqlen, _ = hid.shape
    logits = hid[:, -1, :] @ wte.t()
    _, top_k_ids = torch.topk(logits, dim=-1, k=width)
    top_k_probs = torch.gather(F.softmax(logits, dim=-1).log(), 1, top_k_ids)
    nxt = wte[top_k_ids.reshape(-1)].view(bsz * width, 1, -1)
    next_hidden, _ = gpt2_hidden(nxt, sd, _expand(past, width), pos0=seqlen)
    context_hidden = hid.repeat_interleave(width, 0)
    if input_token is None:
        toks = top_k_ids.view(-1, 1).clone()
    else:
        toks = torch.cat([input_token.repeat_interleave(width, 0), top_k_ids.view(-1, 1)], dim=-1)
    texts = [decode(t) for t in toks]
    clap = clap_log_softmax(audio_embeds, text_encode(texts), temp)
    _, s = ranking(context_hidden, next_hidden, top_k_probs, alpha, beta, clap, width,
                   prefix_length)
    return s.unsqueeze(1), top_k_ids


def generate_beam_magic(embed, sd, decode, text_encode, audio_embeds, temp, beam_size=5,
                        entry_length=20, magic_width=25, alpha=0.1, beta=0.2,
                        stop_token_index=13) -> Tuple[List[List[int]], List[float]]:
    """generate_beam_magic (gpt2_prefix_eval.py:602-689), temperature 1, ``embed`` given.
    Returns (token lists ordered best-first, their length-normalised scores)."""
    wte = sd["gpt.transformer.wte.weight"]
    tokens, scores = None, None
    seq_lengths = torch.ones(beam_size)
    is_stopped = torch.zeros(beam_size, dtype=torch.bool)
    generated = embed
    with torch.no_grad():
        for _ in range(entry_length):
            logits, logits_ids = compute_magic_score(generated, sd, magic_width, tokens, decode,
                                                     text_encode, audio_embeds, temp, alpha, beta, 1)
            logits = logits[:, -1, :]
            if scores is None:
                scores, index = logits.topk(beam_size, -1)
                next_tokens = logits_ids[torch.arange(logits_ids.size(0)).unsqueeze(1), index]
                generated = generated.expand(beam_size, *generated.shape[1:])
                next_tokens, scores = next_tokens.permute(1, 0), scores.squeeze(0)
                tokens = next_tokens
            else:
                logits_ids = logits_ids.view(-1)
                logits[is_stopped] = -float("inf")
                logits[is_stopped, 0] = 0
                scores_sum = scores[:, None] + logits
                seq_lengths[~is_stopped] += 1
                avg = scores_sum / seq_lengths[:, None]
                avg, next_index = avg.view(-1).topk(beam_size, -1)
                src = next_index // scores_sum.shape[1]
                seq_lengths = seq_lengths[src]
                next_tokens = logits_ids[next_index].unsqueeze(1)
                tokens = torch.cat((tokens[src], next_tokens), dim=1)
                generated = generated[src]
                scores = avg * seq_lengths
                is_stopped = is_stopped[src]
            nxt = wte[next_tokens.squeeze()].view(generated.shape[0], 1, -1)
            generated = torch.cat((generated, nxt), dim=1)
            is_stopped = is_stopped + next_tokens.eq(stop_token_index).squeeze()
            if is_stopped.all():
                break
    scores = scores / seq_lengths
    outs = [tokens[i, :int(seq_lengths[i])].tolist() for i in range(beam_size)]
    order = scores.argsort(descending=True)
    return [outs[i] for i in order], [float(scores[i]) for i in order]


def magic_search(embed, sd, decode, text_encode, audio_embeds, temp, beam_width=15, alpha=0.1,
                 decoding_len=35, beta=0.2, stop_token_index=13) -> List[int]:
    """magic_search (gpt2_prefix_eval.py:341-393) with PlugAndPlayContrastiveDecodingOneStepFast
    (396-469): ``decoding_len - prefix_len`` steps, per step top-``beam_width`` candidates by
    logit, softmax PROBABILITIES (not log), one KV-cached candidate forward, argmax of the
    ranking score; stops after emitting ``stop_token_index``.  Returns the generated ids."""
    wte = sd["gpt.transformer.wte.weight"]
    prefix_len = embed.shape[1]
    ids: List[int] = []
    with torch.no_grad():
        last_hidden, past = gpt2_hidden(embed, sd)
        logit = last_hidden[:, -1, :] @ wte.t()
        for _ in range(decoding_len - prefix_len):
            bsz, seqlen, _ = last_hidden.shape
            probs = F.softmax(logit, dim=-1)
            _, top_k_ids = torch.topk(logit, dim=-1, k=beam_width)
            top_k_probs = torch.gather(probs, 1, top_k_ids)
            nxt = wte[top_k_ids.view(-1)].view(-1, 1, D)
            next_hidden, cand_past = gpt2_hidden(nxt, sd, _expand(past, beam_width), pos0=seqlen)
            logits = next_hidden[:, -1, :] @ wte.t()
            context = last_hidden.repeat_interleave(beam_width, 0)
            toks = [ids + [int(t)] for t in top_k_ids.view(-1)]
            texts = [decode(t) for t in toks]
            clap = clap_log_softmax(audio_embeds, text_encode(texts), temp)
            sel, _ = ranking(context, next_hidden, top_k_probs, alpha, beta, clap, beam_width)
            j = int(sel[0])
            nid = int(top_k_ids[0, j])
            ids.append(nid)
            last_hidden = torch.cat([last_hidden, next_hidden[j:j + 1]], dim=1)
            past = [(k[j:j + 1], v[j:j + 1]) for k, v in cand_past]
            logit = logits[j:j + 1]
            if nid == stop_token_index:
                break
    return ids
