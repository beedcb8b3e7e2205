"""Drop-in for the reference's decoding entry points (gpt2_prefix_eval.py):

    generate2(model, tokenizer, tokens=None, prompt=None, embed=None, entry_count=1,
              entry_length=67, top_p=0.8, temperature=1., stop_token='.') -> str      (161-222)
    generate_beam(model, tokenizer, beam_size=5, prompt=None, embed=None, entry_length=67,
                  temperature=1., stop_token='.') -> list[str]                        (99-158)
    get_prefix_tokens(prefix_embed, embeddings, tokenizer) -> (str,)                  (271-278)

``model`` is a ClapCaption_prompt drop-in (anything whose ``.gpt`` is a
zsaac.modules.ZsGPT2LMHeadModel); ``tokenizer`` is duck-typed (``encode``/``decode``).  Decoding
runs on the MI355X kernels with a KV cache (the reference recomputes the whole sequence every
step; identical math).  For throughput use the batched zsaac.pipeline.CaptionPipeline: these
functions keep the reference's one-clip-per-call signature.

``temperature`` divides the logits as the reference does (``temperature if temperature > 0 else
1.0``, lines 121, 196, 629): in the LM-head kernel's top-k / softmax statistics (zs_lmhead_topk_t,
zs_gpt2_decode_persist) and in the magic ranking score (zs_magic_score_t).

Deviation (documented): a stop token emitted as the very first token returns that
one-token caption (the reference crashes there: ``tokens.squeeze()`` is 0-d, line 218).
"""
from typing import List

import torch
import torch.nn.functional as nnf

from zsaac import ops
from zsaac.modules import require_device

__all__ = ["generate2", "generate_beam", "get_prefix_tokens", "generate_beam_magic", "magic_search",
           "compute_audio_text_similarity_via_embeddings", "compute_audio_text_similarity_via_raw_text"]


def _decoder(model, embed, entry_length, beam):
    require_device(embed, "generate")
    if embed.shape[0] != 1:
        raise ValueError("the reference decodes one clip per call (batch 1); use "
                         "zsaac.pipeline.CaptionPipeline for batches")
    P = embed.shape[1]
    dec = model.gpt.engine(max(beam, 1), P, entry_length, embed.device)
    w = dec.w
    zeros = torch.zeros(1, 1, dtype=torch.int32, device=embed.device)
    hl = torch.zeros(1, dtype=torch.int32, device=embed.device)
    emb = embed.float().contiguous()
    ops.prefill_embed(zeros, hl, emb, P * w.wte.shape[1], P, w.wte, w.wpe, 1, P, None, dec.x,
                      dec.plen, dec.last_row)
    return dec, P


def _temperature(temperature) -> float:
    """The reference's divisor: ``temperature if temperature > 0 else 1.0``."""
    return float(temperature) if temperature > 0 else 1.0


def generate2(model, tokenizer, tokens=None, prompt=None, embed=None, entry_count=1, entry_length=67,
              top_p=0.8, temperature=1., stop_token: str = '.'):
    """Greedy: the top-p filter never removes the highest-probability token, so the pick is the
    argmax (gpt2_prefix_eval.py:194-212); stop after appending ``stop_token`` or 764 (' .').
    Like the reference, the returned text starts with the prompt tokens (``tokens`` or the
    encoded ``prompt``) when no ``embed`` is given (lines 182-184, 209-210, 218)."""
    if embed is None:
        if tokens is None:
            tokens = torch.tensor(tokenizer.encode(prompt)).unsqueeze(0)
        dev = next(model.parameters()).device
        embed = model.gpt.transformer.wte(tokens.to(dev))
    head = [] if tokens is None else [int(t) for t in torch.as_tensor(tokens).reshape(-1).tolist()]
    stop = tokenizer.encode(stop_token)[0]
    dec, P = _decoder(model, embed, entry_length, 1)
    dec.prefill(1, P)
    dec.stop0 = stop
    dec.temperature = _temperature(temperature)
    ids, ln = dec.greedy(1, P)
    out = head + ids[0, :int(ln[0])].tolist()
    return tokenizer.decode(out)


def generate_beam(model, tokenizer, beam_size: int = 5, prompt=None, embed=None, entry_length=67,
                  temperature=1., stop_token: str = '.') -> List[str]:
    """Length-normalised beam search with log(softmax) scores, stopped beams extended by id 0 at
    zero cost; texts sorted by score/length descending (gpt2_prefix_eval.py:99-158).  With a
    ``prompt`` and no ``embed`` each beam's token row starts with the prompt ids and is cut at
    ``seq_length`` (which counts generated tokens only), as the reference does (lines 112-130,
    154-155)."""
    head = []
    if embed is None:
        tokens = torch.tensor(tokenizer.encode(prompt)).unsqueeze(0)
        head = [int(t) for t in tokens.reshape(-1).tolist()]
        dev = next(model.parameters()).device
        embed = model.gpt.transformer.wte(tokens.to(dev))
    stop = tokenizer.encode(stop_token)[0]
    dec, P = _decoder(model, embed, entry_length, beam_size)
    dec.prefill(1, P, row_stride=beam_size)
    dec.stop0 = stop
    dec.temperature = _temperature(temperature)
    ids, ln, sc = dec.beam(1, beam_size, P)
    ids, ln, sc = ids[0].cpu(), ln[0].cpu(), sc[0].cpu()
    texts = [tokenizer.decode((head + ids[i].tolist())[:int(ln[i])]) for i in range(beam_size)]
    order = (sc / ln).argsort(descending=True)
    return [texts[i] for i in order]


def get_prefix_tokens(prefix_embed, embeddings, tokenizer) -> str:
    """argmax_n cos(prefix_embed[0, p], embeddings[n]) per position, decoded token by token and
    joined; returns a 1-tuple like the reference (trailing comma at line 275)."""
    require_device(prefix_embed, "get_prefix_tokens")
    x = prefix_embed[0].float().contiguous()
    M, K = x.shape
    w = embeddings.float().contiguous() if embeddings.dtype != torch.bfloat16 else embeddings.contiguous()
    a = x if w.dtype == torch.float32 else x.to(w.dtype)
    V = w.shape[0]
    nblk = ops.lmhead_nblk(V)
    ps = torch.empty(M, nblk, 2, device=x.device)
    pv = torch.empty(M, nblk, 1, device=x.device)
    pi = torch.empty(M, nblk, 1, device=x.device, dtype=torch.int32)
    ops.lmhead_topk(a, w, 1, ps, pv, pi, row_norm=True)
    idx = torch.empty(M, device=x.device, dtype=torch.int32)
    ops.argmax_finalize(pv, pi, M, nblk, idx)
    prefix_tokens = [tokenizer.decode(int(t)) for t in idx.cpu()]
    prefix_sentence = "".join(prefix_tokens),
    return prefix_sentence


# ------------------------------------------------------------------ CLAP-guided ("magic") decoding
def compute_audio_text_similarity_via_embeddings(clap, audio_embeds, text_embeds):
    """gpt2_prefix_eval.py:536-547: log(softmax(normalize(text) @ normalize(audio)^T / temp)^T)
    -> [1, T] (one audio row, as the reference's ``.t()`` requires)."""
    a = audio_embeds.reshape(1, -1).float()
    a = a / a.norm(dim=-1, keepdim=True)
    t = text_embeds / text_embeds.norm(dim=-1, keepdim=True)
    return (torch.matmul(t, a.t()) / clap.temp).T.softmax(dim=1).log()


def compute_audio_text_similarity_via_raw_text(clap, audio_embeds, text_list):
    """gpt2_prefix_eval.py:549-551 (clap.encode_text on the HIP BERT engine)."""
    return compute_audio_text_similarity_via_embeddings(clap, audio_embeds, clap.encode_text(text_list))


def _magic_engine(model, clap, P, beam, width, steps):
    from zsaac.magic import MagicDecoder
    dev = next(model.parameters()).device
    w = model.gpt.weights(dev)
    bert = clap.text_engine()
    key = (P, beam, width, steps, id(bert))
    cache = w.__dict__.setdefault("_magic", {})
    if key not in cache:
        cache.clear()
        cache[key] = MagicDecoder(w, bert, 1, P + 1, beam=beam, width=width, max_steps=steps)
    return cache[key]


def _magic_inputs(embed, audio_embeds):
    require_device(embed, "magic decoding")
    if embed.shape[0] != 1:
        raise ValueError("the reference decodes one clip per call (batch 1); use "
                         "zsaac.magic.MagicDecoder for batches")
    dev = embed.device
    zeros = torch.zeros(1, 1, dtype=torch.int32, device=dev)
    hl = torch.zeros(1, dtype=torch.int32, device=dev)
    # audio_embeds: [1, 1024] (the reference's .t() at line 543 needs 2-D; predict_prompt.py:140
    # passes the collated [1, 1, 1024] prefix, which the reference itself cannot transpose)
    audio = audio_embeds.reshape(1, -1).float().to(dev).contiguous()
    return zeros, hl, embed.float().contiguous(), audio


def generate_beam_magic(model, clap, tokenizer, audio_embeds, beam_size: int = 5, prompt=None,
                        embed=None, entry_length=20, temperature=1., stop_token: str = '.',
                        magic_width=25, alpha=0.1, beta=0.2) -> List[str]:
    """CLAP-guided beam search (gpt2_prefix_eval.py:602-689): per step the top ``magic_width``
    tokens of every beam are scored by (1-alpha) log p - alpha max-cos(context) + beta CLAP
    log-softmax of the candidate text, then length-normalised beam selection; texts sorted best
    first.  ``embed`` is required (with only a ``prompt`` the reference feeds the prompt ids into
    the candidate texts and token rows, a path its own callers never take)."""
    if embed is None:
        raise NotImplementedError("generate_beam_magic needs embed= (predict_prompt.py:140)")
    stop = tokenizer.encode(stop_token)[0]
    hard, hl, soft, audio = _magic_inputs(embed, audio_embeds)
    P = soft.shape[1]
    eng = _magic_engine(model, clap, P, beam_size, magic_width, entry_length)
    (toks, _), = eng.beam_magic(hard, hl, soft, P, audio, tokenizer, clap.text_encoder.tokenizer,
                                beam_size, magic_width, entry_length, alpha, beta,
                                float(clap.temp), stop, temperature=_temperature(temperature))
    return [tokenizer.decode(t) for t in toks]


def magic_search(model, tokenizer, audio_embeds, clap, input_ids=None, prompt=None, embed=None,
                 beam_width=15, alpha=0.1, decoding_len=35, beta=0.2, clip_text_max_len=60,
                 stop_token='.') -> str:
    """CLAP-guided greedy decoding (gpt2_prefix_eval.py:341-393 + 396-469): ``decoding_len -
    prefix_len`` steps, each picking the argmax of (1-alpha) p - alpha max-cos + beta CLAP score
    over the top ``beam_width`` tokens; stops after emitting ``stop_token``; returns the decoded
    generated ids.  ``embed`` is required (the reference's prompt path raises NameError at 349)."""
    if embed is None:
        raise NotImplementedError("magic_search needs embed= (the reference's prompt path "
                                  "references an unbound name, gpt2_prefix_eval.py:349)")
    stop = tokenizer.encode(stop_token)[0]
    hard, hl, soft, audio = _magic_inputs(embed, audio_embeds)
    P = soft.shape[1]
    steps = max(decoding_len - P, 1)
    eng = _magic_engine(model, clap, P, 1, beam_width, steps)
    ids, = eng.search(hard, hl, soft, P, audio, tokenizer, clap.text_encoder.tokenizer,
                      beam_width, decoding_len, alpha, beta, float(clap.temp), stop)
    return tokenizer.decode(ids)
