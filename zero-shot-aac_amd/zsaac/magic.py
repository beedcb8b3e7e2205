"""CLAP-guided ("magic") decoding on the HIP kernels, batched over clips.

Reference (/root/reference/gpt2_prefix_eval.py): ``generate_beam_magic`` 602-689 with
``ComputeMagicScore`` 553-599 (beam search whose per-step candidate score mixes the GPT-2
log-probability, a degeneration penalty -- the max cosine between the candidate's hidden state and
the context's -- and the CLAP audio-text similarity of the candidate continuation), and
``magic_search`` 341-393 with ``PlugAndPlayContrastiveDecodingOneStepFast`` 396-469 (the same
score with probabilities, one hypothesis, argmax).  Driven from predict_prompt.py:121-140
(``--magic``: beam 3, CLAP ``ASE`` loaded from the HTSAT-BERT checkpoint).

One decode step for C clips x b beams x W candidates (R = C*b*W candidate rows):

  logits [C*b, V] (LM head GEMM of each beam's last ln_f row)
  -> zs_row_topk: W candidates + log-softmax (beam) / softmax (search) values
  -> zs_magic_expand: each candidate row inherits its beam's KV history (kvrow indices)
  -> GPT-2 decode forward of the R candidate tokens (KV cache, kvrow indirection) -> ln_f rows
  -> zs_magic_maxcos: degeneration penalty against the beam's context hidden states
  -> host: candidate texts (tokenizer.decode of tokens so far + candidate), BERT tokenisation
  -> BertTextEngine: CLAP text embeddings of the R texts
  -> zs_magic_score: log-softmax of the CLAP similarities per clip, the ranking score
  -> zs_magic_step: beam / argmax selection, histories re-pointed, next LM-head rows gathered

The reference recomputes GPT-2 over the whole sequence every step (generate_beam_magic 627 ->
ComputeMagicScore 554); the KV cache computes the same attention over the same keys.  Text
generation for BERT stays on the host exactly as the reference does it (its tokenizer call).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from . import ops
from .bert import BertTextEngine, tokenize_pieces
from .decoder import D, Gpt2Decoder, Gpt2Weights


class MagicDecoder:
    """Magic decoding for up to ``max_clips`` clips with prompts up to ``max_prompt`` rows."""

    def __init__(self, gpt: Gpt2Weights, bert: BertTextEngine, max_clips: int, max_prompt: int,
                 beam: int = 5, width: int = 25, max_steps: int = 20, text_max_len: int = 30):
        if not (1 <= beam <= 8 and beam <= width <= 64):
            raise ValueError("magic decoding: 1 <= beam <= 8, beam <= width <= 64")
        self.gpt, self.bert = gpt, bert
        self.C, self.b, self.W = max_clips, beam, width
        self.max_steps = max_steps
        self.text_max_len = text_max_len
        R = max_clips * beam * width
        self.R = R
        self.dec = Gpt2Decoder(gpt, R, max_prompt, max_steps, max_prefill_rows=max_clips,
                               use_graph=False, compact=False)
        dev, dt = gpt.wte.device, gpt.dtype
        self.dev, self.dtype = dev, dt
        Lmax = self.dec.Lmax
        nb = max_clips * beam
        i32 = dict(device=dev, dtype=torch.int32)
        self.ctx = torch.zeros(R, Lmax, D, device=dev, dtype=dt)
        self.logits = torch.zeros(nb, gpt.V, device=dev)
        self.pval = torch.empty(nb, width, device=dev)
        self.kvrow = torch.zeros(nb, Lmax, **i32)
        self.kvrow_c = torch.zeros(R, Lmax, **i32)
        self.pos = torch.zeros(nb, **i32)
        self.maxcos = torch.empty(R, device=dev)
        self.score = torch.empty(R, device=dev)
        self.scores = torch.zeros(nb, device=dev)
        self.seq_len = torch.ones(nb, device=dev)
        self.stopped = torch.zeros(nb, **i32)
        self.tokens = torch.zeros(nb, max(max_steps, 1), **i32)
        self.cdone = torch.zeros(max_clips, **i32)
        self.ntok = torch.zeros(max_clips, **i32)
        self.step_limit = torch.zeros(max_clips, **i32)
        self.sel_h = torch.empty(nb, D, device=dev, dtype=dt)
        self.ws = ops.skinny_workspace(dev, [(nb, gpt.V, D)])

    # ------------------------------------------------------------------ prefill
    def _prefill(self, hard_ids, hard_len, soft, n_soft, C, b, W, soft_ld=None):
        """Prompt rows (clap_to_gpt: wte(hard) ; soft) through GPT-2: KV rows k*b*W, the ln_f
        rows of every prompt position into ctx[k*b*W], the last position's LM-head logits into
        beam row k*b."""
        dec = self.dec
        Pmax = int(hard_ids.shape[1]) + n_soft
        ops.prefill_embed(hard_ids, hard_len, soft, soft_ld or soft.stride(0), n_soft, self.gpt.wte,
                          self.gpt.wpe, C, Pmax, None, dec.x, dec.plen, dec.last_row)
        dec.prefill(C, Pmax, row_stride=b * W)
        M = C * Pmax
        hp = dec.h[:M]
        ops.layernorm(dec.x[:M], *self.gpt.lnf, out=hp)
        Lmax = dec.Lmax
        self.ctx[:C * b * W].view(C, b * W, Lmax, D)[:, 0, :Pmax].copy_(hp.view(C, Pmax, D))
        nb = C * b
        self.logits[:nb].zero_()
        ops.gemm(dec.hf[:C], self.gpt.wte, self.logits[:nb].view(C, b * self.gpt.V)[:, :self.gpt.V],
                 split_k=1)
        return Pmax

    def _init_state(self, C, b, W, steps):
        nb = C * b
        base = (torch.arange(nb, device=self.dev, dtype=torch.int32) // b) * (b * W)
        self.kvrow[:nb].copy_(base[:, None].expand(nb, self.dec.Lmax))
        self.pos[:nb].copy_(self.dec.plen[:C].repeat_interleave(b))
        for t in (self.scores, self.stopped, self.tokens, self.cdone, self.ntok):
            t.zero_()
        self.seq_len.fill_(1.0)
        self.step_limit[:C].copy_(steps)

    # ------------------------------------------------------------------ one step
    def _texts(self, tokenizer, cand_h, tok_h, C, b, W, s):
        """The candidate texts ``tokenizer.decode(tokens so far + candidate)`` (ref
        gpt2_prefix_eval.py:582-586) as (prefix, rest) pieces for tokenize_pieces: the prefix is
        the beam's decoded head up to its last space, when the candidate's text starts with it."""
        out = []
        cand = cand_h.tolist()
        # a tokenizer whose decode is a concatenation of per-id pieces (concat_decode) decodes a
        # candidate text as head text + piece; any other decodes the whole id list each time
        concat = getattr(tokenizer, "concat_decode", False)
        pieces = {}
        for j in range(C * b):
            head = tok_h[j, :s].tolist()
            ht = tokenizer.decode(head) if head else ""
            i = ht.rfind(" ")
            cut = ht[:i + 1] if i > 0 else None
            for w in range(W):
                c = cand[j * W + w]
                if concat:
                    pc = pieces.get(c)
                    if pc is None:
                        pc = pieces[c] = tokenizer.decode([c])
                    t = ht + pc
                else:
                    t = tokenizer.decode(head + [c])
                out.append((t[:i], t[i:]) if cut is not None and t.startswith(cut) else ("", t))
        return out

    def _run(self, C, b, W, mode, tokenizer, text_tokenizer, audio, alpha, beta, temp, stop,
             n_steps, score_temp=1.0):
        dec, nb, R = self.dec, C * b, C * b * W
        cand = dec.next_tok[:R]
        greedy = mode == "search"
        if getattr(self, "_cand_h", None) is None or self._cand_h.numel() < self.R:
            self._cand_h = torch.zeros(self.R, dtype=torch.int32, pin_memory=True)
            self._tok_h = torch.zeros_like(self.tokens, device="cpu").pin_memory()
        for s in range(n_steps):
            ops.row_topk(self.logits[:nb], W, self.pval[:nb], cand.view(nb, W),
                         mode=1 if greedy else 0)
            # candidate ids and histories to the host now; the candidate GPT-2 forward runs
            # while the host builds and tokenises the candidate texts
            self._cand_h[:R].copy_(cand, non_blocking=True)
            self._tok_h[:nb].copy_(self.tokens[:nb], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            ops.magic_expand(self.kvrow, self.pos, nb, W, dec.Lmax, self.kvrow_c, dec.pos)
            dec._decode_forward(R, kvrow=self.kvrow_c[:R])
            hf = dec.hf[:R]
            ops.magic_maxcos(hf, R, W, self.ctx, dec.Lmax, self.kvrow, self.pos, self.maxcos)
            ev.synchronize()
            pieces = self._texts(tokenizer, self._cand_h[:R], self._tok_h[:nb, :s], C, b, W, s)
            ids, lens = tokenize_pieces(text_tokenizer, pieces, self.text_max_len, self.dev)
            text = self.bert.encode_ids(ids, lens)
            nact = 1 if (s == 0 and not greedy) else b
            ops.magic_score(self.pval, self.maxcos, text, audio, C, b, W, nact, temp, alpha, beta,
                            self.score, score_temp=score_temp)
            ops.magic_step(self.score, cand, C, b, W, s == 0, greedy, stop, s, self.step_limit,
                           self.scores, self.seq_len, self.stopped, self.tokens, self.kvrow,
                           self.pos, self.cdone, self.ntok, hf, self.sel_h)
            if bool(self.cdone[:C].all()):
                break
            ops.gemm(self.sel_h[:nb], self.gpt.wte, self.logits[:nb], split_k=1)

    def _check(self, C, b, W, Pmax):
        if C > self.C or b * W > self.b * self.W or b > self.b or W > self.W:
            raise ValueError(f"magic decode: C={C} b={b} W={W} exceeds the engine "
                             f"({self.C}, {self.b}, {self.W})")
        if Pmax > self.dec.Pmax:
            raise ValueError(f"magic decode: prompt {Pmax} > {self.dec.Pmax}")

    # ------------------------------------------------------------------ entry points
    def beam_magic(self, hard_ids, hard_len, soft, n_soft, audio, tokenizer, text_tokenizer,
                   beam: int, width: int, entry_length: int, alpha: float = 0.1,
                   beta: float = 0.2, temp: Optional[float] = None, stop: int = 13,
                   soft_ld: Optional[int] = None,
                   temperature: float = 1.0) -> List[Tuple[List[List[int]], List[float]]]:
        """generate_beam_magic for every clip: per clip (token lists best-first, scores/len).
        hard_ids [C, H] int32 / hard_len [C] / soft [C, n_soft, 768] f32 (clap_to_gpt's rows),
        audio [C, 1024] f32 (the CLAP audio embeddings).  ``temp`` is CLAP's logit temperature,
        ``temperature`` generate_beam_magic's (divides the ranking scores, line 629)."""
        C = int(hard_len.shape[0])
        self._check(C, beam, width, int(hard_ids.shape[1]) + n_soft)
        if entry_length > self.max_steps:
            raise ValueError(f"entry_length {entry_length} > engine max_steps {self.max_steps}")
        temp = self.bert.temp if temp is None else temp
        self._prefill(hard_ids, hard_len, soft, n_soft, C, beam, width, soft_ld)
        self._init_state(C, beam, width, torch.full((C,), entry_length, dtype=torch.int32))
        self._run(C, beam, width, "beam", tokenizer, text_tokenizer, audio.float().contiguous(),
                  alpha, beta, temp, stop, entry_length,
                  score_temp=temperature if temperature > 0 else 1.0)
        toks = self.tokens[:C * beam].cpu().view(C, beam, -1)
        ln = self.seq_len[:C * beam].cpu().view(C, beam)
        sc = (self.scores[:C * beam].cpu() / self.seq_len[:C * beam].cpu()).view(C, beam)
        out = []
        for k in range(C):
            order = sc[k].argsort(descending=True)
            out.append(([toks[k, i, :int(ln[k, i])].tolist() for i in order],
                        [float(sc[k, i]) for i in order]))
        return out

    def search(self, hard_ids, hard_len, soft, n_soft, audio, tokenizer, text_tokenizer,
               width: int = 15, decoding_len: int = 35, alpha: float = 0.1, beta: float = 0.2,
               temp: Optional[float] = None, stop: int = 13) -> List[List[int]]:
        """magic_search for every clip: the generated ids (``decoding_len - prompt length``
        steps at most, stop included)."""
        C = int(hard_len.shape[0])
        Pmax = int(hard_ids.shape[1]) + n_soft
        self._check(C, 1, width, Pmax)
        temp = self.bert.temp if temp is None else temp
        plen = (hard_len.cpu().to(torch.int32) + n_soft)
        steps = (decoding_len - plen).clamp(min=0)
        n = int(steps.max())
        if n > self.max_steps:
            raise ValueError(f"decoding_len - prompt = {n} > engine max_steps {self.max_steps}")
        self._prefill(hard_ids, hard_len, soft, n_soft, C, 1, width)
        self._init_state(C, 1, width, steps)
        if n > 0:
            self._run(C, 1, width, "search", tokenizer, text_tokenizer,
                      audio.float().contiguous(), alpha, beta, temp, stop, n)
        toks, nt = self.tokens[:C].cpu(), self.ntok[:C].cpu()
        return [toks[k, :int(nt[k])].tolist() for k in range(C)]
