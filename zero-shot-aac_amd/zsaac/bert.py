"""CLAP text tower on the HIP kernels: ``ASE.encode_text`` (retrieval/models/ase_model.py:57-60)
over HF ``BertModel(add_pooling_layer=False)`` (retrieval/models/text_encoder.py:43-68).

The reference's magic decoding calls it once per decode step with every candidate continuation
as text (gpt2_prefix_eval.py:442-445, 583-586).  Batched here over all candidates of all clips:

  tokenised texts [T, L] (host, the reference's tokenizer call) -> zs_bert_embed_ln ->
  per layer (post-LN, eps 1e-12):  qkv GEMM (q|k|v packed [2304, 768]) -> zs_row_attention
  (bidirectional, keys masked past each text's length) -> out-proj GEMM + residual ->
  zs_layernorm_dual -> FFN GEMM + GELU(erf) -> GEMM + residual -> zs_layernorm_dual
  -> CLS rows -> text_proj (GEMM + ReLU, GEMM) -> L2 normalise   => [T, 1024] f32

Only the CLS row of the last layer is used (``text_feats[:, 0, :]``), so the last layer runs its
attention over every row (the keys) but the out-projection, both LayerNorms and the FFN on the T
CLS rows only.  bf16 operands with f32 accumulation and an f32 residual stream (perf mode) or f32
throughout (parity mode)."""
from __future__ import annotations

import weakref
from typing import Dict, Optional

import torch

from . import ops

D, FF, HEADS, HD = 768, 3072, 12, 64


def _w(t, dev, dtype):
    return t.detach().to(device=dev, dtype=dtype).contiguous()


def _f(t, dev):
    return t.detach().to(device=dev, dtype=torch.float32).contiguous()


class BertTextEngine:
    """Packed BERT + text_proj weights and workspaces for up to ``max_texts`` texts of up to
    ``max_len`` tokens (the reference truncates at 30)."""

    def __init__(self, sd: Dict[str, torch.Tensor], device, dtype=torch.bfloat16,
                 max_texts: int = 256, max_len: int = 30,
                 prefix: str = "text_encoder.text_encoder.", proj_prefix: str = "text_proj."):
        dev = torch.device(device)
        self.dev, self.dtype = dev, dtype
        e = prefix + "embeddings."
        self.word = _f(sd[e + "word_embeddings.weight"], dev)
        self.pos = _f(sd[e + "position_embeddings.weight"], dev)
        self.type0 = _f(sd[e + "token_type_embeddings.weight"][0], dev)
        self.eln = (_f(sd[e + "LayerNorm.weight"], dev), _f(sd[e + "LayerNorm.bias"], dev))
        self.layers = []
        i = 0
        while f"{prefix}encoder.layer.{i}.attention.self.query.weight" in sd:
            p = f"{prefix}encoder.layer.{i}."
            g = lambda n: sd[p + n]
            self.layers.append({
                "qkv_w": _w(torch.cat([g(f"attention.self.{n}.weight") for n in ("query", "key", "value")]), dev, dtype),
                "qkv_b": _f(torch.cat([g(f"attention.self.{n}.bias") for n in ("query", "key", "value")]), dev),
                "o_w": _w(g("attention.output.dense.weight"), dev, dtype),
                "o_b": _f(g("attention.output.dense.bias"), dev),
                "ln1": (_f(g("attention.output.LayerNorm.weight"), dev), _f(g("attention.output.LayerNorm.bias"), dev)),
                "i_w": _w(g("intermediate.dense.weight"), dev, dtype),
                "i_b": _f(g("intermediate.dense.bias"), dev),
                "f_w": _w(g("output.dense.weight"), dev, dtype),
                "f_b": _f(g("output.dense.bias"), dev),
                "ln2": (_f(g("output.LayerNorm.weight"), dev), _f(g("output.LayerNorm.bias"), dev)),
            })
            i += 1
        if not self.layers:
            raise KeyError(f"no BERT layers under {prefix!r}")
        if proj_prefix + "0.weight" not in sd:
            raise KeyError(f"{proj_prefix}0.weight: the text tower needs ASE's text_proj")
        self.p0 = (_w(sd[proj_prefix + "0.weight"], dev, dtype), _f(sd[proj_prefix + "0.bias"], dev))
        self.p2 = (_w(sd[proj_prefix + "2.weight"], dev, dtype), _f(sd[proj_prefix + "2.bias"], dev))
        self.E = self.p2[0].shape[0]
        self.temp = float(sd["temp"]) if "temp" in sd else None
        self.max_texts, self.max_len = max_texts, max_len
        self._alloc(max_texts, max_len)

    def _alloc(self, T, L):
        dev, dt = self.dev, self.dtype
        M = T * L
        self.x = torch.empty(M, D, device=dev)
        self.y = torch.empty(M, D, device=dev)
        self.h = torch.empty(M, D, device=dev, dtype=dt) if dt != torch.float32 else None
        self.qkv = torch.empty(M, 3 * D, device=dev, dtype=dt)
        self.att = torch.empty(M, D, device=dev, dtype=dt)
        self.ff = torch.empty(M, FF, device=dev, dtype=dt)
        self.cls_x = torch.empty(T, D, device=dev)
        self.cls_y = torch.empty(T, D, device=dev)
        self.cls_h = torch.empty(T, D, device=dev, dtype=dt) if dt != torch.float32 else None
        self.p_h = torch.empty(T, self.p0[0].shape[0], device=dev, dtype=dt)
        self.out = torch.empty(T, self.E, device=dev)
        self.cap = (T, L)

    def _op(self, x32, h):
        return x32 if h is None else h

    def hidden(self, ids: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
        """BertModel(...)[0]: the last hidden state [T, L, 768] f32 (every row)."""
        return self.encode_ids(ids, lens, full=True)

    def encode_ids(self, ids: torch.Tensor, lens: torch.Tensor, full: bool = False) -> torch.Tensor:
        """ids [T, L] int32 (device, [PAD]-padded), lens [T] int32 -> normalised text embeddings
        [T, E] f32 (a view of an engine buffer, valid until the next call); ``full``: the last
        hidden state of every row instead (:meth:`hidden`)."""
        T, L = ids.shape
        if T > self.cap[0] or L > self.cap[1]:
            self._alloc(max(T, self.cap[0]), max(L, self.cap[1]))
        M = T * L
        x, y = self.x[:M], self.y[:M]
        h = self.h[:M] if self.h is not None else None
        qkv, att, ff = self.qkv[:M], self.att[:M], self.ff[:M]
        ops.bert_embed_ln(ids.reshape(-1), L, self.word, self.pos, self.type0, *self.eln, x, h)
        a_op = self._op(x, h)
        nl = len(self.layers)
        for li, ly in enumerate(self.layers):
            ops.gemm(a_op, ly["qkv_w"], qkv, bias=ly["qkv_b"], split_k=1)
            ops.row_attention(qkv, 3 * D, qkv[:, D:], qkv[:, 2 * D:], 3 * D, T, L, HEADS, HD, False,
                              1.0 / 8.0, att, D, lens=lens)
            if li + 1 < nl or full:
                ops.gemm(att, ly["o_w"], y, bias=ly["o_b"], residual=x, split_k=1)
                ops.layernorm_dual(y, *ly["ln1"], x, h)
                ops.gemm(a_op, ly["i_w"], ff, bias=ly["i_b"], act=ops.ACT_GELU_ERF, split_k=1)
                ops.gemm(ff, ly["f_w"], y, bias=ly["f_b"], residual=x, split_k=1)
                ops.layernorm_dual(y, *ly["ln2"], x, h)
            else:
                # last layer: only the CLS rows (row t*L of each text) go on
                cx, cy = self.cls_x[:T], self.cls_y[:T]
                ch = self.cls_h[:T] if self.cls_h is not None else None
                a_cls = att.view(T, L * D)[:, :D]
                r_cls = x.view(T, L * D)[:, :D]
                ops.gemm(a_cls, ly["o_w"], cy, bias=ly["o_b"], residual=r_cls, split_k=1)
                ops.layernorm_dual(cy, *ly["ln1"], cx, ch)
                c_op = self._op(cx, ch)
                ffc = ff[:T]
                ops.gemm(c_op, ly["i_w"], ffc, bias=ly["i_b"], act=ops.ACT_GELU_ERF, split_k=1)
                ops.gemm(ffc, ly["f_w"], cy, bias=ly["f_b"], residual=cx, split_k=1)
                ops.layernorm_dual(cy, *ly["ln2"], cx, ch)
        if full:
            return x.view(T, L, D)
        c_op = self._op(self.cls_x[:T], self.cls_h[:T] if self.cls_h is not None else None)
        ph = self.p_h[:T]
        ops.gemm(c_op, self.p0[0], ph, bias=self.p0[1], act=ops.ACT_RELU, split_k=1)
        out = self.out[:T]
        ops.gemm(ph, self.p2[0], out, bias=self.p2[1], split_k=1)
        return ops.l2norm(out, out)

    def encode_texts(self, tokenizer, texts, max_length: Optional[int] = None) -> torch.Tensor:
        """The reference's tokenizer call (text_encoder.py:59-63) + :meth:`encode_ids`."""
        ids, lens = tokenize(tokenizer, texts, max_length or self.max_len, self.dev)
        return self.encode_ids(ids, lens)


# per-tokenizer caches, keyed weakly by the tokenizer object (an id() key could be reused by a
# later tokenizer with another vocabulary)
_BACKENDS = weakref.WeakKeyDictionary()


def _backend(tokenizer, max_length):
    """A private copy of a fast tokenizer's Rust backend configured like the reference's call
    (truncation at max_length, pad to the longest with [PAD]): encode_batch gives the same ids
    as ``tokenizer(..., padding='longest', truncation=True)`` without the Python wrapper's
    per-text overhead (4800 candidate texts per magic step: 0.11 s against 0.36 s)."""
    bk = getattr(tokenizer, "backend_tokenizer", None)
    if bk is None or not getattr(tokenizer, "is_fast", False) or getattr(tokenizer, "padding_side", "right") != "right":
        return None
    per = _BACKENDS.setdefault(tokenizer, {})
    if max_length not in per:
        from tokenizers import Tokenizer
        b = Tokenizer.from_str(bk.to_str())
        b.enable_truncation(max_length)
        b.enable_padding(pad_id=tokenizer.pad_token_id, pad_token=tokenizer.pad_token)
        per[max_length] = b
    return per[max_length]


_RAW = weakref.WeakKeyDictionary()


def _to_dev(t, device):
    if torch.device(device).type == "cpu":
        return t
    return t.pin_memory().to(device, non_blocking=True)


def _raw_backend(tokenizer):
    """The fast tokenizer's Rust backend without truncation / padding (pieces are encoded without
    special tokens and assembled by tokenize_pieces)."""
    bk = getattr(tokenizer, "backend_tokenizer", None)
    if bk is None or not getattr(tokenizer, "is_fast", False) or getattr(tokenizer, "padding_side", "right") != "right":
        return None
    if tokenizer not in _RAW:
        from tokenizers import Tokenizer
        b = Tokenizer.from_str(bk.to_str())
        b.no_truncation()
        b.no_padding()
        _RAW[tokenizer] = (b, {})
    return _RAW[tokenizer]


def tokenize_pieces(tokenizer, pieces, max_length, device):
    """``tokenize`` of the texts ``prefix + rest`` for ``pieces = [(prefix, rest), ...]`` where every
    ``rest`` is empty-prefixed or starts with ' ' (a BERT word boundary: the normalizer and the
    whitespace / punctuation pre-tokenizer never act across it), so the WordPiece ids of the text
    are those of the prefix followed by those of the rest.  The magic decoder's 4800 candidate
    texts per step share one prefix per beam (the text up to the head's last space) and draw
    their rests from a small set ('' + last word + candidate piece), so both are encoded once per
    distinct string (the rests cached across steps) instead of 4800 full texts per step.  Ids
    are [CLS] + (prefix ids + rest ids)[:max_length - 2] + [SEP], padded to the longest with
    [PAD] -- exactly ``tokenizer(texts, padding='longest', truncation=True, max_length=...)``."""
    raw = _raw_backend(tokenizer)
    if raw is None:
        return tokenize(tokenizer, [p + r for p, r in pieces], max_length, device)
    bk, cache = raw
    if len(cache) > 500_000:
        cache.clear()
    pre = {p for p, _ in pieces if p}
    new = list({r for _, r in pieces if r not in cache} | {p for p in pre if p not in cache})
    if new:
        for t, e in zip(new, bk.encode_batch(new, add_special_tokens=False)):
            cache[t] = e.ids
    cls, sep, pad = tokenizer.cls_token_id, tokenizer.sep_token_id, tokenizer.pad_token_id
    body = max_length - 2
    rows = []
    for p, r in pieces:
        t = (cache[p] + cache[r]) if p else cache[r]
        rows.append([cls] + t[:body] + [sep])
    L = max(len(x) for x in rows)
    lens = torch.tensor([len(x) for x in rows], dtype=torch.int32)
    ids = torch.tensor([x + [pad] * (L - len(x)) for x in rows], dtype=torch.int32)
    return _to_dev(ids, device), _to_dev(lens, device)


def tokenize(tokenizer, texts, max_length, device):
    """``tokenizer(texts, padding='longest', truncation=True, max_length=30)`` on the host ->
    device ids [T, L] int32 and lengths [T] int32 (the attention mask as lengths: BERT's
    tokenizer right-pads, so the mask is a prefix of ones)."""
    bk = _backend(tokenizer, max_length)
    if bk is not None:
        enc = bk.encode_batch(list(texts))
        ids = torch.tensor([e.ids for e in enc], dtype=torch.int32)
        lens = torch.tensor([sum(e.attention_mask) for e in enc], dtype=torch.int32)
    else:
        t = tokenizer(list(texts), padding="longest", truncation=True, max_length=max_length,
                      return_tensors="pt")
        ids = t["input_ids"].to(torch.int32)
        lens = t["attention_mask"].sum(1).to(torch.int32)
    return _to_dev(ids, device), _to_dev(lens, device)
