"""Deterministic, seeded random-init state dicts at the reference's exact shapes and key names.

No checkpoint (GPT-2, CLAP/HTSAT, CNN14, mapper) is available offline, so every parity test,
the bench and the golden fixtures use weights from these generators.  The keys are the ones the
reference's modules produce, so the same dicts load into the reference classes (golden
generation, tests/golden/make_goldens.py) and into this package's loaders:

* GPT-2 small: HF ``GPT2LMHeadModel(GPT2Config())`` keys, prefixed ``gpt.`` under
  ``ClapCaption_prompt`` (reference models/caption_model.py:52).
* MLP mapper ``clap_project.model.{0,2}``  (models/mapper.py:6-18, caption_model.py:55-57).
* TransformerMapper ``clap_project.{linear,prefix_const,transformer.layers.*}`` (mapper.py:125-139).
* HTSAT ``audio_encoder.audio_enc.*`` (retrieval/models/htsat.py:588-758, args audio_encoder.py:41-51).
* CNN14 ``audio_encoder.audio_enc.*`` (retrieval/models/cnns.py:137-201).
* ASE ``audio_proj.{0,2}`` (retrieval/models/ase_model.py:34-38).

Values are drawn from one ``torch.Generator`` in a fixed key order, so a (seed, spec) pair
always reproduces the same tensors on any host with the same torch build.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch

GPT2_VOCAB = 50257
GPT2_NPOS = 1024
GPT2_D = 768
GPT2_LAYERS = 12
GPT2_HEADS = 12

HTSAT_DEPTHS = (2, 2, 6, 2)
HTSAT_HEADS = (4, 8, 16, 32)
HTSAT_EMBED = 96
HTSAT_WINDOW = 8
HTSAT_CLASSES = 527
N_MELS = 64

CNN14_CH = (64, 128, 256, 512, 1024, 2048)


def _gen(seed: int) -> torch.Generator:
    g = torch.Generator()
    g.manual_seed(int(seed))
    return g


def _randn(g, shape, std):
    return torch.randn(*shape, generator=g, dtype=torch.float32) * std


def _ln(sd, g, name, dim, wstd=0.1, bstd=0.05):
    sd[name + ".weight"] = 1.0 + _randn(g, (dim,), wstd)
    sd[name + ".bias"] = _randn(g, (dim,), bstd)


def _linear(sd, g, name, out_f, in_f, bias=True, gain=1.0):
    std = gain / math.sqrt(in_f)
    sd[name + ".weight"] = _randn(g, (out_f, in_f), std)
    if bias:
        sd[name + ".bias"] = _randn(g, (out_f,), 0.02)


def _bn(sd, g, name, dim):
    sd[name + ".weight"] = 1.0 + _randn(g, (dim,), 0.1)
    sd[name + ".bias"] = _randn(g, (dim,), 0.1)
    sd[name + ".running_mean"] = _randn(g, (dim,), 0.5)
    sd[name + ".running_var"] = 0.5 + torch.rand(dim, generator=g)
    sd[name + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.int64)


# ----------------------------------------------------------------------------------- GPT-2

def gpt2_state_dict(seed: int = 0, std: float = 0.02, emb_std: float = None,
                    stop_boost: float = 1.0, prefix: str = "gpt.") -> "OrderedDict[str, torch.Tensor]":
    """GPT-2 small (124,439,808 params, tied LM head).

    ``std`` scales every Conv1D weight (HF init uses 0.02; the golden fixtures use a larger value
    so greedy argmax margins are non-degenerate, SURVEY.md §7 "No weights").  ``stop_boost``
    scales rows 13 ('.') and 764 (' .') of ``wte`` so that stop tokens actually fire in some
    fixtures.  Conv1D layout [in, out] as HF stores it (y = x @ W + b).
    """
    g = _gen(seed)
    emb_std = std if emb_std is None else emb_std
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    p = prefix + "transformer."
    wte = _randn(g, (GPT2_VOCAB, GPT2_D), emb_std)
    if stop_boost != 1.0:
        wte[13] *= stop_boost
        wte[764] *= stop_boost
    sd[p + "wte.weight"] = wte
    sd[p + "wpe.weight"] = _randn(g, (GPT2_NPOS, GPT2_D), emb_std * 0.5)
    for i in range(GPT2_LAYERS):
        h = p + f"h.{i}."
        _ln(sd, g, h + "ln_1", GPT2_D)
        sd[h + "attn.c_attn.weight"] = _randn(g, (GPT2_D, 3 * GPT2_D), std)
        sd[h + "attn.c_attn.bias"] = _randn(g, (3 * GPT2_D,), 0.02)
        sd[h + "attn.c_proj.weight"] = _randn(g, (GPT2_D, GPT2_D), std / math.sqrt(2 * GPT2_LAYERS))
        sd[h + "attn.c_proj.bias"] = _randn(g, (GPT2_D,), 0.02)
        _ln(sd, g, h + "ln_2", GPT2_D)
        sd[h + "mlp.c_fc.weight"] = _randn(g, (GPT2_D, 4 * GPT2_D), std)
        sd[h + "mlp.c_fc.bias"] = _randn(g, (4 * GPT2_D,), 0.02)
        sd[h + "mlp.c_proj.weight"] = _randn(g, (4 * GPT2_D, GPT2_D), std / math.sqrt(2 * GPT2_LAYERS))
        sd[h + "mlp.c_proj.bias"] = _randn(g, (GPT2_D,), 0.02)
    _ln(sd, g, p + "ln_f", GPT2_D)
    sd[prefix + "lm_head.weight"] = sd[p + "wte.weight"]  # tied (HF ties lm_head to wte)
    return sd


# ----------------------------------------------------------------------------------- mappers

def mlp_mapper_state_dict(seed: int = 1, prefix_size: int = 1024, prefix_length: int = 10,
                          d: int = GPT2_D, gain: float = 1.0, prefix: str = "clap_project.model."):
    """``MLP((prefix_size, d*L//2, d*L))`` with Tanh (models/mapper.py:6-18)."""
    g = _gen(seed)
    sd = OrderedDict()
    hid = (d * prefix_length) // 2
    _linear(sd, g, prefix + "0", hid, prefix_size, gain=gain)
    _linear(sd, g, prefix + "2", d * prefix_length, hid, gain=gain)
    return sd


def sound_effect_mlp_state_dict(seed: int = 11, prefix_size: int = 1024, d: int = GPT2_D,
                                prefix: str = "sound_effect_project.model."):
    """ClapCaptionModel's ``sound_effect_project = MLP((prefix_size, d // 2, d))`` with Tanh
    (models/caption_model.py:63-64)."""
    g = _gen(seed)
    sd = OrderedDict()
    _linear(sd, g, prefix + "0", d // 2, prefix_size)
    _linear(sd, g, prefix + "2", d, d // 2)
    return sd


def sound_effect_mha_state_dict(seed: int = 12, embed_dim: int = 1024,
                                prefix: str = "sound_effect_project."):
    """ClapCaptionCrossattention[_v2]'s ``nn.MultiheadAttention(prefix_size, 4, batch_first=True)``
    (models/caption_model.py:109, 160): in_proj_weight / in_proj_bias / out_proj."""
    g = _gen(seed)
    sd = OrderedDict()
    sd[prefix + "in_proj_weight"] = _randn(g, (3 * embed_dim, embed_dim), 1.0 / math.sqrt(embed_dim))
    sd[prefix + "in_proj_bias"] = _randn(g, (3 * embed_dim,), 0.02)
    _linear(sd, g, prefix + "out_proj", embed_dim, embed_dim)
    return sd


def transformer_mapper_state_dict(seed: int = 2, prefix_size: int = 1024, prefix_length: int = 10,
                                  clip_length: int = 10, num_layers: int = 8, d: int = GPT2_D,
                                  prefix: str = "clap_project."):
    """``TransformerMapper`` (models/mapper.py:125-139): 8 pre-LN layers, 8 heads, mlp_ratio 2,
    q/kv projections without bias (TransformerLayer bias=False default, mapper.py:83)."""
    g = _gen(seed)
    sd = OrderedDict()
    _linear(sd, g, prefix + "linear", clip_length * d, prefix_size)
    sd[prefix + "prefix_const"] = _randn(g, (prefix_length, d), 1.0)
    for i in range(num_layers):
        L = prefix + f"transformer.layers.{i}."
        _ln(sd, g, L + "norm1", d)
        _linear(sd, g, L + "attn.to_queries", d, d, bias=False)
        _linear(sd, g, L + "attn.to_keys_values", 2 * d, d, bias=False)
        _linear(sd, g, L + "attn.project", d, d)
        _ln(sd, g, L + "norm2", d)
        _linear(sd, g, L + "mlp.fc1", 2 * d, d)
        _linear(sd, g, L + "mlp.fc2", d, 2 * d)
    return sd


# ----------------------------------------------------------------------------------- audio

def htsat_state_dict(seed: int = 3, prefix: str = "audio_encoder.audio_enc.", gain: float = 1.0):
    """HTSAT-Swin (retrieval/models/htsat.py:588-758) with the CLAP args of audio_encoder.py:41-51.

    Only parameters (and BN running stats) are generated; the fixed buffers
    (relative_position_index, attn_mask, torchlibrosa STFT/mel matrices) are not weights and are
    rebuilt by each side.  The dead tscam_conv/head params are included so the dict is a full
    checkpoint for the reference class.
    """
    g = _gen(seed)
    sd = OrderedDict()
    _bn(sd, g, prefix + "bn0", N_MELS)
    sd[prefix + "patch_embed.proj.weight"] = _randn(g, (HTSAT_EMBED, 1, 4, 4), gain / 4.0)
    sd[prefix + "patch_embed.proj.bias"] = _randn(g, (HTSAT_EMBED,), 0.02)
    _ln(sd, g, prefix + "patch_embed.norm", HTSAT_EMBED)
    for i, (depth, heads) in enumerate(zip(HTSAT_DEPTHS, HTSAT_HEADS)):
        dim = HTSAT_EMBED * 2 ** i
        for j in range(depth):
            b = prefix + f"layers.{i}.blocks.{j}."
            _ln(sd, g, b + "norm1", dim)
            sd[b + "attn.relative_position_bias_table"] = _randn(
                g, ((2 * HTSAT_WINDOW - 1) ** 2, heads), 0.5)
            _linear(sd, g, b + "attn.qkv", 3 * dim, dim, gain=gain)
            _linear(sd, g, b + "attn.proj", dim, dim, gain=gain * 0.5)
            _ln(sd, g, b + "norm2", dim)
            _linear(sd, g, b + "mlp.fc1", 4 * dim, dim, gain=gain)
            _linear(sd, g, b + "mlp.fc2", dim, 4 * dim, gain=gain * 0.5)
        if i < len(HTSAT_DEPTHS) - 1:
            d = prefix + f"layers.{i}.downsample."
            sd[d + "reduction.weight"] = _randn(g, (2 * dim, 4 * dim), gain / math.sqrt(4 * dim))
            _ln(sd, g, d + "norm", 4 * dim)
    nf = HTSAT_EMBED * 2 ** (len(HTSAT_DEPTHS) - 1)
    _ln(sd, g, prefix + "norm", nf)
    sd[prefix + "tscam_conv.weight"] = _randn(g, (HTSAT_CLASSES, nf, 2, 3), 0.01)
    sd[prefix + "tscam_conv.bias"] = _randn(g, (HTSAT_CLASSES,), 0.01)
    _linear(sd, g, prefix + "head", HTSAT_CLASSES, HTSAT_CLASSES)
    return sd


def cnn14_state_dict(seed: int = 4, prefix: str = "audio_encoder.audio_enc."):
    """CNN14 (retrieval/models/cnns.py:137-201): bn0 + 6 ConvBlocks (conv3x3 no-bias, BN, ReLU)."""
    g = _gen(seed)
    sd = OrderedDict()
    _bn(sd, g, prefix + "bn0", N_MELS)
    cin = 1
    for i, cout in enumerate(CNN14_CH, start=1):
        b = prefix + f"conv_block{i}."
        sd[b + "conv1.weight"] = _randn(g, (cout, cin, 3, 3), math.sqrt(2.0 / (cin * 9)))
        sd[b + "conv2.weight"] = _randn(g, (cout, cout, 3, 3), math.sqrt(2.0 / (cout * 9)))
        _bn(sd, g, b + "bn1", cout)
        _bn(sd, g, b + "bn2", cout)
        cin = cout
    return sd


def audio_proj_state_dict(seed: int = 5, audio_width: int = 768, embed_size: int = 1024,
                          prefix: str = "audio_proj."):
    """ASE.audio_proj = Linear(w, 1024) -> ReLU -> Linear(1024, 1024) (ase_model.py:34-38)."""
    g = _gen(seed)
    sd = OrderedDict()
    _linear(sd, g, prefix + "0", embed_size, audio_width)
    _linear(sd, g, prefix + "2", embed_size, embed_size)
    return sd


def label_table(seed: int = 6, n_labels: int = 527, dim: int = 1024) -> torch.Tensor:
    """Synthetic stand-in for ``audioset_label.pkl``'s 527 CLAP label-text embeddings (unit rows)."""
    g = _gen(seed)
    t = torch.randn(n_labels, dim, generator=g)
    return t / t.norm(dim=-1, keepdim=True)


def label_token_table(seed: int = 7, n_labels: int = 527, max_len: int = 3,
                      vocab: int = GPT2_VOCAB) -> List[List[int]]:
    """Synthetic stand-in for ``GPT2Tokenizer.encode(' ' + label.lower())`` of every AudioSet
    label (1..max_len BPE ids each).  Ids avoid the stop tokens 13/764 and ',' (11)."""
    g = _gen(seed)
    out = []
    for _ in range(n_labels):
        n = int(torch.randint(1, max_len + 1, (1,), generator=g))
        ids = []
        while len(ids) < n:
            t = int(torch.randint(256, vocab, (1,), generator=g))
            if t not in (11, 13, 764):
                ids.append(t)
        out.append(ids)
    return out


def synthetic_waveforms(n: int, seed: int = 1234, length: int = 320000) -> torch.Tensor:
    """randn(N, 320000)*0.1 clipped to [-1, 1], seed 1234."""
    g = _gen(seed)
    return (torch.randn(n, length, generator=g) * 0.1).clamp_(-1.0, 1.0)


def synthetic_clap_embeddings(n: int, seed: int = 4321, dim: int = 1024) -> torch.Tensor:
    g = _gen(seed)
    e = torch.randn(n, dim, generator=g)
    return e / e.norm(dim=-1, keepdim=True)


def gpt2_vocab(label_names, n_vocab: int = 50257):
    """A GPT-2-format BPE vocabulary (vocab dict, merges list) for offline tests of the real-data
    harness: ids 0..255 are the byte tokens in GPT-2's order (so '.' = 13, ',' = 11 as in GPT-2);
    the prompt template pieces get their real GPT-2 ids ("There" 1858, " are" 389, " something"
    1223, " in" 287, " this" 428, " audio" 6597) and " ." is 764; merges build those pieces and a
    shared " snd" prefix for the synthetic label names; every other id up to n_vocab decodes to a
    filler string, so any generated id decodes."""
    from .bpe import bytes_to_unicode
    b2u = bytes_to_unicode()
    sp = b2u[ord(" ")]
    vocab = {b2u[b]: i for i, b in enumerate(b2u)}      # GPT-2's byte order: bytes_to_unicode's
    merges = []
    fixed = {"There": 1858, sp + "are": 389, sp + "something": 1223, sp + "in": 287,
             sp + "this": 428, sp + "audio": 6597, sp + ".": 764}
    nxt = [256]

    def new_id():
        while nxt[0] in fixed.values():
            nxt[0] += 1
        nxt[0] += 1
        return nxt[0] - 1

    def chain(word):
        cur = word[0]
        for ch in word[1:]:
            merged = cur + ch
            if (cur, ch) not in merges:
                merges.append((cur, ch))
            if merged not in vocab:
                vocab[merged] = fixed.get(merged, new_id())
            cur = merged
    for w in fixed:
        chain(w)
    prefixes = sorted({sp + n.lower()[:3] for n in label_names})
    for p in prefixes:
        chain(p)
    used = set(vocab.values())
    k = 0
    for i in range(n_vocab):
        if i not in used:
            vocab[f"<{k}>"] = i
            k += 1
    return vocab, merges


# ----------------------------------------------------------------------------------- BERT (CLAP text)

BERT_D = 768
BERT_FF = 3072
BERT_HEADS = 12
BERT_NPOS = 512


def bert_vocab() -> List[str]:
    """A small WordPiece vocabulary (the bert-base-uncased vocab file is a name fetch, unavailable
    offline): the special tokens at their BERT positions relative to each other, single
    characters, '##' continuations and a few whole words, so that a WordPiece split of the
    synthetic caption words (:class:`zsaac.tokenizer.WordTokenizer`) exercises greedy
    longest-match-first, [UNK] and truncation."""
    toks = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    chars = [chr(c) for c in range(97, 123)] + [str(d) for d in range(10)]
    toks += [".", ",", "'", "-"] + chars + ["##" + c for c in chars]
    toks += [f"w{i}" for i in range(40)] + [f"##{i}{j}" for i in range(3) for j in range(10)]
    toks += ["there", "are", "in", "this", "audio", "sound", "dog", "bark", "##ing", "##s"]
    return toks


def bert_state_dict(seed: int = 13, vocab: int = None, layers: int = 12,
                    prefix: str = "text_encoder.text_encoder.", proj_prefix: str = "text_proj.",
                    embed_size: int = 1024, temp: float = 0.07):
    """ASE's text tower: HF ``BertModel(add_pooling_layer=False)`` keys under
    ``text_encoder.text_encoder.`` (retrieval/models/text_encoder.py:43-47), ``text_proj.{0,2}``
    and ``temp`` (retrieval/models/ase_model.py:40-46).  bert-base geometry (768 / 12 heads /
    3072), ``layers`` encoder layers (bert-base has 12)."""
    g = _gen(seed)
    vocab = vocab or len(bert_vocab())
    sd = OrderedDict()
    e = prefix + "embeddings."
    sd[e + "word_embeddings.weight"] = _randn(g, (vocab, BERT_D), 0.5)
    sd[e + "position_embeddings.weight"] = _randn(g, (BERT_NPOS, BERT_D), 0.2)
    sd[e + "token_type_embeddings.weight"] = _randn(g, (2, BERT_D), 0.2)
    _ln(sd, g, e + "LayerNorm", BERT_D)
    for i in range(layers):
        L = prefix + f"encoder.layer.{i}."
        for n in ("query", "key", "value"):
            _linear(sd, g, L + f"attention.self.{n}", BERT_D, BERT_D, gain=1.5)
        _linear(sd, g, L + "attention.output.dense", BERT_D, BERT_D)
        _ln(sd, g, L + "attention.output.LayerNorm", BERT_D)
        _linear(sd, g, L + "intermediate.dense", BERT_FF, BERT_D, gain=1.5)
        _linear(sd, g, L + "output.dense", BERT_D, BERT_FF)
        _ln(sd, g, L + "output.LayerNorm", BERT_D)
    _linear(sd, g, proj_prefix + "0", embed_size, BERT_D)
    _linear(sd, g, proj_prefix + "2", embed_size, embed_size)
    sd["temp"] = torch.tensor(float(temp))
    return sd


# ----------------------------------------------------------------------------------- Mistral (C5)

MISTRAL_7B = dict(vocab=32000, hidden=4096, heads=32, kv_heads=8, ffn=14336, layers=32)
MISTRAL_TINY = dict(vocab=32000, hidden=1024, heads=8, kv_heads=2, ffn=3072, layers=2)


def _fp8_exact(w):
    """Round a weight to what per-row fp8 e4m3 (scale amax / 448) represents exactly, so the fp8
    engine and an f32 reference hold the same values."""
    amax = w.abs().amax(dim=1).clamp(min=1e-12)
    s = amax / 448.0
    return (w / s[:, None]).to(torch.float8_e4m3fn).float() * s[:, None]


def mistral_state_dict(seed: int = 21, cfg: dict = None, eos_boost: float = 1.5,
                       fp8_exact: bool = True):
    """MistralForCausalLM keys (``model.embed_tokens``, ``model.layers.*``, ``model.norm``,
    ``lm_head``) at ``cfg`` (default: the tiny test geometry); projection weights rounded to fp8
    values unless ``fp8_exact`` is False; ``eos_boost`` scales lm_head row 2 (eos) so that some
    captions end."""
    c = dict(MISTRAL_TINY if cfg is None else cfg)
    g = _gen(seed)
    D, F, H, KVH, V = c["hidden"], c["ffn"], c["heads"], c["kv_heads"], c["vocab"]
    hd = D // H
    sd = OrderedDict()
    rnd = (lambda o, i, gain=1.0: _fp8_exact(_randn(g, (o, i), gain / math.sqrt(i)))) if fp8_exact \
        else (lambda o, i, gain=1.0: _randn(g, (o, i), gain / math.sqrt(i)))
    sd["model.embed_tokens.weight"] = _randn(g, (V, D), 1.0)
    for i in range(c["layers"]):
        L = f"model.layers.{i}."
        sd[L + "input_layernorm.weight"] = 1.0 + _randn(g, (D,), 0.1)
        sd[L + "self_attn.q_proj.weight"] = rnd(H * hd, D, 2.0)
        sd[L + "self_attn.k_proj.weight"] = rnd(KVH * hd, D, 2.0)
        sd[L + "self_attn.v_proj.weight"] = rnd(KVH * hd, D)
        sd[L + "self_attn.o_proj.weight"] = rnd(D, H * hd)
        sd[L + "post_attention_layernorm.weight"] = 1.0 + _randn(g, (D,), 0.1)
        sd[L + "mlp.gate_proj.weight"] = rnd(F, D, 1.5)
        sd[L + "mlp.up_proj.weight"] = rnd(F, D)
        sd[L + "mlp.down_proj.weight"] = rnd(D, F)
    sd["model.norm.weight"] = 1.0 + _randn(g, (D,), 0.1)
    lm = _randn(g, (V, D), 4.0 / math.sqrt(D))
    lm[2] *= eos_boost
    sd["lm_head.weight"] = lm
    return sd
