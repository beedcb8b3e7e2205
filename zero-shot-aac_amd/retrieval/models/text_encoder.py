"""Drop-in for retrieval/models/text_encoder.py:38-68 ``TextEncoder`` -- the CLAP text tower that
``ASE.encode_text`` runs (and CLAP-guided "magic" decoding calls every step,
gpt2_prefix_eval.py:549-551).

The reference builds ``BertModel.from_pretrained(type, add_pooling_layer=False)`` and its
``BertTokenizer``: name fetches, unavailable offline.  Here the module holds the same parameter
tree (HF BertModel keys, bert-base geometry: hidden 768, 12 heads, FFN 3072; the layer count and
vocabulary size from ``text_encoder_args``, defaulting to bert-base-uncased's 12 / 30522) so a
CLAP checkpoint's ``text_encoder.text_encoder.*`` entries load into it, and the tokenizer comes
from a local vocabulary (``text_encoder_args["vocab"]``: a vocab.txt path or a token->id dict)
or is assigned by the caller (``.tokenizer = ...``).  ``forward`` returns the last hidden state
[T, L, 768] computed by zsaac.bert.BertTextEngine on the HIP kernels.
"""
import torch
import torch.nn as nn

from zsaac.modules import EngineCache, ParamTree, require_device, zs_dtype_of

BERT_FAMILY = {"bert-base-uncased": (30522, 12)}


def bert_spec(vocab: int, layers: int, n_pos: int = 512, d: int = 768, ff: int = 3072):
    """HF BertModel(add_pooling_layer=False) parameter names and shapes (BERT's own init is
    irrelevant here: a checkpoint is loaded over it)."""
    spec = {"embeddings.word_embeddings.weight": torch.zeros(vocab, d),
            "embeddings.position_embeddings.weight": torch.zeros(n_pos, d),
            "embeddings.token_type_embeddings.weight": torch.zeros(2, d),
            "embeddings.LayerNorm.weight": torch.ones(d), "embeddings.LayerNorm.bias": torch.zeros(d)}
    for i in range(layers):
        p = f"encoder.layer.{i}."
        for n in ("query", "key", "value"):
            spec[p + f"attention.self.{n}.weight"] = torch.zeros(d, d)
            spec[p + f"attention.self.{n}.bias"] = torch.zeros(d)
        spec[p + "attention.output.dense.weight"] = torch.zeros(d, d)
        spec[p + "attention.output.dense.bias"] = torch.zeros(d)
        spec[p + "attention.output.LayerNorm.weight"] = torch.ones(d)
        spec[p + "attention.output.LayerNorm.bias"] = torch.zeros(d)
        spec[p + "intermediate.dense.weight"] = torch.zeros(ff, d)
        spec[p + "intermediate.dense.bias"] = torch.zeros(ff)
        spec[p + "output.dense.weight"] = torch.zeros(d, ff)
        spec[p + "output.dense.bias"] = torch.zeros(d)
        spec[p + "output.LayerNorm.weight"] = torch.ones(d)
        spec[p + "output.LayerNorm.bias"] = torch.zeros(d)
    return spec


def _tokenizer(vocab):
    from transformers import BertTokenizer
    if isinstance(vocab, str):
        with open(vocab, encoding="utf-8") as f:
            vocab = {t.rstrip("\n"): i for i, t in enumerate(f)}
    return BertTokenizer(vocab=dict(vocab), do_lower_case=True)


class TextEncoder(nn.Module):

    def __init__(self, config):
        super().__init__()
        args = config["text_encoder_args"]
        kind = args["type"]
        if kind not in BERT_FAMILY and "vocab_size" not in args:
            raise NotImplementedError(f"text encoder {kind!r}: the BERT-base family only")
        vocab, layers = BERT_FAMILY.get(kind, (None, 12))
        vocab = args.get("vocab_size", vocab)
        layers = args.get("num_layers", layers)
        self.text_encoder = ParamTree(bert_spec(vocab, layers))
        self.tokenizer = _tokenizer(args["vocab"]) if args.get("vocab") is not None else None
        self.text_width = 768
        self._cache = EngineCache()

    @property
    def device(self):
        return list(self.parameters())[0].device

    def engine(self, proj_sd=None):
        """The BertTextEngine of this tower (+ ``proj_sd``: ASE's text_proj / temp entries)."""
        from zsaac.bert import BertTextEngine
        dev, dt = self.device, zs_dtype_of(self)

        def build():
            sd = {"text_encoder." + k: v for k, v in self.text_encoder.state_dict().items()}
            sd.update({k: v.detach() for k, v in (proj_sd or {}).items()})
            return BertTextEngine(sd, dev, dt, prefix="text_encoder.")
        extra = tuple((k, v.data_ptr(), v._version) for k, v in sorted((proj_sd or {}).items()))
        return self._cache.get(self, build, (dt, str(dev), extra))

    def forward(self, text):
        if self.tokenizer is None:
            raise RuntimeError("TextEncoder.tokenizer is not set (bert-base-uncased's vocabulary "
                               "is a name fetch; pass text_encoder_args['vocab'] or assign one)")
        from zsaac.bert import tokenize
        require_device(next(self.parameters()), "TextEncoder.forward")
        if getattr(self, "_id_proj", None) is None or self._id_proj["text_proj.0.weight"].device != self.device:
            self._id_proj = _identity_proj(self.device)
        eng = self.engine(self._id_proj)
        ids, lens = tokenize(self.tokenizer, text, 30, self.device)
        return eng.hidden(ids, lens)


def _identity_proj(dev, d=768):
    return {"text_proj.0.weight": torch.eye(d, device=dev), "text_proj.0.bias": torch.zeros(d, device=dev),
            "text_proj.2.weight": torch.eye(d, device=dev), "text_proj.2.bias": torch.zeros(d, device=dev)}
