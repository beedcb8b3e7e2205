"""Import shims that let THIS container import the read-only reference for golden generation only.

Used solely by tests/golden/make_goldens.py (never by tests at run time, never on the GPU box:
/root/reference does not exist there).  What is shimmed and why:

* ``transformers.AdamW`` was removed in transformers 5.x; gpt2_prefix_eval.py:2 and
  dataset/dataset.py:11 import it -> wrapped module adds ``AdamW = torch.optim.AdamW``.
* ``train`` (gpt2_prefix_eval.py:7) names a module absent from the reference -> stub.
* ``GPT2LMHeadModel.from_pretrained('gpt2')`` (models/caption_model.py:52) is a name fetch that is
  unavailable offline -> returns a locally built ``GPT2LMHeadModel(GPT2Config())`` with eager
  attention, into which the caller loads the seeded synthetic state dict.
* torchlibrosa (front end), ruamel.yaml, wandb, loguru, sentence_transformers, librosa are absent
  -> stubs.  The torchlibrosa stub is an IDENTITY module, so the reference HTSAT/CNN14 forward is
  driven from a log-mel input; the front end itself is third-party arithmetic that stays
  "parity unpinned" (DESIGN.md §Oracle).
"""
from __future__ import annotations

import sys
import types

import torch
import torch.nn as nn

REF = "/root/reference"


class _Any:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return self

    def __getattr__(self, name):
        return _Any()


def _stub(name, **attrs):
    m = types.ModuleType(name)

    def __getattr__(attr):  # noqa: N807
        return _Any
    m.__getattr__ = __getattr__
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _Identity(nn.Module):
    def __init__(self, *a, **k):
        super().__init__()

    def forward(self, x):
        return x


_installed = False


def install():
    global _installed
    if _installed:
        return
    import transformers  # import the real package BEFORE stubbing librosa
    from transformers import GPT2Config, GPT2LMHeadModel

    def _from_pretrained(*a, **k):
        cfg = GPT2Config()
        cfg._attn_implementation = "eager"
        m = GPT2LMHeadModel(cfg)
        return m
    GPT2LMHeadModel.from_pretrained = staticmethod(_from_pretrained)

    _stub("train", ClipCocoDataset=type("ClipCocoDataset", (), {}),
          ClipCaptionModel=type("ClipCaptionModel", (nn.Module,), {}))
    tl = _stub("torchlibrosa", Spectrogram=_Identity, LogmelFilterBank=_Identity)
    _stub("torchlibrosa.augmentation", SpecAugmentation=_Identity)
    tl.augmentation = sys.modules["torchlibrosa.augmentation"]
    import yaml as _yaml
    ry = _stub("ruamel")
    ry.yaml = _yaml
    sys.modules["ruamel.yaml"] = _yaml
    for name in ("wandb", "loguru", "sentence_transformers", "librosa", "stanza", "peft",
                 "bitsandbytes", "deepl", "openai"):
        if name not in sys.modules:
            _stub(name)
    sys.modules["loguru"].logger = _Any()
    sys.modules["sentence_transformers"].util = _Any()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    # lazy module: set the missing names directly on it (``from transformers import AdamW``);
    # done last because resolving other lazy attributes can rebuild the module's namespace
    transformers = sys.modules["transformers"]
    transformers.__dict__["AdamW"] = torch.optim.AdamW
    transformers.__dict__.setdefault("get_linear_schedule_with_warmup", lambda *a, **k: None)
    _installed = True


def install_bert(vocab, layers):
    """``BertModel.from_pretrained`` / ``BertTokenizer.from_pretrained`` ('bert-base-uncased',
    retrieval/models/text_encoder.py:43-47) are name fetches, unavailable offline -> a locally
    built ``BertModel(BertConfig(vocab_size=len(vocab), num_hidden_layers=layers))`` (eager
    attention, bert-base geometry otherwise) and a ``BertTokenizer`` over ``vocab``; the caller
    loads the seeded synthetic state dict into the model."""
    install()
    from transformers import BertConfig, BertModel, BertTokenizer

    def _model(*a, add_pooling_layer=True, **k):
        cfg = BertConfig(vocab_size=len(vocab), num_hidden_layers=layers)
        cfg._attn_implementation = "eager"
        return BertModel(cfg, add_pooling_layer=add_pooling_layer)
    BertModel.from_pretrained = staticmethod(_model)
    BertTokenizer.from_pretrained = staticmethod(
        lambda *a, **k: BertTokenizer(vocab={t: i for i, t in enumerate(vocab)}, do_lower_case=True))


def install_mistral(cfg_kw):
    """ClapCaption_Mistralai_prompt (models/caption_model.py:340-370) loads
    ``MistralForCausalLM.from_pretrained('mistralai/Mistral-7B-v0.1', quantization_config=NF4)``
    (a name fetch, unavailable offline) and wraps it with peft LoRA (absent).  Shims: a locally
    built ``MistralForCausalLM(MistralConfig(**cfg_kw))`` (eager attention) into which the caller
    loads the synthetic weights; ``prepare_model_for_kbit_training`` = identity; ``get_peft_model``
    = a wrapper exposing the ``base_model.model.model.embed_tokens`` path and ``generate`` of the
    real PeftModelForCausalLM without adapters (LoRA with B = 0 at init is the identity)."""
    install()
    from transformers import MistralConfig, MistralForCausalLM

    def _model(*a, **k):
        cfg = MistralConfig(**cfg_kw)
        cfg._attn_implementation = "eager"
        return MistralForCausalLM(cfg)
    MistralForCausalLM.from_pretrained = staticmethod(_model)

    class _Lora(nn.Module):
        def __init__(self, m):
            super().__init__()
            self.model = m

    class _Peft(nn.Module):
        def __init__(self, m):
            super().__init__()
            self.base_model = _Lora(m)

        def generate(self, *a, **k):
            return self.base_model.model.generate(*a, **k)

        def forward(self, *a, **k):
            return self.base_model.model(*a, **k)

    peft = sys.modules["peft"]
    peft.prepare_model_for_kbit_training = lambda m, **k: m
    peft.get_peft_model = lambda m, cfg: _Peft(m)
    peft.LoraConfig = lambda **k: None
    transformers = sys.modules["transformers"]
    transformers.__dict__["BitsAndBytesConfig"] = lambda **k: None


def legacy_cache(gpt):
    """The reference's magic decoding handles ``past_key_values`` as transformers 4.24's tuples of
    per-layer (k, v) (gpt2_prefix_eval.py:471-494); transformers 5.x returns and expects a Cache
    object.  Wrap ``gpt.forward`` so tuples go in and come out (same tensors, no arithmetic).
    The candidate steps pass an all-ones ``attention_mask`` of length 1 next to a longer cache
    (gpt2_prefix_eval.py:419,567): transformers 4.24 turned it into a [B,1,1,1] additive mask of
    zeros (no key masked); 5.x reads a short mask as covering only the newest key and masks the
    cache.  An all-ones mask masks nothing under 4.24 whatever its length, so it is dropped."""
    from transformers import DynamicCache
    from transformers.cache_utils import Cache
    orig = gpt.forward

    def fwd(*a, past_key_values=None, **k):
        m = k.get("attention_mask")
        if m is not None and bool((m == 1).all()):
            k.pop("attention_mask")
        if past_key_values is not None and not isinstance(past_key_values, Cache):
            past_key_values = DynamicCache(ddp_cache_data=[tuple(x) for x in past_key_values])
        out = orig(*a, past_key_values=past_key_values, **k)
        pkv = out.past_key_values
        if pkv is not None and hasattr(pkv, "layers"):
            out.past_key_values = tuple((x.keys, x.values) for x in pkv.layers)
        return out
    gpt.forward = fwd
    return gpt


def gpt2_from_state_dict(sd_gpt):
    """A reference-config GPT2LMHeadModel (eager attention) holding ``sd_gpt`` (no 'gpt.' prefix)."""
    install()
    from transformers import GPT2LMHeadModel  # noqa
    m = GPT2LMHeadModel.from_pretrained("gpt2")
    missing, unexpected = m.load_state_dict(sd_gpt, strict=False)
    assert not unexpected, unexpected
    assert all("attn.bias" in k or "masked_bias" in k for k in missing), missing
    return m.eval()
