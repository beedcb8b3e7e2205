"""nn.Module mirrors of the reference classes on the hot path, with the reference's parameter
names and shapes (so reference checkpoints load with ``load_state_dict``), whose forward runs
on the HIP kernels.  The modules only HOLD parameters; the first forward on a device packs them
into a kernel engine (zsaac.decoder / zsaac.encoder) that is cached until the parameters change.

There is no CPU path: a forward on CPU tensors raises ZsError.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn

from ._lib import ZsError

BUFFER_SUFFIXES = ("running_mean", "running_var", "num_batches_tracked")


def zs_dtype_of(module: nn.Module) -> torch.dtype:
    """Compute dtype of the kernel engine: ``module.zs_dtype`` if set (torch.bfloat16 for the
    perf mode), else float32 (parity mode, the reference's precision)."""
    return getattr(module, "zs_dtype", torch.float32)


def require_device(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise ZsError(f"{what}: zsaac runs on the MI355X HIP kernels only (got a CPU tensor); "
                      "move the model and inputs to 'cuda'")


class EngineCache:
    """Caches an engine built from a module's parameters; rebuilt when any parameter's storage
    or version changes (load_state_dict, .to(), in-place edits)."""

    def __init__(self):
        self.key = None
        self.engine = None

    @staticmethod
    def _key(module: nn.Module, extra):
        return (tuple((p.data_ptr(), p._version) for p in module.parameters()), extra)

    def get(self, module: nn.Module, build, extra=None):
        k = self._key(module, extra)
        if k != self.key:
            self.engine = build()
            self.key = k
        return self.engine


class ParamTree(nn.Module):
    """Parameter container with arbitrary dotted names (``layers.0.blocks.1.attn.qkv.weight``);
    BatchNorm running statistics become buffers, like the reference modules'."""

    def __init__(self, spec: Dict[str, torch.Tensor]):
        super().__init__()
        for name, t in spec.items():
            *path, leaf = name.split(".")
            mod = self
            for p in path:
                if p not in mod._modules:
                    mod.add_module(p, nn.Module())
                mod = mod._modules[p]
            if leaf in BUFFER_SUFFIXES:
                mod.register_buffer(leaf, t.clone())
            else:
                mod.register_parameter(leaf, nn.Parameter(t.clone(), requires_grad=False))


def register_tree(module: nn.Module, spec: Dict[str, torch.Tensor], buffers=()) -> None:
    """Register ``spec`` (dotted name -> tensor) on ``module`` as parameters (buffers for BN
    statistics and the names in ``buffers``), creating intermediate submodules."""
    for name, t in spec.items():
        *path, leaf = name.split(".")
        mod = module
        for p in path:
            if p not in mod._modules:
                mod.add_module(p, nn.Module())
            mod = mod._modules[p]
        if leaf in BUFFER_SUFFIXES or name in buffers or leaf in buffers:
            mod.register_buffer(leaf, t.clone())
        else:
            mod.register_parameter(leaf, nn.Parameter(t.clone(), requires_grad=False))


def htsat_reference_spec() -> Dict[str, torch.Tensor]:
    """Every state-dict entry of the reference HTSAT_Swin_Transformer with the CLAP args
    (parameters + persistent buffers relative_position_index / attn_mask), minus the
    audio_feats_extractor (its own module)."""
    from .synthetic import HTSAT_DEPTHS, htsat_state_dict
    spec = dict(htsat_state_dict(3, prefix=""))
    ws = 8
    coords = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")).flatten(1)
    rel = (coords[:, :, None] - coords[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    rpi = rel.sum(-1)
    res = 64
    for i, depth in enumerate(HTSAT_DEPTHS):
        for j in range(depth):
            b = f"layers.{i}.blocks.{j}."
            spec[b + "attn.relative_position_index"] = rpi
            if j % 2 == 1 and res > ws:
                spec[b + "attn_mask"] = _shift_mask(res, ws, ws // 2)
        res //= 2
    return spec


def _shift_mask(H, ws, shift):
    img = torch.zeros(1, H, H, 1)
    sl = (slice(0, -ws), slice(-ws, -shift), slice(-shift, None))
    cnt = 0
    for h in sl:
        for w in sl:
            img[:, h, w, :] = cnt
            cnt += 1
    x = img.view(1, H // ws, ws, H // ws, ws, 1).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws)
    m = x.unsqueeze(1) - x.unsqueeze(2)
    return m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)


class Conv1D(nn.Module):
    """HF transformers Conv1D: weight [in, out], y = x @ W + b (GPT-2 c_attn/c_proj/c_fc)."""

    def __init__(self, nf: int, nx: int):
        super().__init__()
        self.nf = nf
        self.weight = nn.Parameter(torch.empty(nx, nf).normal_(std=0.02))
        self.bias = nn.Parameter(torch.zeros(nf))


class _Attn(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.c_attn = Conv1D(3 * d, d)
        self.c_proj = Conv1D(d, d)


class _Mlp(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.c_fc = Conv1D(4 * d, d)
        self.c_proj = Conv1D(d, 4 * d)


class _Block(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.ln_1 = nn.LayerNorm(d, eps=1e-5)
        self.attn = _Attn(d)
        self.ln_2 = nn.LayerNorm(d, eps=1e-5)
        self.mlp = _Mlp(d)


class _Transformer(nn.Module):
    def __init__(self, vocab, n_pos, d, n_layer):
        super().__init__()
        self.wte = nn.Embedding(vocab, d)
        self.wpe = nn.Embedding(n_pos, d)
        self.h = nn.ModuleList([_Block(d) for _ in range(n_layer)])
        self.ln_f = nn.LayerNorm(d, eps=1e-5)


class GPT2Output:
    def __init__(self, logits):
        self.logits = logits


class ZsGPT2LMHeadModel(nn.Module):
    """GPT-2 small with HF GPT2LMHeadModel's module tree / state-dict keys (tied lm_head).
    ``forward(inputs_embeds=...)`` returns ``.logits`` for every position (the reference's
    full-recompute call, gpt2_prefix_eval.py:118/192) computed by the HIP kernels."""

    def __init__(self, vocab=50257, n_positions=1024, n_embd=768, n_layer=12):
        super().__init__()
        self.transformer = _Transformer(vocab, n_positions, n_embd, n_layer)
        self.lm_head = nn.Linear(n_embd, vocab, bias=False)
        self.lm_head.weight = self.transformer.wte.weight          # tied
        nn.init.normal_(self.transformer.wte.weight, std=0.02)
        nn.init.normal_(self.transformer.wpe.weight, std=0.01)
        self._cache = EngineCache()

    def get_input_embeddings(self):
        return self.transformer.wte

    def engine(self, max_rows: int, max_prompt: int, max_steps: int, device):
        from .decoder import Gpt2Decoder, Gpt2Weights
        dt = zs_dtype_of(self)

        def build():
            sd = {"gpt." + k: v for k, v in self.state_dict().items()}
            return Gpt2Weights(sd, device, dt)
        w = self._cache.get(self, build, (dt, str(device)))
        key = (max_rows, max_prompt, max_steps)
        decs = w.__dict__.setdefault("_decoders", {})
        if key not in decs:
            decs[key] = Gpt2Decoder(w, max_rows, max_prompt, max_steps, max_prefill_rows=max_rows)
        return decs[key]

    def forward(self, input_ids=None, inputs_embeds=None, output_hidden_states=False, **kw):
        from . import ops
        if inputs_embeds is None:
            inputs_embeds = self.transformer.wte(input_ids)
        require_device(inputs_embeds, "GPT2LMHeadModel.forward")
        B, L, D = inputs_embeds.shape
        dec = self.engine(B, L, 1, inputs_embeds.device)
        w = dec.w
        zeros = torch.zeros(B, 1, dtype=torch.int32, device=inputs_embeds.device)
        hl = torch.zeros(B, dtype=torch.int32, device=inputs_embeds.device)
        emb = inputs_embeds.float().contiguous()
        ops.prefill_embed(zeros, hl, emb, L * D, L, w.wte, w.wpe, B, L, None, dec.x, dec.plen,
                          dec.last_row)
        dec.prefill(B, L)
        # logits for every position: ln_f over all rows, then one vocab GEMM
        M = B * L
        hf = torch.empty(M, D, device=emb.device, dtype=w.dtype)
        ops.layernorm(dec.x[:M], *w.lnf, out=hf)
        logits = torch.empty(M, w.V, device=emb.device)
        ops.gemm(hf, w.wte, logits, split_k=1)
        return GPT2Output(logits.view(B, L, w.V))
