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


# architecture constants (retrieval/models/htsat.py:588-758 with the CLAP args of
# audio_encoder.py:41-51; retrieval/models/cnns.py:137-201)
HTSAT_DEPTHS, HTSAT_HEADS, HTSAT_EMBED, HTSAT_WINDOW, HTSAT_CLASSES = (2, 2, 6, 2), (4, 8, 16, 32), 96, 8, 527
CNN14_CH, N_MELS = (64, 128, 256, 512, 1024, 2048), 64


class _RefInit:
    """The reference modules' own initialisers, from a private generator: trunc_normal(0.02) for
    HTSAT Linear / rel-pos tables (htsat.py:300, 745-758), xavier_uniform for CNN14 convs
    (cnns.py:14-29, init_layer), LayerNorm / BatchNorm weight 1 bias 0, running stats 0 / 1."""

    def __init__(self, seed=0):
        self.g = torch.Generator().manual_seed(seed)

    def trunc_normal(self, shape, std=0.02):
        return torch.empty(*shape).normal_(0.0, std, generator=self.g).clamp_(-2 * std, 2 * std)

    def xavier(self, shape):
        fan_in = shape[1] * (shape[2] * shape[3] if len(shape) == 4 else 1)
        fan_out = shape[0] * (shape[2] * shape[3] if len(shape) == 4 else 1)
        a = (6.0 / (fan_in + fan_out)) ** 0.5
        return torch.empty(*shape).uniform_(-a, a, generator=self.g)

    @staticmethod
    def norm(spec, name, dim, bn=False):
        spec[name + ".weight"] = torch.ones(dim)
        spec[name + ".bias"] = torch.zeros(dim)
        if bn:
            spec[name + ".running_mean"] = torch.zeros(dim)
            spec[name + ".running_var"] = torch.ones(dim)
            spec[name + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.int64)


def htsat_reference_spec() -> Dict[str, torch.Tensor]:
    """Every state-dict entry of the reference HTSAT_Swin_Transformer with the CLAP args
    (parameters + persistent buffers relative_position_index / attn_mask), minus the
    audio_feats_extractor (its own module), initialised as the reference initialises them."""
    ri, spec = _RefInit(3), {}
    ri.norm(spec, "bn0", N_MELS, bn=True)
    spec["patch_embed.proj.weight"] = ri.xavier((HTSAT_EMBED, 1, 4, 4))
    spec["patch_embed.proj.bias"] = torch.zeros(HTSAT_EMBED)
    ri.norm(spec, "patch_embed.norm", HTSAT_EMBED)
    ws = HTSAT_WINDOW
    coords = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")).flatten(1)
    rel = (coords[:, :, None] - coords[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    rpi = rel.sum(-1)
    res = 64
    for i, (depth, heads) in enumerate(zip(HTSAT_DEPTHS, HTSAT_HEADS)):
        dim = HTSAT_EMBED * 2 ** i
        for j in range(depth):
            b = f"layers.{i}.blocks.{j}."
            ri.norm(spec, b + "norm1", dim)
            spec[b + "attn.relative_position_bias_table"] = ri.trunc_normal(((2 * ws - 1) ** 2, heads))
            spec[b + "attn.relative_position_index"] = rpi
            for nm, o, k in (("attn.qkv", 3 * dim, dim), ("attn.proj", dim, dim),
                             ("mlp.fc1", 4 * dim, dim), ("mlp.fc2", dim, 4 * dim)):
                spec[b + nm + ".weight"] = ri.trunc_normal((o, k))
                spec[b + nm + ".bias"] = torch.zeros(o)
            ri.norm(spec, b + "norm2", dim)
            if j % 2 == 1 and res > ws:
                spec[b + "attn_mask"] = _shift_mask(res, ws, ws // 2)
        if i < len(HTSAT_DEPTHS) - 1:
            d = f"layers.{i}.downsample."
            spec[d + "reduction.weight"] = ri.trunc_normal((2 * dim, 4 * dim))
            ri.norm(spec, d + "norm", 4 * dim)
        res //= 2
    nf = HTSAT_EMBED * 2 ** (len(HTSAT_DEPTHS) - 1)
    ri.norm(spec, "norm", nf)
    spec["tscam_conv.weight"] = ri.xavier((HTSAT_CLASSES, nf, 2, 3))
    spec["tscam_conv.bias"] = torch.zeros(HTSAT_CLASSES)
    spec["head.weight"] = ri.trunc_normal((HTSAT_CLASSES, HTSAT_CLASSES))
    spec["head.bias"] = torch.zeros(HTSAT_CLASSES)
    return spec


def cnn14_reference_spec() -> Dict[str, torch.Tensor]:
    """Every state-dict entry of the reference Cnn14 encoder (bn0 + 6 ConvBlocks), initialised as
    the reference's init_bn / init_layer do (cnns.py:14-29, 36-52)."""
    ri, spec = _RefInit(4), {}
    ri.norm(spec, "bn0", N_MELS, bn=True)
    cin = 1
    for i, cout in enumerate(CNN14_CH, start=1):
        b = f"conv_block{i}."
        spec[b + "conv1.weight"] = ri.xavier((cout, cin, 3, 3))
        spec[b + "conv2.weight"] = ri.xavier((cout, cout, 3, 3))
        ri.norm(spec, b + "bn1", cout, bn=True)
        ri.norm(spec, b + "bn2", cout, bn=True)
        cin = cout
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

    def weights(self, device):
        """The packed Gpt2Weights of these parameters (cached until they change)."""
        from .decoder import Gpt2Weights
        dt = zs_dtype_of(self)

        def build():
            sd = {"gpt." + k: v for k, v in self.state_dict().items()}
            return Gpt2Weights(sd, device, dt)
        return self._cache.get(self, build, (dt, str(device)))

    def engine(self, max_rows: int, max_prompt: int, max_steps: int, device):
        from .decoder import Gpt2Decoder
        w = self.weights(device)
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
