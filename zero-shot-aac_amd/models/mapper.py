"""Drop-in for the reference's ``models/mapper.py`` (models/mapper.py:6-139): same classes, same
constructor arguments, same parameter names/shapes (checkpoints load unchanged), forward on the
MI355X HIP kernels (zsaac).  Set ``module.zs_dtype = torch.bfloat16`` for the perf mode; the
default float32 is the parity mode.

Only the inference forward is provided (the reference trains these; training is out of scope).
"""
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from zsaac import ops
from zsaac.modules import EngineCache, require_device, zs_dtype_of

__all__ = ["MLP", "MlpTransformer", "MultiHeadAttention", "TransformerLayer", "Transformer",
           "TransformerMapper"]

_ACT = {nn.Tanh: ops.ACT_TANH, nn.ReLU: ops.ACT_RELU, nn.GELU: ops.ACT_GELU_ERF}


class MLP(nn.Module):
    """mapper.py:6-18: Linear / act / ... / Linear (act between, not after the last)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        require_device(x, "MLP.forward")
        dt = zs_dtype_of(self)
        lead = x.shape[:-1]
        h = x.reshape(-1, x.shape[-1]).float().contiguous()
        lins = [m for m in self.model if isinstance(m, nn.Linear)]
        ws = self._cache.get(self, lambda: [(l.weight.detach().to(dt).contiguous(),
                                             None if l.bias is None else l.bias.detach().float().contiguous())
                                            for l in lins], (dt,))
        M = h.shape[0]
        cur =torch.empty(M, h.shape[1], device=x.device, dtype=dt)
        ops.cast(h, cur)
        for i, (w, b) in enumerate(ws):
            last = i == len(ws) - 1
            if M <= 64:
                ops.reserve_skinny_workspace(x.device, M, w.shape[0], w.shape[1])
            out = torch.empty(M, w.shape[0], device=x.device, dtype=torch.float32 if last else dt)
            ops.gemm(cur, w, out, bias=b, act=ops.ACT_NONE if last else self.act_code)
            cur = out
        return cur.view(*lead, -1)

    def __init__(self, sizes: Tuple[int, ...], bias=True, act=nn.Tanh):
        super(MLP, self).__init__()
        layers = []
        for i in range(len(sizes) - 1):
            layers.append(nn.Linear(sizes[i], sizes[i + 1], bias=bias))
            if i < len(sizes) - 2:
                layers.append(act())
        self.model = nn.Sequential(*layers)
        self.act_code = _ACT[act]
        self._cache = EngineCache()


class MlpTransformer(nn.Module):
    """mapper.py:20-35 (parameters only; run inside TransformerMapper's engine)."""

    def __init__(self, in_dim, h_dim, out_d: Optional[int] = None, act=F.relu, dropout=0.):
        super().__init__()
        out_d = out_d if out_d is not None else in_dim
        self.fc1 = nn.Linear(in_dim, h_dim)
        self.act = act
        self.fc2 = nn.Linear(h_dim, out_d)
        self.dropout = nn.Dropout(dropout)


class MultiHeadAttention(nn.Module):
    """mapper.py:37-66 (parameters only)."""

    def __init__(self, dim_self, dim_ref, num_heads, bias=True, dropout=0.):
        super().__init__()
        self.num_heads = num_heads
        head_dim = dim_self // num_heads
        self.scale = head_dim ** -0.5
        self.to_queries = nn.Linear(dim_self, dim_self, bias=bias)
        self.to_keys_values = nn.Linear(dim_ref, dim_self * 2, bias=bias)
        self.project = nn.Linear(dim_self, dim_self)
        self.dropout = nn.Dropout(dropout)


class TransformerLayer(nn.Module):
    """mapper.py:68-87 (parameters only)."""

    def __init__(self, dim_self, dim_ref, num_heads, mlp_ratio=4., bias=False, dropout=0., act=F.relu,
                 norm_layer: nn.Module = nn.LayerNorm):
        super().__init__()
        self.norm1 = norm_layer(dim_self)
        self.attn = MultiHeadAttention(dim_self, dim_ref, num_heads, bias=bias, dropout=dropout)
        self.norm2 = norm_layer(dim_self)
        self.mlp = MlpTransformer(dim_self, int(dim_self * mlp_ratio), act=act, dropout=dropout)


class Transformer(nn.Module):
    """mapper.py:89-123 (parameters only; enc_dec=False as TransformerMapper builds it)."""

    def __init__(self, dim_self: int, num_heads: int, num_layers: int, dim_ref: Optional[int] = None,
                 mlp_ratio: float = 2., act=F.relu, norm_layer: nn.Module = nn.LayerNorm,
                 enc_dec: bool = False):
        super(Transformer, self).__init__()
        dim_ref = dim_ref if dim_ref is not None else dim_self
        if enc_dec:
            raise NotImplementedError("enc_dec Transformer is not on the captioning path")
        self.enc_dec = enc_dec
        self.layers = nn.ModuleList([TransformerLayer(dim_self, dim_ref, num_heads, mlp_ratio, act=act,
                                                      norm_layer=norm_layer) for _ in range(num_layers)])


class TransformerMapper(nn.Module):
    """mapper.py:125-139: Linear -> [x ; prefix_const] -> 8 self-attention layers -> rows
    clip_length:, on zsaac.decoder.TransformerMapperEngine."""

    def forward(self, x):
        from zsaac.decoder import TransformerMapperEngine
        require_device(x, "TransformerMapper.forward")
        dt = zs_dtype_of(self)
        B = x.shape[0]
        cap = max(B, 1)

        def build():
            sd = {"clap_project." + k: v for k, v in self.state_dict().items()}
            return TransformerMapperEngine(sd, x.device, dt, cap, clip_length=self.clip_length,
                                           num_layers=len(self.transformer.layers),
                                           heads=self.transformer.layers[0].attn.num_heads)
        eng = self._cache.get(self, build, (dt, cap, str(x.device)))
        out = eng(x.reshape(B, -1).float().contiguous())
        return out.reshape(B, -1, self.prefix_const.shape[1]).clone()

    def __init__(self, dim_clip: int, dim_embedding: int, prefix_length: int, clip_length: int,
                 num_layers: int = 8):
        super(TransformerMapper, self).__init__()
        self.clip_length = clip_length
        self.transformer = Transformer(dim_embedding, 8, num_layers)
        self.linear = nn.Linear(dim_clip, clip_length * dim_embedding)
        self.prefix_const = nn.Parameter(torch.randn(prefix_length, dim_embedding), requires_grad=True)
        self._cache = EngineCache()
