"""Oracle for the CLAP audio encoders (from log-mel) and ASE.encode_audio.  TEST INFRASTRUCTURE.

HTSAT: retrieval/models/htsat.py — bn0 (949-951), reshape_wav2img (908-923), PatchEmbed (94-126),
SwinTransformerBlock (354-474) with WindowAttention (269-350), PatchMerging (477-516),
BasicLayer (519-584), forward_features latent_output (777-847).  The dead tscam_conv / sigmoid
branch (841-885) does not affect ``embedding`` and is skipped.
CNN14: retrieval/models/cnns.py:36-78 (ConvBlock), 171-201 (forward).
ASE.encode_audio: retrieval/models/ase_model.py:52-55 (+ audio_proj 34-38).
All fp32, weights as a reference-keyed state dict (prefix ``audio_encoder.audio_enc.``).
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

P = "audio_encoder.audio_enc."
DEPTHS, HEADS, EMBED, WIN = (2, 2, 6, 2), (4, 8, 16, 32), 96, 8


def bn_eval(x, sd, name, eps=1e-5):
    """BatchNorm (eval) over dim 1."""
    shape = [1, -1] + [1] * (x.dim() - 2)
    rm, rv = sd[name + ".running_mean"].view(shape), sd[name + ".running_var"].view(shape)
    w, b = sd[name + ".weight"].view(shape), sd[name + ".bias"].view(shape)
    return (x - rm) / torch.sqrt(rv + eps) * w + b


def bn0(logmel, sd, prefix=P):
    """x.transpose(1,3) -> bn0 -> transpose back (htsat.py:949-951, cnns.py:176-178)."""
    return bn_eval(logmel.transpose(1, 3), sd, prefix + "bn0").transpose(1, 3)


def reshape_wav2img(x, spec_size=256, freq_ratio=4):
    """htsat.py:908-923: bicubic (align_corners=True) T 1001->1024, then fold (B,1,1024,64) into
    (B,1,256,256): image row = chunk*64 + mel, column = frame within chunk."""
    B, C, T, Fq = x.shape
    tT = spec_size * freq_ratio
    if T < tT:
        x = F.interpolate(x, (tT, x.shape[3]), mode="bicubic", align_corners=True)
    x = x.permute(0, 1, 3, 2).contiguous()
    x = x.reshape(B, C, x.shape[2], freq_ratio, x.shape[3] // freq_ratio)
    x = x.permute(0, 1, 3, 2, 4).contiguous()
    return x.reshape(B, C, x.shape[2] * x.shape[3], x.shape[4])


def layer_norm(x, sd, name, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[name + ".weight"], sd[name + ".bias"], eps)


def linear(x, sd, name):
    return F.linear(x, sd[name + ".weight"], sd.get(name + ".bias"))


def rel_pos_index(ws=WIN):
    """WindowAttention.relative_position_index (htsat.py:291-301)."""
    coords = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij"))
    cf = coords.flatten(1)
    rel = (cf[:, :, None] - cf[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    return rel.sum(-1)


def window_partition(x, ws):
    B, H, W, C = x.shape
    x = x.view(B, H // ws, ws, W // ws, ws, C)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(-1, ws, ws, C)


def window_reverse(w, ws, H, W):
    B = int(w.shape[0] / (H * W / ws / ws))
    x = w.view(B, H // ws, W // ws, ws, ws, -1)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(B, H, W, -1)


def shift_mask(H, W, ws, shift):
    """SW-MSA attention mask (htsat.py:406-425): 0 within a region, -100 across regions."""
    img = torch.zeros((1, H, W, 1))
    sl = (slice(0, -ws), slice(-ws, -shift), slice(-shift, None))
    cnt = 0
    for h in sl:
        for w in sl:
            img[:, h, w, :] = cnt
            cnt += 1
    mw = window_partition(img, ws).view(-1, ws * ws)
    m = mw.unsqueeze(1) - mw.unsqueeze(2)
    return m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)


def swin_block(x, sd, name, H, W, heads, shift):
    """SwinTransformerBlock.forward (htsat.py:431-470) + WindowAttention.forward (312-347)."""
    B, L, C = x.shape
    ws = WIN
    if min(H, W) <= ws:   # htsat.py:383-386: window = resolution, no shift
        shift, ws = 0, min(H, W)
    shortcut = x
    x = layer_norm(x, sd, name + "norm1").view(B, H, W, C)
    if shift > 0:
        x = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
    xw = window_partition(x, ws).view(-1, ws * ws, C)
    Bw, N, _ = xw.shape
    qkv = linear(xw, sd, name + "attn.qkv").reshape(Bw, N, 3, heads, C // heads).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    q = q * (C // heads) ** -0.5
    attn = q @ k.transpose(-2, -1)
    table = sd[name + "attn.relative_position_bias_table"]
    bias = table[rel_pos_index(ws).view(-1)].view(N, N, -1).permute(2, 0, 1).contiguous()
    attn = attn + bias.unsqueeze(0)
    if shift > 0:
        mask = shift_mask(H, W, ws, shift)
        nW = mask.shape[0]
        attn = attn.view(Bw // nW, nW, heads, N, N) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, heads, N, N)
    attn = attn.softmax(-1)
    xo = (attn @ v).transpose(1, 2).reshape(Bw, N, C)
    xo = linear(xo, sd, name + "attn.proj")
    x = window_reverse(xo.view(-1, ws, ws, C), ws, H, W)
    if shift > 0:
        x = torch.roll(x, shifts=(shift, shift), dims=(1, 2))
    x = shortcut + x.view(B, H * W, C)
    h = layer_norm(x, sd, name + "norm2")
    h = linear(F.gelu(linear(h, sd, name + "mlp.fc1")), sd, name + "mlp.fc2")
    return x + h


def patch_merging(x, sd, name, H, W):
    """PatchMerging.forward (htsat.py:492-513)."""
    B, L, C = x.shape
    x = x.view(B, H, W, C)
    x = torch.cat([x[:, 0::2, 0::2], x[:, 1::2, 0::2], x[:, 0::2, 1::2], x[:, 1::2, 1::2]], -1)
    x = x.view(B, -1, 4 * C)
    return F.linear(layer_norm(x, sd, name + "norm"), sd[name + "reduction.weight"])


def htsat_embedding(logmel: torch.Tensor, sd: Dict[str, torch.Tensor], prefix=P) -> torch.Tensor:
    """HTSAT_Swin_Transformer.forward(...)['embedding'] from the log-mel [B,1,1001,64] -> [B,768]."""
    x = reshape_wav2img(bn0(logmel, sd, prefix))
    x = F.conv2d(x, sd[prefix + "patch_embed.proj.weight"], sd[prefix + "patch_embed.proj.bias"], stride=4)
    x = x.flatten(2).transpose(1, 2)
    x = layer_norm(x, sd, prefix + "patch_embed.norm")
    res = 64
    for i, (depth, heads) in enumerate(zip(DEPTHS, HEADS)):
        for j in range(depth):
            x = swin_block(x, sd, prefix + f"layers.{i}.blocks.{j}.", res, res, heads,
                           0 if j % 2 == 0 else WIN // 2)
        if i < len(DEPTHS) - 1:
            x = patch_merging(x, sd, prefix + f"layers.{i}.downsample.", res, res)
            res //= 2
    x = layer_norm(x, sd, prefix + "norm")
    return x.mean(dim=1)   # avgpool over the (permuted) 64 final tokens (htsat.py:838-847)


def conv_block(x, sd, name):
    """ConvBlock.forward with pool (2,2) avg (cnns.py:63-78)."""
    x = F.relu(bn_eval(F.conv2d(x, sd[name + "conv1.weight"], padding=1), sd, name + "bn1"))
    x = F.relu(bn_eval(F.conv2d(x, sd[name + "conv2.weight"], padding=1), sd, name + "bn2"))
    return F.avg_pool2d(x, kernel_size=(2, 2))


def cnn14_embedding(logmel: torch.Tensor, sd, prefix=P) -> torch.Tensor:
    """Cnn14.forward from log-mel (cnns.py:171-201): [B,1,1001,64] -> [B,2048]."""
    x = bn0(logmel, sd, prefix)
    for i in range(1, 7):
        x = conv_block(x, sd, prefix + f"conv_block{i}.")
    x = torch.mean(x, dim=3)
    return torch.max(x, dim=2)[0] + torch.mean(x, dim=2)


def audio_project(feat: torch.Tensor, sd, prefix="audio_proj.") -> torch.Tensor:
    """ASE.encode_audio's ``F.normalize(audio_proj(feat), dim=-1)`` (ase_model.py:52-55)."""
    h = F.relu(linear(feat, sd, prefix + "0"))
    return F.normalize(linear(h, sd, prefix + "2"), dim=-1)
