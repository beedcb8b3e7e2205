"""Audio encoders on the HIP kernels: HTSAT (default CLAP encoder) and CNN14, plus the ASE
``audio_proj`` + L2 normalisation — i.e. ``ASE.encode_audio`` (retrieval/models/ase_model.py:52-55)
from the raw waveform.

Weights are taken from a reference-keyed state dict (``audio_encoder.audio_enc.*``,
``audio_proj.*``) and repacked once: Linear weights -> [N][K] in the compute dtype, conv weights
-> [Cout][ky][kx][Cin] (NHWC implicit GEMM), biases / norms / BN stats stay f32.
Activations: residual stream f32, GEMM operands in the compute dtype.
"""
from __future__ import annotations

import copy
import os
from typing import Dict

import torch

from . import ops
from .frontend import tables_from_state_dict

DEPTHS, HEADS, EMBED, WIN = (2, 2, 6, 2), (4, 8, 16, 32), 96, 8
CNN14_CH = (64, 128, 256, 512, 1024, 2048)
# stages whose blocks run as ONE fused kernel per block (zs_swin_block, bf16 only); the env var
# ZSAAC_FUSED_SWIN (comma-separated channel widths, "" = none) overrides it for A/B runs.
# Stage 3 (C = 384) runs unfused: its fused kernel holds a whole CU per window (155 KB of LDS) at
# ~17 % MFMA for 133 us, while the unfused block's 16384-row GEMMs are MFMA-efficient; beside the
# decode grids CU time, not latency, is what a begin costs (headline A/B: fused 96,192,384
# 6.32-6.46k, 96,192 6.70-6.88k, 96 6.63-6.66k, none 6.19-6.20k clips/s)
FUSED_SWIN_C = tuple(int(c) for c in os.environ.get("ZSAAC_FUSED_SWIN", "96,192").split(",")
                     if c.strip())


def pack_frags(w: torch.Tensor) -> torch.Tensor:
    """[N][K] -> MFMA fragment order [N/16][K/32][64][8] (csrc/swin.hip): lane l of fragment
    (nt, ks) holds W[16 nt + l % 16][32 ks + 8 (l // 16) .. +8]."""
    N, K = w.shape
    assert N % 16 == 0 and K % 32 == 0, (N, K)
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()


def swin_group(C: int) -> int:
    """Heads per q/k/v group of the fused Swin kernel (csrc/swin.hip SwinCfg::G): one
    (head, 32 queries) per wave, 4 waves for C <= 192, 8 for C = 384."""
    return 4 if C >= 384 else 2


def pack_qkv(w: torch.Tensor, b: torch.Tensor, C: int):
    """qkv.weight [3C][C] / bias [3C] (htsat.py:286, columns part*C + head*24 + d, 304-309) ->
    rows regrouped per group of G heads [q h0.., k h0.., v h0..] x 32 (head dim zero-padded
    24 -> 32) = [heads/G * 96 G][C], fragment-packed; bias [heads/G][96 G]."""
    nh, G = C // 24, swin_group(C)
    wp = torch.zeros(3, nh, 32, C, dtype=w.dtype, device=w.device)
    wp[:, :, :24] = w.reshape(3, nh, 24, C)
    bp = torch.zeros(3, nh, 32, dtype=b.dtype, device=b.device)
    bp[:, :, :24] = b.reshape(3, nh, 24)
    wp = wp.reshape(3, nh // G, G, 32, C).permute(1, 0, 2, 3, 4).reshape(nh * 96, C)
    bp = bp.reshape(3, nh // G, G, 32).permute(1, 0, 2, 3).reshape(nh * 96)
    return pack_frags(wp), bp.contiguous()


def _f32(t, dev):
    return t.detach().to(device=dev, dtype=torch.float32).contiguous()


def _w(t, dev, dtype):
    return t.detach().to(device=dev, dtype=dtype).contiguous()


class HtsatWeights:
    """htsat.py:588-758 parameters (reference keys) in kernel layouts."""

    def __init__(self, sd: Dict[str, torch.Tensor], device, dtype, prefix="audio_encoder.audio_enc."):
        p = prefix
        self.dtype = dtype
        self.bn0 = tuple(_f32(sd[p + "bn0." + k], device)
                         for k in ("running_mean", "running_var", "weight", "bias"))
        self.pe_w = _f32(sd[p + "patch_embed.proj.weight"].reshape(96, 16), device)
        self.pe_b = _f32(sd[p + "patch_embed.proj.bias"], device)
        self.pe_ln = (_f32(sd[p + "patch_embed.norm.weight"], device),
                      _f32(sd[p + "patch_embed.norm.bias"], device))
        self.blocks = []
        self.merges = []
        for i, depth in enumerate(DEPTHS):
            stage = []
            for j in range(depth):
                b = p + f"layers.{i}.blocks.{j}."
                stage.append({
                    "n1": (_f32(sd[b + "norm1.weight"], device), _f32(sd[b + "norm1.bias"], device)),
                    "qkv_w": _w(sd[b + "attn.qkv.weight"], device, dtype),
                    "qkv_b": _f32(sd[b + "attn.qkv.bias"], device),
                    "rel": _f32(sd[b + "attn.relative_position_bias_table"], device),
                    "proj_w": _w(sd[b + "attn.proj.weight"], device, dtype),
                    "proj_b": _f32(sd[b + "attn.proj.bias"], device),
                    "n2": (_f32(sd[b + "norm2.weight"], device), _f32(sd[b + "norm2.bias"], device)),
                    "fc1_w": _w(sd[b + "mlp.fc1.weight"], device, dtype),
                    "fc1_b": _f32(sd[b + "mlp.fc1.bias"], device),
                    "fc2_w": _w(sd[b + "mlp.fc2.weight"], device, dtype),
                    "fc2_b": _f32(sd[b + "mlp.fc2.bias"], device),
                })
                C = EMBED << i
                if dtype == torch.bfloat16 and C in FUSED_SWIN_C:
                    blk = stage[-1]
                    blk["qkv_p"], blk["qkv_bp"] = pack_qkv(blk["qkv_w"], blk["qkv_b"], C)
                    blk["proj_p"] = pack_frags(blk["proj_w"])
                    blk["fc1_p"] = pack_frags(blk["fc1_w"])
                    blk["fc2_p"] = pack_frags(blk["fc2_w"])
            self.blocks.append(stage)
            if i < len(DEPTHS) - 1:
                d = p + f"layers.{i}.downsample."
                self.merges.append({
                    "n": (_f32(sd[d + "norm.weight"], device), _f32(sd[d + "norm.bias"], device)),
                    "red_w": _w(sd[d + "reduction.weight"], device, dtype),
                })
        self.norm = (_f32(sd[p + "norm.weight"], device), _f32(sd[p + "norm.bias"], device))


class Cnn14Weights:
    """cnns.py:137-201 parameters; conv weights [Cout][3][3][Cin] (Cin=1: 9 taps zero-padded to 32),
    eval BN folded into scale = w/sqrt(var+eps), shift = b - mean*scale."""

    def __init__(self, sd, device, dtype, prefix="audio_encoder.audio_enc."):
        p = prefix
        self.dtype = dtype
        self.bn0 = tuple(_f32(sd[p + "bn0." + k], device)
                         for k in ("running_mean", "running_var", "weight", "bias"))
        self.convs = []
        cin = 1
        for i, cout in enumerate(CNN14_CH, start=1):
            b = p + f"conv_block{i}."
            for c, (ci, bn) in enumerate(((cin, "bn1"), (cout, "bn2")), start=1):
                w = sd[b + f"conv{c}.weight"].detach().float()            # [Cout, Cin, 3, 3]
                wp = w.permute(0, 2, 3, 1).reshape(cout, 9 * ci)
                if ci == 1:
                    wp = torch.nn.functional.pad(wp, (0, 32 - 9))
                g = sd[b + bn + ".weight"].float()
                scale = g / torch.sqrt(sd[b + bn + ".running_var"].float() + 1e-5)
                shift = sd[b + bn + ".bias"].float() - sd[b + bn + ".running_mean"].float() * scale
                self.convs.append((ci, cout, _w(wp, device, dtype), _f32(scale, device),
                                   _f32(shift, device)))
            cin = cout


class AudioProjWeights:
    def __init__(self, sd, device, dtype, prefix="audio_proj."):
        self.w0 = _w(sd[prefix + "0.weight"], device, dtype)
        self.b0 = _f32(sd[prefix + "0.bias"], device)
        self.w2 = _w(sd[prefix + "2.weight"], device, dtype)
        self.b2 = _f32(sd[prefix + "2.bias"], device)


class AudioEncoder:
    """``ASE.encode_audio`` for a fixed maximum batch: wav [B, 320000] -> [B, 1024] (unit rows).

    All intermediate buffers are allocated once here, so :meth:`encode` launches only kernels
    (graph-capturable)."""

    def __init__(self, sd, kind="htsat", dtype=torch.bfloat16, max_batch=64, device="cuda",
                 n_samples=320000):
        self.kind, self.dtype, self.B, self.dev = kind, dtype, max_batch, torch.device(device)
        self.T = n_samples
        self.n_frames = n_samples // 320 + 1
        self.tables = tables_from_state_dict(sd, self.dev)
        if kind == "htsat":
            self.w = HtsatWeights(sd, self.dev, dtype)
            width = 768
        elif kind == "cnn14":
            self.w = Cnn14Weights(sd, self.dev, dtype)
            width = 2048
        else:
            raise ValueError(kind)
        self.width = width
        # audio_proj is optional: the bare HTSAT/CNN14 drop-ins return the encoder features
        self.proj = AudioProjWeights(sd, self.dev, dtype) if "audio_proj.0.weight" in sd else None
        self._alloc()

    def twin(self, max_batch=None):
        """Same packed weights, private activation buffers (for another stream), sized for
        ``max_batch`` clips per pass (default: this encoder's)."""
        t = copy.copy(self)
        if max_batch:
            t.B = int(max_batch)
        t._graphs = {}     # captured graphs read / write the parent's buffers: never shared
        t._alloc()
        return t

    def _alloc(self):
        B, dev, dtype, width, kind = self.B, self.dev, self.dtype, self.width, self.kind
        self.logmel = torch.empty(B, self.n_frames, 64, device=dev)
        self.feat = torch.empty(B, width, device=dev)
        self.feat_t = torch.empty(B, width, device=dev, dtype=dtype)
        self.proj_h = torch.empty(B, 1024, device=dev, dtype=dtype)
        self.emb = torch.empty(B, 1024, device=dev)
        self.ws = ops.skinny_workspace(dev, [(B, 1024, width), (B, 1024, 1024)])
        if kind == "htsat":
            M = B * 4096
            self.img = torch.empty(B, 256, 256, device=dev)
            self.x = torch.empty(M * 96, device=dev)            # residual stream (f32), ping
            self.x2 = torch.empty(M * 96 // 2, device=dev)      # after a merge, pong
            # activations of the unfused block sequence: M*C is the same at every stage
            # (tokens / 4, channels * 2 per merge), so size for the first unfused stage only
            # (stages run by zs_swin_block keep theirs in LDS)
            unf = [i for i in range(len(DEPTHS)) if "qkv_p" not in self.w.blocks[i][0]]
            mc = M * 96 if unf else 0
            self.h = torch.empty(mc, device=dev, dtype=dtype)
            self.qkv = torch.empty(mc * 3, device=dev, dtype=dtype)
            self.att = torch.empty(mc, device=dev, dtype=dtype)
            self.hid = torch.empty(mc * 4, device=dev, dtype=dtype)
            self.mrg = torch.empty(M * 96, device=dev, dtype=dtype)
        else:
            H, W = self.n_frames, 64
            big = B * H * W * 64
            self.c_in = torch.empty(B * H * W, device=dev, dtype=dtype)
            self.c_a = torch.empty(big, device=dev, dtype=dtype)
            self.c_b = torch.empty(big, device=dev, dtype=dtype)

    # -------------------------------------------------------------- HTSAT
    def _htsat(self, B):
        w = self.w
        ops.wav2img(self.logmel[:B], out=self.img[:B])
        M, C, res = B * 4096, 96, 64
        x = self.x[:M * C].view(M, C)
        ops.patch_embed(self.img[:B], w.pe_w, w.pe_b, *w.pe_ln, out=x)
        for i, (depth, heads) in enumerate(zip(DEPTHS, HEADS)):
            for j in range(depth):
                blk = w.blocks[i][j]
                shift = 0 if (j % 2 == 0 or res <= WIN) else WIN // 2
                if "qkv_p" in blk:
                    ops.swin_block(x, B, res, res, C, heads, shift, blk)
                    continue
                h = self.h[:M * C].view(M, C)
                qkv = self.qkv[:M * 3 * C].view(M, 3 * C)
                att = self.att[:M * C].view(M, C)
                hid = self.hid[:M * 4 * C].view(M, 4 * C)
                ops.layernorm(x, *blk["n1"], out=h)
                ops.gemm(h, blk["qkv_w"], qkv, bias=blk["qkv_b"])
                ops.window_attention(qkv, B, res, res, C, heads, shift, blk["rel"], att)
                ops.gemm(att, blk["proj_w"], x, bias=blk["proj_b"], residual=x)
                ops.layernorm(x, *blk["n2"], out=h)
                ops.gemm(h, blk["fc1_w"], hid, bias=blk["fc1_b"], act=ops.ACT_GELU_ERF)
                ops.gemm(hid, blk["fc2_w"], x, bias=blk["fc2_b"], residual=x)
            if i < len(DEPTHS) - 1:
                mg = w.merges[i]
                Mo = M // 4
                y = self.mrg[:Mo * 4 * C].view(Mo, 4 * C)
                ops.patch_merge_ln(x, B, res, res, C, *mg["n"], out=y)
                nxt = (self.x2 if x.data_ptr() == self.x.data_ptr() else self.x)[:Mo * 2 * C].view(Mo, 2 * C)
                ops.gemm(y, mg["red_w"], nxt)
                x, M, C, res = nxt, Mo, 2 * C, res // 2
        ops.ln_meanpool(x, B, res * res, C, *w.norm, out=self.feat[:B])

    # -------------------------------------------------------------- CNN14
    def _cnn14(self, B):
        H, W = self.n_frames, 64
        cur = self.c_in[:B * H * W]
        ops.cast(self.logmel[:B].reshape(-1), cur)
        bufs = (self.c_a, self.c_b)
        k = 0
        for blk in range(6):
            for c in range(2):
                ci, co, wt, sc, sh = self.w.convs[blk * 2 + c]
                out = bufs[k % 2][:B * H * W * co]
                ops.conv3x3_bn_relu(cur, B, H, W, ci, wt, co, sc, sh, out)
                cur, k = out, k + 1
            Ho, Wo = H // 2, W // 2
            out = bufs[k % 2][:B * Ho * Wo * co]
            ops.avgpool2(cur, B, H, W, co, out)
            cur, k, H, W = out, k + 1, Ho, Wo
        ops.cnn_head(cur, B, H, W, 2048, self.feat[:B])

    def encode(self, wav: torch.Tensor) -> torch.Tensor:
        """wav [B, T] f32 (device) -> normalised CLAP embeddings [B, 1024] f32 (a view)."""
        B = wav.shape[0]
        assert B <= self.B and wav.shape[1] == self.T, (wav.shape, self.B, self.T)
        ops.logmel(wav, self.tables, bn=self.w.bn0, out=self.logmel[:B])
        return self.encode_logmel(None, B)

    def encode_graphed(self, wav: torch.Tensor) -> torch.Tensor:
        """encode() with everything after the log-mel front end replayed from a hipGraph per batch
        size (captured on first use, on the current -- non-default -- stream, without a device
        sync): one graph launch instead of ~75 kernel launches' host enqueue (~7 ms of Python per
        256-clip pass, which held up the concurrent runner's begins)."""
        B = wav.shape[0]
        assert B <= self.B and wav.shape[1] == self.T, (wav.shape, self.B, self.T)
        ops.logmel(wav, self.tables, bn=self.w.bn0, out=self.logmel[:B])
        if not hasattr(self, "_graphs"):
            self._graphs = {}
        ent = self._graphs.get(B)
        if ent is None:
            g = torch.cuda.CUDAGraph()
            g.capture_begin()
            try:
                out = self.encode_logmel(None, B)
            finally:
                g.capture_end()
            ent = self._graphs[B] = (g, out)
        ent[0].replay()
        return ent[1]

    def encode_logmel(self, logmel, B=None):
        """From a bn0'd log-mel [B, frames, 64] (None: the internal buffer) -> [B, 1024]."""
        if logmel is not None:
            B = logmel.shape[0]
            self.logmel[:B].copy_(logmel)
        if self.kind == "htsat":
            self._htsat(B)
        else:
            self._cnn14(B)
        if self.proj is None:
            return self.feat[:B]
        return self.project(self.feat[:B])

    def project(self, feat):
        B = feat.shape[0]
        assert self.proj is not None, "no audio_proj weights"
        ops.cast(feat, self.feat_t[:B])
        ops.gemm(self.feat_t[:B], self.proj.w0, self.proj_h[:B], bias=self.proj.b0, act=ops.ACT_RELU,
                 workspace=self.ws)
        ops.gemm(self.proj_h[:B], self.proj.w2, self.emb[:B], bias=self.proj.b2, workspace=self.ws)
        return ops.l2norm(self.emb[:B], out=self.emb[:B])
