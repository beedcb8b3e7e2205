"""Mistral-7B caption decoder on the HIP kernels (BASELINE.json config C5).

Reference: predict_mistralai_multilingual.py:90-111 -- per batch of 32 clips and per language tag
(``<en>``, ``<zh>``, ``<fr>``): ``prefix_embed = clap_to_gpt(prefix, embed_tokens(hard prompt),
embed_tokens(tokenizer(tag)))`` (models/caption_model.py:392-413) then
``LMmodel.generate(inputs_embeds=prefix_embed, attention_mask=ones, do_sample=False,
max_length=60, eos_token_id=2, pad_token_id=2)`` -- batched greedy decoding of
``MistralForCausalLM`` (4-bit NF4 base weights + LoRA r=8 on every projection and the LM head,
caption_model.py:355-364).

Here: the LoRA adapters are merged into the base weights at load (W + (alpha / r) B A,
:func:`merge_peft_state_dict`), the RMSNorm weights are folded into the GEMMs that follow them,
and the decoder weights are stored as fp8 e4m3 (OCP) with one f32 scale per output channel
(``mode="fp8"``, the perf mode), bf16 (``"bf16"``) or f32 (``"f32"``, the parity mode: no folding,
zs_gemm f32, ids bit-exact against HF MistralForCausalLM on the same weights).  NF4 itself is a
bitsandbytes storage format (the library is absent here); fp8 is the MI355X-native 8-bit format:
a checkpoint's NF4 tensors are dequantised to f32 on load (:func:`dequantize_bnb_4bit`, in torch on
the host, from the saved quant_state) and :class:`MistralWeights` re-quantises them.

One decode step for M rows (csrc/mistral.hip): per layer
  [add + RMSNorm] -> qkv GEMM (fp8 weights, split-K slabs) -> RoPE + KV append -> GQA attention
  -> o GEMM -> add + RMSNorm -> gate|up GEMM -> SiLU * up -> down GEMM -> (next layer's add+norm)
then the final norm, the LM head (zs_lmhead_topk argmax) and the greedy step (eos -> done).
The prompt (hard prompt padded to the batch's longest with id 0 and attended, as the reference's
all-ones attention mask does; soft rows; language tag ids) is prefilled as B x P rows.
"""
from __future__ import annotations

import math
import time
from typing import Dict, List, Optional, Sequence

import torch

from . import ops
from ._lib import ZS_BF16, ZS_F32, call


# bitsandbytes 4-bit checkpoints (caption_model.py:355-364 loads the base model with
# BitsAndBytesConfig(load_in_4bit, bnb_4bit_quant_type="nf4", bnb_4bit_use_double_quant=True)):
# a quantized Linear's state dict holds ``weight`` (packed uint8, two 4-bit codes per byte, the
# first element in the HIGH nibble), ``weight.absmax`` (one scale per block of `blocksize`
# elements; uint8 codes when double-quantized), ``weight.quant_map`` (the 16-entry NF4 code),
# ``weight.nested_absmax`` / ``weight.nested_quant_map`` (the double quantization of absmax:
# blocks of `nested_blocksize`, a 256-entry dynamic code, plus `nested_offset`) and
# ``weight.quant_state.bitsandbytes__nf4`` (the remaining fields as JSON bytes in a uint8 tensor:
# shape, dtype, blocksize, quant_type, nested_*).  Read with json (nothing executed).
_BNB_STATE = ".quant_state.bitsandbytes__"


def _bnb_state(sd: Dict[str, torch.Tensor], wkey: str) -> Optional[dict]:
    import json
    for qt in ("nf4", "fp4"):
        k = wkey + _BNB_STATE + qt
        if k in sd:
            return json.loads(bytes(sd[k].to(torch.uint8).flatten().tolist()).decode("utf-8"))
    return None


def dequantize_bnb_4bit(sd: Dict[str, torch.Tensor], wkey: str) -> torch.Tensor:
    """The f32 weight of a bitsandbytes 4-bit (NF4 / FP4) Linear saved under ``wkey``
    (bitsandbytes dequantize_4bit: code[nibble] * absmax[i // blocksize], absmax itself
    dequantized as nested_code[q] * nested_absmax[j // nested_blocksize] + nested_offset when
    double-quantized)."""
    st = _bnb_state(sd, wkey)
    if st is None:
        raise ValueError(f"{wkey}: no bitsandbytes quant_state")
    shape = [int(v) for v in st["shape"]]
    n = 1
    for v in shape:
        n *= v
    bs = int(st["blocksize"])
    packed = sd[wkey].to(torch.uint8).flatten()
    codes = torch.empty(packed.numel() * 2, dtype=torch.long)
    codes[0::2] = (packed >> 4).long()
    codes[1::2] = (packed & 0xF).long()
    codes = codes[:n]
    qmap = sd[wkey + ".quant_map"].float().flatten()
    absmax = sd[wkey + ".absmax"]
    if wkey + ".nested_absmax" in sd:
        nbs = int(st.get("nested_blocksize", 256))
        nq = sd[wkey + ".nested_quant_map"].float().flatten()
        na = sd[wkey + ".nested_absmax"].float().flatten()
        aq = absmax.to(torch.uint8).flatten().long()
        idx = torch.arange(aq.numel()) // nbs
        absmax = nq[aq] * na[idx] + float(st.get("nested_offset", 0.0))
    absmax = absmax.float().flatten()
    vals = qmap[codes] * absmax[torch.arange(n) // bs]
    return vals.view(shape)


def dequantize_bnb_state_dict(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """A state dict with bitsandbytes 4-bit Linear weights -> plain f32 weights under the same
    keys (the absmax / quant_map / nested_* / quant_state entries dropped); other entries as is."""
    qkeys = {k.split(_BNB_STATE)[0] for k in sd if _BNB_STATE in k}
    aux = (".absmax", ".quant_map", ".nested_absmax", ".nested_quant_map")
    out = {}
    for k, v in sd.items():
        if _BNB_STATE in k or any(k.endswith(a) and k[:-len(a)] in qkeys for a in aux):
            continue
        out[k] = dequantize_bnb_4bit(sd, k) if k in qkeys else v
    return out


def merge_peft_state_dict(sd: Dict[str, torch.Tensor], lora_alpha: float = 16.0, r: int = 8,
                          prefix: str = "") -> Dict[str, torch.Tensor]:
    """A peft LoRA state dict (``...base_model.model.model.layers.0.self_attn.q_proj.base_layer
    .weight`` + ``lora_A.default.weight`` [r, in] + ``lora_B.default.weight`` [out, r], the
    ``get_peft_model`` of caption_model.py:362-364) -> plain MistralForCausalLM keys with
    W = base + (lora_alpha / r) B @ A.  bitsandbytes 4-bit base weights (the reference's NF4
    checkpoint) are dequantized first (:func:`dequantize_bnb_state_dict`)."""
    if any(_BNB_STATE in k for k in sd):
        sd = dequantize_bnb_state_dict(sd)
    out, lora = {}, {}
    strip = prefix + "base_model.model."
    for k, v in sd.items():
        if not k.startswith(strip):
            continue
        k2 = k[len(strip):]
        if ".lora_A." in k2 or ".lora_B." in k2:
            base = k2.split(".lora_")[0]
            lora.setdefault(base, {})["A" if ".lora_A." in k2 else "B"] = v.float()
        else:
            out[k2.replace(".base_layer.", ".")] = v
    for base, ab in lora.items():
        w = base + ".weight"
        out[w] = out[w].float() + (lora_alpha / r) * (ab["B"] @ ab["A"])
    return out


def quantize_fp8(w: torch.Tensor):
    """Per-output-channel (row) fp8 e4m3fn: returns (uint8 codes [N, K], f32 scales [N])."""
    w = w.float()
    amax = w.abs().amax(dim=1).clamp(min=1e-12)
    scale = amax / 448.0
    q = (w / scale[:, None]).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), scale


def dequantize_fp8(q: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    return q.view(torch.float8_e4m3fn).float() * scale[:, None].float()


def glu_interleave(gu: torch.Tensor) -> torch.Tensor:
    """[gate; up] rows [2F, K] -> the glu-interleaved order the decode GEMM's fused SiLU * up
    epilogue reads (csrc/mistral.hip fp8_gemm_run_kernel, zs_mistral_silu_mul): in every group of
    16 rows, rows 0-3 / 8-11 are gate rows 8 grp + 0..3 / 4..7 and rows 4-7 / 12-15 the matching
    up rows.  F % 8 == 0."""
    F = gu.shape[0] // 2
    if gu.shape[0] != 2 * F or F % 8:
        raise ValueError(f"glu_interleave: {tuple(gu.shape)} is not [2F, K] with F % 8 == 0")
    r = torch.arange(2 * F, device=gu.device)
    c = r % 16
    j = 8 * (r // 16) + 4 * (c // 8) + c % 4
    return gu[torch.where((c // 4) % 2 == 0, j, F + j)]


def fp8_pack_tiles(q: torch.Tensor) -> torch.Tensor:
    """Row-major fp8 codes [N, K] (K % 1024 == 0) -> the tile-packed stream zs_fp8_gemm_rows reads
    (csrc/mistral.hip): [K/1024][ceil(N/128)][8][16][64 lanes][16 B], i.e. the 1 KiB block of
    (k split s, 128-column tile t, 16-column group w, 64-deep k block j) holds, in lane l,
    W[128 t + 16 w + (l & 15)][1024 s + 64 j + 16 (l >> 4) .. +16]; rows past N are zero.  Every
    wave-load of the GEMM is then one contiguous KiB and a workgroup's run of items one
    contiguous stretch of HBM."""
    N, K = q.shape
    if K % 1024:
        raise ValueError(f"fp8_pack_tiles: K={K} must be a multiple of 1024")
    NT = -(-N // 128)
    if NT * 128 != N:
        q = torch.cat([q, q.new_zeros(NT * 128 - N, K)])
    # [t, w, fr, s, j, g, 16] -> [s, t, w, j, g, fr, 16]
    v = q.reshape(NT, 8, 16, K // 1024, 16, 4, 16).permute(3, 0, 1, 4, 5, 2, 6)
    return v.contiguous().view(-1)


class MistralWeights:
    """Packed decoder weights from MistralForCausalLM keys (``model.*``, ``lm_head.weight``)."""

    def __init__(self, sd: Dict[str, torch.Tensor], device, mode: str = "fp8", n_heads: int = 32,
                 n_kv_heads: int = 8, eps: float = 1e-5, rope_theta: float = 10000.0,
                 prefix: str = ""):
        if mode not in ("fp8", "bf16", "f32"):
            raise ValueError(mode)
        dev = torch.device(device)
        self.mode, self.dev = mode, dev
        self.adt = torch.float32 if mode == "f32" else torch.bfloat16   # activation operand dtype
        p = prefix + "model."
        self.emb = sd[p + "embed_tokens.weight"].to(dev, self.adt).contiguous()
        self.V, self.D = self.emb.shape
        self.H, self.KVH, self.HD = n_heads, n_kv_heads, 128
        if self.D != self.H * self.HD:
            raise ValueError("Mistral kernels need head_dim 128 (hidden = heads x 128)")
        self.eps, self.theta = eps, rope_theta
        fold = mode != "f32"
        self.layers = []
        i = 0
        while f"{p}layers.{i}.self_attn.q_proj.weight" in sd:
            L = f"{p}layers.{i}."
            g1 = sd[L + "input_layernorm.weight"].float()
            g2 = sd[L + "post_attention_layernorm.weight"].float()
            qkv = torch.cat([sd[L + f"self_attn.{n}_proj.weight"].float() for n in "qkv"])
            gu = torch.cat([sd[L + "mlp.gate_proj.weight"].float(), sd[L + "mlp.up_proj.weight"].float()])
            ly = {"ln1": None if fold else g1.to(dev), "ln2": None if fold else g2.to(dev),
                  "qkv": self._pack(qkv * g1[None] if fold else qkv),
                  "o": self._pack(sd[L + "self_attn.o_proj.weight"]),
                  "gu": self._pack(glu_interleave(gu * g2[None] if fold else gu)),
                  "down": self._pack(sd[L + "mlp.down_proj.weight"])}
            self.layers.append(ly)
            i += 1
        self.F = self.layers[0]["gu"]["N"] // 2
        gn = sd[p + "norm.weight"].float()
        lm = sd[prefix + "lm_head.weight"].float()
        self.lnf = None if fold else gn.to(dev)
        self.lm = (lm * gn[None] if fold else lm).to(dev, self.adt).contiguous()

    @classmethod
    def synthetic(cls, device, cfg: dict, seed: int = 0, mode: str = "fp8", eos_boost: float = 1.5,
                  shared_values: bool = False, resid_init: bool = False):
        """Random-init weights at ``cfg`` (zsaac.synthetic.MISTRAL_7B geometry for the bench)
        generated and quantised on the device, layer by layer (a 7B f32 state dict on the host
        would take 29 GB).  ``shared_values``: every mode holds the SAME values for one seed --
        the matrices rounded to what per-row fp8 e4m3 represents, the embedding and LM head to
        bf16 -- so an "f32" engine is the exact-arithmetic reference of the "fp8" one.
        ``resid_init``: the residual-branch outputs (o_proj, down_proj) scaled by 1 / sqrt(2 L) and
        unit gains elsewhere (the GPT-2 / Megatron initialisation): a residual stream whose
        per-layer perturbations stay small, as in a trained model, instead of the bench's
        high-gain init, whose 32-layer stack amplifies bf16 rounding ~0.7 % per layer."""
        dev = torch.device(device)
        g = torch.Generator(device=dev).manual_seed(seed)
        self = cls.__new__(cls)
        self.mode, self.dev = mode, dev
        self._shared = shared_values
        self.adt = torch.float32 if mode == "f32" else torch.bfloat16
        D, F, V = cfg["hidden"], cfg["ffn"], cfg["vocab"]
        self.V, self.D, self.F = V, D, F
        self.H, self.KVH, self.HD = cfg["heads"], cfg["kv_heads"], 128
        self.eps, self.theta = 1e-5, 10000.0
        rnd = lambda o, i, gain=1.0: torch.randn(o, i, device=dev, generator=g) * (gain / math.sqrt(i))
        emb = torch.randn(V, D, device=dev, generator=g)
        self.emb = (emb.bfloat16() if shared_values else emb).to(self.adt)
        self.layers = []
        kv = self.KVH * 128
        ro = 1.0 / math.sqrt(2 * cfg["layers"]) if resid_init else 1.0
        gq, gg = (1.0, 1.0) if resid_init else (2.0, 1.5)
        for _ in range(cfg["layers"]):
            self.layers.append({
                "ln1": None, "ln2": None,
                "qkv": self._pack(torch.cat([rnd(D, D, gq), rnd(kv, D, gq), rnd(kv, D)])),
                "o": self._pack(rnd(D, D, ro)),
                "gu": self._pack(glu_interleave(torch.cat([rnd(F, D, gg), rnd(F, D)]))),
                "down": self._pack(rnd(D, F, ro))})
        self.lnf = None
        lm = rnd(V, D, 4.0)
        lm[2] *= eos_boost
        self.lm = (lm.bfloat16() if shared_values else lm).to(self.adt).contiguous()
        return self

    def _pack(self, w):
        w = w.float()
        N, K = w.shape
        if self.mode != "fp8" and getattr(self, "_shared", False):
            w = dequantize_fp8(*quantize_fp8(w))        # the fp8 engine's exact values
        if self.mode == "fp8":
            q, s = quantize_fp8(w)
            return {"N": N, "K": K, "w8": fp8_pack_tiles(q.to(self.dev)),
                    "scale": s.to(self.dev).contiguous()}
        return {"N": N, "K": K, "w": w.to(self.dev, self.adt).contiguous()}

    def nbytes(self) -> int:
        n = 0
        for ly in self.layers:
            for k in ("qkv", "o", "gu", "down"):
                t = ly[k]
                n += t["w8"].numel() + t["scale"].numel() * 4 if "w8" in t else t["w"].numel() * t["w"].element_size()
        return n + self.lm.numel() * self.lm.element_size()


class MistralDecoder:
    """Batched greedy decoding (HF generate, do_sample=False) for up to ``max_batch`` sequences
    with prompts of up to ``max_prompt`` rows and ``max_new`` generated tokens."""

    def __init__(self, w: MistralWeights, max_batch: int = 32, max_prompt: int = 64,
                 max_new: int = 60):
        self.w = w
        dev, adt = w.dev, w.adt
        self.B, self.Pmax, self.max_new = max_batch, max_prompt, max_new
        self.fused_decode_attn = True     # False: decode through rope_kv + attention (A/B, tests)
        self.use_graph = True             # decode steps replayed from hipGraphs (decode_step)
        self.graphs = {}
        self.prefill_unpack = True        # fp8 prefill as unpack + tiled GEMM (A/B knob)
        # fp8 decode (M <= 32) through zs_fp8_gemm_run: gate|up with the SiLU * up epilogue in one
        # launch (GLU), the other projections as (ks splits, 1 / kh of a split) per workgroup
        # (A/B knobs; False: zs_fp8_gemm_rows + zs_mistral_silu_mul)
        self.fused_glu = True
        self.run_cfg = {"qkv": (1, 1), "o": (1, 2), "down": (2, 1)}
        self._wb = None
        ly0 = w.layers[0]
        self._wb_need = max(ly0[k]["N"] * ly0[k]["K"] for k in ("qkv", "o", "gu", "down"))
        self.Lmax = max_prompt + max_new + 1
        Mp = max_batch * max_prompt
        D, H, KVH, HD, F = w.D, w.H, w.KVH, w.HD, w.F
        self.nqkv = (H + 2 * KVH) * HD
        self.x = torch.empty(Mp, D, device=dev)
        self.h = torch.empty(Mp, D, device=dev, dtype=adt)
        self.q = torch.empty(Mp, H * HD, device=dev, dtype=adt)
        self.att = torch.empty(Mp, H * HD, device=dev, dtype=adt)
        self.act = torch.empty(Mp, F, device=dev, dtype=adt)
        # f32 result slabs: decode (M = B <= 64 rows) writes nsplit split-K slabs of B rows; the
        # fp8 prefill (unpack + one tiled GEMM, prefill_unpack) writes one slab of M = B P rows;
        # only the 64-row-chunk fp8 prefill (prefill_unpack False, an A/B knob) needs nsplit x Mp
        # rows, and _gemm grows the slab for it on demand (at 7B: 14 x 2048 x 28672 f32 = 3.3 GB)
        self.nsplit = max(self._splits(w.D), self._splits(F))
        self.slab_ncol = max(self.nqkv, 2 * F, D)
        self.slab = torch.empty(max(self.nsplit * max_batch, Mp) * self.slab_ncol, device=dev)
        self.kc = [torch.empty(max_batch, KVH, self.Lmax, HD, device=dev, dtype=adt) for _ in w.layers]
        self.vc = [torch.empty(max_batch, KVH, self.Lmax, HD, device=dev, dtype=adt) for _ in w.layers]
        inv = 1.0 / (w.theta ** (torch.arange(0, HD, 2, dtype=torch.int64).float() / HD))
        fr = torch.arange(self.Lmax, dtype=torch.float32)[:, None] * inv[None]
        self.cos = fr.cos().to(dev).contiguous()
        self.sin = fr.sin().to(dev).contiguous()
        i32 = dict(device=dev, dtype=torch.int32)
        self.pos = torch.zeros(Mp, **i32)
        self.next_tok = torch.zeros(max_batch, **i32)
        self.done = torch.zeros(max_batch, **i32)
        self.out_ids = torch.zeros(max_batch, max_new, **i32)
        self.out_len = torch.zeros(max_batch, **i32)
        self.step_ctr = torch.zeros(1, **i32)
        self.all_done = torch.zeros(3, **i32)
        self.nblk = ops.lmhead_nblk(w.V)
        self.pval = torch.empty(max_batch, self.nblk, 1, device=dev)
        self.pidx = torch.empty(max_batch, self.nblk, 1, device=dev, dtype=torch.int32)
        self.last = torch.empty(max_batch, D, device=dev, dtype=adt)
        # decode rows before an RMSNorm folded into the next GEMM (zs_mistral_add_ss): bf16 x and
        # the per-512-column partial sums of squares [8][32]
        self.xb = torch.empty(max_batch, D, device=dev, dtype=torch.bfloat16)
        self.rss = torch.empty(8 * 32, device=dev)

    def _wscratch(self, N, K):
        """bf16 [N][K] scratch for one unpacked weight matrix (the largest: gate|up)."""
        if self._wb is None or self._wb.numel() < N * K:
            self._wb = torch.empty(max(N * K, self._wb_need), device=self.w.dev,
                                   dtype=torch.bfloat16)
        return self._wb[:N * K].view(N, K)

    def _splits(self, K):
        return call("zs_fp8_splits", K) if self.w.mode == "fp8" else 1

    def _gemm(self, a, lw, M):
        """f32 result slabs of a @ W^T for M rows: (slab tensor, nsplit, split stride)."""
        N, K = lw["N"], lw["K"]
        if self.w.mode == "fp8" and M > 64 and self.prefill_unpack:
            # prefill: codes -> bf16 once per matrix, one tiled MFMA GEMM over all M rows, then
            # the per-channel scales (the row kernel would re-stream the weights per 64 rows)
            st = torch.cuda.current_stream().cuda_stream
            wb = self._wscratch(N, K)
            call("zs_fp8_unpack_bf16", lw["w8"].data_ptr(), N, K, wb.data_ptr(), st)
            out = self.slab[:M * N].view(M, N)
            ops.gemm(a[:M], wb, out, split_k=1)
            call("zs_scale_cols", out.data_ptr(), M, N, N, lw["scale"].data_ptr(), st)
            return out, 1, M * N
        if self.w.mode == "fp8":
            ns = self._splits(K)
            ss = M * N
            if self.slab.numel() < ns * ss:      # (captured decode graphs point at the old slab)
                self.slab = torch.empty(ns * ss, device=self.w.dev)
                self.graphs.clear()
            out = self.slab[:ns * ss]
            for m0 in range(0, M, 64):
                mm = min(64, M - m0)
                call("zs_fp8_gemm_rows", a[m0:].data_ptr(), a.stride(0), lw["w8"].data_ptr(),
                     lw["scale"].data_ptr(), mm, N, K, out[m0 * N:].data_ptr(), ss, N,
                     torch.cuda.current_stream().cuda_stream)
            return out, ns, ss
        out = self.slab[:M * N].view(M, N)
        ops.gemm(a[:M], lw["w"], out, split_k=1)
        return out, 1, M * N

    def _gemm_run(self, a, lw, M, name, normed=False, act=None):
        """Decode GEMM through zs_fp8_gemm_run (fp8, M <= 32): (slab tensor, nslab, stride).
        normed: ``a`` is xb and the RMSNorm factor comes from rss (zs_mistral_add_ss); act: the
        GLU form writing silu(gate) * up there."""
        N, K = lw["N"], lw["K"]
        ks, kh = (self._splits(K), 1) if act is not None else self.run_cfg[name]
        if self._splits(K) % ks:
            ks = 1
        ns, ss = self._splits(K) // ks * kh, M * N
        y = self.slab[:ns * ss]
        call("zs_fp8_gemm_run", a.data_ptr(), a.stride(0), lw["w8"].data_ptr(),
             lw["scale"].data_ptr(), M, N, K, ks, kh, None if act is not None else y.data_ptr(),
             ss, N, act.data_ptr() if act is not None else None,
             act.stride(0) if act is not None else 0, self.rss.data_ptr() if normed else None,
             self.w.D // 512, float(self.w.eps), torch.cuda.current_stream().cuda_stream)
        return y, ns, ss

    def _add_ss(self, M, y, ns, ss):
        call("zs_mistral_add_ss", self.x.data_ptr(), y.data_ptr() if y is not None else None, ns,
             ss, M, self.w.D, self.xb.data_ptr(), self.rss.data_ptr(),
             torch.cuda.current_stream().cuda_stream)

    def _norm(self, M, y, ns, ss, w):
        call("zs_mistral_add_rmsnorm", self.x.data_ptr(), y.data_ptr() if y is not None else None,
             ns, ss, M, self.w.D, float(self.w.eps), w.data_ptr() if w is not None else None,
             self.h.data_ptr(), ops.dt(self.h), torch.cuda.current_stream().cuda_stream)

    def _layers(self, M, rows_per_seq):
        w, st = self.w, torch.cuda.current_stream().cuda_stream
        dt = ops.dt(self.h)
        nl = len(w.layers)
        # decode through zs_fp8_gemm_run: every RMSNorm but the last as zs_mistral_add_ss + the
        # consuming GEMM's row factor; the last one (the LM head's input h) as before
        run = (self.fused_glu and w.mode == "fp8" and rows_per_seq == 1 and M <= 32
               and w.D % 512 == 0 and w.D <= 4096)
        if run:
            self._add_ss(M, None, 1, 0)
        else:
            self._norm(M, None, 1, 0, w.layers[0]["ln1"])
        for l, ly in enumerate(w.layers):
            y, ns, ss = (self._gemm_run(self.xb, ly["qkv"], M, "qkv", normed=True) if run else
                         self._gemm(self.h, ly["qkv"], M))
            if rows_per_seq == 1 and self.fused_decode_attn:    # decode: RoPE + append + attention
                call("zs_mistral_decode_attention", y.data_ptr(), ns, ss, M, w.H, w.KVH,
                     self.pos.data_ptr(), self.cos.data_ptr(), self.sin.data_ptr(),
                     self.kc[l].data_ptr(), self.vc[l].data_ptr(), self.Lmax,
                     self.att.data_ptr(), dt, st)
            else:                                                # prefill: P rows per sequence
                call("zs_mistral_rope_kv", y.data_ptr(), ns, ss, M, w.H, w.KVH,
                     self.pos.data_ptr(), rows_per_seq, self.cos.data_ptr(), self.sin.data_ptr(),
                     self.q.data_ptr(), self.kc[l].data_ptr(), self.vc[l].data_ptr(), self.Lmax,
                     dt, st)
                call("zs_mistral_attention", self.q.data_ptr(), M, w.H, w.KVH,
                     self.pos.data_ptr(), rows_per_seq, self.kc[l].data_ptr(),
                     self.vc[l].data_ptr(), self.Lmax, self.att.data_ptr(), dt, st)
            if run:
                y, ns, ss = self._gemm_run(self.att, ly["o"], M, "o")
                self._add_ss(M, y, ns, ss)
                self._gemm_run(self.xb, ly["gu"], M, "gu", normed=True, act=self.act)
                y, ns, ss = self._gemm_run(self.act, ly["down"], M, "down")
                if l + 1 < nl:
                    self._add_ss(M, y, ns, ss)
                    continue
            else:
                y, ns, ss = self._gemm(self.att, ly["o"], M)
                self._norm(M, y, ns, ss, ly["ln2"])
                y, ns, ss = self._gemm(self.h, ly["gu"], M)
                call("zs_mistral_silu_mul", y.data_ptr(), ns, ss, M, w.F, self.act.data_ptr(), dt,
                     st)
                y, ns, ss = self._gemm(self.act, ly["down"], M)
            self._norm(M, y, ns, ss, w.layers[l + 1]["ln1"] if l + 1 < nl else w.lnf)

    def _lm_argmax(self, a, B):
        ops.lmhead_topk(a, self.w.lm, 1, None, self.pval, self.pidx, M=B)

    def generate(self, hard_ids: torch.Tensor, soft: torch.Tensor, tail_ids: torch.Tensor,
                 max_length: int = 60, eos: int = 2) -> List[List[int]]:
        """hard_ids [B, H] int32 (padded with 0 like padding_captions), soft [B, ns, D] f32 (the
        mapper rows), tail_ids [nt] int32 (the language tag's token ids) -> per sequence the
        generated ids up to and including eos (HF generate with inputs_embeds: at most
        max_length - P new tokens, finished rows padded, special tokens dropped by the caller)."""
        w, st = self.w, torch.cuda.current_stream().cuda_stream
        B, H = hard_ids.shape
        ns, nt = soft.shape[1], tail_ids.numel()
        P = H + ns + nt
        new = max_length - P
        if B > self.B or P > self.Pmax or new > self.max_new:
            raise ValueError(f"mistral generate: B={B} P={P} new={new} exceeds the engine")
        if new <= 0:
            return [[] for _ in range(B)]
        M = B * P
        call("zs_mistral_embed", hard_ids.data_ptr(), H, soft.data_ptr(), ns, tail_ids.data_ptr(),
             nt, None, w.emb.data_ptr(), w.D, M, self.x.data_ptr(), ops.dt(w.emb), st)
        self.pos[:M].copy_(torch.arange(P, device=w.dev, dtype=torch.int32).repeat(B))
        self._layers(M, P)
        self.last[:B].copy_(self.h[:M].view(B, P, w.D)[:, P - 1])
        self._lm_argmax(self.last[:B], B)
        for t in (self.done, self.out_len, self.step_ctr, self.all_done, self.out_ids):
            t.zero_()
        self.pos[:B].fill_(P - 1)
        # max_steps = the row stride of out_ids (the loop below stops after `new` steps)
        ops.greedy_step(self.pval, self.pidx, B, self.nblk, self.step_ctr, self.max_new, eos, eos,
                        self.out_ids, self.out_len, self.done, self.pos, self.next_tok, self.all_done)
        for s in range(1, new):
            if s % 8 == 0 and int(self.all_done[0]):
                break
            self.decode_step(B, eos)
        ids, ln = self.out_ids[:B].cpu(), self.out_len[:B].cpu()
        return [ids[b, :int(ln[b])].tolist() for b in range(B)]

    # ---------------------------------------------------------------- async form (no host sync)
    def begin(self, hard_ids: torch.Tensor, soft: torch.Tensor, tail_ids: torch.Tensor,
              max_length: int = 60, eos: int = 2) -> bool:
        """:meth:`generate`'s prefill and step 0 enqueued on the current stream; then
        :meth:`advance` chunks of steps and :meth:`ready` / :meth:`ids` (generate_concurrent).
        Returns False when there is nothing to generate."""
        w, st = self.w, torch.cuda.current_stream().cuda_stream
        B, H = hard_ids.shape
        ns, nt = soft.shape[1], tail_ids.numel()
        P = H + ns + nt
        new = max_length - P
        if B > self.B or P > self.Pmax or new > self.max_new:
            raise ValueError(f"mistral begin: B={B} P={P} new={new} exceeds the engine")
        self._aB, self._anew, self._as, self._aeos = B, new, 1, eos
        if new <= 0:
            return False
        M = B * P
        call("zs_mistral_embed", hard_ids.data_ptr(), H, soft.data_ptr(), ns, tail_ids.data_ptr(),
             nt, None, w.emb.data_ptr(), w.D, M, self.x.data_ptr(), ops.dt(w.emb), st)
        self.pos[:M].copy_(torch.arange(P, device=w.dev, dtype=torch.int32).repeat(B))
        self._layers(M, P)
        self.last[:B].copy_(self.h[:M].view(B, P, w.D)[:, P - 1])
        self._lm_argmax(self.last[:B], B)
        for t in (self.done, self.out_len, self.step_ctr, self.all_done, self.out_ids):
            t.zero_()
        self.pos[:B].fill_(P - 1)
        ops.greedy_step(self.pval, self.pidx, B, self.nblk, self.step_ctr, self.max_new, eos, eos,
                        self.out_ids, self.out_len, self.done, self.pos, self.next_tok, self.all_done)
        return True

    def advance(self, n: int = 8):
        """Enqueue up to n more decode steps (the same steps generate's loop runs between its
        all-done checks), then an async copy of the all-done flag and an event after it."""
        stop = min(self._anew, self._as + n)
        while self._as < stop:
            self.decode_step(self._aB, self._aeos)
            self._as += 1
        if not hasattr(self, "_aflag"):
            self._aflag = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._aflag.copy_(self.all_done[:1], non_blocking=True)
        self._aev = torch.cuda.Event()
        self._aev.record()

    def ready(self) -> Optional[bool]:
        """None while the last advance is in flight; else True when generation is over."""
        if not self._aev.query():
            return None
        return bool(int(self._aflag[0])) or self._as >= self._anew

    def ids(self) -> List[List[int]]:
        B = self._aB
        ids, ln = self.out_ids[:B].cpu(), self.out_len[:B].cpu()
        return [ids[b, :int(ln[b])].tolist() for b in range(B)]

    def _step_body(self, B, eos):
        w, st = self.w, torch.cuda.current_stream().cuda_stream
        call("zs_mistral_embed", None, 0, None, 0, None, 0, self.next_tok.data_ptr(),
             w.emb.data_ptr(), w.D, B, self.x.data_ptr(), ops.dt(w.emb), st)
        self._layers(B, 1)
        self._lm_argmax(self.h[:B], B)
        ops.greedy_step(self.pval, self.pidx, B, self.nblk, self.step_ctr, self.max_new, eos, eos,
                        self.out_ids, self.out_len, self.done, self.pos, self.next_tok,
                        self.all_done)

    def decode_step(self, B: int, eos: int = 2):
        """One greedy step of B sequences (every operand on the device: token ids, positions, KV
        caches, stop flags), replayed from a hipGraph captured on first use per (B, eos): the
        ~290 launches of a 32-layer step are one graph launch instead of ~290 host round trips
        through the C-ABI."""
        if not self.use_graph:
            return self._step_body(B, eos)
        key = (B, eos, self.fused_decode_attn, self.fused_glu, tuple(sorted(self.run_cfg.items())))
        g = self.graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):                 # capture only: nothing runs here
                self._step_body(B, eos)
            self.graphs[key] = g
        g.replay()

    def hidden_states(self, embeds: torch.Tensor) -> torch.Tensor:
        """The final-norm hidden states of every row of ``embeds`` [B, P, D] (causal, positions
        0..P-1, the prefill of :meth:`generate`) as f32 [B, P, D]: the logits are ``h @ lm^T``
        (tests: logits and top-1 / top-2 margins along a sequence)."""
        w, st = self.w, torch.cuda.current_stream().cuda_stream
        B, P, _ = embeds.shape
        if B > self.B or P > self.Pmax:
            raise ValueError(f"mistral hidden_states: B={B} P={P} exceeds the engine")
        M = B * P
        x = embeds.float().contiguous()
        call("zs_mistral_embed", None, 0, x.data_ptr(), P, None, 0, None, w.emb.data_ptr(), w.D,
             M, self.x.data_ptr(), ops.dt(w.emb), st)
        self.pos[:M].copy_(torch.arange(P, device=w.dev, dtype=torch.int32).repeat(B))
        self._layers(M, P)
        return self.h[:M].float().view(B, P, w.D).clone()

    def generate_embeds(self, embeds: torch.Tensor, max_length: int = 60,
                        eos: int = 2) -> List[List[int]]:
        """HF ``generate(inputs_embeds=embeds, attention_mask=ones, do_sample=False, ...)`` from
        already assembled prompt rows [B, P, D] (the drop-in's entry point)."""
        B = embeds.shape[0]
        dev = self.w.dev
        empty = torch.zeros(B, 0, dtype=torch.int32, device=dev)
        return self.generate(empty, embeds.float().contiguous(), torch.zeros(0, dtype=torch.int32,
                                                                              device=dev),
                             max_length=max_length, eos=eos)


def generate_concurrent(decoders: Sequence["MistralDecoder"], streams: Sequence, jobs):
    """Several independent greedy generates at once, one decoder (sharing the weights) and one
    stream per job: jobs = [(hard_ids, soft, tail_ids, max_length)], each exactly
    :meth:`MistralDecoder.generate`'s result (the 3 language tags of a C5 batch co-run: every
    step of one is a chain of latency-bound launches the others' weight streams overlap).  The
    host never blocks on one job while another could be advanced."""
    assert len(decoders) >= len(jobs) and len(streams) >= len(jobs)
    caller = torch.cuda.current_stream()
    live = []
    for i, (hard, soft, tail, max_length) in enumerate(jobs):
        s = streams[i]
        s.wait_stream(caller)
        with torch.cuda.stream(s):
            if decoders[i].begin(hard, soft, tail, max_length):
                decoders[i].advance(7)       # generate checks all-done first at step 8
                live.append(i)
    out = [[[] for _ in range(hard.shape[0])] for hard, *_ in jobs]
    while live:
        progressed = False
        for i in list(live):
            r = decoders[i].ready()
            if r is None:
                continue
            progressed = True
            if r:
                with torch.cuda.stream(streams[i]):
                    out[i] = decoders[i].ids()
                live.remove(i)
            else:
                with torch.cuda.stream(streams[i]):
                    decoders[i].advance(8)
        if not progressed:
            time.sleep(20e-6)
    for s in streams[:len(jobs)]:
        caller.wait_stream(s)
    return out

