"""Thin, validated torch-tensor wrappers over the C-ABI (one function per zs_* entry point).

Tensors are device memory owned by the caller; every call is enqueued on the current torch
stream (``torch.cuda.current_stream()``), performs no allocation and no synchronisation, and is
therefore safe inside ``torch.cuda.graph`` capture.  Shape/dtype checks happen here on the host
before the launch (the kernels assume them).
"""
from __future__ import annotations

from typing import Optional

import torch

from ._lib import (ACT_GELU_ERF, ACT_GELU_TANH, ACT_NONE, ACT_RELU, ACT_TANH, ZS_BF16, ZS_F32,
                   ZsError, call)

__all__ = ["dt", "ACT_NONE", "ACT_GELU_ERF", "ACT_GELU_TANH", "ACT_RELU", "ACT_TANH"]


def dt(t) -> int:
    d = t.dtype if isinstance(t, torch.Tensor) else t
    if d == torch.float32:
        return ZS_F32
    if d == torch.bfloat16:
        return ZS_BF16
    raise ZsError(f"unsupported dtype {d} (float32 / bfloat16)")


def _p(t: Optional[torch.Tensor]):
    if t is None:
        return None
    if not t.is_cuda:
        raise ZsError("zsaac ops take device tensors (no CPU fallback)")
    return t.data_ptr()


def _s():
    return torch.cuda.current_stream().cuda_stream


def _need(cond, msg):
    if not cond:
        raise ZsError(msg)


def _i32(t, name):
    _need(t is None or t.dtype == torch.int32, f"{name} must be int32")


# ---------------------------------------------------------------- front end
def logmel(wav, tables, bn=None, out=None):
    """wav [B,T] f32 -> [B, T//320+1, 64] f32 (log-mel, optionally bn0'd)."""
    B, T = wav.shape
    nf = T // 320 + 1
    out = out if out is not None else torch.empty(B, nf, 64, device=wav.device)
    bm, bv, bw, bb = (bn if bn is not None else (None, None, None, None))
    call("zs_logmel", _p(wav), B, T, _p(tables["window"]), _p(tables["twiddle"]),
         _p(tables["melW"]), _p(tables["mel_lo"]), _p(tables["mel_hi"]), _p(bm), _p(bv), _p(bw),
         _p(bb), _p(out), _s())
    return out


def pack_clips(flat, offsets, lengths, T, out):
    """Ragged clips in one flat f32 device buffer -> out [B, T]: crop / zero-pad (zs_pack_clips)."""
    _need(flat.dtype == torch.float32 and offsets.dtype == torch.int64 and lengths.dtype == torch.int32,
          "pack_clips: flat f32, offsets int64, lengths int32")
    B = lengths.numel()
    _need(out.shape[0] >= B and out.shape[1] == T, "pack_clips: out [B, T]")
    call("zs_pack_clips", _p(flat), _p(offsets), _p(lengths), B, T, _p(out), _s())
    return out[:B]


def wav2img(logmel_t, out=None):
    B, T_in, F = logmel_t.shape
    _need(F == 64, "wav2img expects 64 mel bins")
    out = out if out is not None else torch.empty(B, 256, 256, device=logmel_t.device)
    call("zs_wav2img", _p(logmel_t), B, T_in, _p(out), _s())
    return out


def patch_embed(img, w, b, ln_w, ln_b, out=None):
    B = img.shape[0]
    out = out if out is not None else torch.empty(B * 4096, 96, device=img.device)
    call("zs_patch_embed", _p(img), B, _p(w), _p(b), _p(ln_w), _p(ln_b), _p(out), _s())
    return out


# ---------------------------------------------------------------- generic
def layernorm(x, w, b, out, eps=1e-5, rows=None, M=None):
    C = x.shape[-1]
    M = M if M is not None else (rows.numel() if rows is not None else x.numel() // C)
    _i32(rows, "rows")
    call("zs_layernorm", _p(x), M, C, x.stride(-2) if x.dim() > 1 else C, _p(rows), _p(w), _p(b),
         float(eps), _p(out), out.stride(-2) if out.dim() > 1 else C, dt(out), _s())
    return out


_SKINNY_WS = {}


def _devkey(device):
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device(dev.type, torch.cuda.current_device())
    return dev


SKINNY_MAX_M = 256     # gemm_skinny.hip SK_MAX_M (4 row blocks of 64)


def reserve_skinny_workspace(device, M, N, K):
    """Allocate (once, zeroed, before any graph capture) the workspace the auto-mode skinny GEMM
    (M <= SKINNY_MAX_M) needs for this shape; shared by every skinny GEMM on the device's stream order."""
    need = call("zs_gemm_workspace_floats", M, N, K)
    dev = _devkey(device)
    cur = _SKINNY_WS.get(dev)
    if need and (cur is None or cur.numel() < need):
        if cur is not None:
            _RETIRED.append(cur)     # a captured graph may still reference it: never free
        _SKINNY_WS[dev] = torch.zeros(max(need, 4 << 20), device=dev)
    return _SKINNY_WS.get(dev)


_RETIRED = []


def skinny_workspace(device, shapes):
    """A private zeroed workspace for the skinny GEMMs of one engine (one stream): sized for the
    largest of ``shapes`` [(M, N, K)].  Engines that may run concurrently on different streams
    must not share a workspace (its tile counters and slabs are per launch)."""
    need = max([call("zs_gemm_workspace_floats", M, N, K) for M, N, K in shapes] + [0])
    return torch.zeros(max(need, 1), device=device) if need else None


def gemm(a, w, out, bias=None, residual=None, act=ACT_NONE, split_k=0, workspace=None, M=None):
    """out = act(a @ w.T + bias) + residual;  a [M,K], w [N,K] (same dtype), out f32/bf16.
    split_k=0 (auto): M <= SKINNY_MAX_M uses the weight-streaming skinny kernel when a
    workspace is given or was reserved for the device (reserve_skinny_workspace), else the tiled
    kernel."""
    K = a.shape[-1]
    N = w.shape[0]
    M = M if M is not None else a.numel() // K
    _need(w.shape[1] == K and a.dtype == w.dtype, f"gemm: a{tuple(a.shape)} w{tuple(w.shape)}")
    _need(K % 32 == 0, f"gemm: K={K} must be a multiple of 32")
    if split_k == 0:
        need = call("zs_gemm_workspace_floats", M, N, K) if M <= SKINNY_MAX_M else 0
        if workspace is None and need:
            workspace = _SKINNY_WS.get(_devkey(a.device))
            if workspace is not None and need > workspace.numel():
                workspace = None
        elif workspace is not None and need > workspace.numel():
            # an engine's private workspace is sized for its decode shapes: M <= 64 must fit,
            # larger M simply takes the tiled kernel
            _need(M > 64, f"gemm: workspace {workspace.numel()} < {need} floats")
            workspace = None
        # bf16 M <= 64 keeps auto mode without a workspace: zs_gemm takes the row-group kernel
        # (no workspace), and the tiled kernel for shapes that kernel does not cover
        if workspace is None and not (a.dtype == torch.bfloat16 and M <= 64):
            split_k = 1
    lda = a.stride(-2) if a.dim() > 1 else K
    ldo = out.stride(-2) if out.dim() > 1 else N
    ldr = (residual.stride(-2) if residual.dim() > 1 else N) if residual is not None else 0
    _need(bias is None or bias.dtype == torch.float32, "gemm: bias must be f32")
    _need(residual is None or residual.dtype == torch.float32, "gemm: residual must be f32")
    call("zs_gemm", M, N, K, dt(a), _p(a), lda, _p(w), w.stride(0), _p(bias), _p(residual), ldr,
         _p(out), ldo, dt(out), act, split_k, _p(workspace), _s())
    return out


def gemm_ln(x, ln_w, ln_b, w, out, bias=None, residual=None, act=ACT_NONE, eps=1e-5):
    """out = act(LayerNorm(x) @ w.T + bias) + residual in one launch (zs_gemm_ln): x [M, K] f32
    rows (M <= 64), w [N, K] bf16.  The LN output is rounded to bf16 like the zs_layernorm ->
    zs_gemm pair it replaces.  ln_w = ln_b = None: normalise only (affine folded into w, bias)."""
    M, K = x.shape
    N = w.shape[0]
    _need(w.shape[1] == K and w.dtype == torch.bfloat16 and x.dtype == torch.float32,
          f"gemm_ln: x{tuple(x.shape)} {x.dtype} w{tuple(w.shape)} {w.dtype}")
    _need(bias is None or bias.dtype == torch.float32, "gemm_ln: bias must be f32")
    _need(residual is None or residual.dtype == torch.float32, "gemm_ln: residual must be f32")
    ldr = residual.stride(0) if residual is not None else 0
    call("zs_gemm_ln", M, N, K, _p(x), x.stride(0), _p(ln_w), _p(ln_b), float(eps), _p(w),
         w.stride(0), _p(bias), _p(residual), ldr, _p(out), out.stride(0), dt(out), act, _s())
    return out


def gemm_ln_f32(x, ln_w, ln_b, w, out, bias=None, residual=None, act=ACT_NONE, eps=1e-5):
    """out = act(LayerNorm(x) @ w.T + bias) + residual, all f32 (zs_gemm_ln_f32): x [M, K]
    (M <= 64), w [N, K] f32; the LN affine applied in f32 before the product.  ln_w = ln_b =
    None: no LayerNorm (the decode step's projections, K up to 3072)."""
    M, K = x.shape
    N = w.shape[0]
    _need(w.shape[1] == K and w.dtype == torch.float32 and x.dtype == torch.float32
          and out.dtype == torch.float32, f"gemm_ln_f32: x{tuple(x.shape)} w{tuple(w.shape)} {w.dtype}")
    _need((ln_w is None) == (ln_b is None), "gemm_ln_f32: LN weight and bias together")
    _need(bias is None or bias.dtype == torch.float32, "gemm_ln_f32: bias must be f32")
    ldr = residual.stride(0) if residual is not None else 0
    call("zs_gemm_ln_f32", M, N, K, _p(x), x.stride(0), _p(ln_w), _p(ln_b), float(eps), _p(w),
         w.stride(0), _p(bias), _p(residual), ldr, _p(out), out.stride(0), act, _s())
    return out


def l2norm(x, out=None, eps=1e-12):
    out = out if out is not None else torch.empty_like(x)
    C = x.shape[-1]
    call("zs_l2norm_rows", _p(x), x.numel() // C, C, float(eps), _p(out), _s())
    return out


def cast(x, out):
    _need(x.dtype == torch.float32 and x.numel() == out.numel(), "cast: f32 in, same numel")
    call("zs_cast", _p(x), x.numel(), _p(out), dt(out), _s())
    return out


# ---------------------------------------------------------------- HTSAT
def window_attention(qkv, B, H, W, C, heads, shift, rel_table, out, ws=8):
    call("zs_window_attention", _p(qkv), B, H, W, C, heads, ws, shift, _p(rel_table), _p(out),
         dt(qkv), _s())
    return out


def swin_block(x, B, H, W, C, heads, shift, blk):
    """One fused SwinTransformerBlock (htsat.py:427-474) in place on the f32 residual stream x
    [B*H*W, C]; blk holds the fragment-packed bf16 weights (encoder.HtsatWeights)."""
    _need(x.dtype == torch.float32 and x.is_contiguous(), "swin_block: x must be contiguous f32")
    call("zs_swin_block", _p(x), B, H, W, C, heads, shift, _p(blk["n1"][0]), _p(blk["n1"][1]),
         _p(blk["qkv_p"]), _p(blk["qkv_bp"]), _p(blk["rel"]), _p(blk["proj_p"]), _p(blk["proj_b"]),
         _p(blk["n2"][0]), _p(blk["n2"][1]), _p(blk["fc1_p"]), _p(blk["fc1_b"]), _p(blk["fc2_p"]),
         _p(blk["fc2_b"]), _s())
    return x


def patch_merge_ln(x, B, H, W, C, ln_w, ln_b, out):
    call("zs_patch_merge_ln", _p(x), B, H, W, C, _p(ln_w), _p(ln_b), _p(out), dt(out), _s())
    return out


def ln_meanpool(x, B, N, C, ln_w, ln_b, out):
    call("zs_ln_meanpool", _p(x), B, N, C, _p(ln_w), _p(ln_b), _p(out), _s())
    return out


# ---------------------------------------------------------------- CNN14
def conv3x3_bn_relu(x, B, H, W, Cin, w, Cout, scale, shift, out):
    call("zs_conv3x3_bn_relu", _p(x), B, H, W, Cin, _p(w), Cout, _p(scale), _p(shift), _p(out),
         dt(x), _s())
    return out


def avgpool2(x, B, H, W, C, out):
    call("zs_avgpool2", _p(x), B, H, W, C, _p(out), dt(x), _s())
    return out


def cnn_head(x, B, H, W, C, out):
    call("zs_cnn_head", _p(x), B, H, W, C, _p(out), dt(x), _s())
    return out


# ---------------------------------------------------------------- prompt / mapper
def prompt_assemble(emb, labels, k, label_tok, label_len, hard_ids, hard_len, chosen=None):
    B, D = emb.shape
    L = labels.shape[0]
    for t, n in ((label_tok, "label_tok"), (label_len, "label_len"), (hard_ids, "hard_ids"),
                 (hard_len, "hard_len"), (chosen, "chosen")):
        _i32(t, n)
    call("zs_prompt_assemble", _p(emb), B, D, _p(labels), L, k, _p(label_tok), _p(label_len),
         label_tok.shape[1], _p(hard_ids), hard_ids.shape[1], _p(hard_len), _p(chosen), _s())


def row_attention(q, ldq, k, v, ldkv, B, L, heads, hd, causal, scale, out, ldo, lens=None):
    _i32(lens, "lens")
    call("zs_row_attention", _p(q), ldq, _p(k), _p(v), ldkv, B, L, _p(lens), heads, hd,
         int(causal), float(scale), _p(out), ldo, dt(out), _s())
    return out


# ---------------------------------------------------------------- GPT-2
def prefill_embed(hard_ids, hard_len, soft, soft_ld, n_soft, wte, wpe, B, Pmax, embed, x, plen,
                  last_row):
    D = wte.shape[1]
    call("zs_gpt2_prefill_embed", _p(hard_ids), _p(hard_len), hard_ids.shape[1], _p(soft),
         soft_ld, n_soft, _p(wte), _p(wpe), B, Pmax, D, _p(embed), _p(x), _p(plen),
         _p(last_row), dt(wte), _s())


def row_attention_kv(qkv, B, L, heads, scale, out, kc, vc, Lmax, lens, row_stride=1):
    """Causal prefill attention over qkv [B*L, 3*heads*64] bf16 fused with the KV-cache write
    (zs_row_attention_kv: kv_write + row_attention of one layer in one launch, L <= 32)."""
    _i32(lens, "lens")
    call("zs_row_attention_kv", _p(qkv), B, L, _p(lens), heads, float(scale), _p(out),
         out.stride(0), _p(kc), _p(vc), Lmax, row_stride, _s())
    return out


def greedy_init(R, plen, pos, done, out_len, out_ids, max_steps, step_ctr, all_done):
    """generate2's state before step 0 in one launch (zs_greedy_init)."""
    call("zs_greedy_init", R, _p(plen), _p(pos), _p(done), _p(out_len), _p(out_ids), max_steps,
         _p(step_ctr), _p(all_done), _s())


def kv_write(qkv, R, n, D, heads, kc, vc, Lmax, pos0=None, row_stride=1):
    call("zs_kv_write", _p(qkv), R, n, D, heads, _p(pos0), row_stride, _p(kc), _p(vc), Lmax,
         dt(qkv), _s())


def decode_attention(qkv, R, D, heads, kc, vc, Lmax, pos, out, kvrow=None):
    call("zs_decode_attention", _p(qkv), R, D, heads, _p(kc), _p(vc), Lmax, _p(pos), _p(kvrow),
         _p(out), dt(qkv), _s())
    return out


def cross_attention(q, k, v, B, Lq, Lk, heads, out, scale=None):
    """softmax(scale q k^T) v per (row, query, head) for Lk <= 64 keys (zs_cross_attention):
    q [B*Lq, heads*hd], k / v [B*Lk, heads*hd] (row strides taken from the tensors)."""
    D = q.shape[-1]
    hd = D // heads
    _need(D % heads == 0 and q.dtype == k.dtype == v.dtype == out.dtype, "cross_attention: shapes")
    _need(k.stride(0) == v.stride(0), "cross_attention: k and v share a row stride")
    scale = hd ** -0.5 if scale is None else scale
    call("zs_cross_attention", _p(q), q.stride(0), _p(k), _p(v), k.stride(0), B, Lq, Lk, heads, hd,
         float(scale), _p(out), out.stride(0), dt(q), _s())
    return out


def label_topk(emb, labels, k, rows, idx=None):
    """sound_effect_choice: the k most similar label rows per embedding (zs_label_topk):
    emb [B, D] f32, labels [L, D] f32 -> rows [B, k, D] f32 (+ idx [B, k] int32)."""
    B, D = emb.shape
    _i32(idx, "idx")
    call("zs_label_topk", _p(emb), B, D, _p(labels), labels.shape[0], k, _p(idx), _p(rows), _s())
    return rows


def stream_spin(us: int, stream=None):
    """Hold the (current) stream for `us` microseconds on the GPU (zs_stream_spin)."""
    call("zs_stream_spin", int(us), (stream or torch.cuda.current_stream()).cuda_stream)


def dedicated_streams(n: int, device, priority: int = 0) -> list:
    """n new HIP streams bound to distinct hardware queues (zs_stream_create), as torch streams.
    torch's pooled streams get their hardware queue at first use, so concurrent batch streams
    can silently land on one queue and serialize.  priority < 0: the highest stream priority,
    > 0: the lowest."""
    import ctypes as C
    out = []
    with torch.cuda.device(device):
        for _ in range(n):
            h = C.c_void_p()
            call("zs_stream_create", C.byref(h), int(priority))
            out.append(torch.cuda.ExternalStream(h.value, device=device))
    return out


def cu_split_masks(cus: int, n_begin: int):
    """(begin mask, grid mask) as lists of 32-bit words: n_begin of the device's cus CUs for the
    begins, the rest for the decode grids.  The begin CUs are taken evenly over the bit range in
    a pattern that lands on every XCD whether the driver deals mask bits to XCDs in blocks of
    cus / 8 or round-robin: bit i when ((i >> 3) & 3) == (i & 3) (a quarter of the CUs), trimmed
    or padded in bit order to n_begin."""
    words = (cus + 31) // 32
    pick = [i for i in range(cus) if ((i >> 3) & 3) == (i & 3)]
    rest = [i for i in range(cus) if i not in set(pick)]
    chosen = set((pick + rest)[:n_begin])
    b = [0] * words
    g = [0] * words
    for i in range(cus):
        (b if i in chosen else g)[i // 32] |= 1 << (i % 32)
    return b, g


def masked_streams(n: int, device, mask) -> list:
    """n new HIP streams on the CUs of ``mask`` (zs_stream_create_masked), as torch streams."""
    import ctypes as C
    arr = (C.c_uint * len(mask))(*mask)
    out = []
    with torch.cuda.device(device):
        for _ in range(n):
            h = C.c_void_p()
            call("zs_stream_create_masked", C.byref(h), arr, len(mask))
            out.append(torch.cuda.ExternalStream(h.value, device=device))
    return out


def decode_attention_map(qkv, R, rowmap, nphys, D, heads, kc, vc, Lmax, pos, out, cpos=None):
    """decode_attention over compact slots c < R whose physical row is rowmap[c]."""
    call("zs_decode_attention_map", _p(qkv), R, _p(rowmap), nphys, D, heads, _p(kc), _p(vc), Lmax,
         _p(pos), _p(cpos), _p(out), dt(qkv), _s())
    return out


def embed_tokens_map(tok, pos, rowmap, nphys, wte, wpe, x, R, cpos=None):
    call("zs_embed_tokens_map", _p(tok), _p(pos), _p(rowmap), nphys, _p(wte), _p(wpe), R,
         wte.shape[1], _p(x), _p(cpos), dt(wte), _s())
    return x


def compact_rows(done, nrows, rowmap, n_active):
    call("zs_compact_rows", _p(done), nrows, _p(rowmap), _p(n_active), _s())


def embed_tokens(tok, pos, wte, wpe, x, R=None):
    R = R if R is not None else tok.numel()
    call("zs_embed_tokens", _p(tok), _p(pos), _p(wte), _p(wpe), R, wte.shape[1], _p(x), dt(wte),
         _s())
    return x


def lmhead_nblk(V: int) -> int:
    return call("zs_lmhead_nblk", V)


def lmhead_topk(a, w, topk, part_stat, part_val, part_idx, row_norm=False, M=None,
                temperature=1.0):
    K = a.shape[-1]
    M = M if M is not None else a.numel() // K
    _need(a.dtype == w.dtype and w.shape[1] == K, "lmhead: dtype/shape mismatch")
    _need(temperature > 0, "lmhead: temperature > 0")
    call("zs_lmhead_topk_t", M, K, w.shape[0], dt(a), _p(a), a.stride(-2) if a.dim() > 1 else K,
         _p(w), topk, int(row_norm), float(temperature), _p(part_stat), _p(part_val),
         _p(part_idx), _s())


def argmax_finalize(part_val, part_idx, M, nblk, idx):
    call("zs_argmax_finalize", _p(part_val), _p(part_idx), M, nblk, _p(idx), _s())
    return idx


def prefix_ids_assemble(hard_ids, hard_len, soft_idx, n_soft, B, Pmax, out):
    _i32(hard_ids, "hard_ids"), _i32(hard_len, "hard_len"), _i32(soft_idx, "soft_idx"), _i32(out, "out")
    call("zs_prefix_ids_assemble", _p(hard_ids), hard_ids.shape[-1], _p(hard_len), _p(soft_idx),
         n_soft, B, Pmax, _p(out), _s())
    return out


def greedy_step(part_val, part_idx, R, nblk, step_ctr, max_steps, stop0, stop1, out_ids, out_len,
                done, pos, next_tok, all_done):
    call("zs_greedy_step", _p(part_val), _p(part_idx), R, nblk, _p(step_ctr), max_steps, stop0,
         stop1, _p(out_ids), _p(out_len), _p(done), _p(pos), _p(next_tok), _p(all_done), _s())


def greedy_step_map(part_val, part_idx, R, rowmap, nphys, nblk, step_ctr, max_steps, stop0,
                    stop1, out_ids, out_len, done, pos, next_tok, all_done):
    call("zs_greedy_step_map", _p(part_val), _p(part_idx), R, _p(rowmap), nphys, nblk,
         _p(step_ctr), max_steps, stop0, stop1, _p(out_ids), _p(out_len), _p(done), _p(pos),
         _p(next_tok), _p(all_done), _s())


def beam_step(part_stat, part_val, part_idx, C, beam, nblk, topk, first, stop, step_ctr,
              max_steps, scores, seq_len, stopped, tokens, tokens_tmp, kvrow, kvrow_tmp, Lmax,
              pos, next_tok, all_done):
    call("zs_beam_step", _p(part_stat), _p(part_val), _p(part_idx), C, beam, nblk, topk,
         int(first), stop, _p(step_ctr), max_steps, _p(scores), _p(seq_len), _p(stopped),
         _p(tokens), _p(tokens_tmp), _p(kvrow), _p(kvrow_tmp), Lmax, _p(pos), _p(next_tok),
         _p(all_done), _s())


# ---------------------------------------------------------------- CLAP text tower + magic decoding
def bert_embed_ln(ids, L, word, pos, type0, ln_w, ln_b, x, h=None, eps=1e-12):
    """ids [T*L] int32 -> x f32 [T*L, 768] (+ operand copy h): BertEmbeddings + LayerNorm."""
    _i32(ids, "ids")
    rows = ids.numel()
    call("zs_bert_embed_ln", _p(ids), rows, L, _p(word), _p(pos), _p(type0), _p(ln_w), _p(ln_b),
         float(eps), _p(x), _p(h), dt(h) if h is not None else ZS_F32, _s())
    return x


def layernorm_dual(y, ln_w, ln_b, x, h=None, eps=1e-12, M=None):
    C = y.shape[-1]
    M = M if M is not None else y.numel() // C
    call("zs_layernorm_dual", _p(y), M, C, y.stride(0), _p(ln_w), _p(ln_b), float(eps), _p(x),
         x.stride(0), _p(h), h.stride(0) if h is not None else C,
         dt(h) if h is not None else ZS_F32, _s())
    return x


def row_topk(logits, k, out_val, out_idx, mode=0, R=None, V=None):
    """top-k of each logits row with log(softmax) (mode 0) or softmax (mode 1) values."""
    _need(logits.dtype == torch.float32, "row_topk: f32 logits")
    _i32(out_idx, "out_idx")
    R = R if R is not None else logits.shape[0]
    V = V if V is not None else logits.shape[1]
    call("zs_row_topk", _p(logits), R, V, logits.stride(0), k, mode, _p(out_val), _p(out_idx), _s())
    return out_val, out_idx


def magic_expand(kvrow, pos, nbeams, W, Lmax, kvrow_c, pos_c):
    for t, n in ((kvrow, "kvrow"), (pos, "pos"), (kvrow_c, "kvrow_c"), (pos_c, "pos_c")):
        _i32(t, n)
    call("zs_magic_expand", _p(kvrow), _p(pos), nbeams, W, Lmax, _p(kvrow_c), _p(pos_c), _s())


def magic_maxcos(hid, ncand, W, ctx, Lmax, kvrow, pos, maxcos):
    _need(hid.dtype == ctx.dtype, "magic_maxcos: hid / ctx dtype")
    call("zs_magic_maxcos", _p(hid), ncand, W, _p(ctx), Lmax, _p(kvrow), _p(pos), _p(maxcos),
         dt(hid), _s())
    return maxcos


def magic_score(pval, maxcos, text, audio, C, b, W, nact, temp, alpha, beta, score,
                score_temp=1.0):
    E = audio.shape[-1]
    call("zs_magic_score_t", _p(pval), _p(maxcos), _p(text), _p(audio), C, E, b, W, nact,
         float(temp), float(alpha), float(beta), float(score_temp), _p(score), _s())
    return score


def magic_step(score, cand, C, b, W, first, greedy, stop, step, max_steps, scores, seq_len,
               stopped, tokens, kvrow, pos, cdone, ntok, hid, sel_h):
    _need(hid.dtype == sel_h.dtype, "magic_step: hid / sel_h dtype")
    call("zs_magic_step", _p(score), _p(cand), C, b, W, int(first), int(greedy), stop, step,
         _p(max_steps), _p(scores), _p(seq_len), _p(stopped), _p(tokens), tokens.shape[1],
         _p(kvrow), kvrow.shape[1], _p(pos), _p(cdone), _p(ntok), _p(hid), _p(sel_h), dt(hid), _s())


# ---------------------------------------------------------------- greedy decode on a grid (bs <= 64)
PERSIST_GRIDS = (48, 96, 192)     # workgroups of 256 threads (half a CU each) per launch


def decode_persist_workspace(device) -> torch.Tensor:
    n = call("zs_decode_persist_workspace_bytes")
    return torch.zeros(n + 256, dtype=torch.uint8, device=device)


def decode_persist_grid(grid: int = 48) -> int:
    """Workgroups of one zs_gpt2_decode_persist launch (48, 96 or 192, each 256 threads)."""
    _need(grid in PERSIST_GRIDS, f"decode grid {grid} (one of {PERSIST_GRIDS})")
    return grid


def pack_b_fragments(W: torch.Tensor) -> torch.Tensor:
    """W [N][K] (bf16, K % 32 == 0) -> MFMA 16x16x32 B-fragment order [ceil(N/16)][K/32][64][8]:
    block j, k-step s, lane l holds W[16 j + l % 16][32 s + 8 (l // 16) .. + 8]; rows past N are
    zero.  One KiB per (block, k-step): each wave-load of a fragment is contiguous."""
    N, K = W.shape
    _need(K % 32 == 0, "pack_b_fragments: K % 32")
    Np = -(-N // 16) * 16
    Wp = torch.zeros(Np, K, dtype=W.dtype, device=W.device)
    Wp[:N] = W
    return (Wp.view(Np // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
            .view(Np // 16, K // 32, 64, 8))


def pack_f32_fragments(W: torch.Tensor) -> torch.Tensor:
    """W [N][K] (f32, K % 16 == 0) -> the f32 grid decode's fragment order
    [ceil(N/16)][K/16][64][4]: block j, k-step s, lane l holds W[16 j + l % 16][16 s + 4 (l // 16)
    .. + 4] (v_mfma_f32_16x16x4_f32, four MFMAs per fragment); rows past N are zero."""
    N, K = W.shape
    _need(W.dtype == torch.float32 and K % 16 == 0, "pack_f32_fragments: f32, K % 16")
    Np = -(-N // 16) * 16
    Wp = torch.zeros(Np, K, dtype=W.dtype, device=W.device)
    Wp[:N] = W
    return (Wp.view(Np // 16, 16, K // 16, 4, 4).permute(0, 2, 3, 1, 4).contiguous()
            .view(Np // 16, K // 16, 64, 4))


def decode_persist_f32_workspace(device) -> torch.Tensor:
    n = call("zs_decode_persist_f32_workspace_bytes")
    return torch.zeros(n + 256, dtype=torch.uint8, device=device)


PERSIST_GRIDS_F32 = (192,)


def _decode_grid_args(R, Lmax, max_steps, stop0, stop1, V, wte, wpe, wte_packed, temperature,
                      layer_ptrs, lm_bias, kv_ptrs, pos, next_tok, done, out_ids, out_len,
                      step_ctr, all_done, ws, grid, f32=False):
    _need(1 <= R <= 64, "gpt2 decode grid: 1 <= R <= 64")
    dt = torch.float32 if f32 else torch.bfloat16
    _need(wte.dtype == dt and wpe.dtype == dt and wte_packed.dtype == dt,
          f"gpt2 decode grid: {dt} wte / wpe / wte_packed")
    for t, n in ((pos, "pos"), (next_tok, "next_tok"), (done, "done"), (out_ids, "out_ids"),
                 (out_len, "out_len"), (step_ctr, "step_ctr"), (all_done, "all_done")):
        _i32(t, n)
    _need(out_ids.shape[-1] == max_steps, "gpt2 decode grid: out_ids [R, max_steps]")
    nb = (1 if f32 else 2) * (-(-V // 16) * 16)
    _need(lm_bias.dtype == torch.float32 and lm_bias.numel() >= nb,
          f"gpt2 decode grid: lm_bias f32 [{nb}]")
    _need(temperature > 0, "gpt2 decode grid: temperature > 0")
    if f32:
        _need(grid in PERSIST_GRIDS_F32, f"f32 decode grid {grid} (one of {PERSIST_GRIDS_F32})")
    else:
        decode_persist_grid(grid)
    base = ws.data_ptr()
    off = (-base) % 256
    return (R, Lmax, max_steps, stop0, stop1, V, _p(wte), _p(wpe), _p(wte_packed),
            float(temperature), layer_ptrs, _p(lm_bias), kv_ptrs, _p(pos), _p(next_tok), _p(done),
            _p(out_ids), _p(out_len), _p(step_ctr), _p(all_done), base + off, ws.numel() - off)


def gpt2_decode_persist(*args, grid=48, exclusive=False):
    """The remaining greedy steps of one bs <= 64 batch in one persistent launch
    (zs_gpt2_decode_persist) of `grid` 256-thread workgroups (`exclusive`: one per CU at most
    among exclusive launches).  Arguments as _decode_grid_args (layer_ptrs / kv_ptrs: ctypes
    arrays of 96 / 24 device pointers; the weights in fragment order,
    Gpt2Weights.packed_layer_ptrs)."""
    call("zs_gpt2_decode_persist", *_decode_grid_args(*args, grid), int(grid), int(bool(exclusive)),
         _s())


def gpt2_decode_phases(*args, steps=1, grid=96):
    """`steps` decode steps of the same computation as phase launches (zs_gpt2_decode_phases:
    bit-identical to the persistent launch at any grid; graph-capturable)."""
    call("zs_gpt2_decode_phases", *_decode_grid_args(*args, grid), int(steps), int(grid), _s())


def gpt2_decode_persist_f32(*args, grid=192, exclusive=False):
    """gpt2_decode_persist in f32 (zs_gpt2_decode_persist_f32: the parity mode; weights in f32
    fragment order, Gpt2Weights.packed_layer_ptrs of an f32 model)."""
    call("zs_gpt2_decode_persist_f32", *_decode_grid_args(*args, grid, f32=True), int(grid),
         int(bool(exclusive)), _s())


def gpt2_decode_phases_f32(*args, steps=1, grid=192):
    """The f32 decode's phase launches (zs_gpt2_decode_phases_f32, bit-identical to the persistent
    f32 launch)."""
    call("zs_gpt2_decode_phases_f32", *_decode_grid_args(*args, grid, f32=True), int(steps),
         int(grid), _s())
