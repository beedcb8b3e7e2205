"""Prefix mappers + GPT-2 decode (greedy / beam, KV cache) on the HIP kernels.

Replaces, for a whole batch of clips at once:
  * ``MLP`` / ``TransformerMapper`` (models/mapper.py) and ``clap_to_gpt``
    (models/caption_model.py:315-329),
  * ``get_prefix_tokens`` (gpt2_prefix_eval.py:271-278),
  * ``generate2`` (gpt2_prefix_eval.py:161-222) and ``generate_beam`` (99-158).

The reference decodes one clip at a time and recomputes the whole sequence every step
(``model.gpt(inputs_embeds=generated)``); here every clip is a row of a batched KV-cache decode
with per-row prompt lengths and positions.  Stop handling, tie rules and the beam arithmetic are
kept.  The per-step work — embed, 12 blocks, ln_f, LM head + row reduction, step
bookkeeping — runs on device and is captured once into a hipGraph (``torch.cuda.CUDAGraph``) that
is replayed until every row has stopped; the host only checks a flag every ``chunk`` steps.
"""
from __future__ import annotations

import copy
import math
import os
from typing import Dict, List, Optional, Tuple

import torch

from . import ops

# bench.py sets a list here: every persistent decode launch then appends (start event, end event,
# id(decoder)), recorded on the launching stream around the launch (the roofline's live timing)
PERSIST_LOG: Optional[list] = None

D, NH, HD, NL = 768, 12, 64, 12
STOP_DOT, STOP_SPACE_DOT = 13, 764


def _f32(t, dev):
    return t.detach().to(device=dev, dtype=torch.float32).contiguous()


def _w(t, dev, dtype):
    return t.detach().to(device=dev, dtype=dtype).contiguous()


# ------------------------------------------------------------------------------- mappers
class MlpMapper:
    """MLP((1024, 3840, 7680)) + Tanh (mapper.py:6-18): prefix [B,1024] -> soft [B, 10*768]."""

    def __init__(self, sd, device, dtype, max_batch, prefix="clap_project.model."):
        self.dtype = dtype
        self.w0, self.b0 = _w(sd[prefix + "0.weight"], device, dtype), _f32(sd[prefix + "0.bias"], device)
        self.w2, self.b2 = _w(sd[prefix + "2.weight"], device, dtype), _f32(sd[prefix + "2.bias"], device)
        self.in_dim = self.w0.shape[1]
        self.out_dim = self.w2.shape[0]
        self.soft_ld = self.out_dim
        self.device, self.max_batch = device, max_batch
        self._alloc()

    def _alloc(self):
        device, max_batch, dtype = self.device, self.max_batch, self.dtype
        self.x_t = torch.empty(max_batch, self.in_dim, device=device, dtype=dtype)
        self.h = torch.empty(max_batch, self.w0.shape[0], device=device, dtype=dtype)
        self.out = torch.empty(max_batch, self.out_dim, device=device)
        self.ws = ops.skinny_workspace(device, [(max_batch, self.w0.shape[0], self.in_dim),
                                                (max_batch, self.out_dim, self.w2.shape[1])])

    def twin(self):
        """Same weights, private activation buffers/workspace (for another stream)."""
        t = copy.copy(self)
        t._alloc()
        return t

    def __call__(self, prefix):
        B = prefix.shape[0]
        ops.cast(prefix, self.x_t[:B])
        ops.gemm(self.x_t[:B], self.w0, self.h[:B], bias=self.b0, act=ops.ACT_TANH, workspace=self.ws)
        ops.gemm(self.h[:B], self.w2, self.out[:B], bias=self.b2, workspace=self.ws)
        return self.out[:B]           # clip b's soft prefix at out + b*soft_ld


class TransformerMapperEngine:
    """TransformerMapper (mapper.py:125-139): linear -> concat prefix_const -> 8 pre-LN layers
    (8 heads x 96, no q/kv bias, softmax over keys, ReLU MLP x2) -> rows clip_length: ."""

    def __init__(self, sd, device, dtype, max_batch, prefix="clap_project.", clip_length=10,
                 num_layers=8, heads=8):
        self.dtype, self.cl, self.heads = dtype, clip_length, heads
        self.lin_w = _w(sd[prefix + "linear.weight"], device, dtype)
        self.lin_b = _f32(sd[prefix + "linear.bias"], device)
        self.pc = _f32(sd[prefix + "prefix_const"], device)
        self.pl = self.pc.shape[0]
        self.L = clip_length + self.pl
        self.layers = []
        for i in range(num_layers):
            p = prefix + f"transformer.layers.{i}."
            self.layers.append({
                "n1": (_f32(sd[p + "norm1.weight"], device), _f32(sd[p + "norm1.bias"], device)),
                "q": _w(sd[p + "attn.to_queries.weight"], device, dtype),
                "kv": _w(sd[p + "attn.to_keys_values.weight"], device, dtype),
                "proj_w": _w(sd[p + "attn.project.weight"], device, dtype),
                "proj_b": _f32(sd[p + "attn.project.bias"], device),
                "n2": (_f32(sd[p + "norm2.weight"], device), _f32(sd[p + "norm2.bias"], device)),
                "fc1_w": _w(sd[p + "mlp.fc1.weight"], device, dtype),
                "fc1_b": _f32(sd[p + "mlp.fc1.bias"], device),
                "fc2_w": _w(sd[p + "mlp.fc2.weight"], device, dtype),
                "fc2_b": _f32(sd[p + "mlp.fc2.bias"], device),
            })
        self.in_dim = self.lin_w.shape[1]
        self.soft_ld = self.L * D
        self.device, self.max_batch = device, max_batch
        self._alloc()

    def twin(self):
        t = copy.copy(self)
        t._alloc()
        return t

    def _alloc(self):
        device, dtype, B, L = self.device, self.dtype, self.max_batch, self.L
        self.x_t = torch.empty(B, self.in_dim, device=device, dtype=dtype)
        self.hs = torch.empty(B, L, D, device=device)
        self.a = torch.empty(B * L, D, device=device, dtype=dtype)
        self.q = torch.empty(B * L, D, device=device, dtype=dtype)
        self.kv = torch.empty(B * L, 2 * D, device=device, dtype=dtype)
        self.o = torch.empty(B * L, D, device=device, dtype=dtype)
        self.mid = torch.empty(B * L, 2 * D, device=device, dtype=dtype)

    def __call__(self, prefix):
        B, L = prefix.shape[0], self.L
        ops.cast(prefix, self.x_t[:B])
        hs = self.hs[:B]
        # linear(x).view(B, clip_length, D) written straight into rows 0..cl-1 of every clip
        ops.gemm(self.x_t[:B], self.lin_w, hs.view(B, L * D)[:, :self.cl * D], bias=self.lin_b)
        hs[:, self.cl:].copy_(self.pc.unsqueeze(0).expand(B, -1, -1))
        x = hs.view(B * L, D)
        scale = (D // self.heads) ** -0.5
        for ly in self.layers:
            M = B * L
            ops.layernorm(x, *ly["n1"], out=self.a[:M])
            ops.gemm(self.a[:M], ly["q"], self.q[:M])
            ops.gemm(self.a[:M], ly["kv"], self.kv[:M])
            kv = self.kv[:M]
            ops.row_attention(self.q[:M], D, kv, kv[:, D:], 2 * D, B, L, self.heads, D // self.heads,
                              False, scale, self.o[:M], D)
            ops.gemm(self.o[:M], ly["proj_w"], x, bias=ly["proj_b"], residual=x)
            ops.layernorm(x, *ly["n2"], out=self.a[:M])
            ops.gemm(self.a[:M], ly["fc1_w"], self.mid[:M], bias=ly["fc1_b"], act=ops.ACT_RELU)
            ops.gemm(self.mid[:M], ly["fc2_w"], x, bias=ly["fc2_b"], residual=x)
        return hs.view(B, L * D)[:, self.cl * D:]   # clip b's soft prefix at base + b*soft_ld


def build_mapper(sd, mapping_type, device, dtype, max_batch, clip_length=10, num_layers=8):
    """ClapCaptionModel's clap_project (models/caption_model.py:55-60): MLP, or TransformerMapper
    with params.json's prefix_length_clip / num_layers."""
    if mapping_type == "mlp":
        return MlpMapper(sd, device, dtype, max_batch)
    if mapping_type != "transformer":
        raise ValueError(f"mapping_type {mapping_type!r} (mlp | transformer)")
    return TransformerMapperEngine(sd, device, dtype, max_batch, clip_length=clip_length,
                                   num_layers=num_layers)


# ------------------------------------------------------------------------------- GPT-2
def colsum(W: torch.Tensor) -> torch.Tensor:
    """Per output column n of a [N][K] bf16 weight: sum_k W[n][k] of the bf16 values (f64, then
    f32) -- the LayerNorm fold's mean correction in the grid decode's epilogues."""
    return W.double().sum(dim=1).float().contiguous()


class Gpt2Weights:
    """HF GPT-2 small (``gpt.`` keys under ClapCaption_prompt): Conv1D [in,out] -> [out,in]."""

    def __init__(self, sd, device, dtype, prefix="gpt.transformer."):
        self.dtype = dtype
        p = prefix
        self.wte = _w(sd[p + "wte.weight"], device, dtype)
        self.wpe = _w(sd[p + "wpe.weight"], device, dtype)
        wn = torch.nn.functional.normalize(sd[p + "wte.weight"].float(), 2, 1)
        self.wte_norm = _w(wn, device, dtype)          # predict_prompt.py:117-118
        self.V = self.wte.shape[0]
        self.layers = []
        # bf16: the ln_1 / ln_2 affine is folded into c_attn / c_fc (W'[n,k] = W[n,k] * g[k],
        # b'[n] = b[n] + sum_k W[n,k] * beta[k], in f32 before the bf16 rounding of W'), so the
        # LayerNorm before them only normalises: zs_gemm_ln then skips the LN weight / bias loads
        # its 16 row-threads each repeat (half the bytes its workgroups pull through L1 at decode
        # shapes).  f32 parity mode keeps the reference's exact LN -> GEMM order.
        self.folded = dtype == torch.bfloat16
        one = torch.ones(D, device=device)
        zero = torch.zeros(D, device=device)
        for i in range(NL):
            h = p + f"h.{i}."
            t = lambda k: _w(sd[h + k].t(), device, dtype)

            def lin_ln(wk, bk, lnk):
                W = sd[h + wk].float().t()
                b = sd[h + bk].float()
                g, beta = sd[h + lnk + ".weight"].float(), sd[h + lnk + ".bias"].float()
                if not self.folded:
                    return (_w(W, device, dtype), _f32(b, device),
                            (_f32(g, device), _f32(beta, device)), (_f32(g, device), _f32(beta, device)))
                Wf = W * g[None, :]
                bf = (b.double() + W.double() @ beta.double()).float()
                return _w(Wf, device, dtype), _f32(bf, device), (one, zero), (None, None)
            aw, ab, ln1, ln1g = lin_ln("attn.c_attn.weight", "attn.c_attn.bias", "ln_1")
            fw, fb, ln2, ln2g = lin_ln("mlp.c_fc.weight", "mlp.c_fc.bias", "ln_2")
            self.layers.append({
                "ln1": ln1, "ln1_gemm": ln1g, "attn_w": aw, "attn_b": ab,
                "proj_w": t("attn.c_proj.weight"), "proj_b": _f32(sd[h + "attn.c_proj.bias"], device),
                "ln2": ln2, "ln2_gemm": ln2g, "fc_w": fw, "fc_b": fb,
                "mproj_w": t("mlp.c_proj.weight"), "mproj_b": _f32(sd[h + "mlp.c_proj.bias"], device),
            })
        self.lnf = (_f32(sd[p + "ln_f.weight"], device), _f32(sd[p + "ln_f.bias"], device))
        self._layer_ptrs = None
        self._wte_packed = self._lm_bias = None
        if self.folded:
            # the bs <= 64 greedy decode (zs_gpt2_decode_persist / _phases) folds ln_f's affine into
            # the tied LM head as ln_1 / ln_2 into c_attn / c_fc: logit[v] = y . (g o wte[v]) +
            # beta . wte[v] with y the normalised row (g o wte rounded to bf16 once, from f32)
            # lm_bias [2][16 nvb]: beta . wte[v], then the column sums of the folded head (the
            # grid decode runs the LayerNorm in the GEMM epilogue: rstd (x W' - mean cs) + b')
            wte32 = sd[p + "wte.weight"].to(device=device, dtype=torch.float32)
            g, beta = self.lnf
            wg = (wte32 * g[None, :]).to(torch.bfloat16)
            self._wte_packed = ops.pack_b_fragments(wg)
            nvb = -(-self.V // 16)
            lmb = torch.zeros(2, nvb * 16, device=device)
            lmb[0, :self.V] = (wte32.double() @ beta.double()).float()
            lmb[1, :self.V] = colsum(wg)
            self._lm_bias = lmb
            del wte32, wg

    def packed_layer_ptrs(self):
        """The 12 x 8 device pointers zs_gpt2_decode_persist / _phases take: per block c_attn W,
        b, attn.c_proj W, b, c_fc W, b, mlp.c_proj W, b -- each W (bf16, LN affine folded) in MFMA
        fragment order (ops.pack_b_fragments), packed once.  f32 model: the same table for
        zs_gpt2_decode_persist_f32 / _phases_f32 (_pack_f32)."""
        if self._layer_ptrs is None:
            import ctypes
            if self.dtype == torch.float32:
                self._pack_f32()
            else:
                assert self.folded, "the grid decode runs the bf16 (LN-folded) weights"
                # the LayerNorm-fed GEMMs' biases as [2][N]: b' (beta folded), then the folded
                # weight's column sums cs[n] = sum_k W'[n][k] (the epilogue's rstd (x W' - mean cs) + b')
                self._packed = [{k: (ops.pack_b_fragments(ly[k]) if k.endswith("_w") else
                                     torch.stack([ly[k], colsum(ly[k[:-2] + "_w"])])
                                     if k in ("attn_b", "fc_b") else ly[k])
                                 for k in ("attn_w", "attn_b", "proj_w", "proj_b", "fc_w", "fc_b",
                                           "mproj_w", "mproj_b")} for ly in self.layers]
            keys = ("attn_w", "attn_b", "proj_w", "proj_b", "fc_w", "fc_b", "mproj_w", "mproj_b")
            self._layer_ptrs = (ctypes.c_void_p * (8 * NL))(
                *[pl[k].data_ptr() for pl in self._packed for k in keys])
        return self._layer_ptrs

    def _pack_f32(self):
        """The f32 grid decode's tables (the parity mode): ln_1 / ln_2's affine folded into c_attn /
        c_fc in f32 (W' = W diag(g), b' = b + W beta summed in f64), ln_f's into the tied LM head
        (g o wte, per-token bias beta . wte[v]); every W in f32 fragment order
        (ops.pack_f32_fragments)."""
        def fold(W, b, ln):
            g, beta = ln
            return (ops.pack_f32_fragments(W * g[None, :]),
                    (b.double() + W.double() @ beta.double()).float().contiguous())
        self._packed = []
        for ly in self.layers:
            aw, ab = fold(ly["attn_w"], ly["attn_b"], ly["ln1"])
            fw, fb = fold(ly["fc_w"], ly["fc_b"], ly["ln2"])
            self._packed.append({"attn_w": aw, "attn_b": ab,
                                 "proj_w": ops.pack_f32_fragments(ly["proj_w"]), "proj_b": ly["proj_b"],
                                 "fc_w": fw, "fc_b": fb,
                                 "mproj_w": ops.pack_f32_fragments(ly["mproj_w"]), "mproj_b": ly["mproj_b"]})
        g, beta = self.lnf
        self._wte_packed = ops.pack_f32_fragments(self.wte * g[None, :])
        nvb = -(-self.V // 16)
        lmb = torch.zeros(nvb * 16, device=self.wte.device)
        lmb[:self.V] = (self.wte.double() @ beta.double()).float()
        self._lm_bias = lmb

    def wte_packed(self):
        """The tied LM head with ln_f's weight folded in, MFMA fragment order (bf16, or f32 after
        packed_layer_ptrs of an f32 model)."""
        assert self._wte_packed is not None, "the grid decode runs the bf16 (LN-folded) weights"
        return self._wte_packed

    def lm_bias(self):
        """ln_f's bias through the tied LM head, beta . wte[v], f32 [ceil(V/16) 16] (bf16 model:
        [2][ceil(V/16) 16], the folded head's column sums in row 1)."""
        assert self._lm_bias is not None, "the grid decode runs the bf16 (LN-folded) weights"
        return self._lm_bias

    def nbytes(self) -> int:
        n = self.wte.numel() + self.wpe.numel()
        for ly in self.layers:
            n += sum(ly[k].numel() for k in ("attn_w", "proj_w", "fc_w", "mproj_w"))
        return n * self.wte.element_size()


class Gpt2Decoder:
    """Batched GPT-2 prefix decoder with a KV cache.

    ``max_rows`` decode rows (B for greedy, C*beam for beam), prompts up to ``max_prompt``
    tokens, ``max_steps`` generated tokens (entry_length)."""

    def __init__(self, w: Gpt2Weights, max_rows: int, max_prompt: int, max_steps: int = 67,
                 max_prefill_rows: Optional[int] = None, topk: int = 8, chunk: int = 0,
                 use_graph: bool = True, compact: Optional[bool] = None,
                 persist: Optional[bool] = None, alloc_kv: bool = True):
        """alloc_kv False: no KV cache of its own -- share_rows gives it rows of another
        decoder's (a group begin's sub-decoder)."""
        if chunk <= 0:   # a divisor of the steps after step 0, near 6 (no wasted tail steps)
            n = max(max_steps - 1, 1)
            cands = [c for c in range(4, 13) if n % c == 0]
            chunk = min(cands, key=lambda c: abs(c - 6)) if cands else 6
        self.w, self.dtype = w, w.dtype
        # f32 decode on the f32 row-group kernels (zs_gemm_ln_f32); 0 = layernorm + skinny GEMMs
        self.rows_f32 = os.environ.get("ZSAAC_ROWS_F32", "1") != "0"
        dev = w.wte.device
        self.dev = dev
        self.R = max_rows
        self.Rp = max_prefill_rows or max_rows
        self.Pmax = max_prompt
        self.max_steps = max_steps
        self.topk, self.chunk, self.use_graph = topk, chunk, use_graph
        self.stop0, self.stop1 = STOP_DOT, STOP_SPACE_DOT   # generate2 stops on '.' and ' .'
        self.temperature = 1.0      # logits / temperature (gpt2_prefix_eval.py:121, 196)
        # + chunk: a replayed graph chunk may run a few steps past entry_length (no-ops)
        self.Lmax = max_prompt + max_steps + chunk + 1
        dt = self.dtype
        Mp = max(self.Rp * max_prompt, self.R)
        self.x = torch.empty(Mp, D, device=dev)
        self.h = torch.empty(Mp, D, device=dev, dtype=dt)
        self.qkv = torch.empty(Mp, 3 * D, device=dev, dtype=dt)
        self.att = torch.empty(Mp, D, device=dev, dtype=dt)
        self.hid = torch.empty(Mp, 4 * D, device=dev, dtype=dt)
        kv_rows = self.R if alloc_kv else 0
        self.kc = [torch.empty(kv_rows, NH, self.Lmax, HD, device=dev, dtype=dt) for _ in range(NL)]
        self.vc = [torch.empty(kv_rows, NH, self.Lmax, HD, device=dev, dtype=dt) for _ in range(NL)]
        self.hf = torch.empty(max(self.R, self.Rp), D, device=dev, dtype=dt)
        self.nblk = ops.lmhead_nblk(w.V)
        R = max(self.R, self.Rp)
        self.pstat = torch.empty(R, self.nblk, 2, device=dev)
        self.pval = torch.empty(R, self.nblk, topk, device=dev)
        self.pidx = torch.empty(R, self.nblk, topk, device=dev, dtype=torch.int32)
        self.pval1 = torch.empty(R, self.nblk, 1, device=dev)
        self.pidx1 = torch.empty(R, self.nblk, 1, device=dev, dtype=torch.int32)
        # decode state
        i32 = dict(device=dev, dtype=torch.int32)
        self.pos = torch.zeros(self.R, **i32)
        self.next_tok = torch.zeros(self.R, **i32)
        self.done = torch.zeros(self.R, **i32)
        self.out_ids = torch.zeros(self.R, max_steps, **i32)
        self.out_len = torch.zeros(self.R, **i32)
        self.step_ctr = torch.zeros(1, **i32)
        # [flag, greedy_step arrival counter, rows still decoding]
        self.all_done = torch.zeros(3, **i32)
        # greedy row compaction: decode only the rows that have not stopped, in buckets of
        # `bucket` rows (>= `min_bucket`, so the GEMMs stay in the tiled regime); bf16 only
        # (decode_attn5), and the per-row arithmetic of every kernel is independent of the row
        # count, so the ids equal the uncompacted decode's.
        self.bucket, self.min_bucket = 256, 512
        if compact is None:
            compact = dt == torch.bfloat16
        self.compact = (compact and dt == torch.bfloat16 and self.Lmax <= 128
                        and self.R >= self.min_bucket)
        # greedy bf16 decode of one eval batch (<= 64 rows): the grid decode (decode_grid.hip)
        # -- every step after step 0 in one persistent launch (zs_gpt2_decode_persist), or, as
        # the per-step path (persist off, or the give-up fallback), the same computation as phase
        # launches (zs_gpt2_decode_phases); ids and state are identical at every grid size
        self.grid_decode = (dt == torch.bfloat16 and w.folded and self.R <= 64
                            and os.environ.get("ZSAAC_GRID_DECODE", "1") != "0")   # 0: A/B only
        # f32 parity mode: the same grid decode in f32 (zs_gpt2_decode_persist_f32, G = 192)
        self.f32_grid = (dt == torch.float32 and self.R <= 64
                         and os.environ.get("ZSAAC_GRID_DECODE_F32", "1") != "0")
        self.grid_decode = self.grid_decode or self.f32_grid
        if persist is None:
            persist = os.environ.get("ZSAAC_PERSIST", "1") != "0"
        self.persist = bool(persist) and self.grid_decode
        # workgroups (256 threads, half a CU each) of the persistent launch: 48 / 96 / 192,
        # chosen per batch by pipeline.ConcurrentRunner (more when CUs are free)
        self.persist_grid = int(os.environ.get("ZSAAC_PERSIST_GRID", "48"))
        self.phase_grid = 96           # the phase launches' grid (any size gives the same ids)
        if self.f32_grid:
            self.persist_grid = self.phase_grid = ops.PERSIST_GRIDS_F32[0]
        if self.grid_decode:
            import ctypes
            self.persist_ws = (ops.decode_persist_f32_workspace(dev) if self.f32_grid
                               else ops.decode_persist_workspace(dev))
            # the shared packed weights and pointer table, built now and synchronised: a twin
            # decoder launched on another stream must never read a half-written copy
            w.packed_layer_ptrs()
            torch.cuda.synchronize(dev)
            self._kv_ptrs = (ctypes.c_void_p * (2 * NL))(
                *[t.data_ptr() for t in self.kc], *[t.data_ptr() for t in self.vc])
        self.rowmap = torch.zeros(self.R, **i32)
        self.cpos = torch.zeros(self.R, **i32)      # this step's positions in compact order
        self.n_act = torch.zeros(1, **i32)
        self._cgreedy = None
        self.plen = torch.zeros(self.Rp, **i32)
        self.last_row = torch.zeros(self.Rp, **i32)
        # beam state
        self.scores = torch.zeros(self.R, device=dev)
        self.seq_len = torch.ones(self.R, device=dev)
        self.kvrow = torch.zeros(self.R, self.Lmax, **i32)
        self.kvrow_tmp = torch.zeros(self.R, self.Lmax, **i32)
        self.tok_tmp = torch.zeros(self.R, max_steps, **i32)
        self.graphs: Dict[Tuple, torch.cuda.CUDAGraph] = {}
        self.n_captures = 0
        self.rows_stepped = 0       # decode rows x steps run (work counter; persistent launches
                                    # add theirs when the host sees them finish: note_persist_steps)
        self.gave_up = 0            # persistent launches that gave up and resumed stepwise
        self._eager = False         # step_chunk without graphs (the give-up fallback)
        self._persist_R = 0         # rows of the persistent launch in flight (0: none)
        self._persist_pending = 0   # rows of a greedy begin whose launch is deferred
        self.defer_launch = False   # greedy_begin leaves the persistent launch to launch_pending
        self.persist_exclusive = False   # the launch takes a CU per workgroup (runner's choice)
        self.ws = ops.skinny_workspace(dev, [(M, N, K) for M in {self.R, self.Rp}
                                             for N, K in ((3 * D, D), (D, D), (4 * D, D), (D, 4 * D))])

    def share_rows(self, src: "Gpt2Decoder", r0: int):
        """Decode rows r0 .. r0 + R of ``src``'s prefill: this decoder's KV cache, last-position
        hidden rows (hf, step 0's LM-head input) and prompt lengths become views of src's rows
        (pipeline.CaptionPipeline.begin_group runs the prefill of several eval batches at once;
        each batch then takes step 0 and its persistent decode on its own decoder)."""
        R = self.R
        assert src.Lmax == self.Lmax and r0 + R <= src.R and src.dtype == self.dtype
        self.kc = [t[r0:r0 + R] for t in src.kc]
        self.vc = [t[r0:r0 + R] for t in src.vc]
        self.hf = src.hf[r0:r0 + R]
        self.plen = src.plen[r0:r0 + R]
        if self.grid_decode:
            import ctypes
            self._kv_ptrs = (ctypes.c_void_p * (2 * NL))(
                *[t.data_ptr() for t in self.kc], *[t.data_ptr() for t in self.vc])

    # ---------------------------------------------------------------- blocks
    def _layers(self, M, attn_fn):
        x = self.x[:M]
        if self.dtype == torch.bfloat16 and M <= 64:
            # decode at the reference's eval batch: LayerNorm fused into the c_attn / c_fc
            # launches (zs_gemm_ln), row-group GEMMs for the projections (5 launches per block)
            for l, ly in enumerate(self.w.layers):
                qkv, att, hid = self.qkv[:M], self.att[:M], self.hid[:M]
                ops.gemm_ln(x, *ly["ln1_gemm"], ly["attn_w"], qkv, bias=ly["attn_b"])
                attn_fn(l, qkv, att)
                ops.gemm(att, ly["proj_w"], x, bias=ly["proj_b"], residual=x, workspace=self.ws)
                ops.gemm_ln(x, *ly["ln2_gemm"], ly["fc_w"], hid, bias=ly["fc_b"], act=ops.ACT_GELU_TANH)
                ops.gemm(hid, ly["mproj_w"], x, bias=ly["mproj_b"], residual=x, workspace=self.ws)
            return
        if self.dtype == torch.float32 and M <= 64 and self.rows_f32:
            # the f32 parity mode's decode: ln_1 / ln_2 fused into f32 row-group GEMMs
            # (zs_gemm_ln_f32; the affine applied in f32, exact f32 products), the same kernels
            # without LayerNorm for the projections
            for l, ly in enumerate(self.w.layers):
                qkv, att, hid = self.qkv[:M], self.att[:M], self.hid[:M]
                ops.gemm_ln_f32(x, *ly["ln1"], ly["attn_w"], qkv, bias=ly["attn_b"])
                attn_fn(l, qkv, att)
                ops.gemm_ln_f32(att, None, None, ly["proj_w"], x, bias=ly["proj_b"], residual=x)
                ops.gemm_ln_f32(x, *ly["ln2"], ly["fc_w"], hid, bias=ly["fc_b"], act=ops.ACT_GELU_TANH)
                ops.gemm_ln_f32(hid, None, None, ly["mproj_w"], x, bias=ly["mproj_b"], residual=x)
            return
        for l, ly in enumerate(self.w.layers):
            h, qkv, att, hid = self.h[:M], self.qkv[:M], self.att[:M], self.hid[:M]
            ops.layernorm(x, *ly["ln1"], out=h)
            ops.gemm(h, ly["attn_w"], qkv, bias=ly["attn_b"], workspace=self.ws)
            attn_fn(l, qkv, att)
            ops.gemm(att, ly["proj_w"], x, bias=ly["proj_b"], residual=x, workspace=self.ws)
            ops.layernorm(x, *ly["ln2"], out=h)
            ops.gemm(h, ly["fc_w"], hid, bias=ly["fc_b"], act=ops.ACT_GELU_TANH, workspace=self.ws)
            ops.gemm(hid, ly["mproj_w"], x, bias=ly["mproj_b"], residual=x, workspace=self.ws)

    def prefill(self, B: int, Pmax: int, row_stride: int = 1):
        """Runs the prompt rows already in ``self.x[:B*Pmax]`` (zs_gpt2_prefill_embed) through the
        12 blocks, fills the KV cache (row b -> cache row b*row_stride) and leaves ln_f of every
        row's last prompt position in ``self.hf[:B]``."""
        M = B * Pmax

        fused = self.dtype == torch.bfloat16 and Pmax <= 32

        def attn(l, qkv, att):
            if fused:       # one launch: attention + the layer's KV-cache write
                ops.row_attention_kv(qkv, B, Pmax, NH, 1.0 / math.sqrt(HD), att, self.kc[l],
                                     self.vc[l], self.Lmax, self.plen[:B], row_stride=row_stride)
                return
            ops.kv_write(qkv, B, Pmax, D, NH, self.kc[l], self.vc[l], self.Lmax, row_stride=row_stride)
            ops.row_attention(qkv, 3 * D, qkv[:, D:], qkv[:, 2 * D:], 3 * D, B, Pmax, NH, HD, True,
                              1.0 / math.sqrt(HD), att, D, lens=self.plen[:B])

        self._layers(M, attn)
        ops.layernorm(self.x, *self.w.lnf, out=self.hf[:B], rows=self.last_row[:B])

    def _decode_forward(self, R, kvrow=None):
        ops.embed_tokens(self.next_tok[:R], self.pos[:R], self.w.wte, self.w.wpe, self.x[:R])

        def attn(l, qkv, att):
            ops.decode_attention(qkv, R, D, NH, self.kc[l], self.vc[l], self.Lmax, self.pos[:R],
                                 att, kvrow=kvrow)

        self._layers(R, attn)
        ops.layernorm(self.x[:R], *self.w.lnf, out=self.hf[:R])

    def _decode_forward_c(self, R, Rb):
        """_decode_forward over the Rb compact slots of rowmap (physical rows < R)."""
        ops.embed_tokens_map(self.next_tok, self.pos, self.rowmap, R, self.w.wte, self.w.wpe,
                             self.x[:Rb], Rb, cpos=self.cpos)

        def attn(l, qkv, att):
            ops.decode_attention_map(qkv, Rb, self.rowmap, R, D, NH, self.kc[l], self.vc[l],
                                     self.Lmax, self.pos, att, cpos=self.cpos)

        self._layers(Rb, attn)
        ops.layernorm(self.x[:Rb], *self.w.lnf, out=self.hf[:Rb])

    def _greedy_step_body_c(self, R, Rb):
        self._decode_forward_c(R, Rb)
        ops.lmhead_topk(self.hf[:Rb], self.w.wte, 1, None, self.pval1, self.pidx1,
                        temperature=self.temperature)
        ops.greedy_step_map(self.pval1, self.pidx1, Rb, self.rowmap, R, self.nblk, self.step_ctr,
                            self.max_steps, self.stop0, self.stop1, self.out_ids, self.out_len,
                            self.done, self.pos, self.next_tok, self.all_done)

    def _bucket_rows(self, R, alive):
        if alive is None:
            return R
        return min(R, max(self.min_bucket, -(-alive // self.bucket) * self.bucket))

    def _chunk_plan(self, alive=None):
        """(graph key, step body, chunk prologue) of the active decode; ``alive`` is the host's
        latest view of all_done[2] (None = unknown -> every row)."""
        if self._cgreedy is None:
            key, body = self._active
            return key, body, None
        R = self._cgreedy
        Rb = self._bucket_rows(R, alive)
        return (("greedy_c", R, Rb, self.stop0, self.stop1, self.temperature),
                lambda: self._greedy_step_body_c(R, Rb),
                lambda: ops.compact_rows(self.done, R, self.rowmap, self.n_act))

    @staticmethod
    def _rows_of(key):
        return key[1] * key[2] if key[0] == "beam" else key[1]

    def capture_buckets(self):
        """Capture every compacted-greedy bucket graph of the active decode up front (so a timed
        run never captures)."""
        if self._cgreedy is None or not self.use_graph:
            return
        R = self._cgreedy
        for Rb in sorted({self._bucket_rows(R, a) for a in range(0, R + 1, self.bucket)}):
            self._graph(*self._chunk_plan(Rb))

    def _grid_args(self, R):
        w = self.w
        return (R, self.Lmax, self.max_steps, self.stop0, self.stop1, w.V, w.wte, w.wpe,
                w.wte_packed(), self.temperature, w.packed_layer_ptrs(), w.lm_bias(),
                self._kv_ptrs, self.pos, self.next_tok, self.done, self.out_ids, self.out_len,
                self.step_ctr, self.all_done, self.persist_ws)

    def _greedy_step_body(self, R):
        if self.grid_decode:      # the persistent launch's computation, one launch per phase
            phases = ops.gpt2_decode_phases_f32 if self.f32_grid else ops.gpt2_decode_phases
            phases(*self._grid_args(R), steps=1, grid=self.phase_grid)
            return
        self._decode_forward(R)
        ops.lmhead_topk(self.hf[:R], self.w.wte, 1, None, self.pval1, self.pidx1,
                        temperature=self.temperature)
        ops.greedy_step(self.pval1, self.pidx1, R, self.nblk, self.step_ctr, self.max_steps,
                        self.stop0, self.stop1, self.out_ids, self.out_len, self.done, self.pos,
                        self.next_tok, self.all_done)

    def _graph(self, key, body, pre=None):
        """The captured hipGraph of ``chunk`` consecutive decode steps, after the optional chunk
        prologue ``pre`` (captured on first use: one eager warm-up step on a side stream with
        the decode state saved/restored, then capture)."""
        g = self.graphs.get(key)
        if g is None:
            cur = torch.cuda.current_stream()
            if getattr(self, "_cap_stream", None) is None:
                self._cap_stream = torch.cuda.Stream()    # one side stream per decoder
            s = self._cap_stream
            s.wait_stream(cur)
            saved = [t.clone() for t in self._state()]
            with torch.cuda.stream(s):
                if pre is not None:
                    pre()
                body()
            cur.wait_stream(s)
            for t, v in zip(self._state(), saved):
                t.copy_(v)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                if pre is not None:
                    pre()
                for _ in range(self.chunk):
                    body()
            cur.wait_stream(torch.cuda.current_stream())
            self.graphs[key] = g
            self.n_captures += 1
        return g

    @property
    def n_chunks(self) -> int:
        """Chunks after the prefill step that cover entry_length (step 0 runs with the prefill)."""
        return max(0, -(-(self.max_steps - 1) // self.chunk))

    def step_chunk(self, alive=None):
        """Enqueue ``chunk`` decode steps of the active decode (no host sync).  ``alive``: an
        upper bound on the rows still decoding (all_done[2] read after the previous chunk);
        it only picks the compaction bucket, so None is always safe."""
        key, body, pre = self._chunk_plan(alive)
        self.rows_stepped += (key[2] if key[0] == "greedy_c" else self._rows_of(key)) * self.chunk
        if self.use_graph and not self._eager:
            self._graph(key, body, pre).replay()
        else:
            if pre is not None:
                pre()
            for _ in range(self.chunk):
                body()

    def finished_async(self):
        """Enqueue a copy of all_done + step_ctr to pinned host memory; returns (event, host
        tensor): [0] = finished flag, [1] < 0 = a persistent launch gave up, [2] = rows still
        decoding, [3] = decode steps done."""
        if not hasattr(self, "_flag_host"):
            self._flag_host = torch.zeros(4, dtype=torch.int32, pin_memory=True)
            self._flag_dev = torch.zeros(4, dtype=torch.int32, device=self.dev)
        self._flag_dev[:3].copy_(self.all_done)
        self._flag_dev[3:].copy_(self.step_ctr)
        self._flag_host.copy_(self._flag_dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return ev, self._flag_host

    def run_to_completion(self):
        """Synchronous loop: replay chunks until every row stopped or entry_length reached."""
        if self._persist_R:
            flag, arr, alive = self.all_done.tolist()
            if arr >= 0:
                self.note_persist_steps(int(self.step_ctr.item()))
                return
            self.resume_stepwise()
        for _ in range(self.n_chunks):
            flag, arr, alive = self.all_done.tolist()
            if flag:
                break
            self.step_chunk(alive)

    def note_persist_steps(self, steps: int):
        """The host saw the persistent launch finish after ``steps`` decode steps (step_ctr):
        count the rows it stepped (the launch runs steps 1 .. steps - 1)."""
        if self._persist_R:
            self.rows_stepped += self._persist_R * max(0, steps - 1)
            self._persist_R = 0

    def resume_stepwise(self):
        """After a persistent launch gave up (all_done[1] = -1: its grid was not co-resident in
        time): the kernel commits ids, out_len, pos / done / next_tok and step_ctr after every
        step it completes (workgroup 0, once every workgroup's LM-head keys are in), so the state
        in memory is the last completed step's; K/V rows written past it are rewritten with the
        same values.  Re-arm the flags; the remaining steps run as phase launches (the same
        arithmetic: ids equal an uninterrupted launch's), eagerly (no graph capture while other
        streams run).  Enqueued on the current stream."""
        self.all_done[:2].zero_()
        self.gave_up += 1
        self._persist_R = 0
        self._eager = True

    def _state(self):
        return [self.pos, self.next_tok, self.done, self.out_ids, self.out_len, self.step_ctr,
                self.all_done, self.scores, self.seq_len, self.kvrow, self.kvrow_tmp, self.tok_tmp]

    # ---------------------------------------------------------------- greedy (generate2)
    def greedy_begin(self, B: int):
        """Enqueue step 0 of generate2 from the prefill rows (no host sync); afterwards
        :meth:`step_chunk` advances ``chunk`` steps at a time."""
        self.greedy_begin_device(B)
        self.greedy_begin_host(B)

    def greedy_begin_device(self, R: int):
        """The device work of :meth:`greedy_begin` (LM head, step-0 bookkeeping): no host
        state, so a pipeline can capture it in its begin graph."""
        ops.lmhead_topk(self.hf[:R], self.w.wte, 1, None, self.pval1, self.pidx1,
                        temperature=self.temperature)
        ops.greedy_init(R, self.plen, self.pos, self.done, self.out_len, self.out_ids,
                        self.max_steps, self.step_ctr, self.all_done)
        ops.greedy_step(self.pval1, self.pidx1, R, self.nblk, self.step_ctr, self.max_steps,
                        self.stop0, self.stop1, self.out_ids, self.out_len, self.done, self.pos,
                        self.next_tok, self.all_done)

    def greedy_begin_host(self, R: int):
        """The host state of :meth:`greedy_begin` and, for the persistent decode, its launch (a
        grid shape chosen per batch by the runner: never captured)."""
        self._active = (("greedy", R, self.stop0, self.stop1, self.temperature),
                        lambda: self._greedy_step_body(R))
        self._cgreedy = R if (self.compact and R >= self.min_bucket) else None
        self._eager = False
        self._persist_R = 0
        if self.persist and R <= 64:
            self._persist_pending = R
            if not self.defer_launch:
                self.launch_pending()

    def launch_pending(self):
        """Enqueues the persistent decode launch greedy_begin set up (at once, or -- with
        ``defer_launch`` set during the begin -- when the runner has room for its grid)."""
        R = self._persist_pending
        assert R, "launch_pending: no greedy begin waiting for its persistent launch"
        ev = PERSIST_LOG
        if ev is not None:          # bench.py's roofline: HIP events around each launch
            ev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
                       id(self)))
            ev[-1][0].record()
        persist = ops.gpt2_decode_persist_f32 if self.f32_grid else ops.gpt2_decode_persist
        persist(*self._grid_args(R), grid=self.persist_grid, exclusive=self.persist_exclusive)
        if ev is not None:
            ev[-1][1].record()
        self._persist_R = R
        self._persist_pending = 0

    def greedy(self, B: int, Pmax: int):
        """After :meth:`prefill` (row_stride 1): generate2 for all B rows.
        Returns (ids [B, max_steps] int32, lengths [B] int32) device tensors."""
        self.greedy_begin(B)
        self.run_to_completion()
        return self.out_ids[:B], self.out_len[:B]

    # ---------------------------------------------------------------- beam (generate_beam)
    def _beam_step_body(self, C, beam):
        R = C * beam
        self._decode_forward(R, kvrow=self.kvrow[:R])
        ops.lmhead_topk(self.hf[:R], self.w.wte, self.topk, self.pstat, self.pval, self.pidx,
                        temperature=self.temperature)
        ops.beam_step(self.pstat, self.pval, self.pidx, C, beam, self.nblk, self.topk, False,
                      self.stop0, self.step_ctr, self.max_steps, self.scores, self.seq_len,
                      self.done, self.out_ids, self.tok_tmp, self.kvrow, self.kvrow_tmp, self.Lmax,
                      self.pos, self.next_tok, self.all_done)

    def beam(self, C: int, beam: int, Pmax: int):
        """After :meth:`prefill` (C rows, row_stride=beam): generate_beam per clip.
        Returns (tokens [C, beam, steps], seq_len [C, beam], scores [C, beam]) device tensors
        (rows unsorted; the caller orders by scores/seq_len like the reference)."""
        self.beam_begin(C, beam)
        self.run_to_completion()
        R = C * beam
        return (self.out_ids[:R].view(C, beam, -1), self.seq_len[:R].view(C, beam),
                self.scores[:R].view(C, beam))

    def beam_begin(self, C: int, beam: int):
        assert beam <= self.topk and C * beam <= self.R
        R = C * beam
        self._eager = False
        self._persist_R = 0
        ops.lmhead_topk(self.hf[:C], self.w.wte, self.topk, self.pstat, self.pval, self.pidx,
                        temperature=self.temperature)
        for t in (self.done, self.step_ctr, self.all_done, self.out_ids, self.scores):
            t.zero_()
        self.seq_len.fill_(1.0)
        self.pos[:R].view(C, beam)[:, 0].copy_(self.plen[:C])
        ops.beam_step(self.pstat, self.pval, self.pidx, C, beam, self.nblk, self.topk, True,
                      self.stop0, self.step_ctr, self.max_steps, self.scores, self.seq_len,
                      self.done, self.out_ids, self.tok_tmp, self.kvrow, self.kvrow_tmp, self.Lmax,
                      self.pos, self.next_tok, self.all_done)
        self._active = (("beam", C, beam, self.stop0, self.temperature),
                        lambda: self._beam_step_body(C, beam))
        self._cgreedy = None

    # ---------------------------------------------------------------- get_prefix_tokens
    def prefix_tokens(self, embed_rows: torch.Tensor, out_idx: torch.Tensor):
        """argmax_n cos(embed_row, wte[n]) for every row of ``embed_rows`` [M, 768] f32."""
        M = embed_rows.shape[0]
        a = self.h[:M]
        ops.cast(embed_rows, a)
        ops.lmhead_topk(a, self.w.wte_norm, 1, None, self.pval_big(M), self.pidx_big(M),
                        row_norm=True)
        ops.argmax_finalize(self._pv_big, self._pi_big, M, self.nblk, out_idx)
        return out_idx

    def prefix_tokens_soft(self, soft_rows: torch.Tensor, hard_ids: torch.Tensor,
                           hard_len: torch.Tensor, B: int, Pmax: int, out_idx: torch.Tensor):
        """get_prefix_tokens with the cosine argmax over the soft-prompt rows only
        (``soft_rows`` [B * n_soft, 768] f32, contiguous): a hard row is wte[id], whose own
        cosine is the maximum whenever :meth:`hard_rows_safe` holds for every possible id, so its
        result is the id itself (zs_prefix_ids_assemble)."""
        M = soft_rows.shape[0]
        n_soft = M // B
        a = self.h[:M]
        ops.cast(soft_rows, a)
        ops.lmhead_topk(a, self.w.wte_norm, 1, None, self.pval_big(M), self.pidx_big(M),
                        row_norm=True)
        if getattr(self, "_soft_idx", None) is None or self._soft_idx.numel() < M:
            self._soft_idx = torch.empty(M, device=self.dev, dtype=torch.int32)
        ops.argmax_finalize(self._pv_big, self._pi_big, M, self.nblk, self._soft_idx)
        return ops.prefix_ids_assemble(hard_ids, hard_len, self._soft_idx, n_soft, B, Pmax, out_idx)

    def hard_rows_safe(self, ids, margin) -> bool:
        """True when for every token id in ``ids`` the cosine argmax of the row wte[id] against
        normalize(wte) — computed by the same LM-head kernel get_prefix_tokens uses — is id
        itself, ahead of every other vocabulary row by more than ``margin``."""
        ids = torch.as_tensor(sorted(set(int(i) for i in ids)), device=self.dev, dtype=torch.long)
        C = ids.numel()
        if C == 0:
            return True
        a = self.w.wte.index_select(0, ids).contiguous()
        pv = torch.empty(C, self.nblk, 2, device=self.dev)
        pi = torch.empty(C, self.nblk, 2, device=self.dev, dtype=torch.int32)
        ops.lmhead_topk(a, self.w.wte_norm, 2, None, pv, pi, row_norm=True)
        v, i = pv.view(C, -1), pi.view(C, -1).long()
        own = i == ids[:, None]
        neg = torch.full_like(v, -float("inf"))
        best_own = torch.where(own, v, neg).amax(1)
        best_other = torch.where(own, neg, v).amax(1)
        return bool(((best_own - best_other) > margin).all())

    def _ensure_big(self, M):
        if getattr(self, "_big_M", 0) < M:
            self._ps_big = torch.empty(M, self.nblk, 2, device=self.dev)
            self._pv_big = torch.empty(M, self.nblk, 1, device=self.dev)
            self._pi_big = torch.empty(M, self.nblk, 1, device=self.dev, dtype=torch.int32)
            self._big_M = M

    def pstat_big(self, M):
        self._ensure_big(M)
        return self._ps_big

    def pval_big(self, M):
        self._ensure_big(M)
        return self._pv_big

    def pidx_big(self, M):
        self._ensure_big(M)
        return self._pi_big
