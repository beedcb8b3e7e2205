"""End-to-end batched caption pipeline (the hot path of BASELINE.json ``north_star``):

  wav [B, 320000] --zs_logmel(+bn0)--> HTSAT/CNN14 --audio_proj, L2--> CLAP emb [B,1024]
  --zs_prompt_assemble--> hard prompt ids --normalize_prefix--> mapper --prefill_embed-->
  GPT-2 prefill (KV cache) --get_prefix_tokens--> greedy (generate2) or beam (generate_beam)
  --> token ids [B, <=67] (+ lengths), all on one GPU, one stream.

What the reference does per clip in Python (predict_prompt.py:129-148 over the dataset of
dataset/dataset.py:441-453 fed by data_handing/embeddings_generator.py:44-73) is done here for a
batch of clips.  Multi-GPU sharding and the token-id all-gather live in zsaac/dist.py.
"""
from __future__ import annotations

import copy
import dataclasses
import os
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import ops
from .decoder import Gpt2Decoder, Gpt2Weights, MlpMapper, build_mapper
from .encoder import AudioEncoder


@dataclass
class CaptionConfig:
    encoder: str = "htsat"            # "htsat" | "cnn14"
    mapping_type: str = "mlp"         # "mlp" | "transformer"
    dtype: torch.dtype = torch.bfloat16
    batch: int = 64
    sound_effect_num: int = 3
    normalize_prefix: bool = True
    prefix_length: int = 10
    entry_length: int = 67
    beam: int = 0                     # 0 -> greedy generate2, else generate_beam(beam_size)
    prefix_tokens: bool = True        # also compute get_prefix_tokens (predict_prompt.py:137)
    use_graph: bool = True
    compact_decode: bool = True       # greedy bf16: decode only the rows that have not stopped
    clip_length: int = 10             # TransformerMapper clip_length (params.json prefix_length_clip)
    mapper_layers: int = 8            # TransformerMapper num_layers (params.json num_layers)
    persist_decode: Optional[bool] = None   # greedy bf16 at <= 64 rows: the persistent decode
                                      # launch (zs_gpt2_decode_persist); None = env ZSAAC_PERSIST (on)
    encoder_batch: int = 64           # clips per encoder pass (the reference's eval batch size);
                                      # a larger ``batch`` is encoded in chunks of this size and
                                      # decoded together (clip results do not depend on it)


@dataclass
class CaptionBatch:
    ids: torch.Tensor          # greedy: [B, steps] int32; beam: [B, beam, steps]
    lengths: torch.Tensor      # greedy: [B] int32; beam: [B, beam] f32 seq_len
    scores: Optional[torch.Tensor]
    hard_ids: torch.Tensor     # [B, h_cap] int32 (0-padded)
    hard_len: torch.Tensor     # [B]
    plen: torch.Tensor         # [B] prompt length H + 10
    prefix_ids: Optional[torch.Tensor]   # [B, Pmax] int32 get_prefix_tokens ids
    clap_emb: torch.Tensor     # [B, 1024]

    def captions(self) -> List[List[int]]:
        """Per clip: the reference's output token list (beam: best beam first)."""
        if self.scores is None:
            ids, ln = self.ids.cpu().numpy(), self.lengths.cpu().numpy()
            return [ids[b, :ln[b]].tolist() for b in range(ids.shape[0])]
        return [beams[0] for beams in self.beams()]

    def beams(self) -> List[List[List[int]]]:
        ids = self.ids.cpu().numpy()
        ln = self.lengths.cpu().numpy()
        sc = self.scores.cpu().numpy()
        out = []
        for c in range(ids.shape[0]):
            avg = sc[c] / ln[c]                       # scores / seq_lengths (line 153)
            order = np.argsort(-avg, kind="stable")   # scores.argsort(descending=True)
            out.append([ids[c, i, :int(ln[c, i])].tolist() for i in order])
        return out

    def prefix_token_lists(self) -> List[List[int]]:
        pid, pl = self.prefix_ids.cpu().numpy(), self.plen.cpu().numpy()
        return [pid[b, :pl[b]].tolist() for b in range(pid.shape[0])]


# token ids prompt_kernel (csrc/gpt2.hip) writes around the labels: "There", " are",
# " something", ",", " in", " this", " audio", "."
PROMPT_TEMPLATE_IDS = (1858, 389, 1223, 11, 287, 428, 6597, 13)


class CaptionPipeline:
    """Weights from reference-keyed state dicts; all buffers sized for ``cfg.batch`` clips."""

    def __init__(self, caption_sd, audio_sd, label_table: torch.Tensor,
                 label_tokens: Sequence[Sequence[int]], cfg: CaptionConfig = CaptionConfig(),
                 device="cuda"):
        self.cfg = cfg
        dev = torch.device(device)
        self.dev = dev
        B = cfg.batch
        eb = min(B, max(1, cfg.encoder_batch))
        self.encoder = AudioEncoder(audio_sd, cfg.encoder, cfg.dtype, eb, dev) if audio_sd else None
        self.mapper = build_mapper(caption_sd, cfg.mapping_type, dev, cfg.dtype, B,
                                   clip_length=cfg.clip_length, num_layers=cfg.mapper_layers)
        self.gpt = Gpt2Weights(caption_sd, dev, cfg.dtype)
        self._setup_tables(label_table, label_tokens)
        self._alloc()
        # get_prefix_tokens on the soft rows only when every id a hard prompt can hold (the
        # template tokens of prompt_kernel, gpt2.hip, and the label table's tokens) is its own
        # cosine argmax by a margin above the dtype's rounding (bf16 2e-2, f32 1e-4)
        cand = list(PROMPT_TEMPLATE_IDS) + [t for toks in label_tokens for t in toks]
        margin = 2e-2 if cfg.dtype == torch.bfloat16 else 1e-4
        self.hard_skip = cfg.prefix_tokens and self.decoder.hard_rows_safe(cand, margin)

    def twin(self) -> "CaptionPipeline":
        """A pipeline sharing every packed weight with this one but owning its activation
        buffers, KV cache, skinny-GEMM workspace and decode graphs — so it can run a different
        batch concurrently on another HIP stream (ConcurrentRunner)."""
        t = copy.copy(self)
        t.encoder = self.encoder.twin() if self.encoder is not None else None
        t.mapper = self.mapper.twin()
        t._alloc()
        return t

    def group_twin(self, k: int) -> "CaptionPipeline":
        """A twin sized for k eval batches (k x cfg.batch clips) whose begin (encode, prompt,
        mapper, get_prefix_tokens, prefill) runs for all of them at once (begin_group); each
        batch then takes step 0 and its persistent decode on a sub-decoder of its own whose KV
        cache rows are this twin's (Gpt2Decoder.share_rows).  Greedy bf16 / f32 decoding with
        the MLP mapper only."""
        assert not self.cfg.beam and isinstance(self.mapper, MlpMapper)
        sb = self.cfg.batch
        t = copy.copy(self)
        t.cfg = dataclasses.replace(self.cfg, batch=k * sb, encoder_batch=k * sb)
        t.encoder = self.encoder.twin(max_batch=k * sb) if self.encoder is not None else None
        t.mapper = self.mapper.twin()        # (called per eval batch: sb rows)
        t._alloc()
        t.sub_batch = sb
        t.soft_buf = torch.empty(k * sb, self.mapper.soft_ld, device=self.dev)
        t.subs = []
        for j in range(k):
            d = Gpt2Decoder(self.gpt, sb, self.Pmax, self.cfg.entry_length, max_prefill_rows=1,
                            use_graph=self.cfg.use_graph, topk=8, compact=self.cfg.compact_decode,
                            persist=self.cfg.persist_decode, alloc_kv=False)
            d.share_rows(t.decoder, j * sb)
            t.subs.append(d)
        return t

    def begin_group(self, emb: torch.Tensor, sizes: Optional[Sequence[int]] = None):
        """The begins of the consecutive eval batches of ``emb`` [<= k x sub_batch, 1024] at once
        (``sizes``: the batches' clip counts, each <= sub_batch; default: sub_batch each, the last
        ragged)
        (group_twin): prompt assembly, L2 norm, the mapper (one launch pair per eval batch, as a
        batch's own begin runs it), prefill_embed, get_prefix_tokens and the prefill over every
        row, then step 0 of each batch on its sub-decoder, persistent launches deferred
        (sub-decoder.launch_pending).  Every kernel's per-row arithmetic is independent of the
        rows it runs with (the tiled GEMMs accumulate k in order whatever the tile), so each
        batch's ids equal its own begin's (tests/test_gpu_persist.py)."""
        cfg, B, Pmax, sb = self.cfg, emb.shape[0], self.Pmax, self.sub_batch
        assert B <= cfg.batch
        if sizes is None:
            sizes = [min(sb, B - r) for r in range(0, B, sb)]
        sizes = [int(z) for z in sizes]
        assert sum(sizes) == B and len(sizes) <= len(self.subs) and all(0 < z <= sb for z in sizes)
        self._B, self._emb, self._sizes = B, emb, sizes
        self._offs = [sum(sizes[:j]) for j in range(len(sizes))]
        ops.prompt_assemble(emb, self.labels, cfg.sound_effect_num, self.label_tok, self.label_len,
                            self.hard_ids[:B], self.hard_len[:B])
        prefix = self.prefix[:B]
        if cfg.normalize_prefix:
            ops.l2norm(emb, out=prefix)               # dataset.py:448-449
        else:
            prefix.copy_(emb)
        soft = self.soft_buf[:B]
        for c0, z in zip(self._offs, sizes):      # the mapper per eval batch, as its own begin
            soft[c0:c0 + z].copy_(self.mapper(prefix[c0:c0 + z]))
        dec = self.decoder
        ops.prefill_embed(self.hard_ids[:B], self.hard_len[:B], soft, self.mapper.soft_ld,
                          cfg.prefix_length, self.gpt.wte, self.gpt.wpe, B, Pmax,
                          self.embed[:B * Pmax], dec.x, dec.plen, dec.last_row)
        if cfg.prefix_tokens:
            self.prefix_tokens(B, soft)
        dec.prefill(B, Pmax)
        for j, (r0, r) in enumerate(zip(self._offs, sizes)):
            d = self.subs[j]
            if d.kc[0].data_ptr() != dec.kc[0][r0:].data_ptr():
                d.share_rows(dec, r0)           # (batch j's rows start at r0 this time)
            d.greedy_begin_device(r)
            d.defer_launch = True
            try:
                d.greedy_begin_host(r)
            finally:
                d.defer_launch = False

    def sub_result(self, j: int) -> CaptionBatch:
        """Batch j of the last begin_group's outputs (views, valid until the next begin_group)."""
        Pmax = self.Pmax
        r0, r = self._offs[j], self._sizes[j]
        d = self.subs[j]
        pid = (self.prefix_ids[r0 * Pmax:(r0 + r) * Pmax].view(r, Pmax)
               if self.cfg.prefix_tokens else None)
        return CaptionBatch(d.out_ids[:r], d.out_len[:r], None, self.hard_ids[r0:r0 + r],
                            self.hard_len[r0:r0 + r], d.plen[:r], pid, self._emb[r0:r0 + r])

    def _alloc(self):
        cfg, dev, B = self.cfg, self.dev, self.cfg.batch
        beam = max(cfg.beam, 1)
        # beam: per-block top-`beam` lists suffice for the global top-beam (fewer candidates to
        # sort in the LM head's epilogue and to merge in beam_step)
        self.decoder = Gpt2Decoder(self.gpt, B * beam, self.Pmax, cfg.entry_length,
                                   max_prefill_rows=B, use_graph=cfg.use_graph,
                                   topk=cfg.beam if cfg.beam else 8,
                                   compact=cfg.compact_decode, persist=cfg.persist_decode)
        i32 = dict(device=dev, dtype=torch.int32)
        self.hard_ids = torch.zeros(B, self.h_cap, **i32)
        self.hard_len = torch.zeros(B, **i32)
        self.prefix = torch.empty(B, 1024, device=dev)
        self.embed = torch.empty(B * self.Pmax, 768, device=dev)
        self.prefix_ids = torch.zeros(B * self.Pmax, **i32)
        self.emb_buf = torch.empty(B, 1024, device=dev)
        self.emb_in = torch.empty(B, 1024, device=dev)     # begin_emb_graphed's input
        self._begin_graphs = {}

    def _setup_tables(self, label_table, label_tokens):
        cfg, dev = self.cfg, self.dev
        self.labels = label_table.to(device=dev, dtype=torch.float32).contiguous()
        mt = max(len(t) for t in label_tokens)
        lt = np.zeros((len(label_tokens), mt), dtype=np.int32)
        for i, t in enumerate(label_tokens):
            lt[i, :len(t)] = t
        self.label_tok = torch.from_numpy(lt).to(dev)
        self.label_len = torch.tensor([len(t) for t in label_tokens], dtype=torch.int32, device=dev)
        k = cfg.sound_effect_num
        # longest possible hard prompt: "There are" + k labels + (k-1) commas + " in this audio."
        self.h_cap = 2 + k * mt + max(k - 1, 0) + 4 if k > 0 else 7
        self.Pmax = self.h_cap + cfg.prefix_length

    def encode(self, wav: torch.Tensor) -> torch.Tensor:
        """CLAP embeddings [B, 1024] of a waveform batch, encoder_batch clips per pass."""
        assert self.encoder is not None, "no audio encoder weights"
        B, eb = wav.shape[0], self.encoder.B
        if B <= eb:
            return self.encoder.encode(wav)
        for c0 in range(0, B, eb):
            c1 = min(B, c0 + eb)
            self.emb_buf[c0:c1].copy_(self.encoder.encode(wav[c0:c1]))
        return self.emb_buf[:B]

    def caption_wav(self, wav: torch.Tensor) -> CaptionBatch:
        return self.caption_emb(self.encode(wav))

    def caption_emb(self, emb: torch.Tensor) -> CaptionBatch:
        """From CLAP audio embeddings [B, 1024] (the pickle's ``audio_embedding``)."""
        self.begin_emb(emb)
        self.decoder.run_to_completion()
        return self.result()

    # ------------------------------------------------------------------ async (no host sync)
    def begin_wav(self, wav: torch.Tensor):
        self.begin_emb(self.encode(wav))

    def result(self) -> CaptionBatch:
        """Views of the current batch's outputs (valid until the next begin_*)."""
        B, cfg, dec = self._B, self.cfg, self.decoder
        if cfg.beam:
            R = B * cfg.beam
            ids = dec.out_ids[:R].view(B, cfg.beam, -1)
            ln, sc = dec.seq_len[:R].view(B, cfg.beam), dec.scores[:R].view(B, cfg.beam)
        else:
            ids, ln, sc = dec.out_ids[:B], dec.out_len[:B], None
        pid = self.prefix_ids[:B * self.Pmax].view(B, self.Pmax) if cfg.prefix_tokens else None
        return CaptionBatch(ids, ln, sc, self.hard_ids[:B], self.hard_len[:B], dec.plen[:B], pid,
                            self._emb)

    def prefix_tokens(self, B: int, soft: torch.Tensor):
        """get_prefix_tokens ids of the current batch into prefix_ids (after prefill_embed)."""
        n, Pmax, dec = self.cfg.prefix_length, self.Pmax, self.decoder
        if (self.hard_skip and self.mapper.soft_ld == n * 768 and soft.is_contiguous()
                and soft.dtype == torch.float32):
            dec.prefix_tokens_soft(soft.reshape(-1)[:B * n * 768].view(B * n, 768),
                                   self.hard_ids[:B], self.hard_len[:B], B, Pmax,
                                   self.prefix_ids[:B * Pmax])
        else:
            dec.prefix_tokens(self.embed[:B * Pmax], self.prefix_ids[:B * Pmax])

    def begin_emb(self, emb: torch.Tensor):
        """Enqueue prompt assembly, mapper, prefill, get_prefix_tokens and decode step 0 for a
        batch of CLAP embeddings, without any host synchronisation."""
        cfg, B = self.cfg, emb.shape[0]
        self._B, self._emb = B, emb
        assert B <= cfg.batch
        self._begin_device(emb)
        dec = self.decoder
        if cfg.beam:
            dec.beam_begin(B, cfg.beam)
        else:
            dec.greedy_begin_host(B)

    def begin_emb_graphed(self, emb: torch.Tensor):
        """begin_emb with its device work (prompt .. step 0: ~100 kernels) replayed from a hipGraph
        per batch size, captured on first use on the current (non-default) stream: the embedding
        is copied into a fixed buffer first, every other operand already lives in this pipeline's
        buffers.  Greedy decoding only (beam search: begin_emb).  A kernel trace of the headline
        showed a begin's stream idle between its kernels for 50-75 % of the begin's wall time
        (tools/tl_phases.py: 14-30 ms wall, 5-13 ms of kernels beside the decode grids)."""
        cfg, B = self.cfg, emb.shape[0]
        assert B <= cfg.batch and not cfg.beam
        self.emb_in[:B].copy_(emb)
        if not hasattr(self, "_begin_graphs"):
            self._begin_graphs = {}
        g = self._begin_graphs.get(B)
        if g is None:
            g = torch.cuda.CUDAGraph()
            g.capture_begin()
            try:
                self._begin_device(self.emb_in[:B])
            finally:
                g.capture_end()
            self._begin_graphs[B] = g
            self.decoder.n_captures += 1
        g.replay()
        self._B, self._emb = B, self.emb_in[:B]
        self.decoder.greedy_begin_host(B)

    def _begin_device(self, emb: torch.Tensor):
        """The device work of a begin (no host state: capturable)."""
        cfg, B, Pmax = self.cfg, emb.shape[0], self.Pmax
        ops.prompt_assemble(emb, self.labels, cfg.sound_effect_num, self.label_tok, self.label_len,
                            self.hard_ids[:B], self.hard_len[:B])
        prefix = self.prefix[:B]
        if cfg.normalize_prefix:
            ops.l2norm(emb, out=prefix)               # dataset.py:448-449
        else:
            prefix.copy_(emb)
        soft = self.mapper(prefix)
        dec = self.decoder
        ops.prefill_embed(self.hard_ids[:B], self.hard_len[:B], soft, self.mapper.soft_ld,
                          cfg.prefix_length, self.gpt.wte, self.gpt.wpe, B, Pmax,
                          self.embed[:B * Pmax], dec.x, dec.plen, dec.last_row)
        if cfg.prefix_tokens:
            self.prefix_tokens(B, soft)
        if cfg.beam:
            dec.prefill(B, Pmax, row_stride=cfg.beam)
        else:
            dec.prefill(B, Pmax)
            dec.greedy_begin_device(B)


def persist_grids(env: Optional[str] = None) -> List[int]:
    """The persistent-decode grid sizes (workgroups of 256 threads, ops.PERSIST_GRIDS) a runner
    may use, largest first: ``env`` or ZSAAC_PERSIST_GRIDS ("192,96,48"); with ``env`` None and
    ZSAAC_PERSIST_GRID set, that one size alone.  Every size gives the same ids (decode_grid.hip's
    canonical arithmetic), so the choice is a scheduling decision only."""
    if env is None:
        env = (os.environ["ZSAAC_PERSIST_GRID"] if "ZSAAC_PERSIST_GRID" in os.environ
               else os.environ.get("ZSAAC_PERSIST_GRIDS", DEFAULT_PERSIST_GRIDS))
    grids = sorted({int(t) for t in env.replace(" ", "").split(",") if t}, reverse=True)
    for g in grids:
        assert g in ops.PERSIST_GRIDS, f"persist grid {g} (one of {ops.PERSIST_GRIDS})"
    return grids


# largest first; the last is the throughput grid every batch can fall back to (192 stays
# available: alone it has the shortest step, but beside other grids 96 wins -- a 131-clip shard
# 3.47k vs 2.42k clips/s, the headline equal)
DEFAULT_PERSIST_GRIDS = "96,48"


def persist_budget(cus: int, staged: bool = False) -> int:
    """Workgroup slots the in-flight persistent grids may hold together: a grid workgroup takes
    half a CU (4 waves x <= 256 registers), so 2 x CUs is the chip.  The pipelined schedule's
    default, 1.5 x CUs (8 grids of 48), leaves a quarter of the slots to the begins' kernels:
    measured in one process (tools/headline_ab.py, 12 reps, encode-ahead 256, grids sized at
    launch): 5.73k clips/s against 5.33k at 2 x CUs and 4.71k at 1 x CUs.  ``staged``
    (begin_first: the begins have run before the grids) 2 x CUs less a sixteenth, ten grids of 48
    on 256 CUs (profiles/r6/begin_first_ab.txt: 448 / 480 / 512 slots 7.03k / 7.02k / 7.11k on
    the 1045-clip set, 480 / 512 6.96k / 6.81k on 1280 clips).  ZSAAC_PERSIST_BUDGET overrides."""
    dflt = 2 * cus - cus // 8 if staged else 3 * cus // 2
    return int(os.environ.get("ZSAAC_PERSIST_BUDGET", str(dflt)))


def choose_persist_grid(in_flight: int, to_begin: int, grids: List[int], budget: int) -> int:
    """Grid size of the persistent decode launch of the next batch to begin, given the workgroups
    of the grids already in flight and the batches still to begin (this one included): the
    largest grid that, beside the grids in flight and every other batch still to begin at the
    smallest size, fits the budget.  Then every later begin still has room for the smallest grid,
    so (with at most budget // smallest batches in flight) the grids in flight never exceed the
    budget and every persistent launch can be co-resident."""
    g_min = grids[-1]
    for g in grids:
        if in_flight + g + g_min * (to_begin - 1) <= budget:
            return g
    return g_min


_SPLIT_STREAMS = {}     # (device, CUs, begin CUs) -> (begin streams, grid streams)
# a staged run that sees no event complete for this long raises (with its state) instead of
# spinning: a persistent launch that cannot become co-resident gives up after ~2^22 polls (s)
STALL_S = float(os.environ.get("ZSAAC_RUNNER_STALL_S", "60"))
# the first wave of a staged run's grids, released by one gate, start STAGGER_US apart (each
# waits k x STAGGER_US after the gate on the GPU, zs_stream_spin): released together, one grid of
# ten sometimes found no room for all its workgroups until another ended -- a 1280-clip
# repetition 0.16 or 0.18 s at random; staggered by 300 us every repetition took 0.162-0.164 s
# (profiles/r6/begin_first_ab.txt, r6u; 100 us: 2 late grids in 8 repetitions; with begin groups
# of 2, 150 / 200 / 300 us: none in 8 each, 8.01k / 7.99k / 7.97k clips/s, r6ee)
STAGGER_US = int(os.environ.get("ZSAAC_STAGGER_US", "200"))


class ConcurrentRunner:
    """Keeps several independent bs=`cfg.batch` batches in flight on one GPU; the host only
    polls events and a pinned all-done flag (no blocking syncs).  Two schedules:

    * pipelined (run's main loop): pipeline twins (shared weights, private buffers / KV cache /
      graphs), each on its own HIP stream; a batch's begin (encode .. step 0) is enqueued when a
      pipeline frees, its persistent decode grid when the begin has finished -- begins and grids
      share the chip.  Also the path of a run with no more batches than grids fit at once.
    * staged (begin_first, the bench's headline schedule; _run_grouped with begin_group, else
      _run_staged): every begin runs first -- with begin_group k, one begin per k consecutive
      batches on a group twin, each batch decoding on a sub-decoder that shares the twin's KV
      cache rows -- and the decode grids launch once every begin has finished, in batch order as
      the budget frees, on a pool of budget / 48 streams, the first wave released STAGGER_US
      apart.  Ids are the same under either schedule (tests/test_gpu_persist.py).

    Results are copied out on the pipeline's stream before it takes the next batch."""

    def __init__(self, pipe: CaptionPipeline, n_inflight: int = 2, streams: Optional[list] = None,
                 grids: Optional[List[int]] = None, budget: Optional[int] = None,
                 encode_ahead: int = 0, encode_first: bool = False, begin_first: bool = False,
                 extra_pipes: int = 0, enc_stream=None, cu_split: int = 0,
                 begin_gate: int = 0, begin_group: int = 0, n_batches: int = 0):
        self.cus = torch.cuda.get_device_properties(pipe.dev).multi_processor_count
        # persistent grids (greedy bf16 at <= 64 rows; beam search never launches one), one size
        # per batch from `grids` (largest first, see choose_persist_grid)
        self.persist = pipe.decoder.persist and not pipe.cfg.beam
        self.grids = grids or (list(ops.PERSIST_GRIDS_F32) if getattr(pipe.decoder, "f32_grid", False)
                               else persist_grids())
        self.budget = budget or persist_budget(self.cus)
        # begin_first (persistent decode only): every pipeline begins its batch (prompt .. step 0)
        # at once, and the persistent launches follow as the budget frees, the first ones after
        # every first-round begin -- the begins run on the whole chip instead of beside the grids
        self.begin_first = bool(begin_first) and self.persist
        # begin_first: the first persistent launches wait for the first `begin_gate` begins (0:
        # every begin of the first round), so those begins run beside no decode grid
        self.begin_gate = int(begin_gate)
        # begin_group k > 0 (begin_first, greedy, MLP mapper): the begins of k consecutive eval
        # batches run as ONE begin of k x batch clips on a group twin (CaptionPipeline.group_twin:
        # encoder pass, prefill and get_prefix_tokens at k x the rows), each batch then decodes
        # on a sub-decoder sharing the twin's KV cache rows; n_batches sizes the group twins
        # warmup() prepares
        self.begin_group = (int(begin_group) if self.begin_first and not pipe.cfg.beam
                            and isinstance(pipe.mapper, MlpMapper) else 0)
        self.n_batches = int(n_batches)
        self.gpipes: List[CaptionPipeline] = []
        self.late_grid = True     # grid size chosen when the begin has finished (False: at begin)
        # one begin per pass over the pipelines: a begin costs milliseconds of host enqueue, so
        # beginning every idle pipeline in one pass delayed the first grids' launches until the
        # last begin was enqueued (~43 ms into the headline, tools/timeline.py)
        self.one_begin = True
        # the encoder's up-front passes replayed from per-size hipGraphs (Encoder.encode_graphed)
        self.enc_graph = True
        self.spread = False       # A/B: exclusive (one CU per workgroup) grids while CUs allow
        # A/B (ZSAAC_GRAPH_BEGINS=1): greedy begins replayed from per-pipeline hipGraphs
        # (CaptionPipeline.begin_emb_graphed), captured in warmup -- measured 5.75k vs 5.86k and
        # 5.09k vs 5.30k clips/s (same box, medians of 5): the idle time between a begin's kernels
        # beside the grids is waiting for CU resources, not host enqueue
        self.graph_begins = self.persist and os.environ.get("ZSAAC_GRAPH_BEGINS", "0") != "0"
        if self.persist and (not self.begin_first or self.begin_group):
            # persistent decode grids must be co-resident: at most budget // (smallest grid)
            n_inflight = max(1, min(n_inflight, self.budget // self.grids[-1]))
        self.n_inflight = n_inflight
        # extra_pipes: pipelines beyond the grids the budget holds, so the next batches' begins
        # (prefill etc.) run while every grid slot decodes and launch the moment one frees
        n_pipes = n_inflight + (max(0, int(extra_pipes)) if self.persist else 0)
        self.pipes = [pipe] + [pipe.twin() for _ in range(n_pipes - 1)]
        # encode_ahead > 0 (waveform inputs): one encoder twin sized for that many clips encodes
        # every batch's clips up front, in passes of up to encode_ahead clips (consecutive
        # batches), on a stream of its own; a batch's begin (mapper .. step 0) waits only for its
        # own pass.  The encoder then runs at its most efficient size and before the decode grids
        # fill the chip; captions do not depend on it (a clip's embedding is its own).
        # encode_first: every begin waits for the LAST pass (encoding and decoding do not share
        # the chip).
        self.encode_ahead = int(encode_ahead) if pipe.encoder is not None else 0
        self.encode_first = bool(encode_first)
        self.enc = pipe.encoder.twin(max_batch=self.encode_ahead) if self.encode_ahead else None
        # dedicated streams on distinct hardware queues: pooled torch streams take their queue at
        # first use and can end up sharing one, which serializes the batches
        # (``streams``: reuse another runner's, at least as many -- tools/headline_ab.py)
        need = len(self.pipes)
        if self.begin_first:
            # begin_first keeps a pipeline per batch but only as many streams as grids can run at
            # once: every stream is a hardware queue, and a process holding more queues than the
            # scheduler maps at once gets its queues time-sliced (a stream per pipeline, 20 at
            # 1280 clips, slowed every later multi-stream run 5-27 %; a pool of 12 still cost C3
            # 9 % and C5's step 2.7 -> 3.8 ms, a pool of 10 nothing: profiles/r6/begin_first_ab.txt)
            cap = self.budget // self.grids[-1]
            need = cap if self.begin_group else min(need, cap)
        # cu_split > 0 (persistent decode, A/B option): the chip is split by CU masks -- the
        # pipelines' begins (prompt .. step 0, and a give-up's phase launches) on cu_split CUs,
        # the decode grids on the rest (each pipeline launches its grid on a second stream of
        # its own); the budget then holds the grids to two workgroups per grid CU
        self.cu_split = int(cu_split) if self.persist else 0
        self.gstreams = None
        if self.cu_split:
            key = (str(pipe.dev), self.cus, self.cu_split)
            have = _SPLIT_STREAMS.setdefault(key, ([], []))   # reused by later runners
            bmask, gmask = ops.cu_split_masks(self.cus, self.cu_split)
            if len(have[0]) < need:
                have[0].extend(ops.masked_streams(need - len(have[0]), pipe.dev, bmask))
                have[1].extend(ops.masked_streams(need - len(have[1]), pipe.dev, gmask))
            streams, self.gstreams = have[0][:need], have[1][:need]
            self.budget = min(self.budget, 2 * (self.cus - self.cu_split))
        streams = (list(streams[:need]) if streams is not None
                   else ops.dedicated_streams(need, pipe.dev, priority=-1))
        assert len(streams) == need, "ConcurrentRunner: too few streams given"
        self.streams = streams
        # the encoder running ahead yields to the begins and grids: a low-priority stream
        self.enc_stream = None
        if self.enc is not None:
            self.enc_stream = (enc_stream if enc_stream is not None
                               else ops.dedicated_streams(1, pipe.dev, priority=1)[0])

    def warmup(self, wav: torch.Tensor):
        """Runs one batch per pipeline synchronously (captures every decode graph, and with
        graph_begins the begin graph of this batch size)."""
        for i, p in enumerate(self.pipes):
            s = self.streams[i % len(self.streams)]
            s.wait_stream(torch.cuda.current_stream(p.dev))
            with torch.cuda.stream(s):
                if self.graph_begins:
                    p.begin_emb(p.encode(wav))          # (eager first: every lazy buffer exists)
                    p.decoder.run_to_completion()
                    p.begin_emb_graphed(p.encode(wav))
                    p.decoder.run_to_completion()
                else:
                    p.caption_wav(wav)
                p.decoder.capture_buckets()
            s.synchronize()
        self._warm_groups(wav, "wav")

    def warmup_emb(self, emb: torch.Tensor):
        for i, p in enumerate(self.pipes):
            s = self.streams[i % len(self.streams)]
            s.wait_stream(torch.cuda.current_stream(p.dev))
            with torch.cuda.stream(s):
                p.caption_emb(emb)
                if self.graph_begins:
                    p.begin_emb_graphed(emb)
                    p.decoder.run_to_completion()
                p.decoder.capture_buckets()
            s.synchronize()
        self._warm_groups(emb, "emb")

    def decoders(self) -> List[Gpt2Decoder]:
        """Every decoder this runner steps: the pipelines' and the group twins' sub-decoders."""
        return [p.decoder for p in self.pipes] + [d for G in self.gpipes for d in G.subs]

    def _warm_groups(self, x: torch.Tensor, inputs: str):
        """begin_group: the group twins a run of n_batches needs, each run once (a full group of
        x's rows repeated) with its sub-decoders' persistent launches, synchronously."""
        k = self.begin_group
        if not k or not self.n_batches:
            return
        need = -(-self.n_batches // k)
        while len(self.gpipes) < need:
            self.gpipes.append(self.pipes[0].group_twin(k))
        sb = self.pipes[0].cfg.batch
        xs = x.repeat((-(-k * sb // x.shape[0]),) + (1,) * (x.dim() - 1))[:k * sb].contiguous()
        s = self.streams[0]
        s.wait_stream(torch.cuda.current_stream(self.pipes[0].dev))
        for G in self.gpipes:
            with torch.cuda.stream(s):
                G.begin_group(G.encode(xs) if inputs == "wav" else xs)
                for d in G.subs:
                    d.persist_grid = self.grids[-1]
                    d.persist_exclusive = False
                    d.launch_pending()
                    d.run_to_completion()
            s.synchronize()

    def run(self, batches: Sequence[torch.Tensor], keep=None, inputs: str = "wav") -> List[CaptionBatch]:
        """Captions every batch (waveforms [B, n] or, with inputs="emb", CLAP embeddings
        [B, 1024]; B <= cfg.batch, ragged last batch allowed); returns CaptionBatch copies in
        input order.  ``keep`` optionally post-processes a result on its pipeline's stream; the
        completion order is timing-dependent, so it must not issue collectives (gather after
        run() instead, in input order — see bench.py)."""
        assert inputs in ("wav", "emb")
        self.bdec = None                 # (_run_grouped: batch -> the sub-decoder that decoded it)
        results: List[Optional[CaptionBatch]] = [None] * len(batches)
        caller = torch.cuda.current_stream(self.pipes[0].dev)
        for s in self.streams:           # inputs were produced on the caller's stream
            s.wait_stream(caller)
        staged = self.begin_first and len(batches) > self.budget // self.grids[-1]
        ahead = None
        if inputs == "wav" and self.enc is not None and not staged and len(batches) > len(self.pipes):
            # (a pipelined run that fits its pipelines at once begins sooner encoding per batch:
            # measured on a 131-clip shard, 37.5 vs 40 ms.  A staged run encodes on its begins'
            # streams: with the encoder's passes on their low-priority stream every repetition
            # took 2-32 s instead of 0.15 s -- profiles/r6/begin_first_ab.txt, r6i)
            ahead = self._encode_ahead(batches, caller)
        if staged and self.begin_group:
            return self._run_grouped(batches, keep, inputs, caller)
        if staged:
            # (more batches than grids the budget holds at once; fewer take the pipelined path
            # below, whose small-run form gives each batch an exclusive grid)
            return self._run_staged(batches, keep, inputs, caller, ahead)
        # a run that fits its pipelines at once (a small shard) has no later begins to leave room
        # for: its grids may fill the chip, and they take one CU per workgroup (exclusive
        # launches) while the CUs allow -- left to itself the dispatcher doubles workgroups up on
        # CUs while others idle (tools/placement.py: 3 grids of 96 covered 185 CUs, 103 twice)
        small = self.persist and len(batches) <= len(self.pipes)
        exclusive = False
        spread = self.spread or small
        budget = 2 * self.cus if small else self.budget
        excl_slots = {}
        excl_in_flight = lambda: sum(excl_slots.values())
        active = {}
        nxt = 0
        trace = self.trace = [] if os.environ.get("ZSAAC_RUNNER_TRACE") else None
        t_run = time.perf_counter()
        self.decode_steps = [0] * len(batches)     # per batch: decode steps actually enqueued
        self.assign = []                           # (pipeline index, batch index), in begin order
        self.grid = [0] * len(batches)             # persistent grid size per batch (0: none)
        self.gave_up = 0                           # launches of this run that resumed stepwise
        slots = {}                                 # pipeline index -> its launch's workgroups
        while nxt < len(batches) or active:
            progressed = False
            if ahead is not None:
                ahead.pump()
            for i, (p, s) in enumerate(zip(self.pipes, self.streams)):
                st = active.get(i)
                if st is None:
                    if nxt < len(batches):
                        # persistent decode: the begin is enqueued now, the grid launch when the
                        # begin has finished (its size chosen then, from the grids in flight and
                        # the batches not yet launched: bigger grids once few batches remain)
                        if self.persist and not self.late_grid:    # (A/B: size at begin)
                            g = choose_persist_grid(sum(slots.values()), len(batches) - nxt,
                                                    self.grids, budget)
                            self.grid[nxt] = slots[i] = g
                            p.decoder.persist_grid = g
                            p.decoder.persist_exclusive = exclusive
                        p.decoder.defer_launch = self.persist and self.late_grid
                        try:
                            self._begin(i, nxt, batches, inputs, ahead)
                        finally:
                            p.decoder.defer_launch = False
                        with torch.cuda.stream(s):
                            if self.persist and self.late_grid:
                                ev = torch.cuda.Event()
                                ev.record(s)
                                active[i] = ("begun", nxt, ev)
                            else:
                                ev, flag = p.decoder.finished_async()
                                active[i] = (nxt, 0, ev, flag)
                        self.assign.append((i, nxt))
                        if trace is not None:
                            trace.append(("begin", nxt, round((time.perf_counter() - t_run) * 1e3, 2)))
                        nxt += 1
                        progressed = True
                        if self.one_begin:
                            break       # launches / completions before the next begin
                    continue
                if st[0] == "begun":
                    _, bi, ev = st
                    if not ev.query():
                        continue
                    unlaunched = len(batches) - nxt + sum(1 for a in active.values()
                                                          if a[0] == "begun")
                    g = choose_persist_grid(sum(slots.values()), unlaunched, self.grids,
                                            budget)
                    if sum(slots.values()) + g > budget:
                        continue               # (extra pipelines: wait for a grid to finish)
                    # spread (A/B option): while the exclusive workgroups in flight leave room,
                    # a grid takes one CU per workgroup (it shares CUs with normal grids only)
                    excl = exclusive or (spread and excl_in_flight() + g <= self.cus)
                    p.decoder.persist_grid = g
                    p.decoder.persist_exclusive = excl
                    slots[i] = g
                    excl_slots[i] = g if excl else 0
                    self.grid[bi] = g
                    gs = self.gstreams[i] if self.gstreams else s
                    if gs is not s:
                        gs.wait_stream(s)
                    with torch.cuda.stream(gs):
                        p.decoder.launch_pending()
                        ev, flag = p.decoder.finished_async()
                    active[i] = (bi, 0, ev, flag)
                    if trace is not None:
                        trace.append(("launch", bi, round((time.perf_counter() - t_run) * 1e3, 2)))
                    progressed = True
                    continue
                bi, n, ev, flag = st
                if not ev.query():
                    continue
                progressed = True
                if self.gstreams and n == 0:
                    s.wait_stream(self.gstreams[i])   # (the grid ran on its own stream)
                if int(flag[1]) < 0:
                    # the persistent launch gave up waiting (its grid was not co-resident): finish
                    # this batch on the per-step path from the state it started from
                    self.gave_up += 1
                    with torch.cuda.stream(s):
                        p.decoder.resume_stepwise()
                        p.decoder.step_chunk(None)
                        ev, flag = p.decoder.finished_async()
                    slots.pop(i, None)
                    excl_slots.pop(i, None)
                    active[i] = (bi, 1, ev, flag)
                    continue
                if int(flag[0]) or n >= p.decoder.n_chunks:
                    p.decoder.note_persist_steps(int(flag[3]))
                    self.decode_steps[bi] = int(flag[3]) if not p.cfg.beam else 1 + n * p.decoder.chunk
                    with torch.cuda.stream(s):
                        r = p.result()
                        results[bi] = _copy_batch(r, caller)
                        if keep is not None:
                            keep(results[bi])
                    del active[i]
                    slots.pop(i, None)
                    excl_slots.pop(i, None)
                else:
                    with torch.cuda.stream(s):
                        p.decoder.step_chunk(int(flag[2]))
                        ev, flag = p.decoder.finished_async()
                    active[i] = (bi, n + 1, ev, flag)
            if not progressed:
                time.sleep(20e-6)
        for s in self.streams:           # results are consumed on the caller's stream
            caller.wait_stream(s)
        for s in self.gstreams or []:
            caller.wait_stream(s)
        if ahead is not None:
            caller.wait_stream(self.enc_stream)
        return results

    def _begin(self, i, bi, batches, inputs, ahead):
        p, s = self.pipes[i], self.streams[i % len(self.streams)]
        begin = p.begin_emb_graphed if self.graph_begins else p.begin_emb
        with torch.cuda.stream(s):
            if ahead is not None:
                s.wait_event(ahead.ready(bi))
                begin(ahead.embs[bi])
            elif inputs == "wav":
                begin(p.encode(batches[bi]))
            else:
                begin(batches[bi])

    def _run_staged(self, batches, keep, inputs, caller, ahead):
        """run() with begin_first: a begin on every free pipeline (persistent launches deferred),
        one begin per pass over the loop so finished batches and launches are handled between
        begins; launches in batch order while the grids in flight fit the budget, each on a
        stream no grid is running on, after its own begin and -- the first ones -- after the
        first `begin_gate` begins (0: every begin of the first round) have finished on the GPU.
        With a pipeline per batch every begin runs before (or beside few) decode grids and every
        later launch finds its batch begun."""
        n = len(batches)
        S = len(self.streams)
        results: List[Optional[CaptionBatch]] = [None] * n
        self.decode_steps = [0] * n
        self.assign, self.grid, self.gave_up = [], [0] * n, 0
        free = list(range(len(self.pipes)))
        n_gate = min(n, len(free)) if self.begin_gate <= 0 else min(n, self.begin_gate)
        begun, active, slots = [], {}, {}
        gate, bev, sbusy = [], {}, set()
        nxt = 0
        trace = self.trace = [] if os.environ.get("ZSAAC_RUNNER_TRACE") else None
        t_run = t_prog = time.perf_counter()
        while nxt < n or begun or active:
            progressed = False
            if ahead is not None:
                ahead.pump()
            if nxt < n and free:
                i = free.pop(0)
                self.pipes[i].decoder.defer_launch = True
                try:
                    self._begin(i, nxt, batches, inputs, ahead)
                finally:
                    self.pipes[i].decoder.defer_launch = False
                ev = torch.cuda.Event()
                ev.record(self.streams[i % S])
                bev[nxt] = ev
                if len(gate) < n_gate:
                    gate.append(ev)
                begun.append((nxt, i))
                self.assign.append((i, nxt))
                if trace is not None:
                    trace.append(("begin", nxt, round((time.perf_counter() - t_run) * 1e3, 2)))
                nxt += 1
                progressed = True
            while begun and len(gate) >= n_gate and len(sbusy) < S:
                bi, i = begun[0]
                used = sum(slots.values())
                g = choose_persist_grid(used, len(begun) + n - nxt, self.grids, self.budget)
                if used + g > self.budget:
                    break
                k = next(k for k in range(S) if k not in sbusy)
                p, s = self.pipes[i], self.streams[k]
                p.decoder.persist_grid = g
                p.decoder.persist_exclusive = False    # (not a value left over from run())
                with torch.cuda.stream(s):
                    s.wait_event(bev.pop(bi))
                    for ev in gate:          # the first launches: after the gating begins
                        s.wait_event(ev)
                    if gate and STAGGER_US:      # (released in turn, as _run_grouped)
                        ops.stream_spin(STAGGER_US * len(sbusy), s)
                    p.decoder.launch_pending()
                    ev, flag = p.decoder.finished_async()
                slots[i] = g
                sbusy.add(k)
                self.grid[bi] = g
                active[i] = (bi, 0, ev, flag, k)
                begun.pop(0)
                if trace is not None:
                    trace.append(("launch", bi, round((time.perf_counter() - t_run) * 1e3, 2)))
                progressed = True
            if len(gate) >= n_gate and active:
                gate = []                    # (launches after the first ones: no gate)
                n_gate = 0
            for i in list(active):
                bi, c, ev, flag, k = active[i]
                if not ev.query():
                    continue
                progressed = True
                p, s = self.pipes[i], self.streams[k]
                if int(flag[1]) < 0:          # gave up (not co-resident): finish stepwise
                    self.gave_up += 1
                    with torch.cuda.stream(s):
                        p.decoder.resume_stepwise()
                        p.decoder.step_chunk(None)
                        ev, flag = p.decoder.finished_async()
                    slots.pop(i, None)
                    active[i] = (bi, 1, ev, flag, k)
                    continue
                if int(flag[0]) or c >= p.decoder.n_chunks:
                    p.decoder.note_persist_steps(int(flag[3]))
                    self.decode_steps[bi] = int(flag[3])
                    with torch.cuda.stream(s):
                        results[bi] = _copy_batch(p.result(), caller)
                        if keep is not None:
                            keep(results[bi])
                    del active[i]
                    slots.pop(i, None)
                    sbusy.discard(k)
                    free.append(i)
                else:
                    with torch.cuda.stream(s):
                        p.decoder.step_chunk(int(flag[2]))
                        ev, flag = p.decoder.finished_async()
                    active[i] = (bi, c + 1, ev, flag, k)
            if progressed:
                t_prog = time.perf_counter()
            else:
                time.sleep(20e-6)
                if time.perf_counter() - t_prog > STALL_S:
                    raise RuntimeError(
                        f"ConcurrentRunner (begin_first): no progress for {STALL_S} s; begun "
                        f"{begun}, active {[(i, a[0], a[1], a[4]) for i, a in active.items()]}, "
                        f"grids {slots}, next batch {nxt} of {n}")
        for s in self.streams:
            caller.wait_stream(s)
        if ahead is not None:
            caller.wait_stream(self.enc_stream)
        return results

    def _run_grouped(self, batches, keep, inputs, caller):
        """run() with begin_first and begin_group k: one begin per group of k consecutive eval
        batches (CaptionPipeline.begin_group on a group twin: the encoder pass, prefill and
        get_prefix_tokens at k x the rows), the groups' begins spread over the streams and all
        enqueued first; the decode grids then launch in batch order within the budget, each on
        a stream no grid is running on, after its group's begin -- the first ones after every
        group's begin has finished on the GPU."""
        n, k, S = len(batches), self.begin_group, len(self.streams)
        budget = self.budget
        groups = [list(range(g, min(n, g + k))) for g in range(0, n, k)]
        while len(self.gpipes) < len(groups):
            self.gpipes.append(self.pipes[0].group_twin(k))
        results: List[Optional[CaptionBatch]] = [None] * n
        self.decode_steps = [0] * n
        self.assign, self.grid, self.gave_up = [], [0] * n, 0
        gev = []
        trace = self.trace = [] if os.environ.get("ZSAAC_RUNNER_TRACE") else None
        if trace is not None:
            self.traces = getattr(self, "traces", []) + [trace]
        t_run = t_prog = time.perf_counter()
        for gi, bl in enumerate(groups):      # (on one stream: 5.3k instead of 7.3k clips/s)
            G, s = self.gpipes[gi], self.streams[gi % S]
            with torch.cuda.stream(s):
                x = _rows_span([batches[b] for b in bl])
                G.begin_group(G.encode(x) if inputs == "wav" else x,
                              [int(batches[b].shape[0]) for b in bl])
                ev = torch.cuda.Event()
                ev.record(s)
            gev.append(ev)
            if trace is not None:
                trace.append(("begin_group", gi, round((time.perf_counter() - t_run) * 1e3, 2)))
        pending = [(gi, j, b) for gi, bl in enumerate(groups) for j, b in enumerate(bl)]
        self.bdec = {b: self.gpipes[gi].subs[j] for gi, j, b in pending}
        gate = list(gev)    # (gating on fewer groups brought the late grid back: r6w)
        active, slots, sbusy = {}, {}, set()
        while pending or active:
            progressed = False
            while pending and len(sbusy) < S:
                gi, j, b = pending[0]
                used = sum(slots.values())
                g = choose_persist_grid(used, len(pending), self.grids, budget)
                if used + g > budget:
                    break
                kk = next(q for q in range(S) if q not in sbusy)
                d, s = self.gpipes[gi].subs[j], self.streams[kk]
                d.persist_grid = g
                d.persist_exclusive = False
                with torch.cuda.stream(s):
                    s.wait_event(gev[gi])
                    for ev in gate:          # the first launches: after every group's begin
                        s.wait_event(ev)
                    if gate and STAGGER_US:      # the first wave's grids released in turn
                        ops.stream_spin(STAGGER_US * len(sbusy), s)
                    d.launch_pending()
                    ev, flag = d.finished_async()
                slots[b] = g
                sbusy.add(kk)
                self.grid[b] = g
                self.assign.append((gi, b))
                active[b] = (gi, j, 0, ev, flag, kk)
                pending.pop(0)
                if trace is not None:
                    trace.append(("launch", b, round((time.perf_counter() - t_run) * 1e3, 2)))
                progressed = True
            if active:
                gate = []
            for b in list(active):
                gi, j, c, ev, flag, kk = active[b]
                if not ev.query():
                    continue
                progressed = True
                G, s = self.gpipes[gi], self.streams[kk]
                d = G.subs[j]
                if int(flag[1]) < 0:          # gave up (not co-resident): finish stepwise
                    self.gave_up += 1
                    with torch.cuda.stream(s):
                        d.resume_stepwise()
                        d.step_chunk(None)
                        ev, flag = d.finished_async()
                    slots.pop(b, None)
                    active[b] = (gi, j, 1, ev, flag, kk)
                    continue
                if int(flag[0]) or c >= d.n_chunks:
                    d.note_persist_steps(int(flag[3]))
                    self.decode_steps[b] = int(flag[3])
                    if trace is not None:
                        trace.append(("done", b, round((time.perf_counter() - t_run) * 1e3, 2)))
                    with torch.cuda.stream(s):
                        results[b] = _copy_batch(G.sub_result(j), caller)
                        if keep is not None:
                            keep(results[b])
                    del active[b]
                    slots.pop(b, None)
                    sbusy.discard(kk)
                else:
                    with torch.cuda.stream(s):
                        d.step_chunk(int(flag[2]))
                        ev, flag = d.finished_async()
                    active[b] = (gi, j, c + 1, ev, flag, kk)
            if progressed:
                t_prog = time.perf_counter()
            else:
                time.sleep(20e-6)
                if time.perf_counter() - t_prog > STALL_S:
                    raise RuntimeError(
                        f"ConcurrentRunner (begin_group): no progress for {STALL_S} s; pending "
                        f"{pending[:4]}.., active {[(b, a[0], a[2], a[5]) for b, a in active.items()]}, "
                        f"grids {slots}")
        for s in self.streams:
            caller.wait_stream(s)
        return results

    def _encode_ahead(self, batches, caller):
        """The encoder passes of every batch on the encoder stream: consecutive batches grouped
        up to encode_ahead clips (one view when they are adjacent rows of one tensor, as the
        bench's are, else concatenated), enqueued one pass at a time (_EncodeAhead.pump): a pass
        queued far ahead would hold the GPU ahead of the begins issued after it."""
        return _EncodeAhead(self, batches, caller)


class _EncodeAhead:
    def __init__(self, runner, batches, caller):
        E = runner.encode_ahead
        self.enc, self.es, self.batches = runner.enc, runner.enc_stream, batches
        n = sum(int(b.shape[0]) for b in batches)
        self.emb = torch.empty(n, 1024, device=runner.pipes[0].dev)
        self.es.wait_stream(caller)
        self.passes, self.pass_of, self.embs = [], [], []
        i, c0 = 0, 0
        while i < len(batches):
            j, m = i, 0
            while j < len(batches) and m + int(batches[j].shape[0]) <= E:
                m += int(batches[j].shape[0])
                j += 1
            assert j > i, f"a batch of {batches[i].shape[0]} clips > encode_ahead {E}"
            self.passes.append((i, j, c0, m))
            for b in batches[i:j]:
                self.pass_of.append(len(self.passes) - 1)
                self.embs.append(self.emb[c0:c0 + int(b.shape[0])])
                c0 += int(b.shape[0])
            i = j
        self.events = []
        self.graph = runner.enc_graph
        self.first = runner.encode_first
        self.pump(force=1)

    def pump(self, force=0):
        """Enqueues the next pass when none is in flight (or until `force` passes are)."""
        while len(self.events) < len(self.passes):
            if len(self.events) >= force and self.events and not self.events[-1].query():
                return
            i, j, c0, m = self.passes[len(self.events)]
            with torch.cuda.stream(self.es):
                enc = self.enc.encode_graphed if self.graph else self.enc.encode
                self.emb[c0:c0 + m].copy_(enc(_rows_span(self.batches[i:j])))
                ev = torch.cuda.Event()
                ev.record(self.es)
            self.events.append(ev)

    def ready(self, b):
        """The event batch b's begin waits for (its pass enqueued first if needed)."""
        k = len(self.passes) - 1 if self.first else self.pass_of[b]
        self.pump(force=k + 1)
        return self.events[k]


def _rows_span(ts: Sequence[torch.Tensor]) -> torch.Tensor:
    """The row-wise concatenation of 2-D tensors: a view when they are adjacent row ranges of one
    contiguous tensor, else a copy."""
    if len(ts) == 1:
        return ts[0]
    t0 = ts[0]
    adjacent = all(t.is_contiguous() and t.dtype == t0.dtype and t.shape[1:] == t0.shape[1:]
                   for t in ts)
    ptr = t0.data_ptr()
    for t in ts:
        adjacent = adjacent and t.data_ptr() == ptr
        ptr += t.numel() * t.element_size()
    if adjacent:
        rows = sum(int(t.shape[0]) for t in ts)
        return t0.as_strided((rows,) + tuple(t0.shape[1:]), t0.stride())
    return torch.cat(list(ts))


def _copy_batch(r: CaptionBatch, consumer=None) -> CaptionBatch:
    """Clones of a result, made on the current (pipeline) stream; ``consumer`` is the stream
    that will read and free them, recorded so the caching allocator does not recycle the blocks
    for the pipeline stream while consumer-stream kernels may still read them."""
    def c(t):
        if t is None:
            return None
        t = t.clone()
        if consumer is not None:
            t.record_stream(consumer)
        return t
    return CaptionBatch(c(r.ids), c(r.lengths), c(r.scores), c(r.hard_ids), c(r.hard_len),
                        c(r.plen), c(r.prefix_ids), c(r.clap_emb))
