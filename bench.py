#!/usr/bin/env python3
"""Benchmark of the zero-shot audio-captioning hot path on MI355X (BASELINE.json metric):

    audio clips/sec end-to-end (encode + mapper + GPT-2 decode), Clotho-eval bs=64

Headline (BASELINE.json configs[1], "C2"): a Clotho-eval-sized set of 1045 synthetic 10 s / 32 kHz
waveforms per rank (randn*0.1, clipped), resident in HBM before the timed region, captioned in
eval batches of 64 clips exactly as the reference evaluates them: STFT/log-mel + bn0 -> HTSAT ->
audio_proj + L2 -> sound-effect hard prompt -> MLP mapper -> GPT-2 small prefill +
get_prefix_tokens + greedy generate2 (entry_length 67, stop ids 13 / 764), bf16 operands / f32
accumulation.  Every decode GEMM of a batch is a 64-row GEMM.  One "step" = one eval batch of
64 clips (the last batch of the 1045 holds 21).  Independent batches are in flight per GPU, each
on its own HIP stream (pipeline twins sharing the weights, zsaac/pipeline.py ConcurrentRunner),
each decoding in its own persistent launch of 48 half-CU workgroups (a larger grid when few
batches wait, zsaac.pipeline.choose_persist_grid; the grid never changes an id, decode_grid.hip).
Schedule (--begin-first 1, the default): a pipeline per batch; every batch's begin (prompt,
mapper, prefill, get_prefix_tokens, step 0) runs as the encoder's passes deliver, before the
first decode grid launches; the grids then launch in batch order within --persist-budget slots
(default 2 x CUs less a sixteenth: ten grids of 48); --begin-first 0 is round 5's pipelined
schedule (at most --inflight batches, begins beside the grids).  The timed region runs --reps
times (median reported); GPU_MAX_HW_QUEUES is raised to --hw-queues (default 16, the runtime
allows up to 32; streams beyond it share queues in order).  With N ranks the
clips are sharded (zsaac/dist.py shard_range) and ONE RCCL all-gather of the generated token ids
+ lengths (zsaac/dist.py collect_captions) is inside the timed region.

    python bench.py                                  # 1045 clips per rank (weak scaling)
    python bench.py --steps K                        # K full batches of 64 per rank (weak)
    python bench.py --clips N                        # N clips in total, sharded (strong)
    torchrun --nproc-per-node N bench.py --gpus N    # one process per GPU, RCCL

Rank 0 prints ONE JSON line.  Besides the contract fields (value = whole-job clips/s) it holds
  roofline:          the dominant kernel, dg_persist_kernel (zs_gpt2_decode_persist: every
                     decode step after step 0 of one eval batch in one launch), HBM-bound:
                     algorithmic bytes per launch (weights per step + every row's K/V reads and
                     appends, persist_launch_bytes) / its average duration over the timed region's
                     launches (HIP events on each launch's stream); traffic from the committed
                     PMC passes (profiles/r3_pmc_persist.json);
  roofline_decode_step: one decode step of one batch on one stream (nothing else running);
  stages:            per-stage ms on one stream with each stage's roofline fraction (front end
                     HBM, encoder MFMA, prompt+mapper HBM, prefill MFMA, decode HBM);
  roofline_stepwise_*, roofline_decode_attention: the per-step path's kernels (beam, f32, > 64
                     rows) at the bs-64 shapes, cold weights / cold K/V;
  strong_scaling_proxy: T(1045 clips) / T(one rank's 131-clip shard) on this GPU = the predicted
                     1 -> 8 GPU speed-up;
  c3_beam5:          BASELINE configs[2] (beam 5, batch 256) with its LM head's MFMA roofline;
  throughput_mode:   the same path with 128 eval batches decoded per step (8192-row GEMMs) —
                     a different configuration, NOT the metric;
  f32_parity_mode:   the bs-64 headline (1045 clips) in f32 (the mode whose greedy ids are
                     bit-exact);
  c5_mistral:        BASELINE configs C5 (Mistral-7B fp8 decoder, 3 language tags, bs 32) with its
                     decode-step HBM roofline (also alone: --mistral);
  id_agreement:      greedy ids against the reference goldens (bf16 and f32), first divergence
                     and the reference's own top-2 logit margin there (tools/idparity.py);
  cpu_baseline:      the oracle (reference semantics: batch 1, full recompute, fp32) on bounded
                     samples of C2, C1 and C3 (beam 5) on this host's CPU (rank 0, N=1 only);
                     --cpu-baseline-full times BASELINE.md §3's 64 / 50 / 64 clips.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time


def _hw_queues_from_argv(default=16):
    for i, a in enumerate(sys.argv):
        if a == "--hw-queues" and i + 1 < len(sys.argv):
            return int(sys.argv[i + 1])
        if a.startswith("--hw-queues="):
            return int(a.split("=", 1)[1])
    return default


# must precede the HIP runtime's initialisation (the first device call).  The pool's boxes export
# HIP's default of 4 (one of them the null stream's); the bench's concurrent batch streams each
# want a queue of their own (measured at 4 in flight: 3.16k clips/s with 4 queues, 3.68k with 8)
os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(1, _hw_queues_from_argv())))

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
MFMA_F32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: dense f32 MFMA
# the decoder weights: GPT-2's own init scale (blocks and embeddings std 0.02, the c2_gpt2init
# golden's weights), where the reference's own bf16 logit error (0.032) is far below most step
# margins, so the bf16 id-parity gate compares ~64 % of the tokens the bench generates
# (id_agreement.bench_weights); the stop-token boost makes '.' fire for part of the clips
GPT2_KW = dict(seed=11, std=0.02, emb_std=0.02, stop_boost=2.0)
BENCH_WEIGHTS_GOLDEN = "c2_gpt2init"
HEADLINE_REPS = 3
CLOTHO_EVAL_CLIPS = 1045
METRIC = "audio clips/sec end-to-end (encode+mapper+GPT-2 decode), Clotho-eval bs=64"
DATA = ("synthetic 10 s / 32 kHz waveforms (randn*0.1) resident in HBM; seeded random-init "
        "weights at the reference architecture (no checkpoints offline)")


_T0 = time.time()


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.time() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="eval batches of --batch clips per rank (default: the 1045-clip "
                         "Clotho-eval set, 17 batches, the last holding 21 clips)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clips", type=int, default=None,
                    help="strong scaling: this many clips in total, sharded across ranks")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--encoder", default="htsat", choices=["htsat", "cnn14"])
    ap.add_argument("--mapper", default="mlp", choices=["mlp", "transformer"])
    ap.add_argument("--beam", type=int, default=0)
    ap.add_argument("--entry-length", type=int, default=67)
    ap.add_argument("--encoder-batch", type=int, default=0,
                    help="clips per encoder pass (0 = --batch * --group)")
    ap.add_argument("--group", type=int, default=1,
                    help="eval batches decoded together in one decode step (1 = the metric's "
                         "bs=64; > 1 is the labelled throughput mode)")
    ap.add_argument("--inflight", type=int, default=10,
                    help="independent batches in flight per GPU, each on its own HIP stream "
                         "(capped by --persist-budget // the smallest grid)")
    ap.add_argument("--encode-ahead", type=int, default=256,
                    help="clips per up-front encoder pass of the caption runs (the encoder twin "
                         "encodes consecutive eval batches together on a stream of its own, each "
                         "batch's begin waits for its own pass; 0 = every batch encodes its own "
                         "clips at --batch)")
    ap.add_argument("--cu-split", type=int, default=0,
                    help="A/B: CUs reserved (by stream CU masks) for the begins; the decode "
                         "grids get the rest (0: no split)")
    ap.add_argument("--begin-first", type=int, default=1,
                    help="1 (default): a pipeline per batch, every begin (prompt .. step 0) "
                         "enqueued first; the first grid launches wait for --begin-gate begins "
                         "(0: all of them); 0: round 5's pipelined schedule (begins beside grids)")
    ap.add_argument("--begin-gate", type=int, default=0)
    ap.add_argument("--begin-group", type=int, default=2,
                    help="with --begin-first: eval batches per begin (one encoder pass, prefill "
                         "and get_prefix_tokens for all of them; 0 = a begin per batch; 2 / 3 / 4 "
                         "/ 5 measured 7.93k / 7.98k / 7.83k / 7.95k clips/s at 1280 clips and "
                         "7.31k / 7.20k / 7.25k at 1045, profiles/r6/begin_first_ab.txt r6dd)")
    ap.add_argument("--persist-budget", type=int, default=0,
                    help="workgroup slots (half a CU each) the in-flight persistent decode grids "
                         "may hold together (0: ZSAAC_PERSIST_BUDGET or 1.5 per CU)")
    ap.add_argument("--reps", type=int, default=HEADLINE_REPS,
                    help="timed repetitions of the headline region (value = their median)")
    ap.add_argument("--hw-queues", type=int, default=16,
                    help="GPU_MAX_HW_QUEUES for this process (read before HIP initialises)")
    ap.add_argument("--compact", type=int, default=1,
                    help="greedy bf16 at >= 512 rows: decode only the rows that have not stopped")
    ap.add_argument("--extras", type=int, default=1,
                    help="N=1: also measure the throughput mode, the f32 mode and id agreement")
    ap.add_argument("--cpu-baseline-clips", type=int, default=32,
                    help="C2 clips timed on the CPU oracle (C1: all 50 golden clips, C3 beam 5: "
                         "a quarter of this, at least 4)")
    ap.add_argument("--cpu-baseline-full", action="store_true",
                    help="the BASELINE.md §3 plan: 64 C2 clips, all 50 C1 clips, 64 C3 clips")
    ap.add_argument("--no-scaling-proxy", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--stages", action="store_true", help="also report per-stage ms (extra syncs)")
    ap.add_argument("--magic", action="store_true",
                    help="CLAP-guided beam decoding (generate_beam_magic: beam 3, width 25, "
                         "entry 20, predict_prompt.py --magic) on bs=64 batches: a labelled "
                         "secondary line, not the metric")
    ap.add_argument("--magic-bert-layers", type=int, default=12)
    ap.add_argument("--mistral", action="store_true",
                    help="C5: wav -> HTSAT -> prompt + MLP mapper -> Mistral-7B (fp8 weights) "
                         "greedy generate for the en / zh / fr tags, bs=32 (a labelled "
                         "secondary line, not the metric)")
    ap.add_argument("--embeddings-only", action="store_true",
                    help="C4: batched HTSAT/CNN14 encode_audio + one RCCL all-gather of the "
                         "[N,1024] embeddings (no caption decode)")
    return ap.parse_args(argv)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))   # RCCL on ROCm
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def build(args, device, dtype=None, group=None, encoder_batch=None):
    from zsaac import synthetic as S
    from zsaac.pipeline import CaptionConfig, CaptionPipeline
    dtype = dtype or (torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    group = group or args.group
    csd = S.gpt2_state_dict(**GPT2_KW)
    csd.update(S.mlp_mapper_state_dict(1) if args.mapper == "mlp" else S.transformer_mapper_state_dict(2))
    if args.encoder == "htsat":
        asd = S.htsat_state_dict(3)
        asd.update(S.audio_proj_state_dict(5, audio_width=768))
    else:
        asd = S.cnn14_state_dict(4)
        asd.update(S.audio_proj_state_dict(5, audio_width=2048))
    B = args.batch * group
    eb = encoder_batch or getattr(args, "encoder_batch", 0) or B
    cfg = CaptionConfig(encoder=args.encoder, mapping_type=args.mapper, dtype=dtype, batch=B,
                        encoder_batch=eb, beam=args.beam, entry_length=args.entry_length,
                        compact_decode=bool(getattr(args, "compact", 1)))
    pipe = CaptionPipeline(csd, asd, S.label_table(), S.label_token_table(), cfg, device=device)
    return pipe, csd, asd


def synthetic_clips(n, first, device):
    """Clips first..first+n-1 of the synthetic eval set (each clip its own seed, so a clip is the
    same waveform whichever rank or batch takes it)."""
    out = torch.empty(n, 320000, device=device)
    g = torch.Generator(device=device)
    for i in range(n):
        g.manual_seed(1234 + first + i)
        out[i].normal_(generator=g).mul_(0.1).clamp_(-1, 1)
    return out


# ------------------------------------------------------------------ caption runs
def split_batches(n, B, parts=0):
    """[start, end) ranges of n clips in eval batches of at most B: consecutive full batches (the
    reference's DataLoader), or with ``parts`` > 0 at least that many near-equal batches (a small
    shard spread over every in-flight stream; each batch still <= B rows)."""
    k = -(-n // B)
    if parts:
        k = max(k, min(parts, n))
    if not parts:
        return [(i, min(n, i + B)) for i in range(0, n, B)]
    base, rem = divmod(n, k)
    out, a = [], 0
    for j in range(k):
        b = a + base + (1 if j < rem else 0)
        out.append((a, b))
        a = b
    return out


_STREAMS = {}


def run_streams(device, n):
    """n dedicated HIP streams (distinct hardware queues), created once per process and shared by
    every runner of this bench: a fresh set per runner would wrap past GPU_MAX_HW_QUEUES and put
    a later runner's batches on shared queues (serialized)."""
    from zsaac import ops
    have = _STREAMS.setdefault(str(device), [])
    if len(have) < n:        # the pipelines' streams at high priority (the encoder's is low)
        have += ops.dedicated_streams(n - len(have), device, priority=-1)
    return have[:n]


def enc_stream(device):
    """The low-priority stream the caption runs' encoder twin runs ahead on (one per process)."""
    from zsaac import ops
    key = "enc:" + str(device)
    if key not in _STREAMS:       # (ZSAAC_ENC_PRIO: A/B of the encoder stream's priority)
        _STREAMS[key] = ops.dedicated_streams(1, device, priority=int(os.environ.get("ZSAAC_ENC_PRIO", "1")))[0]
    return _STREAMS[key]


def run_captions(args, world, rank, device, pipe, n_local, first, counts, inflight, warmup,
                 parts=0, log_pass=False, reps=1):
    """Times the captioning of this rank's n_local clips (clip ids first..) in batches of
    pipe.cfg.batch (split_batches) on `inflight` streams, then the all-gather; returns (seconds
    max over ranks, outs, runner, info)."""
    from zsaac.pipeline import ConcurrentRunner, persist_budget
    from zsaac import decoder as zdec, dist as zd
    B = pipe.cfg.batch
    pool = synthetic_clips(n_local, first, device)
    batches = [pool[a:b] for a, b in split_batches(n_local, B, parts)]
    log(f"{n_local} clips in {len(batches)} batches of <= {B}, {inflight} in flight: capturing")
    if len(batches) == 0:
        raise ValueError("no clips on this rank")
    ahead = getattr(args, "encode_ahead", 0)
    if getattr(args, "beam", 0) or ahead < B:      # beam runs / larger batches: encoder per batch
        ahead = 0
    extra = getattr(args, "extra_pipes", 0)
    # (bf16 only: the f32 parity mode's two co-resident G192 grids ran 1.49k vs 1.58k clips/s
    # staged, profiles/r6/begin_first_ab.txt)
    bfirst = (bool(getattr(args, "begin_first", 0)) and pipe.decoder.persist and not pipe.cfg.beam
              and pipe.cfg.batch <= 64 and not getattr(pipe.decoder, "f32_grid", False))
    budget = getattr(args, "persist_budget", 0) or None
    bgroup = int(getattr(args, "begin_group", 2)) if bfirst and args.mapper == "mlp" else 0
    if bfirst:
        if not bgroup:          # a pipeline per batch: every begin runs before the grids
            inflight = max(inflight, len(batches))
        budget = budget or persist_budget(torch.cuda.get_device_properties(device).multi_processor_count,
                                          staged=True)
    nstreams = max(1, inflight) + extra
    if bfirst:                  # (as ConcurrentRunner: the grids the budget holds + 2)
        pool = budget // 48
        nstreams = pool if bgroup else min(nstreams, pool)
    runner = ConcurrentRunner(pipe, max(1, inflight),
                              streams=run_streams(device, nstreams),
                              budget=budget,
                              encode_ahead=ahead, enc_stream=enc_stream(device) if ahead else None,
                              extra_pipes=extra, cu_split=getattr(args, "cu_split", 0),
                              begin_first=bfirst, begin_gate=getattr(args, "begin_gate", 0),
                              begin_group=bgroup, n_batches=len(batches))
    for size in sorted({b.shape[0] for b in batches}, reverse=True):   # captures every graph
        runner.warmup(next(b for b in batches if b.shape[0] == size))
        log(f"captured the decode graphs of {size}-clip batches")
    if warmup:
        runner.run([batches[i % len(batches)] for i in range(warmup)])
        log(f"warmed up ({warmup} batches)")
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    cap0 = sum(d.n_captures for d in runner.decoders())
    rows0 = sum(d.rows_stepped for d in runner.decoders())
    times, gave_up = [], 0
    for _ in range(reps):          # every repetition the whole region; the median is reported
        t0 = time.perf_counter()
        outs = runner.run(batches)
        if world > 1:
            zd.collect_captions(outs, counts)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        dt_r = time.perf_counter() - t0
        if world > 1:             # the job's time of this repetition: the slowest rank's
            t = torch.tensor([dt_r], device=device, dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            dt_r = float(t)
        times.append(dt_r)
        gave_up += getattr(runner, "gave_up", 0)
    rows1 = sum(d.rows_stepped for d in runner.decoders())     # (before the log pass)
    dt = sorted(times)[len(times) // 2]
    log(f"timed: {n_local} clips in {dt:.3f} s (median of {reps}: {[round(t, 4) for t in times]})")
    if gave_up:
        log(f"WARNING: {gave_up} persistent launches gave up and finished on the phase launches")
    runner.timed_log, runner.log_outs = [], None
    if log_pass and pipe.decoder.persist:
        # the roofline's live launch timing: the same batches once more, untimed, with HIP events
        # around every persistent launch (events recorded inside the timed region cost it 3-5 %)
        zdec.PERSIST_LOG = []
        try:
            runner.log_outs = runner.run(batches)
            torch.cuda.synchronize()
            runner.timed_log = list(zdec.PERSIST_LOG)
        finally:
            zdec.PERSIST_LOG = None         # no events around launches outside this pass
        ALL_PERSIST_LOGS.extend(runner.timed_log)
    info = {"graph_captures_timed": sum(d.n_captures for d in runner.decoders()) - cap0,
            "timed_reps_s": [round(t, 5) for t in times],
            "persist_gave_up": gave_up,
            "persist_grids": grid_counts(runner),
            "persist_budget_wg_slots": getattr(runner, "budget", None),
            "batches_in_flight": runner.n_inflight,
            "schedule": (("begin_first: " + (f"one begin per {runner.begin_group} eval batches "
                                             "(encoder pass, prefill, get_prefix_tokens at "
                                             f"{runner.begin_group * B} clips), a decoder per batch"
                                             if runner.begin_group else "a pipeline per batch")
                          + ", every begin before the first grid launches, grids launched as the "
                            "budget frees")
                         if getattr(runner, "begin_first", False) and len(batches) > runner.budget // runner.grids[-1]
                         else "pipelined: begins beside the decode grids"),
            # decode rows stepped per clip in ONE repetition of the timed region
            "decode_rows_stepped_per_clip": round((rows1 - rows0) / max(1, reps) / max(1, n_local), 2),
            "decode_steps_mean": round(sum(runner.decode_steps) / max(1, len(runner.decode_steps)), 2),
            "tokens_rank0": int(sum(int(o.lengths.sum()) if o.scores is None
                                    else int(o.lengths[:, 0].sum()) for o in outs))}
    del pool
    return dt, outs, runner, info


def sub_run(args, device, dtype, group, inflight, n_clips, warmup, encoder_batch=None, reps=1):
    """A secondary single-GPU configuration (throughput mode / f32 mode): value (the median of
    `reps` timed repetitions) + config."""
    pipe, _, _ = build(args, device, dtype=dtype, group=group, encoder_batch=encoder_batch)
    dt, outs, runner, info = run_captions(args, 1, 0, device, pipe, n_clips, 10 ** 6, [n_clips],
                                          inflight, warmup, reps=reps)
    B = pipe.cfg.batch
    res = {"value": round(n_clips / dt, 2), "unit": "clips/s", "clips": n_clips,
           "ms_per_step": round(dt / math.ceil(n_clips / B) * 1e3, 3),
           "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
           "config": {"eval_batch": args.batch, "eval_batches_per_step": group,
                      "decode_rows_per_step": B, "encoder_batch": pipe.encoder.B,
                      "steps_in_flight_per_gpu": inflight, **info}}
    del runner, pipe, outs
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


# ------------------------------------------------------------------ rooflines
def _graph_time(launch, reps):
    """Average duration of `reps` back-to-back launches captured in one graph, HIP events on the
    launching stream, 5 replays."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            launch(i)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(reps):
                launch(i)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            g.replay()
        e1.record(s)
    e1.synchronize()
    torch.cuda.current_stream().wait_stream(s)
    return e0.elapsed_time(e1) / 1e3 / (5 * reps)


def _cold_copies(W, cold_bytes=640 << 20):
    return [W] + [W.clone() for _ in range(max(0, -(-cold_bytes // W.nbytes) - 1))]


def _hbm_entry(kernel, byts, avg_s, extra=None):
    gbs = byts / avg_s / 1e9
    r = {"kernel": kernel, "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "avg_launch_us": round(avg_s * 1e6, 3),
         "algo_bytes_per_launch": int(byts)}
    if extra:
        r.update(extra)
    return r


PMC_FILE = os.path.join(ROOT, "profiles", "r2_pmc_traffic.json")


def roofline_gemm_ln(pipe):
    """Dominant kernel of the bs-64 decode: zs_gemm_ln (row-group GEMM with ln_2 fused) at the
    c_fc shape out[64, 3072] = gelu_new(LN(x[64, 768]) @ W[3072, 768]^T + b), bf16 out, as the
    decoder launches it.  Algorithmic bytes = W (bf16) + x (f32) + LN params + bias + out."""
    from zsaac import ops
    dec, ly = pipe.decoder, pipe.gpt.layers[0]
    M = min(64, pipe.cfg.batch)
    x, hid = dec.x[:M], dec.hid[:M]
    W, b = ly["fc_w"], ly["fc_b"]
    N, K = W.shape
    copies = _cold_copies(W)

    def launch(i):
        ops.gemm_ln(x, *ly["ln2_gemm"], copies[i % len(copies)], hid, bias=b, act=ops.ACT_GELU_TANH)
    avg = _graph_time(launch, 2 * len(copies))
    byts = N * K * 2 + M * K * 4 + (2 * K * 4 if ly["ln2_gemm"][0] is not None else 0) + N * 4 + M * N * 2
    flops = 2 * M * N * K
    traffic, tsrc = None, None
    if os.path.exists(PMC_FILE):            # rocprofv3 --pmc passes (tools/pmc_traffic.py)
        with open(PMC_FILE) as f:
            pmc = json.load(f)
        if pmc.get("shape") == [M, N, K] and pmc.get("kernel", "").startswith("gemm_rows"):
            traffic, tsrc = pmc["hbm_bytes_per_launch"], os.path.relpath(PMC_FILE, ROOT)
    return _hbm_entry(f"gemm_rows_kernel<48,4,LN,6> (zs_gemm_ln) decode c_fc [{M}x{K}]x[{K}x{N}] "
                      f"+ln_2 (affine folded into W) +bias +gelu_new (cold W)", byts, avg,
                      {"traffic": traffic, "traffic_source": tsrc,
                       "attainable_tflops_at_this_AI": round(flops / byts * HBM_PEAK_GBS / 1e3, 1),
                       "achieved_tflops": round(flops / avg / 1e12, 2)})


def roofline_rows_gemm(pipe, which):
    from zsaac import ops
    dec, ly = pipe.decoder, pipe.gpt.layers[0]
    M = min(64, pipe.cfg.batch)
    if which == "mproj":
        a, W, b, K = dec.hid[:M], ly["mproj_w"], ly["mproj_b"], 3072
    else:
        a, W, b, K = dec.att[:M], ly["proj_w"], ly["proj_b"], 768
    N = W.shape[0]
    out = torch.empty(M, N, device=W.device)
    copies = _cold_copies(W)

    def launch(i):
        ops.gemm(a, copies[i % len(copies)], out, bias=b, residual=out, workspace=dec.ws)
    avg = _graph_time(launch, 2 * len(copies))
    byts = N * K * 2 + M * K * 2 + N * 4 + 2 * M * N * 4
    return _hbm_entry(f"gemm_rows_kernel decode {which} [{M}x{K}]x[{K}x{N}] +bias +residual "
                      f"(cold W)", byts, avg)


def roofline_attention(pipe, L_mean=None, cold_bytes=320 << 20):
    """decode attention at the bench's decode rows, every row at the mean key count of a 67-step
    greedy decode (prompt Pmax + 34): bytes = K and V of every key once + q/k/v + output.  Cold:
    the launches rotate over copies of the layer's K/V caches totalling > 256 MiB (more than the
    8 x 4 MiB L2s and the 256 MiB Infinity Cache), as the GEMM rooflines rotate weight copies."""
    from zsaac import ops
    dec = pipe.decoder
    R = pipe.cfg.batch * max(1, pipe.cfg.beam)
    D, H, Lmax = 768, 12, dec.Lmax
    L = L_mean or min(Lmax - 1, pipe.Pmax + 34)
    kc, vc = dec.kc[0], dec.vc[0]
    n = max(1, -(-cold_bytes // (kc.nbytes + vc.nbytes)))
    caches = [(kc, vc)] + [(kc.clone(), vc.clone()) for _ in range(n - 1)]
    qkv = dec.qkv[:R]
    pos = torch.full((R,), L - 1, device=pipe.dev, dtype=torch.int32)
    out = torch.empty(R, D, device=pipe.dev, dtype=qkv.dtype)

    def launch(i):
        k, v = caches[i % n]
        ops.decode_attention(qkv, R, D, H, k, v, Lmax, pos, out)
    avg = _graph_time(launch, 2 * n)
    es = qkv.element_size()
    byts = R * H * (2 * L * 64 * es) + R * 3 * D * es + R * D * es
    r = _hbm_entry(f"decode_attn6_kernel<bf16,{'32,SPLIT=2' if R <= 128 else 16}> R={R} heads=12 "
                   f"keys={L} (cold K/V: {n} cache copies, {n * (kc.nbytes + vc.nbytes) >> 20} MiB)",
                   byts, avg)
    del caches
    return r


# ------------------------------------------------------------------ persistent decode roofline
def gpt2_step_weight_bytes(pipe):
    """Bytes of weights one greedy decode step reads: the 12 blocks' bf16 c_attn / attn.c_proj /
    c_fc / mlp.c_proj matrices and f32 biases, the tied LM head (bf16 wte) and ln_f."""
    D, F = 768, 3072
    es = pipe.gpt.wte.element_size()
    per_layer = (3 * D * D + D * D + D * F + F * D) * es + (3 * D + D + F + D) * 4
    return len(pipe.gpt.layers) * per_layer + pipe.gpt.V * D * es + 2 * D * 4


def persist_launch_bytes(w_step, plen, steps, kv_row=12 * 2 * 768 * 2):
    """Algorithmic HBM bytes of one persistent launch (decode steps 1 .. steps-1 of a batch whose
    rows have prompt lengths ``plen``): per step the weights once, and per row its cached K/V
    (keys 0 .. pos-1 of all 12 layers, pos = plen - 1 + t at step t) read plus the new K/V row
    written.  Every row is counted every step (the kernel computes rows that already stopped)."""
    n = steps - 1
    if n <= 0:
        return 0
    keys = sum(n * (p - 1) + n * (n + 1) // 2 for p in plen)
    return n * w_step + kv_row * (keys + len(plen) * n)


PMC_PERSIST_FILE = os.path.join(ROOT, "profiles", "r6", "pmc_persist_g48.json")
F32_INFLIGHT = 4


def grid_counts(runner):
    """{"<workgroups> WGs": launches} of a runner's last run (persistent decode grids)."""
    out = {}
    for g in getattr(runner, "grid", []):
        if g:
            out[f"{g} WGs"] = out.get(f"{g} WGs", 0) + 1
    return out


def persist_roofline(pipe, runner, outs, dt, log):
    """roofline of the dominant kernel, decode_persist_kernel: every launch of a repeat of the
    timed region (same batches, same streams and concurrency, untimed: HIP events recorded on each
    launch's own stream around it, zsaac.decoder.PERSIST_LOG -- recorded inside the timed region
    they cost it 3-5 %), algorithmic bytes of each launch from its batch's prompt lengths and step
    count / its duration."""
    from zsaac import ops
    w_step = gpt2_step_weight_bytes(pipe)
    by_dec = {}
    for e0, e1, tag in log:
        by_dec.setdefault(tag, []).append((e0, e1))
    durs, byts = [], []
    bdec = getattr(runner, "bdec", None)      # (begin groups: batch -> its sub-decoder)
    for i, b in runner.assign:
        e0, e1 = by_dec[id(bdec[b] if bdec else runner.pipes[i].decoder)].pop(0)
        durs.append(e0.elapsed_time(e1) / 1e3)
        byts.append(persist_launch_bytes(w_step, outs[b].plen.tolist(), runner.decode_steps[b]))
    n = len(durs)
    avg_s, avg_b = sum(durs) / n, sum(byts) / n
    traffic, tsrc = None, None
    if os.path.exists(PMC_PERSIST_FILE):     # rocprofv3 --pmc passes (tools/pmc_traffic.py persist)
        with open(PMC_PERSIST_FILE) as f:
            pmc = json.load(f)
        if pmc.get("kernel", "").startswith("dg_persist_kernel"):
            traffic, tsrc = pmc["hbm_bytes_per_launch"], os.path.relpath(PMC_PERSIST_FILE, ROOT)
    steps = sum(runner.decode_steps) / max(1, len(runner.decode_steps))
    return _hbm_entry(
        f"dg_persist_kernel (zs_gpt2_decode_persist): decode steps 1..{steps - 1:.0f} of one "
        f"bs-64 eval batch in one launch (grids {grid_counts(runner)} of 256-thread workgroups), "
        f"the {n} launches of a repeat of the timed region, {runner.n_inflight} batches in flight",
        avg_b, avg_s,
        {"launches": n, "avg_launch_ms": round(avg_s * 1e3, 3),
         "grids": grid_counts(runner),
         "weight_bytes_per_step": int(w_step), "steps_per_launch_mean": round(steps - 1, 2),
         "traffic": traffic, "traffic_source": tsrc,
         "traffic_note": "PMC FETCH_SIZE*2*1024 + WRITE_SIZE*1024 per launch, single-stream "
                         "launches of the same workload (tools/pmc_traffic.py persist)",
         "concurrent_aggregate": {"algo_GBps": round(sum(byts) / dt / 1e9, 1),
                                  "frac": round(sum(byts) / dt / 1e9 / HBM_PEAK_GBS, 4),
                                  "note": "all launches' algorithmic bytes / the headline's timed wall"}})


ALL_PERSIST_LOGS = []     # (start, end, decoder) events of every logged persistent launch


def persist_all_launches(log):
    """Average duration of the logged persistent launches (the roofline's repeat of the timed
    region and the single-stream step runs); rocprofv3 --kernel-trace --stats over the same
    command also counts the warmup and timed-region launches."""
    d = [e0.elapsed_time(e1) for e0, e1, _ in log]
    return {"launches": len(d), "avg_ms": round(sum(d) / max(1, len(d)), 3)}


def decode_step_roofline(pipe, wav, agg_steps_per_s=None, reps=3):
    """One greedy decode step of one batch on ONE stream (nothing else running): the persistent
    launch (all steps after step 0) timed with HIP events / its steps, or, on the per-step path,
    a graph-replayed chunk / its steps.  Bytes = persist_launch_bytes per step."""
    from zsaac import decoder as zdec
    dec, B = pipe.decoder, wav.shape[0]
    w_step = gpt2_step_weight_bytes(pipe)
    if dec.persist:
        per = []
        for _ in range(reps):
            zdec.PERSIST_LOG = []
            try:
                pipe.begin_wav(wav)
                dec.run_to_completion()
                torch.cuda.synchronize()
            finally:
                log, zdec.PERSIST_LOG = zdec.PERSIST_LOG, None
            ALL_PERSIST_LOGS.extend(log)
            e0, e1, _ = log[-1]
            steps = int(dec.step_ctr.item())
            per.append((e0.elapsed_time(e1) / 1e3, steps))
        dur, steps = sorted(per)[len(per) // 2]
        byts = persist_launch_bytes(w_step, dec.plen[:B].tolist(), steps) / (steps - 1)
        step_s = dur / (steps - 1)
        what = "decode_persist_kernel launch / its steps"
    else:
        pipe.begin_wav(wav)
        dec.done.zero_()
        gr = dec._graph(*dec._chunk_plan(None))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            gr.replay()
        e1.record()
        e1.synchronize()
        step_s = e0.elapsed_time(e1) / 1e3 / 10 / dec.chunk
        L = min(dec.Lmax - 1, pipe.Pmax + 34)
        byts = w_step + B * L * 12 * 2 * 768 * 2
        what = "graph-replayed chunk / its steps"
    r = _hbm_entry(f"one greedy decode step, {B} rows (12 blocks + ln_f + LM head + greedy step), "
                   f"single stream ({what})", byts, step_s, {"avg_step_us": round(step_s * 1e6, 1)})
    r.pop("avg_launch_us")
    if agg_steps_per_s:
        agg = byts * agg_steps_per_s / 1e9
        r["concurrent_aggregate"] = {"decode_steps_per_s": round(agg_steps_per_s, 1),
                                     "achieved_GBps": round(agg, 1),
                                     "frac": round(agg / HBM_PEAK_GBS, 4)}
    return r


def htsat_flops(B):
    """Multiply-add flops x 2 of HTSAT forward_features for B clips (patch embed, every Swin
    block's qkv / window attention (64-token windows) / proj / MLP, the patch merges)."""
    from zsaac.encoder import DEPTHS, EMBED, WIN
    M, C = B * 4096, EMBED
    f = 2 * M * C * 16                                   # 4 x 4 patch embed, 1 channel
    for i, depth in enumerate(DEPTHS):
        blk = 2 * M * C * 3 * C + 2 * 2 * M * WIN * WIN * C + 2 * M * C * C + 2 * 2 * M * C * 4 * C
        f += depth * blk
        if i < len(DEPTHS) - 1:
            f += 2 * (M // 4) * 4 * C * 2 * C
            M, C = M // 4, 2 * C
    return f


def cnn14_flops(B, frames):
    from zsaac.encoder import CNN14_CH
    H, W, ci, f = frames, 64, 1, 0
    for co in CNN14_CH:
        f += 2 * B * H * W * 9 * (ci * co + co * co)
        H, W, ci = H // 2, W // 2, co
    return f


def stage_times(pipe, wav, reps=3):
    """Per-stage device time of one batch on one stream (events between stages, outside the timed
    region) and each stage's roofline fraction: front end (STFT/log-mel, HBM), encoder (HTSAT /
    CNN14 + audio_proj, MFMA), prompt + mapper (HBM: the mapper's weights), prefill (GPT-2 over
    B x Pmax rows + get_prefix_tokens, MFMA) and decode (HBM, persist_launch_bytes + step 0)."""
    from zsaac import ops
    dec, cfg, enc = pipe.decoder, pipe.cfg, pipe.encoder
    B, Pmax = wav.shape[0], pipe.Pmax
    names = ("front_end", "encoder", "prompt_mapper", "prefill", "decode")
    out = {k: [] for k in names}
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        ev[0].record()
        ops.logmel(wav, enc.tables, bn=enc.w.bn0, out=enc.logmel[:B])
        ev[1].record()
        emb = enc.encode_logmel(None, B)
        ev[2].record()
        ops.prompt_assemble(emb, pipe.labels, cfg.sound_effect_num, pipe.label_tok, pipe.label_len,
                            pipe.hard_ids[:B], pipe.hard_len[:B])
        soft = pipe.mapper(ops.l2norm(emb, out=pipe.prefix[:B]))
        ev[3].record()
        ops.prefill_embed(pipe.hard_ids[:B], pipe.hard_len[:B], soft, pipe.mapper.soft_ld,
                          cfg.prefix_length, pipe.gpt.wte, pipe.gpt.wpe, B, Pmax,
                          pipe.embed[:B * Pmax], dec.x, dec.plen, dec.last_row)
        pipe.prefix_tokens(B, soft)
        dec.prefill(B, Pmax)
        ev[4].record()
        dec.greedy_begin(B)
        dec.run_to_completion()
        ev[5].record()
        torch.cuda.synchronize()
        for i, k in enumerate(names):
            out[k].append(ev[i].elapsed_time(ev[i + 1]))
    ms = {k: sorted(v)[len(v) // 2] for k, v in out.items()}
    steps = int(dec.step_ctr.item())
    es = 2 if cfg.dtype == torch.bfloat16 else 4
    peak_mfma = MFMA_BF16_PEAK_TFLOPS if es == 2 else MFMA_F32_PEAK_TFLOPS
    frames = enc.n_frames
    mp = pipe.mapper
    if hasattr(mp, "w0"):
        map_bytes = (mp.w0.numel() + mp.w2.numel()) * mp.w0.element_size()
    else:
        map_bytes = sum(t.numel() * t.element_size() for ly in mp.layers for t in ly.values()
                        if torch.is_tensor(t))
    n_gpt = sum(ly[k].numel() for ly in pipe.gpt.layers for k in ("attn_w", "proj_w", "fc_w", "mproj_w"))
    rows = B * Pmax
    prefill_flops = (2 * rows * n_gpt + 2 * 2 * B * 12 * Pmax * Pmax * 64 // 2
                     + 2 * B * cfg.prefix_length * pipe.gpt.V * 768)
    enc_flops = htsat_flops(B) if cfg.encoder == "htsat" else cnn14_flops(B, frames)
    dec_bytes = (persist_launch_bytes(gpt2_step_weight_bytes(pipe), dec.plen[:B].tolist(), steps)
                 + pipe.gpt.V * 768 * es)
    fe_bytes = wav.numel() * 4 + B * frames * 64 * 4

    def hbm(b, k):
        gbs = b / (ms[k] / 1e3) / 1e9
        return {"ms": round(ms[k], 3), "bound": "hbm", "algo_bytes": int(b), "achieved_GBps": round(gbs, 1),
                "frac": round(gbs / HBM_PEAK_GBS, 4)}

    def mfma(f, k):
        tf = f / (ms[k] / 1e3) / 1e12
        return {"ms": round(ms[k], 3), "bound": "mfma", "flops": int(f), "achieved_TFLOPs": round(tf, 1),
                "frac": round(tf / peak_mfma, 4)}
    return {"clips": B, "single_stream": True, "decode_steps": steps,
            "front_end": hbm(fe_bytes, "front_end"),
            "encoder": mfma(enc_flops, "encoder"),
            "prompt_mapper": hbm(map_bytes, "prompt_mapper"),
            "prefill": mfma(prefill_flops, "prefill"),
            "decode": hbm(dec_bytes, "decode")}


# ------------------------------------------------------------------ CPU baseline
def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(args, csd, asd, n_c2, n_c1, n_c3):
    """Oracle = reference semantics (batch 1 per clip, full-sequence recompute every step, fp32)
    on the BASELINE.md §3 configs, bounded by default: n_c2 clips of the C2 workload (wav ->
    HTSAT -> MLP -> greedy), n_c1 of C1's 50 reference-golden CLAP embeddings (-> MLP -> greedy)
    and n_c3 clips of C3 (wav -> HTSAT -> MLP -> beam 5); --cpu-baseline-full times the plan's
    64 / 50 / 64.  On the CPUs this process may use (sched affinity; os.cpu_count() may count the
    whole machine)."""
    import numpy as np
    from oracle import audio as A, caption as OC, frontend as OF
    from zsaac import synthetic as S
    visible = os.cpu_count() or 1
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else visible
    # the CPU share this job may use: OMP_NUM_THREADS when the host sets it (a GPU box of the
    # pool sets it to its per-GPU share; affinity there still lists every core of the machine)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(avail, visible, share) if share > 0 else min(avail, visible))
    torch.set_num_threads(threads)
    table, lt = S.label_table(), S.label_token_table()

    def caption(emb, ntok, beam=0):
        idx = OC.sound_effect_choice(emb, table, 3)[0].tolist()
        hard = torch.tensor([OC.prompt_ids(idx, lt)])
        pe = OC.clap_to_gpt(torch.nn.functional.normalize(emb, dim=-1)[None], hard, csd, args.mapper)
        OC.prefix_tokens(pe, csd)
        if beam:
            lists, _ = OC.generate_beam(pe, csd, beam_size=beam, entry_length=args.entry_length)
            ntok[0] += len(lists[0])
        else:
            ntok[0] += len(OC.generate2(pe, csd, entry_length=args.entry_length))

    def wav_clips(n, first, beam, label):
        wav = synthetic_clips(n, first, torch.device("cpu"))
        ntok = [0]
        t0 = time.perf_counter()
        with torch.no_grad():
            for i in range(n):
                lm = OF.logmel(wav[i:i + 1])
                feat = A.htsat_embedding(lm, asd) if args.encoder == "htsat" else A.cnn14_embedding(lm, asd)
                caption(A.audio_project(feat, asd), ntok, beam)
                log(f"cpu baseline {label} clip {i + 1}/{n}")
        return time.perf_counter() - t0, ntok[0]

    log(f"cpu baseline: C2 {n_c2} clips, C1 {n_c1} clips, C3 {n_c3} clips, {threads} threads")
    dt2, tok2 = wav_clips(n_c2, 777, 0, "C2")
    c1 = np.load(os.path.join(ROOT, "tests", "golden", "c1_greedy.npz"))
    emb = torch.from_numpy(c1["clap_emb"][:n_c1])
    ntok1 = [0]
    t0 = time.perf_counter()
    with torch.no_grad():
        for i in range(n_c1):
            caption(emb[i:i + 1], ntok1)
            if i % 4 == 3:
                log(f"cpu baseline C1 clip {i + 1}/{n_c1}")
    dt1 = time.perf_counter() - t0
    res = {"value": round(n_c2 / dt2, 4), "unit": "clips/s", "cores": threads, "kind": "port",
           "threads": threads, "cpus_visible": visible, "cpus_available": avail,
           "omp_num_threads_env": share or None,
           "cpu_model": _cpu_model(),
           "sample": f"C2: {n_c2} clips of the headline workload (wav -> log-mel -> "
                     f"{args.encoder.upper()} -> audio_proj -> prompt -> {args.mapper} mapper -> "
                     f"get_prefix_tokens -> greedy, {tok2} tokens) in {dt2:.1f} s; batch 1, "
                     f"full-sequence recompute per step (reference semantics), fp32, "
                     f"{threads} threads.  " + ("The BASELINE.md §3 slice (64 clips)" if n_c2 >= 64 else
                     f"A bounded sample (BASELINE.md §3 plans 64 clips; the full 1045 would take "
                     f"~{CLOTHO_EVAL_CLIPS / max(n_c2 / dt2, 1e-9) / 60:.0f} min; "
                     f"bench.py --cpu-baseline-full times the plan)"),
           "c1_plumbing": {"value": round(n_c1 / dt1, 4), "unit": "clips/s", "clips": n_c1,
                           "tokens": ntok1[0], "seconds": round(dt1, 1),
                           "sample": f"C1: {n_c1} of the 50 reference-golden CLAP embeddings -> "
                                     f"MLP -> greedy" + ("" if n_c1 >= 50 else
                                     " (bounded; --cpu-baseline-full times all 50)")}}
    if n_c3 > 0:
        dt3, _ = wav_clips(n_c3, 5555, 5, "C3")
        res["c3_beam5"] = {"value": round(n_c3 / dt3, 4), "unit": "clips/s", "clips": n_c3,
                           "seconds": round(dt3, 1),
                           "sample": f"C3: {n_c3} clips wav -> {args.encoder.upper()} -> MLP -> "
                                     f"generate_beam (beam 5, softmax().log() scores, entry_length "
                                     f"{args.entry_length}), batch 1" + ("" if n_c3 >= 64 else
                                     " (bounded; BASELINE.md §3 plans 64, --cpu-baseline-full)")}
    return res


# ------------------------------------------------------------------ C4
def main_embeddings(args, world, rank, device, pipe):
    """BASELINE.json configs[3] (C4): embedding extraction, data_handing/embeddings_generator.py
    realised as batched encode_audio over synthetic clips sharded across ranks, then one RCCL
    all-gather of the [N,1024] f32 embeddings (zsaac/dist.py gather_rows)."""
    from zsaac import dist as zd
    B = pipe.encoder.B
    steps = args.steps or 16
    n_total = args.clips or B * steps * world
    lo, hi = zd.shard_range(n_total, rank, world)
    counts = zd.shard_counts(n_total, world)
    # (clip c of the shard encodes pool[c % len(pool)]: the waveforms are regenerated per
    # pass-sized window to bound memory; the encoder work per clip is the same)
    pool = synthetic_clips(min(hi - lo, 2 * B), lo, device)
    embs = torch.empty(hi - lo, 1024, device=device)
    gathered = [embs]
    dist_on = torch.distributed.is_available() and torch.distributed.is_initialized()

    def run(n_batches, keep):
        for i in range(n_batches):
            c0 = i * B
            c1 = min(hi - lo, c0 + B)
            e = pipe.encode(pool[(c0 % pool.shape[0]):(c0 % pool.shape[0]) + (c1 - c0)])
            if keep:
                embs[c0:c1].copy_(e)
        if keep and dist_on:          # the RCCL all-gather (at world 1 too, under a process group)
            gathered[0] = zd.gather_rows(embs, counts)
    nb = -(-(hi - lo) // B)
    run(min(args.warmup, nb), False)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(nb, True)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    res = {"metric": "audio clips/sec embedding extraction (STFT/log-mel + " + args.encoder.upper()
                     + " + audio_proj + L2), C4",
           "value": round(n_total / dt, 2), "unit": "clips/s", "n_gpus": world,
           "steps": nb, "warmup": args.warmup, "ms_per_step": round(dt / nb * 1e3, 3),
           "higher_is_better": True, "scaling": "strong" if args.clips else "weak",
           "vs_baseline": None, "dtype": args.dtype,
           "data": DATA,
           "config": {"workload": "C4 embedding extraction, RCCL all-gather of [N,1024] f32",
                      "encoder_batch": B, "clips_total": n_total, "clips_per_rank": counts,
                      "parallelism": f"dp{world} (clip-sharded)"}}
    if rank == 0:
        print(json.dumps(res), flush=True)
    return res, gathered[0]


# ------------------------------------------------------------------ main
def main_magic(args, device):
    """CLAP-guided decoding throughput (predict_prompt.py:121-140 with --magic): wav -> HTSAT ->
    prompt + mapper -> generate_beam_magic(beam 3, width 25, alpha 0.1, beta 0.2, entry 20) with
    a bert-base text tower (12 layers, synthetic WordPiece vocabulary), bs=64 batches, one
    stream.  Host work per step (candidate texts + BERT tokenisation, as the reference) is
    inside the timed region."""
    from transformers import BertTokenizer
    from zsaac import ops, synthetic as S
    from zsaac.bert import BertTextEngine
    from zsaac.magic import MagicDecoder
    from zsaac.tokenizer import WordTokenizer
    args.group = 1
    pipe, _, _ = build(args, device, encoder_batch=args.batch)
    vocab = S.bert_vocab()
    bsd = S.bert_state_dict(layers=args.magic_bert_layers)
    bert = BertTextEngine(bsd, device, pipe.cfg.dtype, max_texts=args.batch * 75)
    tok = BertTokenizer(vocab={t: i for i, t in enumerate(vocab)}, do_lower_case=True)
    beam, width, entry = 3, 25, 20
    mag = MagicDecoder(pipe.gpt, bert, args.batch, pipe.Pmax, beam=beam, width=width,
                       max_steps=entry)
    n = args.steps or 2
    wav = synthetic_clips(args.batch, 0, device)

    def one():
        emb = pipe.encode(wav)
        B = emb.shape[0]
        ops.prompt_assemble(emb, pipe.labels, pipe.cfg.sound_effect_num, pipe.label_tok,
                            pipe.label_len, pipe.hard_ids[:B], pipe.hard_len[:B])
        prefix = ops.l2norm(emb, out=pipe.prefix[:B])
        soft = pipe.mapper(prefix)
        return mag.beam_magic(pipe.hard_ids[:B], pipe.hard_len[:B], soft, 10, prefix,
                              WordTokenizer(), tok, beam, width, entry, 0.1, 0.2, bert.temp,
                              soft_ld=pipe.mapper.soft_ld)
    for _ in range(max(1, warmup)):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    toks = 0
    for _ in range(n):
        res = one()
        toks += sum(len(r[0][0]) for r in res)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    clips = n * args.batch
    # dominant kernel: the text tower's GEMMs over ~144k token rows per step (78 % of the GPU
    # time); timed at the BERT intermediate (fc1) shape with HIP events on the launch stream
    T = args.batch * beam * width * 30
    bdt = pipe.cfg.dtype
    ga = torch.randn(T, 768, device=device).to(bdt)
    gw = (torch.randn(3072, 768, device=device) * 0.03).to(bdt)
    gb = torch.zeros(3072, device=device)
    go = torch.empty(T, 3072, device=device, dtype=bdt)
    for _ in range(2):
        ops.gemm(ga, gw, go, bias=gb, act=ops.ACT_GELU_ERF, split_k=1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        ops.gemm(ga, gw, go, bias=gb, act=ops.ACT_GELU_ERF, split_k=1)
    e1.record()
    e1.synchronize()
    g_s = e0.elapsed_time(e1) / 1e3 / reps
    g_fl = 2.0 * T * 768 * 3072
    peak = MFMA_BF16_PEAK_TFLOPS if bdt == torch.bfloat16 else None
    roof = {"kernel": f"gemm_lean_kernel (zs_gemm) BERT intermediate [{T}x768]x[768x3072] "
                      "+bias +gelu(erf), bf16 out", "bound": "mfma",
            "achieved": round(g_fl / g_s / 1e12, 1), "peak": peak, "unit": "TFLOP/s",
            "frac": round(g_fl / g_s / 1e12 / peak, 4) if peak else None,
            "avg_launch_us": round(g_s * 1e6, 1), "algo_flops_per_launch": g_fl,
            "algo_bytes_per_launch": int(T * 768 * 2 + 3072 * 768 * 2 + T * 3072 * 2)}
    del ga, go
    print(json.dumps({
        "metric": "audio clips/sec, CLAP-guided beam decoding (generate_beam_magic), bs=64",
        "value": round(clips / dt, 3), "unit": "clips/s", "n_gpus": 1, "steps": n,
        "warmup": args.warmup, "ms_per_step": round(dt / n * 1e3, 1), "higher_is_better": True,
        "dtype": args.dtype, "data": DATA + "; bert-base text tower (synthetic weights/vocab)",
        "config": {"workload": "wav -> HTSAT -> prompt + MLP mapper -> generate_beam_magic "
                               "(beam 3, magic_width 25, entry_length 20, alpha 0.1, beta 0.2)",
                   "batch": args.batch, "bert_layers": args.magic_bert_layers,
                   "candidate_rows_per_step": args.batch * beam * width,
                   "tokens_best_beam": toks},
        "roofline": roof,
        "note": "secondary decode mode (predict_prompt.py --magic); not the headline metric"}),
        flush=True)


def main_mistral(args, device):
    """`--mistral`: the C5 line alone (c5_mistral)."""
    print(json.dumps(c5_mistral(args, device, args.steps or 2, args.warmup)), flush=True)


def c5_mistral(args, device, n=2, warmup=1):
    """C5 (predict_mistralai_multilingual.py:90-111): per batch of 32 clips, HTSAT encode ->
    hard prompt (Mistral ids, padded to the batch's longest) -> MLP mapper (1024 -> 20480 ->
    40960) -> for each language tag a batched greedy generate(max_length 60, eos 2) on a
    Mistral-7B geometry decoder (32 layers, 4096, GQA 32/8, FFN 14336) with fp8 e4m3 weights.
    Roofline: one decode step's bytes (fp8 weights + scales + bf16 LM head) / its time."""
    from zsaac import ops, synthetic as S
    from zsaac.decoder import MlpMapper
    from zsaac.encoder import AudioEncoder
    from zsaac.mistral import MistralDecoder, MistralWeights, generate_concurrent
    B = 32
    dt = torch.bfloat16
    asd = S.htsat_state_dict(3)
    asd.update(S.audio_proj_state_dict(5, audio_width=768))
    enc = AudioEncoder(asd, "htsat", dt, B, device)
    w = MistralWeights.synthetic(device, S.MISTRAL_7B, seed=1)
    log(f"mistral-7B fp8 weights: {w.nbytes() / 1e9:.2f} GB on the device")
    g = torch.Generator(device=device).manual_seed(2)
    D = 4096
    msd = {"clap_project.model.0.weight": torch.randn(D * 5, 1024, device=device, generator=g) / 32,
           "clap_project.model.0.bias": torch.zeros(D * 5, device=device),
           "clap_project.model.2.weight": torch.randn(D * 10, D * 5, device=device, generator=g) / (D * 5) ** 0.5,
           "clap_project.model.2.bias": torch.zeros(D * 10, device=device)}
    mapper = MlpMapper(msd, device, dt, B)
    del msd
    labels = S.label_table().to(device)
    lt = torch.randint(3, 32000, (527, 3), generator=torch.Generator().manual_seed(3)).to(torch.int32)
    label_tok, label_len = lt.to(device), torch.full((527,), 3, dtype=torch.int32, device=device)
    Hc = 2 + 3 * 3 + 2 + 4
    hard_ids = torch.zeros(B, Hc, dtype=torch.int32, device=device)
    hard_len = torch.zeros(B, dtype=torch.int32, device=device)
    tags = {"en": [1, 523, 269, 28767], "zh": [1, 523, 26715, 28767], "fr": [1, 523, 1642, 28767]}
    tags = {k: torch.tensor(v, dtype=torch.int32, device=device) for k, v in tags.items()}
    # the 3 language tags of a batch decode concurrently (generate_concurrent: one decoder per
    # tag sharing the weights, one stream each); ZS_MISTRAL_CONCURRENT=0 runs them one by one
    conc = os.environ.get("ZS_MISTRAL_CONCURRENT", "1") != "0"
    decs = [MistralDecoder(w, max_batch=B, max_prompt=Hc + 10 + 4, max_new=60)
            for _ in range(3 if conc else 1)]
    for dec in decs:
        dec.fused_decode_attn = os.environ.get("ZS_MISTRAL_FUSED_ATTN", "1") != "0"   # A/B knobs
        dec.use_graph = os.environ.get("ZS_MISTRAL_GRAPH", "1") != "0"
        dec.prefill_unpack = os.environ.get("ZS_MISTRAL_UNPACK", "1") != "0"
        dec.fused_glu = os.environ.get("ZS_MISTRAL_RUN", "1") != "0"
        for kv in filter(None, os.environ.get("ZS_MISTRAL_RUN_CFG", "").split(",")):   # e.g. down=2x2
            k, v = kv.split("=")
            dec.run_cfg[k] = tuple(int(t) for t in v.split("x"))
    dec = decs[0]
    streams = run_streams(device, 3) if conc else None   # (the process pool: no new HW queues)
    wav = synthetic_clips(B, 0, device)

    def one():
        emb = enc.encode(wav)
        ops.prompt_assemble(emb, labels, 3, label_tok, label_len, hard_ids, hard_len)
        H = int(hard_len.max())          # padding_captions pads to the batch's longest
        soft = mapper(ops.l2norm(emb)).view(B, 10, D).float().contiguous()
        hard = hard_ids[:, :H].contiguous()
        if conc:
            return generate_concurrent(decs, streams, [(hard, soft, tags[t], 60)
                                                       for t in ("en", "zh", "fr")])
        return [dec.generate(hard, soft, tags[t], max_length=60) for t in ("en", "zh", "fr")]
    for _ in range(max(1, warmup)):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ntok = 0
    for _ in range(n):
        res = one()
        ntok += sum(len(r) for lang in res for r in lang)
    torch.cuda.synchronize()
    dt_s = time.perf_counter() - t0
    # decode-step roofline: one 32-row greedy step (M = 32, rows_per_seq 1: embed, 32 layers,
    # LM-head argmax, stop bookkeeping) as generate runs it (graph replay), timed with HIP events
    dec.next_tok.zero_()
    for t in (dec.step_ctr, dec.done, dec.all_done):
        t.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    dec.pos[:B].fill_(30)
    dec.decode_step(B)                              # captured already by generate
    e0.record()
    for _ in range(reps):
        dec.decode_step(B)
    e1.record()
    e1.synchronize()
    step_s = e0.elapsed_time(e1) / 1e3 / reps
    byts = w.nbytes()
    res = {
        "metric": "audio clips/sec, Mistral-7B caption decoder (en+zh+fr greedy generate), bs=32",
        "value": round(n * B / dt_s, 3), "unit": "clips/s", "n_gpus": 1, "steps": n,
        "warmup": warmup, "ms_per_step": round(dt_s / n * 1e3, 1), "higher_is_better": True,
        "dtype": "fp8 weights (e4m3, per-channel scale) x bf16 activations, f32 accumulation",
        "data": DATA + "; Mistral-7B geometry, synthetic fp8 weights",
        "config": {"workload": "C5: wav -> HTSAT -> prompt + MLP mapper (1024->20480->40960) -> "
                               "Mistral-7B greedy generate(max_length 60, eos 2) x 3 language tags",
                   "batch": B, "generated_tokens": ntok,
                   "language_tags_concurrent": conc},
        "roofline": {"kernel": "one Mistral-7B decode step at 32 rows (32 layers: fp8 GEMMs + "
                               "RoPE/attention/norms, bf16 LM head argmax)", "bound": "hbm",
                     "achieved": round(byts / step_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(byts / step_s / 1e9 / HBM_PEAK_GBS, 4),
                     "step_us": round(step_s * 1e6, 1), "algo_bytes_per_step": int(byts)},
        "note": "secondary config C5 (predict_mistralai_multilingual.py); not the headline metric"}
    del dec, decs, w, enc, mapper
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def roofline_lmhead_beam(pipe, reps=20):
    """The C3 beam decode's dominant GEMM: the LM head over all C x beam rows (1280 at B = 256,
    beam 5) against the tied wte [50257 x 768] bf16, with its fused per-row max / sum-exp /
    top-k epilogue (zs_lmhead_topk, the call _beam_step_body makes), MFMA-bound: 2 M V K flops
    per launch / its average duration (HIP events, back-to-back launches in one graph)."""
    from zsaac import ops
    dec = pipe.decoder
    R = pipe.cfg.batch * pipe.cfg.beam
    V, K = pipe.gpt.wte.shape
    a = dec.hf[:R]

    def launch(i):
        ops.lmhead_topk(a, pipe.gpt.wte, dec.topk, dec.pstat, dec.pval, dec.pidx)
    avg = _graph_time(launch, reps)
    fl = 2.0 * R * V * K
    tf = fl / avg / 1e12
    return {"kernel": f"lmhead_kernel<bf16,128,8> (zs_lmhead_topk) M={R} V={V} K={K}, top-{dec.topk} "
                      f"+ softmax statistics per 128-token block", "bound": "mfma",
            "achieved": round(tf, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / MFMA_BF16_PEAK_TFLOPS, 4), "avg_launch_us": round(avg * 1e6, 2),
            "flops_per_launch": int(fl)}


def roofline_c3_step(pipe, reps=20):
    """C3's dominant kernels per beam decode step at its rows (256 clips x beam 5 = 1280):
    the four decode GEMMs of a block as _layers issues them (qkv, attn.c_proj + residual, c_fc
    + gelu_new, mlp.c_proj + residual; HIP events, back-to-back launches in one graph), their
    MFMA fraction as sum(FLOP) / sum(time) over the 12 blocks, the decode attention's HBM
    fraction (unique K / V bytes, cold caches: roofline_attention) and the LM head's MFMA
    fraction (roofline_lmhead_beam); shares of the modelled step time."""
    from zsaac import ops
    dec, ly = pipe.decoder, pipe.gpt.layers[0]
    R = pipe.cfg.batch * max(1, pipe.cfg.beam)
    h, qkv, att, hid, x = dec.h[:R], dec.qkv[:R], dec.att[:R], dec.hid[:R], dec.x[:R]
    shapes = {
        "qkv": (lambda i: ops.gemm(h, ly["attn_w"], qkv, bias=ly["attn_b"], workspace=dec.ws), 3 * 768, 768),
        "proj": (lambda i: ops.gemm(att, ly["proj_w"], x, bias=ly["proj_b"], residual=x,
                                    workspace=dec.ws), 768, 768),
        "fc": (lambda i: ops.gemm(h, ly["fc_w"], hid, bias=ly["fc_b"], act=ops.ACT_GELU_TANH,
                                  workspace=dec.ws), 3072, 768),
        "mproj": (lambda i: ops.gemm(hid, ly["mproj_w"], x, bias=ly["mproj_b"], residual=x,
                                     workspace=dec.ws), 768, 3072),
    }
    gem, fl_tot, t_tot = {}, 0.0, 0.0
    for name, (launch, N, K) in shapes.items():
        avg = _graph_time(launch, reps)
        fl = 2.0 * R * N * K
        gem[name] = {"avg_us": round(avg * 1e6, 2), "tflops": round(fl / avg / 1e12, 1)}
        fl_tot += fl
        t_tot += avg
    tf = fl_tot / t_tot / 1e12
    attn = roofline_attention(pipe)
    lm = roofline_lmhead_beam(pipe)
    step = {"gemms": 12 * t_tot, "attention": 12 * attn["avg_launch_us"] * 1e-6,
            "lm_head": lm["avg_launch_us"] * 1e-6}
    tot = sum(step.values())
    return {"decode_gemms": {"kernel": f"the 4 decode GEMMs of a block at M={R} (zs_gemm: lean "
                                       f"bf16 MFMA tiles)", "bound": "mfma",
                             "achieved": round(tf, 1), "peak": MFMA_BF16_PEAK_TFLOPS,
                             "unit": "TFLOP/s", "frac": round(tf / MFMA_BF16_PEAK_TFLOPS, 4),
                             "per_gemm": gem},
            "decode_attention": attn, "lm_head": lm,
            "step_share": {k: round(v / tot, 3) for k, v in step.items()},
            "modelled_step_us": round(tot * 1e6, 1)}


def c3_beam5(args, device, n_clips=1024, inflight=4):
    """C3 (BASELINE.json configs[2]): the same wav -> HTSAT -> MLP -> GPT-2 path with
    generate_beam (beam 5) on eval batches of 256 clips (1280 decode rows), 1024 synthetic clips,
    `inflight` batches in flight; plus the rooflines of its dominant kernels per decode step
    (roofline_c3_step: the decode GEMMs' MFMA fraction, attention, LM head).  With every batch
    co-running, 128 x 128 tiles for all GEMMs (`lean_min128` 0: the CU-cheapest tile, not the
    fastest alone) -- tools/c3_probe.py, profiles/r4/c3_probe.txt: 2 in flight 3.17k, 4: 3.41k,
    4 + 128 x 128 tiles 3.56k clips/s."""
    import copy
    from zsaac._lib import call
    a3 = copy.copy(args)
    a3.beam, a3.batch, a3.group, a3.encoder_batch = 5, 256, 1, 0
    pipe, _, _ = build(a3, device, dtype=torch.bfloat16, group=1)
    call("zs_tune_set", b"lean_min128", 0)
    try:
        dt, outs, runner, info = run_captions(a3, 1, 0, device, pipe, n_clips, 3 * 10 ** 6,
                                              [n_clips], inflight, 1)
    finally:
        call("zs_tune_set", b"lean_min128", 256)
    res = {"metric": "audio clips/sec end-to-end (encode+mapper+GPT-2 decode), AudioCaps-eval "
                     "beam 5 bs=256", "value": round(n_clips / dt, 2), "unit": "clips/s",
           "clips": n_clips, "ms_per_step": round(dt / math.ceil(n_clips / 256) * 1e3, 3),
           "dtype": "bf16", "config": {"workload": "C3: HTSAT + MLP mapper + GPT-2 generate_beam, "
                                                   "beam 5, entry_length 67", "eval_batch": 256,
                                       "decode_rows_per_gemm": 1280,
                                       "steps_in_flight_per_gpu": inflight,
                                       "gemm_tiles": "128x128 for every lean GEMM (lean_min128 0)",
                                       **info},
           "roofline": None}
    step = roofline_c3_step(pipe)
    res["roofline"] = step["decode_gemms"]
    res["roofline_step"] = step
    del runner, outs, pipe
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def strong_scaling_proxy(args, device, pipe, t_full, n_full, n_ranks=8, full_src=None):
    """Predicted 1 -> 8 GPU strong-scaling speed-up on Clotho-eval from ONE GPU: one rank's
    1/8 shard (shard_range: 131 clips) timed alone, T(1045) / T(131).  Two batchings of the
    shard: the reference's consecutive bs-64 batches (64 + 64 + 3) and near-equal batches over
    every in-flight stream (split_batches parts=inflight); the faster is what a rank runs."""
    from zsaac import dist as zd
    full_src = full_src or "the headline's timed region"
    if t_full is None:
        t_full = run_captions(args, 1, 0, device, pipe, n_full, 0, [n_full], args.inflight, 3,
                              reps=3)[0]
        full_src = "a separate run of the full set (median of 3, not the headline's timed region)"
    lo, hi = zd.shard_range(n_full, 0, n_ranks)
    n = hi - lo
    out = {"clips_full": n_full, "seconds_full": round(t_full, 4), "full_timing": full_src,
           "ranks": n_ranks, "clips_per_rank": n}
    best = None
    # the reference's consecutive bs-64 batches (64 + 64 + 3), and the same number of batches
    # balanced (44 + 44 + 43); each warmed up, the median of 5 runs
    for name, parts in (("bs64_batches", 0), ("balanced_batches", -(-n // pipe.cfg.batch))):
        dt, outs, runner, _ = run_captions(args, 1, 0, device, pipe, n, lo, [n], args.inflight,
                                           3, parts=parts, reps=5)
        sizes = [int(o.ids.shape[0]) for o in outs]
        out[name] = {"seconds": round(dt, 4), "batches": sizes,
                     "grids": [g for g in getattr(runner, "grid", [])],
                     "predicted_speedup": round(t_full / dt, 2)}
        best = max(best or 0.0, t_full / dt)
        del outs, runner
    out["predicted_speedup"] = round(best, 2)
    out["note"] = ("one GPU, one rank's shard alone; the 8-rank run adds one RCCL all-gather of "
                   "token ids (zsaac/dist.py collect_captions)")
    return out


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    device = torch.device("cuda", local)
    from zsaac import dist as zd
    if args.magic:
        return main_magic(args, torch.device("cuda", 0))
    if args.mistral:
        return main_mistral(args, torch.device("cuda", 0))
    pipe, csd, asd = build(args, device)
    if args.embeddings_only:
        main_embeddings(args, world, rank, device, pipe)
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    B = pipe.cfg.batch
    if args.clips:                              # strong scaling: a fixed clip set, sharded
        n_total, scaling = args.clips, "strong"
        lo, hi = zd.shard_range(n_total, rank, world)
        counts = zd.shard_counts(n_total, world)
    else:                                       # weak scaling: a fixed clip count per rank
        per = args.steps * B if args.steps else CLOTHO_EVAL_CLIPS
        n_total, scaling = per * world, "weak"
        lo, hi = rank * per, (rank + 1) * per
        counts = [per] * world
    n_local = hi - lo
    steps = -(-n_local // B)
    want_roof = (rank == 0 and not args.no_roofline and args.group == 1 and B <= 64
                 and not args.beam and args.dtype == "bf16")
    dt, outs, runner, info = run_captions(args, world, rank, device, pipe, n_local, lo, counts,
                                          args.inflight, args.warmup, log_pass=want_roof,
                                          reps=max(1, args.reps))
    workload = (("C3 AudioCaps-eval" if args.beam else "C2 Clotho-eval")
                + (" (1045 clips per rank)" if not (args.steps or args.clips) else "")
                + ": STFT/log-mel + " + args.encoder.upper() + " + " + args.mapper
                + " mapper + GPT-2 small " + ("greedy generate2" if not args.beam else f"beam {args.beam}")
                + f", entry_length {args.entry_length}, + get_prefix_tokens")
    metric = METRIC if not args.beam and args.group == 1 else (
        f"audio clips/sec end-to-end (encode+mapper+GPT-2 decode), "
        + (f"AudioCaps-eval beam {args.beam} bs={args.batch * args.group}" if args.beam
           else f"Clotho-eval {args.group}x{args.batch} clips per decode step (throughput mode)"))
    res = {
        "metric": metric, "value": round(n_total / dt, 2), "unit": "clips/s", "n_gpus": world,
        "steps": steps, "warmup": args.warmup, "ms_per_step": round(dt / steps * 1e3, 3),
        "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
        "dtype": "bf16" if args.dtype == "bf16" else "f32", "data": DATA,
        "config": {"workload": workload, "eval_batch": args.batch,
                   "eval_batches_per_step": args.group, "batch_per_gpu": B,
                   "decode_rows_per_gemm": B * max(1, args.beam),
                   "clips_per_rank": n_local, "clips_total": n_total,
                   "global_batch": B * world, "steps_in_flight_per_gpu": max(1, args.inflight),
                   "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                   "encoder_batch": (runner.enc.B if getattr(runner, "enc", None) is not None
                                     else pipe.encoder.B),
                   "encoder_note": ("the encoder (wav -> CLAP embedding) runs ahead in passes of "
                                    "encoder_batch clips (consecutive eval batches; the reference "
                                    "extracts embeddings offline, data_handing/"
                                    "embeddings_generator.py), the caption path at eval_batch"),
                   "parallelism": f"dp{world} (clip-sharded, RCCL all-gather of token ids)",
                   **info},
    }
    reps_t = info["timed_reps_s"]
    res["value_spread"] = {"median": res["value"], "min": round(n_total / max(reps_t), 2),
                           "max": round(n_total / min(reps_t), 2), "reps": len(reps_t),
                           "note": "value = the median of the timed repetitions of the whole "
                                   "region (each: barrier + sync on both sides, max over ranks)"}
    if info["persist_gave_up"]:
        res["warning"] = (f"{info['persist_gave_up']} persistent decode launches gave up (grid "
                          "not co-resident) and finished on the phase launches")
    if world > 1 and not args.clips and args.group == 1 and not args.beam:
        # strong scaling on the Clotho-eval set itself: its 1045 clips sharded over the ranks
        # (what north_star's ">= 6x from 1 to 8 GPUs on Clotho-eval" measures), timed beside the
        # weak-scaling value
        slo, shi = zd.shard_range(CLOTHO_EVAL_CLIPS, rank, world)
        scounts = zd.shard_counts(CLOTHO_EVAL_CLIPS, world)
        dts, _, srun, sinfo = run_captions(args, world, rank, device, pipe, shi - slo, slo, scounts,
                                           args.inflight, 1, reps=max(1, args.reps))
        res["strong_1045"] = {"value": round(CLOTHO_EVAL_CLIPS / dts, 2), "unit": "clips/s",
                              "clips_total": CLOTHO_EVAL_CLIPS, "clips_per_rank": scounts,
                              "seconds": round(dts, 5), "timed_reps_s": sinfo["timed_reps_s"],
                              "scaling": "strong",
                              "grids_rank0": sinfo["persist_grids"]}
        del srun
    headline_cfg = rank == 0 and args.group == 1 and B <= 64 and not args.beam
    if rank == 0 and not args.no_roofline and headline_cfg and args.dtype == "bf16":
        log("rooflines")
        from zsaac import decoder as zdec
        if pipe.decoder.persist:
            res["roofline"] = persist_roofline(pipe, runner, runner.log_outs, dt, runner.timed_log)
        else:
            res["roofline"] = roofline_gemm_ln(pipe)
        wav = synthetic_clips(B, 0, device)
        agg = info["decode_steps_mean"] * steps / dt if world == 1 else None
        res["roofline_decode_step"] = decode_step_roofline(pipe, wav, agg)
        res["stages"] = stage_times(pipe, wav)
        # the per-step-path kernels (configs the persistent launch does not take: beam, f32,
        # > 64 rows), at the bs-64 decode shapes, cold weights / K/V
        res["roofline_stepwise_c_fc"] = roofline_gemm_ln(pipe)
        res["roofline_stepwise_mproj"] = roofline_rows_gemm(pipe, "mproj")
        res["roofline_stepwise_proj"] = roofline_rows_gemm(pipe, "proj")
        res["roofline_decode_attention"] = roofline_attention(pipe)
        res["persist_launches_all"] = persist_all_launches(ALL_PERSIST_LOGS)
        del wav
    elif rank == 0 and args.stages:
        res["stages"] = stage_times(pipe, synthetic_clips(B, 0, device))
    t_full = None
    if rank == 0 and world == 1 and headline_cfg and not args.clips:
        # the metric's own set: the 1045-clip Clotho-eval set, the headline itself when it ran on
        # it, else timed here (median of 3) when --steps sized the headline differently
        if n_total == CLOTHO_EVAL_CLIPS:
            t_full, c_reps, c_src = dt, info["timed_reps_s"], "the headline's timed region"
        else:
            t_full, _, _, c_info = run_captions(args, 1, 0, device, pipe, CLOTHO_EVAL_CLIPS, 0,
                                                [CLOTHO_EVAL_CLIPS], args.inflight, 3, reps=3)
            c_reps, c_src = c_info["timed_reps_s"], "a separate run after the headline (median of 3)"
        res["clotho_1045"] = {"value": round(CLOTHO_EVAL_CLIPS / t_full, 2), "unit": "clips/s",
                              "clips": CLOTHO_EVAL_CLIPS, "seconds": round(t_full, 5),
                              "timed_reps_s": c_reps, "source": c_src}
    if (rank == 0 and world == 1 and headline_cfg and not args.clips
            and not args.no_scaling_proxy):
        # on the 1045-clip Clotho-eval set (clotho_1045 above)
        res["strong_scaling_proxy"] = strong_scaling_proxy(
            args, device, pipe, t_full, CLOTHO_EVAL_CLIPS,
            full_src=res["clotho_1045"]["source"] if "clotho_1045" in res else None)
    del runner, outs

    def release():
        # (runners hold reference cycles: collect them so their buffers return to the device
        # before the next configuration allocates its own)
        import gc
        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and args.extras and args.group == 1 and not args.beam:
        del pipe
        release()
        log("f32 parity mode")
        # the f32 grid decode (G = 192): two grids co-resident, so 2 pipelines run (4 asked;
        # tools/f32_profile.py, profiles/r5/f32_sweep.txt)
        res["f32_parity_mode"] = sub_run(args, device, torch.float32, 1, F32_INFLIGHT,
                                         CLOTHO_EVAL_CLIPS, 1, reps=3)
        res["f32_parity_mode"]["note"] = ("the headline's 1045 clips at bs=64 in f32: the mode "
                                          "whose greedy ids are bit-exact")
        release()
        log("throughput mode")
        res["throughput_mode"] = sub_run(args, device, torch.bfloat16, 128, 3, 3 * 8192, 1,
                                         encoder_batch=256)
        res["throughput_mode"]["note"] = ("128 eval batches decoded together (8192-row decode "
                                          "GEMMs), 3 in flight: NOT the metric's bs=64")
        release()
        log("C3 beam 5")
        res["c3_beam5"] = c3_beam5(args, device)
        release()
        log("C5 Mistral-7B")
        res["c5_mistral"] = c5_mistral(args, device)
        log("id agreement")
        from tools import idparity
        res["id_agreement"] = {"bench_weights": BENCH_WEIGHTS_GOLDEN,
                               "bf16": idparity.summary(torch.bfloat16, device),
                               "f32": idparity.summary(torch.float32, device)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_baseline_clips > 0:
        n2, n1, n3 = ((64, 50, 64) if args.cpu_baseline_full else
                      (args.cpu_baseline_clips, 50, max(4, args.cpu_baseline_clips // 4)))
        res["cpu_baseline"] = cpu_baseline(args, csd, asd, n2, n1, n3)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
