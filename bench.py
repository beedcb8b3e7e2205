#!/usr/bin/env python3
"""Benchmark of the zero-shot audio-captioning hot path on MI355X (BASELINE.json metric):

    audio clips/sec end-to-end (encode + mapper + GPT-2 decode), Clotho-eval bs=64

Workload (BASELINE.json configs[1], "C2"): synthetic 10 s / 32 kHz waveforms (randn*0.1, clipped)
already resident in HBM -> STFT/log-mel + bn0 -> HTSAT -> audio_proj + L2 -> sound-effect hard
prompt -> MLP mapper -> GPT-2 small prefill + get_prefix_tokens + greedy generate2
(entry_length 67, stop ids 13/764), bf16 operands / f32 accumulation, batch 64 clips per GPU.
One "step" = one batch of 64 clips through the whole path on every rank.  --inflight (default 4)
independent bs=64 batches are decoded concurrently per GPU on separate HIP streams (pipeline
twins sharing the weights, zsaac/pipeline.py ConcurrentRunner) — the batch size the reference
evaluates with stays 64; the GPU just works on several such batches at once.  After the K timed
steps, ONE RCCL all-gather of every batch's generated token ids + lengths (the only collective,
SURVEY §8e) is inside the timed region.  Weights are seeded random init at the reference
architecture (no checkpoints offline).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

Rank 0 prints ONE JSON line.  Besides the contract fields it carries
  roofline:     the dominant kernel family (bf16 MFMA GEMM) at the decode MLP up-projection
                shape the bench runs (R = decode rows) — algorithmic flops per launch / its
                average duration, timed live with HIP events on the stream it runs on;
                roofline_decode_attention: the HBM-bound decode attention, same method;
  cpu_baseline: the oracle (reference semantics: batch 1, full recompute, fp32) on a bounded
                sample of the same workload, timed on this host's CPU (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
GPT2_KW = dict(seed=0, std=0.1, emb_std=0.1, stop_boost=2.0)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--encoder", default="htsat", choices=["htsat", "cnn14"])
    ap.add_argument("--mapper", default="mlp", choices=["mlp", "transformer"])
    ap.add_argument("--beam", type=int, default=0)
    ap.add_argument("--entry-length", type=int, default=67)
    ap.add_argument("--encoder-batch", type=int, default=256,
                    help="clips per encoder pass (0 = --batch); per-clip results do not depend on it")
    ap.add_argument("--group", type=int, default=128,
                    help="eval batches of --batch clips decoded together (one decode step over "
                         "group*batch rows; measured 32 -> 64 -> 128: 10.9k -> 12.1k -> 12.3k "
                         "clips/s); encoded --encoder-batch clips per pass")
    ap.add_argument("--inflight", type=int, default=3,
                    help="independent groups in flight per GPU, each on its own HIP stream "
                         "(A/B in one box at group 128: 3 -> 12.73-12.75k, 2 -> 12.51-12.60k, "
                         "4 -> 12.70k clips/s; 1: -11 %%)")
    ap.add_argument("--compact", type=int, default=1,
                    help="greedy bf16: decode only the rows that have not stopped (0 = all rows)")
    ap.add_argument("--cpu-baseline-clips", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--stages", action="store_true", help="also report per-stage ms (extra syncs)")
    ap.add_argument("--embeddings-only", action="store_true",
                    help="C4: batched HTSAT/CNN14 encode_audio + one RCCL all-gather of the "
                         "[N,1024] embeddings (no caption decode)")
    return ap.parse_args()


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


def build(args, device):
    from zsaac import synthetic as S
    from zsaac.pipeline import CaptionConfig, CaptionPipeline
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    csd = S.gpt2_state_dict(**GPT2_KW)
    csd.update(S.mlp_mapper_state_dict(1) if args.mapper == "mlp" else S.transformer_mapper_state_dict(2))
    if args.encoder == "htsat":
        asd = S.htsat_state_dict(3)
        asd.update(S.audio_proj_state_dict(5, audio_width=768))
    else:
        asd = S.cnn14_state_dict(4)
        asd.update(S.audio_proj_state_dict(5, audio_width=2048))
    cfg = CaptionConfig(encoder=args.encoder, mapping_type=args.mapper, dtype=dtype,
                        batch=args.batch * getattr(args, "group", 1),
                        encoder_batch=getattr(args, "encoder_batch", 0) or args.batch,
                        beam=args.beam, entry_length=args.entry_length,
                        compact_decode=bool(getattr(args, "compact", 1)))
    pipe = CaptionPipeline(csd, asd, S.label_table(), S.label_token_table(), cfg, device=device)
    return pipe, csd, asd


PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic_r1.json")
MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)


def roofline_setup(pipe, cold_bytes=640 << 20):
    """The dominant kernel family is the bf16 MFMA GEMM (gemm_lean_kernel: HTSAT stage 4 and the
    GPT-2 decode/prefill linears).  Its roofline is taken at the decode-step MLP up-projection
    as the bench runs it: c_fc out[R,3072] = gelu_new(h[R,768] @ W[3072,768]^T + b), R = the
    decode rows of one step (eval batches x 64), through ops.gemm exactly as the decoder calls
    it.  Launches rotate over enough distinct copies of W (> the 256 MiB Infinity Cache) that
    every launch streams its weights from HBM, as in the real decode.  Returns (launch fn,
    algorithmic flops, algorithmic bytes, number of W copies, kernel-name substring)."""
    from zsaac import ops
    dec = pipe.decoder
    ly = pipe.gpt.layers[0]
    M = pipe.cfg.batch * max(1, pipe.cfg.beam)
    h, hid = dec.h[:M], dec.hid[:M]
    W, b = ly["fc_w"], ly["fc_b"]
    N, K = W.shape
    es = W.element_size()
    copies = [W] + [W.clone() for _ in range(max(0, -(-cold_bytes // W.nbytes) - 1))]
    flops = 2 * M * N * K
    algo_bytes = N * K * es + M * K * es + N * 4 + M * N * es
    kname = "gemm_skinny_kernel" if M <= 64 else "gemm_lean_kernel"

    def launch(i):
        ops.gemm(h, copies[i % len(copies)], hid, bias=b, act=ops.ACT_GELU_TANH, workspace=dec.ws)
    return launch, flops, algo_bytes, len(copies), kname, (M, N, K)


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


def kernel_roofline(pipe):
    """roofline (dominant kernel, MFMA-bound at the bench's decode rows) + a secondary HBM-bound
    entry for the decode attention (the largest single-shape kernel)."""
    launch, flops, algo_bytes, ncopy, kname, (M, N, K) = roofline_setup(pipe)
    avg_s = _graph_time(launch, 2 * ncopy)
    tflops = flops / avg_s / 1e12
    traffic, tsrc = None, None
    if os.path.exists(PMC_FILE):          # rocprofv3 --pmc passes of tools/pmc_traffic.py
        with open(PMC_FILE) as f:
            pmc = json.load(f)
        if pmc.get("shape") == [M, N, K]:
            traffic, tsrc = pmc["hbm_bytes_per_launch"], os.path.relpath(PMC_FILE, ROOT)
    res = {"kernel": f"{kname}<bf16> decode c_fc [{M}x{K}]x[{K}x{N}] +bias +gelu_new (cold W)",
           "bound": "mfma", "achieved": round(tflops, 1), "peak": MFMA_BF16_PEAK_TFLOPS,
           "unit": "TFLOP/s", "frac": round(tflops / MFMA_BF16_PEAK_TFLOPS, 4),
           "traffic": traffic, "traffic_source": tsrc, "avg_launch_us": round(avg_s * 1e6, 3),
           "algo_flops_per_launch": flops, "algo_bytes_per_launch": algo_bytes,
           "hbm_GBps_algorithmic": round(algo_bytes / avg_s / 1e9, 1)}
    return res, attention_roofline(pipe)


def attention_roofline(pipe, L_mean=None):
    """decode attention (decode_attn6_kernel, the default) at the bench's decode rows, every row at the mean key count of a
    67-step greedy decode (prompt Pmax + 34): algorithmic bytes = K and V of every key read once
    + q/k/v of the new token + the output, per (row, head)."""
    from zsaac import ops
    dec = pipe.decoder
    R = pipe.cfg.batch * max(1, pipe.cfg.beam)
    D, H, Lmax = 768, 12, dec.Lmax
    L = L_mean or min(Lmax - 1, pipe.Pmax + 34)
    lay = dec.kc[0] if isinstance(dec.kc, (list, tuple)) else None
    kc = lay if lay is not None else torch.randn(R, H, Lmax, 64, device=pipe.dev).bfloat16()
    vc = (dec.vc[0] if isinstance(dec.vc, (list, tuple)) else torch.randn_like(kc))
    qkv = dec.qkv[:R] if hasattr(dec, "qkv") else torch.randn(R, 3 * D, device=pipe.dev).bfloat16()
    pos = torch.full((R,), L - 1, device=pipe.dev, dtype=torch.int32)
    out = torch.empty(R, D, device=pipe.dev, dtype=qkv.dtype)

    def launch(i):
        ops.decode_attention(qkv, R, D, H, kc, vc, Lmax, pos, out)
    avg_s = _graph_time(launch, 50)
    es = qkv.element_size()
    byts = R * H * (2 * L * 64 * es) + R * 3 * D * es + R * D * es
    gbs = byts / avg_s / 1e9
    return {"kernel": f"decode_attn6_kernel<bf16> R={R} heads=12 keys={L}", "bound": "hbm",
            "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "avg_launch_us": round(avg_s * 1e6, 3),
            "algo_bytes_per_launch": byts}


def stage_times(pipe, wav, reps=3):
    """Per-stage device time of one batch (events between stages; extra syncs, so outside the
    timed region): front end + encoder + proj, prompt + mapper + prefill + prefix tokens, decode."""
    from zsaac import ops
    dec, cfg = pipe.decoder, pipe.cfg
    B, Pmax = wav.shape[0], pipe.Pmax
    out = {"encode": [], "prompt_mapper_prefill": [], "decode": []}
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        emb = pipe.encode(wav)
        ev[1].record()
        ops.prompt_assemble(emb, pipe.labels, cfg.sound_effect_num, pipe.label_tok, pipe.label_len,
                            pipe.hard_ids[:B], pipe.hard_len[:B])
        soft = pipe.mapper(ops.l2norm(emb, out=pipe.prefix[:B]))
        ops.prefill_embed(pipe.hard_ids[:B], pipe.hard_len[:B], soft, pipe.mapper.soft_ld,
                          cfg.prefix_length, pipe.gpt.wte, pipe.gpt.wpe, B, Pmax,
                          pipe.embed[:B * Pmax], dec.x, dec.plen, dec.last_row)
        pipe.prefix_tokens(B, soft)
        dec.prefill(B, Pmax)
        ev[2].record()
        dec.greedy(B, Pmax)
        ev[3].record()
        torch.cuda.synchronize()
        for i, k in enumerate(out):
            out[k].append(ev[i].elapsed_time(ev[i + 1]))
    res = {k: round(sorted(v)[len(v) // 2], 3) for k, v in out.items()}
    res["decode_steps"] = int(dec.step_ctr.item())
    return res


def cpu_baseline(args, csd, asd, n_clips):
    """Oracle = reference semantics (batch 1 per clip, full-sequence recompute every step, fp32)
    on `n_clips` clips of the same synthetic workload, on this host's CPU."""
    sys.path.insert(0, ROOT)
    from oracle import audio as A, caption as OC, frontend as OF
    from zsaac import synthetic as S
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    table, lt = S.label_table(), S.label_token_table()
    wav = S.synthetic_waveforms(n_clips, seed=777)
    t0 = time.perf_counter()
    ntok = 0
    with torch.no_grad():
        for i in range(n_clips):
            lm = OF.logmel(wav[i:i + 1])
            if args.encoder == "htsat":
                feat = A.htsat_embedding(lm, asd)
            else:
                feat = A.cnn14_embedding(lm, asd)
            emb = A.audio_project(feat, asd)
            idx = OC.sound_effect_choice(emb, table, 3)[0].tolist()
            hard = torch.tensor([OC.prompt_ids(idx, lt)])
            pe = OC.clap_to_gpt(torch.nn.functional.normalize(emb, dim=-1)[None], hard, csd,
                                args.mapper)
            OC.prefix_tokens(pe, csd)
            if args.beam:
                OC.generate_beam(pe, csd, beam_size=args.beam, entry_length=args.entry_length)
            else:
                ntok += len(OC.generate2(pe, csd, entry_length=args.entry_length))
    dt = time.perf_counter() - t0
    return {"value": round(n_clips / dt, 4), "unit": "clips/s", "cores": threads, "kind": "port",
            "sample": f"{n_clips} clips of the same workload, batch 1, full recompute per step "
                      f"(reference semantics), fp32, {ntok} tokens, {dt:.1f} s"}


def main_embeddings(args, world, rank, device, pipe):
    """BASELINE.json configs[3] (C4): embedding extraction, data_handing/embeddings_generator.py
    realised as batched encode_audio over synthetic clips sharded across ranks, then one RCCL
    all-gather of the [N,1024] f32 embeddings (SURVEY §8d "C4 reinterpretation")."""
    B = args.batch * args.group
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    pool = [(torch.randn(B, 320000, device=device, generator=g) * 0.1).clamp_(-1, 1)
            for _ in range(min(2, args.steps + args.warmup))]
    embs = torch.empty(args.steps, B, 1024, device=device)

    def run(first, n, keep):
        for i in range(n):
            e = pipe.encode(pool[(first + i) % len(pool)])
            if keep:
                embs[i].copy_(e)
        if keep and world > 1:
            gathered = torch.empty(world * embs.numel(), device=device)
            torch.distributed.all_gather_into_tensor(gathered, embs.view(-1))
    run(0, args.warmup, False)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.warmup, args.steps, True)
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
           "value": round(world * B * args.steps / dt, 2), "unit": "clips/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "bf16" if args.dtype == "bf16" else "f32",
           "data": "synthetic 10 s / 32 kHz waveforms (randn*0.1) resident in HBM; seeded weights",
           "config": {"workload": "C4 embedding extraction, RCCL all-gather of [N,1024] f32",
                      "encoder_batch": pipe.encoder.B, "batch_per_gpu": B, "global_batch": B * world,
                      "parallelism": f"dp{world} (clip-sharded)"}}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    device = torch.device("cuda", local)
    from zsaac import synthetic as S
    pipe, csd, asd = build(args, device)
    if args.embeddings_only:
        return main_embeddings(args, world, rank, device, pipe)
    B = args.batch * args.group           # clips per step (group eval batches, decoded together)
    # input pool resident in HBM before timing: distinct synthetic clips per step and rank
    pool = []
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    for _ in range(min(4, args.steps + args.warmup)):
        pool.append((torch.randn(B, 320000, device=device, generator=g) * 0.1).clamp_(-1, 1))
    from zsaac.pipeline import ConcurrentRunner
    runner = ConcurrentRunner(pipe, max(1, args.inflight))

    def run(first, n):
        """n batches through the runner (inflight batches decoding concurrently on separate
        streams), then ONE RCCL all-gather of every batch's token ids + lengths in input order
        (completion order is timing-dependent, so no per-batch collective)."""
        outs = runner.run([pool[(first + i) % len(pool)] for i in range(n)])
        if world > 1 and outs:
            import torch.distributed as dist
            ids = torch.cat([(o.ids if o.ids.dim() == 2 else o.ids[:, 0]).reshape(-1) for o in outs])
            ln = torch.cat([(o.lengths if o.lengths.dim() == 1 else o.lengths[:, 0]).int() for o in outs])
            ids_all = torch.empty(world * ids.numel(), dtype=ids.dtype, device=device)
            len_all = torch.empty(world * ln.numel(), dtype=ln.dtype, device=device)
            dist.all_gather_into_tensor(ids_all, ids)
            dist.all_gather_into_tensor(len_all, ln)
        return outs

    runner.warmup(pool[0])          # one batch per twin: captures every decode graph
    run(0, args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    cap0 = sum(p.decoder.n_captures for p in runner.pipes)
    rows0 = sum(p.decoder.rows_stepped for p in runner.pipes)
    t0 = time.perf_counter()
    ntok = 0
    outs = run(args.warmup, args.steps)
    last = outs[-1] if outs else None
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    if last is not None:
        ntok = int(last.lengths.sum()) if last.scores is None else int(last.lengths[:, 0].sum())
    clips = world * B * args.steps
    res = {
        "metric": "audio clips/sec end-to-end (encode+mapper+GPT-2 decode), Clotho-eval bs=64",
        "value": round(clips / dt, 2),
        "unit": "clips/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if args.dtype == "bf16" else "f32",
        "data": "synthetic 10 s / 32 kHz waveforms (randn*0.1) resident in HBM; seeded random-init "
                "weights at the reference architecture (no checkpoints offline)",
        "config": {"workload": ("C3 AudioCaps-eval" if args.beam else "C2 Clotho-eval")
                               + ": STFT/log-mel + " + args.encoder.upper() + " + "
                               + args.mapper + " mapper + GPT-2 small "
                               + ("greedy generate2" if not args.beam else f"beam {args.beam}")
                               + f", entry_length {args.entry_length}, + get_prefix_tokens",
                   "eval_batch": args.batch, "eval_batches_per_step": args.group,
                   "batch_per_gpu": B, "global_batch": B * world,
                   "steps_in_flight_per_gpu": max(1, args.inflight),
                   "parallelism": f"dp{world} (clip-sharded, RCCL all-gather of token ids)",
                   "tokens_last_batch_rank0": ntok,
                   "decode_rows_stepped_per_clip": round(
                       (sum(p.decoder.rows_stepped for p in runner.pipes) - rows0) / max(1, args.steps * B), 2),
                   "graph_captures_timed": sum(p.decoder.n_captures for p in runner.pipes) - cap0,
                   "decode_steps_mean": round(sum(runner.decode_steps) / max(1, len(runner.decode_steps)), 2)},
    }
    if args.stages and rank == 0:
        res["stages_ms"] = stage_times(pipe, pool[0])
    if rank == 0 and not args.no_roofline:
        res["roofline"], res["roofline_decode_attention"] = kernel_roofline(pipe)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_baseline_clips > 0:
        res["cpu_baseline"] = cpu_baseline(args, csd, asd, args.cpu_baseline_clips)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
