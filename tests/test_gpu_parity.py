"""End-to-end parity of the HIP path against the reference goldens (tests/golden/*.npz, produced
by running the reference) and the oracle.

Tolerances (stated per north_star):
  * greedy token ids: BIT-EXACT in f32 parity mode (C1 fixture: 50 clips, 67 steps, with stops);
  * beam token lists and order: exact in f32 mode;
  * encoder embeddings: f32 mode max |err| <= 2e-4 * max|ref| (HTSAT) / 5e-4 (CNN14 deep convs);
    bf16 mode cosine(ref, got) >= 0.995;
  * mapper outputs: f32 1e-4 relative.
  * bf16 perf mode, first-step logits: rms error / std(logits) no worse than torch's own bf16
    execution of the same network on the CPU (+10%), max |err| < 0.5 std, first token agrees on
    >= 3/4 clips.
bf16 greedy ids are reported (agreement fraction), not asserted bit-exact: with these synthetic
weights (std 0.1, chaotic) bf16 moves logits by ~6% of their std, which exceeds the oracle's
top-2 margin on some steps.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GPT2_KW = dict(seed=0, std=0.1, emb_std=0.1, stop_boost=2.0)


@pytest.fixture(scope="module")
def caption_sd():
    from zsaac import synthetic as S
    sd = S.gpt2_state_dict(**GPT2_KW)
    sd.update(S.mlp_mapper_state_dict(1))
    sd.update(S.transformer_mapper_state_dict(2))
    return sd


def _pipeline(caption_sd, dtype, batch, beam=0, mapping="mlp", audio_sd=None, encoder="htsat",
              entry_length=67):
    from zsaac import synthetic as S
    from zsaac.pipeline import CaptionConfig, CaptionPipeline
    cfg = CaptionConfig(encoder=encoder, mapping_type=mapping, dtype=dtype, batch=batch, beam=beam,
                        entry_length=entry_length)
    return CaptionPipeline(caption_sd, audio_sd, S.label_table(), S.label_token_table(), cfg)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


def test_c1_greedy_f32_bit_exact(cuda, golden, caption_sd):
    g = golden("c1_greedy.npz")
    pipe = _pipeline(caption_sd, torch.float32, 50)
    out = pipe.caption_emb(torch.from_numpy(g["clap_emb"]).to(cuda))
    # hard prompt assembled on device == the reference dataset's __getitem__ + collate
    hl = out.hard_len.cpu().numpy()
    assert hl.tolist() == g["hard_len"].tolist()
    hi = out.hard_ids.cpu().numpy()
    for b in range(50):
        assert hi[b, :hl[b]].tolist() == g["hard_ids"][b, :hl[b]].tolist()
    # prefix embeddings (clap_to_gpt) for the stored clips
    pe = pipe.embed.view(50, pipe.Pmax, 768).cpu().numpy()
    for b in range(g["prefix_embed"].shape[0]):
        n = hl[b] + 10
        assert _rel(pe[b, :n], g["prefix_embed"][b, :n]) < 1e-5
    # get_prefix_tokens ids
    pt = out.prefix_token_lists()
    for b in range(50):
        assert pt[b] == g["prefix_tokens"][b, :len(pt[b])].tolist(), b
    # generate2 ids, bit-exact
    caps = out.captions()
    mism = [b for b in range(50) if caps[b] != g["greedy_ids"][b, :g["greedy_len"][b]].tolist()]
    assert not mism, f"greedy mismatch on clips {mism}"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_prefix_tokens_soft_rows_equal_full(cuda, golden, caption_sd, dtype):
    """get_prefix_tokens over the soft rows + hard ids (zs_prefix_ids_assemble) gives exactly the
    ids of the cosine argmax over every prefix row; the margin check passes for these weights."""
    g = golden("c1_greedy.npz")
    pipe = _pipeline(caption_sd, dtype, 50)
    assert pipe.hard_skip
    out = pipe.caption_emb(torch.from_numpy(g["clap_emb"]).to(cuda))
    fast = out.prefix_ids.clone()
    full = torch.zeros_like(pipe.prefix_ids[:50 * pipe.Pmax])
    pipe.decoder.prefix_tokens(pipe.embed[:50 * pipe.Pmax], full)
    full = full.view(50, pipe.Pmax)
    pl = out.plen.cpu().numpy()
    for b in range(50):
        assert fast[b, :pl[b]].tolist() == full[b, :pl[b]].tolist(), b
    # an id whose own row is NOT its cosine argmax (a duplicated wte row) disables the shortcut
    w = pipe.gpt.wte
    saved = w[5].clone()
    w[5].copy_(w[7])
    pipe.gpt.wte_norm[5].copy_(pipe.gpt.wte_norm[7])
    try:
        assert not pipe.decoder.hard_rows_safe([5, 11], 1e-4)
    finally:
        w[5].copy_(saved)
        pipe.gpt.wte_norm[5].copy_(torch.nn.functional.normalize(saved.float(), dim=0).to(w.dtype))


def test_concurrent_runner_f32_bit_exact(cuda, golden, caption_sd):
    """3 pipeline twins in flight on separate streams, 7 batches of <=8 clips (ragged last batch
    of 2): every clip's generate2 ids still equal the reference's, in input order."""
    from zsaac.pipeline import ConcurrentRunner
    g = golden("c1_greedy.npz")
    pipe = _pipeline(caption_sd, torch.float32, 8)
    emb = torch.from_numpy(g["clap_emb"]).to(cuda)
    runner = ConcurrentRunner(pipe, 3)
    runner.warmup_emb(emb[:8])
    outs = runner.run([emb[i:i + 8] for i in range(0, 50, 8)], inputs="emb")
    assert [o.ids.shape[0] for o in outs] == [8] * 6 + [2]
    caps = [c for o in outs for c in o.captions()]
    mism = [b for b in range(50) if caps[b] != g["greedy_ids"][b, :g["greedy_len"][b]].tolist()]
    assert not mism, f"greedy mismatch on clips {mism}"
    pt = [p for o in outs for p in o.prefix_token_lists()]
    assert all(pt[b] == g["prefix_tokens"][b, :len(pt[b])].tolist() for b in range(50))


def test_c1_bf16_logits_and_agreement(cuda, golden, caption_sd):
    """bf16 perf mode: the first-step logits stay within a stated tolerance of the f32 oracle
    (max |err| <= 0.05 * std(logits)); greedy-id agreement is REPORTED (not asserted): with these
    synthetic weights the oracle's top-1/top-2 margin is often below the bf16 logit error, so ids
    diverge after a few tokens."""
    from oracle import caption as OC
    from zsaac import ops
    g = golden("c1_greedy.npz")
    B = 16
    pipe = _pipeline(caption_sd, torch.bfloat16, B)
    emb = torch.from_numpy(g["clap_emb"][:B]).to(cuda)
    cfg, dec = pipe.cfg, pipe.decoder
    ops.prompt_assemble(emb, pipe.labels, cfg.sound_effect_num, pipe.label_tok, pipe.label_len,
                        pipe.hard_ids[:B], pipe.hard_len[:B])
    soft = pipe.mapper(ops.l2norm(emb, out=pipe.prefix[:B]))
    ops.prefill_embed(pipe.hard_ids[:B], pipe.hard_len[:B], soft, pipe.mapper.soft_ld, 10,
                      pipe.gpt.wte, pipe.gpt.wpe, B, pipe.Pmax, pipe.embed[:B * pipe.Pmax], dec.x,
                      dec.plen, dec.last_row)
    dec.prefill(B, pipe.Pmax)
    got = (dec.hf[:B].float() @ pipe.gpt.wte.float().t()).cpu()
    sd16 = {k: (v.bfloat16() if v.is_floating_point() else v) for k, v in caption_sd.items()
            if k.startswith("gpt.")}
    worst, worst_rms, t16_rms, first_ok = 0.0, 0.0, 0.0, 0
    for b in range(B):
        n = int(g["hard_len"][b])
        pe = torch.from_numpy(g["prefix_embed"][b, :n + 10])[None] if b < 4 else \
            OC.clap_to_gpt(torch.nn.functional.normalize(torch.from_numpy(g["clap_emb"][b:b + 1]), dim=-1)[None],
                           torch.from_numpy(g["hard_ids"][b:b + 1, :n]), caption_sd)
        with torch.no_grad():
            ref = OC.gpt2_logits(pe, caption_sd)[0][0, -1]
            # yardstick: the same network run by torch in bf16 on the CPU
            r16 = OC.gpt2_logits(pe.bfloat16(), sd16)[0][0, -1].float()
        sd_ = ref.std()
        worst = max(worst, float((got[b] - ref).abs().max() / sd_))
        worst_rms = max(worst_rms, float((got[b] - ref).pow(2).mean().sqrt() / sd_))
        t16_rms = max(t16_rms, float((r16 - ref).pow(2).mean().sqrt() / sd_))
        first_ok += int(got[b].argmax()) == int(ref.argmax())
    print(f"bf16 first-step logits: rms err/std = {worst_rms:.4f} (torch-bf16 CPU: {t16_rms:.4f}), "
          f"max|err|/std = {worst:.4f}; first token agrees {first_ok}/{B}")
    # tolerance: no worse than torch's own bf16 execution of the network (+10%), and the first
    # greedy token agrees on >= 3/4 of the clips
    assert worst_rms <= 1.1 * t16_rms + 0.01 and worst < 0.5 and first_ok >= B * 3 // 4
    caps = pipe.caption_emb(emb).captions()
    agree = sum(next((i for i, (x, y) in enumerate(zip(caps[b], g["greedy_ids"][b])) if x != y),
                     min(len(caps[b]), int(g["greedy_len"][b]))) for b in range(B))
    print(f"bf16 greedy: {agree}/{int(g['greedy_len'][:B].sum())} leading tokens agree")


def test_bf16_compacted_decode_equals_full(cuda, golden, caption_sd):
    """Greedy row compaction (decode only the rows that have not stopped, in 256-row buckets)
    gives ids and lengths identical to the uncompacted bf16 decode: 640 clips (buckets 512 and
    640), through the synchronous loop and the concurrent runner."""
    from zsaac import synthetic as S
    from zsaac.pipeline import CaptionConfig, CaptionPipeline, ConcurrentRunner
    g = golden("c1_greedy.npz")
    B = 640
    base = torch.from_numpy(g["clap_emb"]).to(cuda)
    gen = torch.Generator(device="cpu").manual_seed(7)
    emb = base[torch.arange(B) % base.shape[0]] + \
        0.05 * torch.randn(B, base.shape[1], generator=gen).to(cuda)
    outs = {}
    for compact in (False, True):
        cfg = CaptionConfig(dtype=torch.bfloat16, batch=B, compact_decode=compact)
        pipe = CaptionPipeline(caption_sd, None, S.label_table(), S.label_token_table(), cfg)
        assert pipe.decoder.compact == compact
        r = pipe.caption_emb(emb)
        outs[compact] = (r.ids.cpu().numpy(), r.lengths.cpu().numpy())
        if compact:
            runner = ConcurrentRunner(pipe, 2)
            runner.warmup_emb(emb)
            rr = runner.run([emb, emb.flip(0)], inputs="emb")
            outs["runner"] = (rr[0].ids.cpu().numpy(), rr[0].lengths.cpu().numpy())
            outs["runner_flip"] = (rr[1].ids.cpu().numpy()[::-1], rr[1].lengths.cpu().numpy()[::-1])
    ln = outs[False][1]
    print(f"compaction test: mean length {ln.mean():.1f}, stopped early {(ln < 67).mean():.2f}")
    assert (ln < 67).any(), "no row stopped early: the test would not exercise compaction"
    for k in (True, "runner", "runner_flip"):
        assert np.array_equal(outs[k][1], ln), k
        for b in range(B):
            assert outs[k][0][b, :ln[b]].tolist() == outs[False][0][b, :ln[b]].tolist(), (k, b)


@pytest.mark.parametrize("beam", [5, 3])
def test_beam_f32(cuda, golden, caption_sd, beam):
    g = golden("beam.npz")
    C = g["clap_emb"].shape[0]
    pipe = _pipeline(caption_sd, torch.float32, C, beam=beam)
    # feed the fixture's fixed hard prompts: bypass prompt assembly
    from zsaac import ops
    dec = pipe.decoder
    B, Pmax = C, pipe.Pmax
    hard = torch.zeros(C, pipe.h_cap, dtype=torch.int32)
    hard[:, :g["hard_ids"].shape[1]] = torch.from_numpy(np.maximum(g["hard_ids"], 0))
    hard_len = torch.from_numpy(g["hard_len"]).int()
    emb = torch.from_numpy(g["clap_emb"]).to(cuda)
    soft = pipe.mapper(emb)
    ops.prefill_embed(hard.to(cuda), hard_len.to(cuda), soft, pipe.mapper.soft_ld, 10,
                      pipe.gpt.wte, pipe.gpt.wpe, B, Pmax, pipe.embed[:B * Pmax], dec.x, dec.plen,
                      dec.last_row)
    dec.prefill(B, Pmax, row_stride=beam)
    ids, ln, sc = dec.beam(C, beam, Pmax)
    from zsaac.pipeline import CaptionBatch
    cb = CaptionBatch(ids, ln, sc, hard, hard_len, dec.plen[:B], None, emb)
    got = cb.beams()
    for c in range(C):
        ref = [g[f"beam{beam}_ids"][c, i, :g[f"beam{beam}_len"][c, i]].tolist() for i in range(beam)]
        assert got[c] == ref, c


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_mappers(cuda, golden, caption_sd, dtype):
    from zsaac.decoder import MlpMapper, TransformerMapperEngine
    g = golden("mappers.npz")
    x = torch.from_numpy(g["x"][:, 0]).to(cuda)
    m = MlpMapper(caption_sd, cuda, dtype, 3)
    t = TransformerMapperEngine(caption_sd, cuda, dtype, 3)
    ym = m(x).cpu().numpy().reshape(3, 1, -1)
    yt = t(x).cpu().numpy().reshape(3, 10, 768)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    assert _rel(ym, g["mlp_out"]) < tol
    assert _rel(yt, g["tmapper_out"]) < tol


@pytest.mark.parametrize("kind,fixture,width", [("htsat", "htsat.npz", 768), ("cnn14", "cnn14.npz", 2048)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_encoder_from_logmel(cuda, golden, kind, fixture, width, dtype):
    from zsaac import synthetic as S
    from zsaac.encoder import AudioEncoder
    from oracle import audio as A
    g = golden(fixture)
    sd = S.htsat_state_dict(3) if kind == "htsat" else S.cnn14_state_dict(4)
    sd.update(S.audio_proj_state_dict(5, audio_width=width))
    enc = AudioEncoder(sd, kind, dtype, max_batch=2, device=cuda)
    lm = torch.from_numpy(g["logmel"])               # [2,1,1001,64] (pre-bn0)
    bn = A.bn0(lm, {k: v for k, v in sd.items()})[:, 0]   # bn0 is fused into zs_logmel normally
    emb = enc.encode_logmel(bn.to(cuda)).cpu().numpy()
    feat = enc.feat[:2].cpu().numpy()
    key = "embedding768" if kind == "htsat" else "embedding2048"
    if dtype == torch.float32:
        assert _rel(feat, g[key]) < (2e-4 if kind == "htsat" else 5e-4)
        assert _rel(emb, g["clap_emb"]) < 5e-4
    else:
        cos = (emb * g["clap_emb"]).sum(-1) / np.linalg.norm(emb, axis=-1) / np.linalg.norm(g["clap_emb"], axis=-1)
        assert cos.min() > 0.995, cos


def test_pipeline_from_wav_f32_vs_oracle(cuda, caption_sd):
    """wav -> log-mel -> HTSAT -> proj -> prompt -> mapper -> greedy (f32) vs the oracle chain."""
    from oracle import audio as A, caption as OC, frontend as OF
    from zsaac import synthetic as S
    asd = S.htsat_state_dict(3)
    asd.update(S.audio_proj_state_dict(5))
    pipe = _pipeline(caption_sd, torch.float32, 2, audio_sd=asd, entry_length=20)
    wav = S.synthetic_waveforms(2)
    out = pipe.caption_wav(wav.to(cuda))
    with torch.no_grad():
        lm = OF.logmel(wav)
        emb = A.audio_project(A.htsat_embedding(lm, asd), asd)
    assert _rel(out.clap_emb.cpu().numpy(), emb.numpy()) < 2e-3
    table, lt = S.label_table(), S.label_token_table()
    caps = out.captions()
    for b in range(2):
        idx = OC.sound_effect_choice(out.clap_emb[b:b + 1].cpu(), table, 3)[0].tolist()
        hard = torch.tensor([OC.prompt_ids(idx, lt)])
        assert out.hard_ids[b, :hard.shape[1]].cpu().tolist() == hard[0].tolist()
        pe = OC.clap_to_gpt(torch.nn.functional.normalize(out.clap_emb[b:b + 1].cpu(), dim=-1)[None],
                            hard, caption_sd)
        ref = OC.generate2(pe, caption_sd, entry_length=20, use_cache=True)
        assert caps[b] == ref
