"""Generate the golden fixtures of tests/golden/*.npz by RUNNING THE REFERENCE (read-only, imported
from /root/reference through tests/golden/_refshim.py) on seeded synthetic weights and inputs.

The reference has no tests, fixtures or golden vectors of its own, so these
fixtures are the pin for oracle/ and for the HIP path.  Only arrays are written; no reference
source travels.  Weights come from zsaac.synthetic (seeded, regenerated identically by the tests),
so the fixtures hold inputs + outputs only.

    python tests/golden/make_goldens.py            # all fixtures (several minutes on 8 cores)
    python tests/golden/make_goldens.py htsat cnn14  # a subset

Fixture list (reference call sites in brackets):
  c1_greedy.npz   C1 harness: 50 CLAP embeddings -> ClapTestDataset_withHardPrompt.__getitem__ +
                  collate (dataset/dataset.py:441-453,632-647) -> clap_to_gpt
                  (models/caption_model.py:315-329) -> get_prefix_tokens + generate2
                  (gpt2_prefix_eval.py:161-222,271-278), as predict_prompt.py:129-148 drives them.
  beam.npz        generate_beam beam 5 and beam 3 (gpt2_prefix_eval.py:99-158).
  mappers.npz     MLP and TransformerMapper forward + clap_to_gpt (models/mapper.py, caption_model.py).
  htsat.npz       HTSAT forward from log-mel (retrieval/models/htsat.py:941-958) + ASE
                  audio_proj/normalize (ase_model.py:52-55).
  cnn14.npz       CNN14 forward from log-mel (cnns.py:171-201) + audio_proj/normalize.
  prompt.npz      compose_discrete_prompts strings + padding_captions (utils.py:158-208).
  variants.npz    ClapCaptionModel + sound-effect MLP, ClapCaptionCrossattention[_v2],
                  ClapCaptionPrefix: clap_to_gpt outputs and generate2 ids.
  c2_margin.npz   generate2 with the reference's top-1/top-2 logit margin at every generated
  c2_margin_flat.npz  step, on smaller decoder weights (the bf16 id-parity check);
  c2_gpt2init.npz     c2_gpt2init at GPT-2's own init scale.  "tolerance" adds to these and
                  c1_greedy the reference's own bf16-vs-f32 logit error (bf16_ref_err*).
  beam_tol.npz    the C3 bf16 beam tolerance: the reference's own bf16-vs-f32 first-step
                  log-prob error and best-beam score loss (generate_beam, gpt2_prefix_eval.py:
                  99-158) on the two weight sets of the C3 tests.
  mistral.npz     C5 Mistral decoder path: ClapCaption_Mistralai_prompt.clap_to_gpt
                  (caption_model.py:392-413) + LMmodel.generate(inputs_embeds, attention_mask=ones,
                  do_sample=False, max_length=60, eos/pad 2) as predict_mistralai_multilingual.py:
                  97-111 drive them, on a 2-layer / 1024-wide Mistral (head_dim 128, GQA 8/2).
  magic.npz       CLAP-guided decoding: ASE.encode_text on sample texts (text_encoder.py:58-68,
                  ase_model.py:57-60), generate_beam_magic (gpt2_prefix_eval.py:602-689) at two
                  (beam, width, alpha, beta) settings and magic_search (341-469), BERT text tower
                  at MAGIC_BERT_LAYERS layers.
"""
from __future__ import annotations

import os
import pickle
import sys
import tempfile
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "zero-shot-aac_amd"))
sys.path.insert(1, REPO)                 # oracle/ (prompt ids, pinned by tests/test_oracle.py)

import _refshim  # noqa: E402

_refshim.install()  # puts /root/reference first on sys.path

from zsaac import synthetic as S  # noqa: E402
from zsaac.tokenizer import IdTokenizer, TableTokenizer, synthetic_label_names  # noqa: E402

# the golden decoder weights (scaled-up init for non-degenerate argmax margins;
# stop_boost makes '.'/' .' fire within 67 steps for part of the clips)
GPT2_KW = dict(seed=0, std=0.1, emb_std=0.1, stop_boost=2.0)
SOUND_EFFECT_NUM = 3


def _save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1e3:.1f} kB)", flush=True)


def _pad(rows, fill=-1):
    n = max([len(r) for r in rows] + [1])
    out = np.full((len(rows), n), fill, dtype=np.int64)
    for i, r in enumerate(rows):
        out[i, :len(r)] = r
    return out, np.array([len(r) for r in rows], dtype=np.int64)


def _caption_model(mapping_type="mlp", stop_boost=None):
    from models.caption_model import ClapCaption_prompt
    kw = dict(GPT2_KW)
    if stop_boost is not None:
        kw["stop_boost"] = stop_boost
    sd = S.gpt2_state_dict(**kw)
    if mapping_type == "mlp":
        sd.update(S.mlp_mapper_state_dict(1))
    else:
        sd.update(S.transformer_mapper_state_dict(2))
    m = ClapCaption_prompt(10, clip_length=10, prefix_size=1024, num_layers=8,
                           mapping_type=mapping_type, only_prefix=False, only_soft_prompt=False)
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("attn.bias" in k or "masked_bias" in k for k in missing), missing
    return m.eval()


class _PrefixTok(IdTokenizer):
    """decode(token) -> 'id|' so get_prefix_tokens' "".join stays parseable."""

    def decode(self, ids):
        return super().decode(ids) + "|"


def gen_c1(n_clips=50, entry_length=67):
    import transformers
    import gpt2_prefix_eval as G
    names = synthetic_label_names()
    label_ids = S.label_token_table()
    tok = TableTokenizer.for_labels(names, label_ids)
    transformers.GPT2Tokenizer.from_pretrained = staticmethod(lambda *a, **k: tok)
    from dataset.dataset import ClapTestDataset_withHardPrompt, collate
    table = S.label_table()
    emb = S.synthetic_clap_embeddings(n_clips)
    tmp = tempfile.mkdtemp()
    data_p, lab_p = os.path.join(tmp, "data.pkl"), os.path.join(tmp, "labels.pkl")
    with open(data_p, "wb") as f:
        pickle.dump([{"audio_embedding": emb[i:i + 1].clone(), "audio_id": f"clip{i:04d}",
                      "caption": ["x"]} for i in range(n_clips)], f)
    with open(lab_p, "wb") as f:
        pickle.dump([{"label_id": i, "label": names[i], "label_embedding": table[i:i + 1].clone()}
                     for i in range(len(names))], f)
    ds = ClapTestDataset_withHardPrompt(data_p, normalize_prefix=True, sound_effect_path=lab_p,
                                        sound_effect_num=SOUND_EFFECT_NUM)
    model = _caption_model("mlp")
    embeddings = torch.nn.functional.normalize(model.gpt.get_input_embeddings().weight.data, 2, 1)
    hard_rows, greedy_rows, pref_rows, pe_keep, margin_rows = [], [], [], [], []
    t0 = time.time()
    for i in range(n_clips):
        audio_id, prefix, hard, mask = collate([ds[i]])
        prefix = prefix.to(dtype=torch.float32)
        with torch.no_grad():
            emb_h = model.gpt.transformer.wte(hard)
            pe, _ = model.clap_to_gpt(prefix, emb_h)
            ps = G.get_prefix_tokens(pe, embeddings, _PrefixTok())
            out = G.generate2(model, IdTokenizer(), embed=pe, entry_length=entry_length)
            ids = [int(t) for t in out.split()]
            margin_rows.append(_step_margins(model, pe, ids))
        hard_rows.append(hard[0].tolist())
        pref_rows.append([int(t) for t in ps[0].split("|") if t])
        greedy_rows.append(ids)
        if i < 4:
            pe_keep.append(pe[0].numpy())
        if i % 10 == 0:
            print(f"  c1 clip {i}: H={hard.shape[1]} gen={len(greedy_rows[-1])} "
                  f"({time.time() - t0:.0f}s)", flush=True)
    hard, hard_len = _pad(hard_rows)
    greedy, greedy_len = _pad(greedy_rows)
    pref, _ = _pad(pref_rows)
    pe_pad = np.zeros((len(pe_keep), max(p.shape[0] for p in pe_keep), 768), np.float32)
    for i, p in enumerate(pe_keep):
        pe_pad[i, :p.shape[0]] = p
    marg = np.zeros(greedy.shape, np.float32)
    for i, m in enumerate(margin_rows):
        marg[i, :len(m)] = m
    _save("c1_greedy.npz", clap_emb=emb.numpy(), hard_ids=hard, hard_len=hard_len,
          greedy_ids=greedy, greedy_len=greedy_len, prefix_tokens=pref,
          prefix_embed=pe_pad, entry_length=np.int64(entry_length),
          sound_effect_num=np.int64(SOUND_EFFECT_NUM), normalize_prefix=np.int64(1), margin=marg)


def _step_margins(model, pe, ids):
    """The reference's top-1 minus top-2 logit at every generated step: one teacher-forced
    forward of the reference GPT2LMHeadModel over prompt + generated ids (the computation
    generate2 repeats at every step, gpt2_prefix_eval.py:187-190); checks its argmax = ids."""
    seq = torch.cat([pe, model.gpt.transformer.wte(torch.tensor([ids[:-1]]))], 1) \
        if len(ids) > 1 else pe
    logits = model.gpt(inputs_embeds=seq).logits[0, pe.shape[1] - 1:]
    assert torch.equal(logits.argmax(-1), torch.tensor(ids)), "teacher forcing != generate2"
    top2 = logits.topk(2, -1).values
    return (top2[:, 0] - top2[:, 1]).tolist()


# bf16 id-parity goldens: block weights at std 0.05 give varied captions (10-20 distinct tokens
# per clip) with step margins from ~0.01 to ~4 (logit std ~3); at GPT-2's own init scale 0.02
# every caption collapses to one repeated token after a first step whose margin varies by clip
MARGIN_GPT2_KW = {"c2_margin": dict(seed=7, std=0.05, emb_std=0.1, stop_boost=2.0),
                  "c2_margin_flat": dict(seed=7, std=0.02, emb_std=0.1, stop_boost=2.0),
                  # GPT-2's own init scale everywhere (blocks and embeddings 0.02, positions
                  # 0.01): the regime of a trained model's small activations, where bf16 rounding
                  # stays far below the logit margins at most steps
                  "c2_gpt2init": dict(seed=11, std=0.02, emb_std=0.02, stop_boost=2.0)}


def gen_margin(n_clips=32, entry_length=67, name="c2_margin"):
    """c2_margin.npz / c2_margin_flat.npz: greedy goldens for the bf16 id-parity check, with the
    reference's top-1 / top-2 logit margin at every generated step (teacher-forced full-sequence
    forward of the reference GPT2LMHeadModel over the prompt + generated ids: the computation
    generate2 repeats every step, gpt2_prefix_eval.py:187-190).  Decoder block weights at a
    smaller scale than the chaotic std-0.1 goldens (MARGIN_GPT2_KW).  Hard prompts as C1
    (dataset.py:441-453)."""
    import gpt2_prefix_eval as G
    from models.caption_model import ClapCaption_prompt
    kw = MARGIN_GPT2_KW[name]
    sd = S.gpt2_state_dict(**kw)
    sd.update(S.mlp_mapper_state_dict(1))
    model = ClapCaption_prompt(10, clip_length=10, prefix_size=1024, num_layers=8,
                               mapping_type="mlp", only_prefix=False, only_soft_prompt=False)
    model.load_state_dict(sd, strict=False)
    model.eval()
    from oracle import caption as OC     # prompt ids exactly as dataset.py builds them (pinned)
    table, label_ids = S.label_table(), S.label_token_table()
    emb = S.synthetic_clap_embeddings(n_clips, seed=4242)
    hard_rows, greedy_rows, margin_rows, std_rows = [], [], [], []
    t0 = time.time()
    for i in range(n_clips):
        e = torch.nn.functional.normalize(emb[i:i + 1], dim=-1)
        idx = OC.sound_effect_choice(emb[i:i + 1], table, SOUND_EFFECT_NUM)[0].tolist()
        hard = torch.tensor([OC.prompt_ids(idx, label_ids)])
        with torch.no_grad():
            pe, _ = model.clap_to_gpt(e.unsqueeze(0), model.gpt.transformer.wte(hard))
            out = G.generate2(model, IdTokenizer(), embed=pe, entry_length=entry_length)
            ids = [int(t) for t in out.split()]
            seq = torch.cat([pe, model.gpt.transformer.wte(torch.tensor([ids[:-1]]))], 1) \
                if len(ids) > 1 else pe
            logits = model.gpt(inputs_embeds=seq).logits[0, pe.shape[1] - 1:]
        hard_rows.append(hard[0].tolist())
        greedy_rows.append(ids)
        margin_rows.append(_step_margins(model, pe, ids))
        std_rows.append(logits.std(-1).tolist())
        if i % 8 == 0:
            print(f"  margin clip {i}: gen={len(ids)} min margin {min(margin_rows[-1]):.3g} "
                  f"logit std {std_rows[-1][0]:.3g} ({time.time() - t0:.0f}s)", flush=True)
    hard, hard_len = _pad(hard_rows)
    greedy, greedy_len = _pad(greedy_rows)
    marg = np.zeros(greedy.shape, np.float32)
    lstd = np.zeros(greedy.shape, np.float32)
    for i, (m, s) in enumerate(zip(margin_rows, std_rows)):
        marg[i, :len(m)] = m
        lstd[i, :len(s)] = s
    _save(name + ".npz", clap_emb=emb.numpy(), hard_ids=hard, hard_len=hard_len,
          greedy_ids=greedy, greedy_len=greedy_len, margin=marg, logit_std=lstd,
          entry_length=np.int64(entry_length), gpt2_kw=np.array(
              [kw["seed"], kw["std"], kw["emb_std"], kw["stop_boost"]], np.float64))


def gen_tolerance(names=("c1_greedy", "c2_margin", "c2_margin_flat", "c2_gpt2init")):
    """The stated bf16 tolerance of each margin golden: the reference's OWN bf16 execution
    (the same GPT2LMHeadModel cast to bfloat16, torch on the CPU) against its f32 execution,
    teacher-forced over every golden clip's prompt + generated ids (the computation generate2
    repeats each step, gpt2_prefix_eval.py:187-190).  Adds to the existing fixture (ids and
    margins unchanged):
      bf16_ref_err        max |logit_bf16 - logit_f32| of the first generated step over the clips
      bf16_ref_err_steps  [B, L] the same per generated step
    tests/test_gpu_idparity.py derives its fixed margin threshold from bf16_ref_err and asserts
    the GPU's bf16 first-step error against it."""
    import copy
    from models.caption_model import ClapCaption_prompt
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import idparity
    for name in names:
        path = os.path.join(HERE, name + ".npz")
        g = dict(np.load(path))
        sd = S.gpt2_state_dict(**idparity.golden_gpt2_kw(g))
        sd.update(S.mlp_mapper_state_dict(1))
        model = ClapCaption_prompt(10, clip_length=10, prefix_size=1024, num_layers=8,
                                   mapping_type="mlp", only_prefix=False, only_soft_prompt=False)
        model.load_state_dict(sd, strict=False)
        model.eval()
        m16 = copy.deepcopy(model.gpt).to(torch.bfloat16).eval()
        emb = torch.from_numpy(g["clap_emb"])
        B = emb.shape[0]
        steps = np.zeros(g["greedy_ids"].shape, np.float32)
        t0 = time.time()
        for b in range(B):
            e = torch.nn.functional.normalize(emb[b:b + 1], dim=-1)
            hard = torch.from_numpy(g["hard_ids"][b, :g["hard_len"][b]]).long()[None]
            ids = g["greedy_ids"][b, :g["greedy_len"][b]].tolist()
            with torch.no_grad():
                pe, _ = model.clap_to_gpt(e.unsqueeze(0), model.gpt.transformer.wte(hard))
                seq = torch.cat([pe, model.gpt.transformer.wte(torch.tensor([ids[:-1]]))], 1) \
                    if len(ids) > 1 else pe
                l32 = model.gpt(inputs_embeds=seq).logits[0, pe.shape[1] - 1:]
                assert torch.equal(l32.argmax(-1), torch.tensor(ids)), f"{name} clip {b}"
                l16 = m16(inputs_embeds=seq.to(torch.bfloat16)).logits[0, pe.shape[1] - 1:].float()
            steps[b, :len(ids)] = (l16 - l32).abs().max(-1).values.numpy()
        g["bf16_ref_err_steps"] = steps
        g["bf16_ref_err"] = np.float32(steps[:, 0].max())
        _save(name + ".npz", **g)
        print(f"  {name}: bf16 reference error first step {float(g['bf16_ref_err']):.4f}, all steps "
              f"max {float(steps.max()):.4f} ({time.time() - t0:.0f}s)", flush=True)


# C3 beam-search tolerance: the weight sets of tests/test_gpu_configs.py's beam checks
BEAM_TOL_SETS = {"std01": (dict(GPT2_KW), 31), "gpt2init": (MARGIN_GPT2_KW["c2_gpt2init"], 37)}


def gen_beam_tolerance(n_clips=4, beam=5, entry_length=67):
    """beam_tol.npz: the stated tolerance of the C3 bf16 beam score rule, from the REFERENCE's
    own bf16 execution.  For each weight set (BEAM_TOL_SETS: decoder weights, CLAP-embedding seed
    of the test) and each of the first n_clips clips (hard prompt as dataset.py:441-453):
      {set}_first_err   max |log_softmax(logits_bf16) - log_softmax(logits_f32)| of the first
                        generated step, the reference's GPT2LMHeadModel cast to bfloat16 (torch
                        CPU) against its f32 run, softmax taken exactly on both logit sets;
      {set}_score_loss  f32 length-normalised score (gpt2_prefix_eval.py:150-156) of the best beam
                        of the reference's generate_beam run in bf16, minus that of its f32 run's
                        best beam (teacher-forced f32 rescoring): what bf16 costs the reference;
      {set}_tau_b       4 x max first_err: the beam score rule's bound (tests/test_gpu_configs.py:
                        an exact maximiser of the bf16 score ends within 2 e, beam search is not
                        exact, hence twice that)."""
    import copy
    import gpt2_prefix_eval as G
    from models.caption_model import ClapCaption_prompt
    from oracle import caption as OC

    class _Gpt(torch.nn.Module):        # generate_beam only touches model.gpt
        def __init__(self, gpt):
            super().__init__()
            self.gpt = gpt

    def score(model, pe, toks):
        wte = model.gpt.transformer.wte
        seq = torch.cat([pe, wte(torch.tensor([toks[:-1]]))], 1) if len(toks) > 1 else pe
        lp = model.gpt(inputs_embeds=seq).logits[0, pe.shape[1] - 1:].log_softmax(-1)
        return float(lp[torch.arange(len(toks)), torch.tensor(toks)].mean())

    table, label_ids = S.label_table(), S.label_token_table()
    out = {}
    for name, (kw, seed) in BEAM_TOL_SETS.items():
        sd = S.gpt2_state_dict(**kw)
        sd.update(S.mlp_mapper_state_dict(1))
        model = ClapCaption_prompt(10, clip_length=10, prefix_size=1024, num_layers=8,
                                   mapping_type="mlp", only_prefix=False, only_soft_prompt=False)
        model.load_state_dict(sd, strict=False)
        model.eval()
        m16 = _Gpt(copy.deepcopy(model.gpt).to(torch.bfloat16)).eval()
        emb = S.synthetic_clap_embeddings(n_clips, seed=seed)
        first, loss = [], []
        t0 = time.time()
        for i in range(n_clips):
            e = torch.nn.functional.normalize(emb[i:i + 1], dim=-1)
            idx = OC.sound_effect_choice(emb[i:i + 1], table, SOUND_EFFECT_NUM)[0].tolist()
            hard = torch.tensor([OC.prompt_ids(idx, label_ids)])
            with torch.no_grad():
                pe, _ = model.clap_to_gpt(e.unsqueeze(0), model.gpt.transformer.wte(hard))
                l32 = model.gpt(inputs_embeds=pe).logits[0, -1]
                l16 = m16.gpt(inputs_embeds=pe.to(torch.bfloat16)).logits[0, -1].float()
                first.append(float((l16.log_softmax(-1) - l32.log_softmax(-1)).abs().max()))
                t32 = G.generate_beam(model, IdTokenizer(), beam_size=beam, embed=pe,
                                      entry_length=entry_length)
                t16 = G.generate_beam(m16, IdTokenizer(), beam_size=beam,
                                      embed=pe.to(torch.bfloat16), entry_length=entry_length)
                b32 = [int(t) for t in t32[0].split()]
                b16 = [int(t) for t in t16[0].split()]
                loss.append(score(model, pe, b16) - score(model, pe, b32))
            print(f"  {name} clip {i}: first err {first[-1]:.4f} score loss {loss[-1]:.4f} "
                  f"exact {b16 == b32} ({time.time() - t0:.0f}s)", flush=True)
        out[f"{name}_clap_emb"] = emb.numpy()
        out[f"{name}_first_err"] = np.array(first, np.float32)
        out[f"{name}_score_loss"] = np.array(loss, np.float32)
        out[f"{name}_tau_b"] = np.float32(4.0 * max(first))
    _save("beam_tol.npz", **out)


VARIANTS = ("se_mlp", "xattn", "xattn_v2", "prefix")


def gen_variants(n_clips=3, entry_length=30):
    """variants.npz: the other caption-model classes of models/caption_model.py on the same
    decoder weights: ClapCaptionModel with sound_effect_embeddings (sound-effect MLP tokens,
    lines 15-21, 63-82), ClapCaptionCrossattention (100-149), ClapCaptionCrossattention_v2 at
    eval (151-206) and ClapCaptionPrefix (90-98): clap_to_gpt outputs for a prefix + text tokens,
    and generate2 ids (gpt2_prefix_eval.py:161-222) on each clip's clap_to_gpt(prefix)."""
    import gpt2_prefix_eval as G
    from models import caption_model as CM
    table = S.label_table()
    emb = torch.nn.functional.normalize(S.synthetic_clap_embeddings(n_clips, seed=77), dim=-1)
    prefix = emb.unsqueeze(1)                                      # [n, 1, 1024]
    tokens = torch.tensor([[1858, 389, 1223, 287, 428, 6597]] * n_clips)
    out = {"prefix": prefix.numpy(), "tokens": tokens.numpy(), "table_seed": np.int64(6),
           "sound_effect_num": np.int64(SOUND_EFFECT_NUM), "entry_length": np.int64(entry_length)}
    for name in VARIANTS:
        sd = S.gpt2_state_dict(**GPT2_KW)
        sd.update(S.mlp_mapper_state_dict(1))
        kw = dict(prefix_size=1024, mapping_type="mlp")
        if name == "se_mlp":
            m = CM.ClapCaptionModel(10, sound_effect_embeddings=table,
                                    sound_effect_num=SOUND_EFFECT_NUM, **kw)
            sd.update(S.sound_effect_mlp_state_dict(11))
        elif name == "prefix":
            m = CM.ClapCaptionPrefix(10, **kw)
        else:
            cls = CM.ClapCaptionCrossattention if name == "xattn" else CM.ClapCaptionCrossattention_v2
            m = cls(10, sound_effect_embeddings=table, sound_effect_num=SOUND_EFFECT_NUM, **kw)
            sd.update(S.sound_effect_mha_state_dict(12))
        missing, unexpected = m.load_state_dict(sd, strict=False)
        assert not unexpected, unexpected
        assert all("attn.bias" in k or "masked_bias" in k for k in missing), missing
        m.eval()
        with torch.no_grad():
            cat, _ = m.clap_to_gpt(prefix, m.gpt.transformer.wte(tokens))
            ids = []
            for i in range(n_clips):
                pe, _ = m.clap_to_gpt(prefix[i:i + 1])
                ids.append([int(t) for t in G.generate2(m, IdTokenizer(), embed=pe,
                                                        entry_length=entry_length).split()])
        g_ids, g_len = _pad(ids)
        out[f"{name}_cat"] = cat.numpy()
        out[f"{name}_ids"], out[f"{name}_len"] = g_ids, g_len
        print(f"  {name}: clap_to_gpt {tuple(cat.shape)}, greedy lengths {g_len.tolist()}", flush=True)
    _save("variants.npz", **out)


def gen_beam(n_clips=4, entry_length=67):
    import gpt2_prefix_eval as G
    model = _caption_model("mlp")
    emb = S.synthetic_clap_embeddings(n_clips, seed=99)
    label_ids = S.label_token_table()
    out = {}
    hard_rows = []
    for i in range(n_clips):
        # fixed hard prompt: "There are <label i>, <label 2i+1> in this audio."
        hard_rows.append([1858, 389] + label_ids[i] + [11] + label_ids[2 * i + 1] + [287, 428, 6597, 13])
    hard, hard_len = _pad(hard_rows)
    for beam in (5, 3):
        rows = []
        for i in range(n_clips):
            h = torch.tensor([hard_rows[i]])
            with torch.no_grad():
                pe, _ = model.clap_to_gpt(emb[i:i + 1].unsqueeze(0), model.gpt.transformer.wte(h))
                texts = G.generate_beam(model, IdTokenizer(), beam_size=beam, embed=pe,
                                        entry_length=entry_length)
            rows.append([[int(t) for t in s.split()] for s in texts])
            print(f"  beam{beam} clip {i}: lens {[len(r) for r in rows[-1]]}", flush=True)
        flat = [r for clip in rows for r in clip]
        ids, lens = _pad(flat)
        out[f"beam{beam}_ids"] = ids.reshape(n_clips, beam, -1)
        out[f"beam{beam}_len"] = lens.reshape(n_clips, beam)
    _save("beam.npz", clap_emb=emb.numpy(), hard_ids=hard, hard_len=hard_len,
          entry_length=np.int64(entry_length), **out)


def gen_temperature(n_clips=4, entry_length=24):
    """generate_beam (beam 3, temperature 0.7 and 1.6) and generate2 (temperature 0.7) on the
    beam.npz clips: the reference divides the logits by temperature before softmax().log()
    (gpt2_prefix_eval.py:121-122) / the top-p sort (196)."""
    import gpt2_prefix_eval as G
    model = _caption_model("mlp")
    emb = S.synthetic_clap_embeddings(n_clips, seed=99)
    label_ids = S.label_token_table()
    hard_rows = [[1858, 389] + label_ids[i] + [11] + label_ids[2 * i + 1] + [287, 428, 6597, 13]
                 for i in range(n_clips)]
    hard, hard_len = _pad(hard_rows)
    out = {}
    for tag, T in (("t07", 0.7), ("t16", 1.6)):
        rows = []
        for i in range(n_clips):
            h = torch.tensor([hard_rows[i]])
            with torch.no_grad():
                pe, _ = model.clap_to_gpt(emb[i:i + 1].unsqueeze(0), model.gpt.transformer.wte(h))
                texts = G.generate_beam(model, IdTokenizer(), beam_size=3, embed=pe,
                                        entry_length=entry_length, temperature=T)
            rows.append([[int(t) for t in s.split()] for s in texts])
        ids, lens = _pad([r for clip in rows for r in clip])
        out[f"beam3_{tag}_ids"] = ids.reshape(n_clips, 3, -1)
        out[f"beam3_{tag}_len"] = lens.reshape(n_clips, 3)
        print(f"  beam3 T={T}: lens {lens.tolist()}", flush=True)
    g = []
    for i in range(n_clips):
        h = torch.tensor([hard_rows[i]])
        with torch.no_grad():
            pe, _ = model.clap_to_gpt(emb[i:i + 1].unsqueeze(0), model.gpt.transformer.wte(h))
            g.append([int(t) for t in G.generate2(model, IdTokenizer(), embed=pe,
                                                  entry_length=entry_length, temperature=0.7).split()])
    gi, gl = _pad(g)
    _save("temperature.npz", clap_emb=emb.numpy(), hard_ids=hard, hard_len=hard_len,
          entry_length=np.int64(entry_length), greedy_t07_ids=gi, greedy_t07_len=gl, **out)


def gen_mappers():
    from models.mapper import MLP, TransformerMapper
    x = S.synthetic_clap_embeddings(3, seed=11).unsqueeze(1)  # [3,1,1024] as in make_preds
    mlp = MLP((1024, 3840, 7680))
    mlp.load_state_dict({k.replace("clap_project.", ""): v for k, v in S.mlp_mapper_state_dict(1).items()})
    tm = TransformerMapper(1024, 768, 10, 10, 8)
    tm.load_state_dict({k.replace("clap_project.", ""): v
                        for k, v in S.transformer_mapper_state_dict(2).items()})
    with torch.no_grad():
        y_mlp = mlp.eval()(x)
        y_tm = tm.eval()(x)
        model = _caption_model("transformer")
        h = torch.tensor([[1858, 389, 1223, 287, 428, 6597, 13]])
        pe_tm, _ = model.clap_to_gpt(x[:1], model.gpt.transformer.wte(h))
    _save("mappers.npz", x=x.numpy(), mlp_out=y_mlp.numpy(), tmapper_out=y_tm.numpy(),
          tm_hard_ids=h.numpy(), tm_prefix_embed=pe_tm[0].numpy())


def _audio_config(kind):
    return {"audio_args": {"sr": 32000, "n_fft": 1024, "hop_length": 320, "f_min": 50,
                           "f_max": 14000, "n_mels": 64, "max_length": 10, "mono": True},
            "audio_encoder_args": {"type": kind, "model": "Cnn14", "pretrained": False,
                                   "freeze": False},
            "training": {"spec_augmentation": True, "dropout": 0.2}}


def _logmel_input(n, seed):
    g = torch.Generator().manual_seed(seed)
    # log-mel-like magnitudes (dB), [B,1,T=1001,F=64]: what AudioFeature hands to bn0
    return torch.randn(n, 1, 1001, 64, generator=g) * 8.0 - 20.0


def _encode(kind, audio_sd, width):
    from retrieval.models.audio_encoder import AudioEncoder
    enc = AudioEncoder(_audio_config(kind))
    missing, unexpected = enc.load_state_dict(
        {k.replace("audio_encoder.", ""): v for k, v in audio_sd.items()}, strict=False)
    assert not unexpected, unexpected
    proj = torch.nn.Sequential(torch.nn.Linear(width, 1024), torch.nn.ReLU(), torch.nn.Linear(1024, 1024))
    proj.load_state_dict({k.replace("audio_proj.", ""): v
                          for k, v in S.audio_proj_state_dict(5, audio_width=width).items()})
    return enc.eval(), proj.eval(), missing


def gen_htsat():
    enc, proj, missing = _encode("transformer", S.htsat_state_dict(3), 768)
    assert all(("relative_position_index" in k) or ("attn_mask" in k) for k in missing), missing
    x = _logmel_input(2, 21)
    with torch.no_grad():
        feat = enc(x)
        emb = torch.nn.functional.normalize(proj(feat), dim=-1)  # ASE.encode_audio, ase_model.py:52-55
    _save("htsat.npz", logmel=x.numpy(), embedding768=feat.numpy(), clap_emb=emb.numpy())


def gen_cnn14():
    enc, proj, missing = _encode("cnn", S.cnn14_state_dict(4), 2048)
    assert not missing, missing
    x = _logmel_input(2, 22)
    with torch.no_grad():
        feat = enc(x)
        emb = torch.nn.functional.normalize(proj(feat), dim=-1)
    _save("cnn14.npz", logmel=x.numpy(), embedding2048=feat.numpy(), clap_emb=emb.numpy())


def gen_prompt():
    import utils as U

    class CharTok:
        def encode(self, s):
            return [ord(c) for c in s]
    names = synthetic_label_names()
    sets = [[], [names[0]], [names[5], names[77]], [names[1], names[2], names[3], names[526]]]
    strings = ["".join(chr(c) for c in U.parse_entities(CharTok(), s, 0).tolist()) for s in sets]
    hp = [torch.tensor([5, 6, 7]), torch.tensor([1]), torch.tensor([9, 8, 7, 6, 5])]
    padded, mask = U.padding_captions(hp, [3, 1, 5])
    enc = np.array([s.encode() for s in strings], dtype=object)
    _save("prompt.npz", strings=np.array(strings), n_labels=np.array([len(s) for s in sets]),
          pad_ids=padded.numpy(), pad_mask=mask.numpy())
    del enc


def gen_keys():
    """Reference state-dict key -> shape maps of the modules the drop-ins mirror."""
    import json
    from models.caption_model import ClapCaption_prompt
    from retrieval.models.audio_encoder import AudioEncoder
    out = {}
    for mt in ("mlp", "transformer"):
        m = ClapCaption_prompt(10, clip_length=10, prefix_size=1024, num_layers=8, mapping_type=mt)
        out[f"ClapCaption_prompt[{mt}]"] = {k: list(v.shape) for k, v in m.state_dict().items()}
    for kind in ("transformer", "cnn"):
        enc = AudioEncoder(_audio_config(kind))
        out[f"AudioEncoder[{kind}]"] = {k: list(v.shape) for k, v in enc.state_dict().items()}
    path = os.path.join(HERE, "state_dict_keys.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote", path)



MAGIC_BERT_LAYERS = 2
# beam, width, alpha, beta, entry_length, GPT-2 stop_boost (3.0: some beams stop on '.')
MAGIC_CFGS = ((3, 25, 0.1, 0.2, 12, 2.0), (2, 8, 0.3, 1.0, 10, 2.0), (3, 25, 0.1, 0.2, 16, 3.0))


def _clap_ase(layers):
    """The reference ASE (audio + text towers) with the synthetic BERT loaded (text side)."""
    _refshim.install_bert(S.bert_vocab(), layers)
    from retrieval.models.ase_model import ASE
    cfg = _audio_config("transformer")
    cfg.update({"embed_size": 1024, "temp": 0.07, "embed_regularization": True,
                "text_encoder_args": {"type": "bert-base-uncased", "freeze": False}})
    clap = ASE(cfg)
    missing, unexpected = clap.load_state_dict(S.bert_state_dict(layers=layers), strict=False)
    assert not unexpected, unexpected
    assert all(m.startswith("audio") or "position_ids" in m for m in missing), missing
    return clap.eval()


def gen_magic(n_clips=3):
    import gpt2_prefix_eval as G
    from zsaac.tokenizer import WordTokenizer
    L = MAGIC_BERT_LAYERS
    clap = _clap_ase(L)
    tok = WordTokenizer()
    texts = [tok.decode(t) for t in ([5, 123, 13], [7], [1000, 2005, 3, 11, 764, 49999, 50000],
                                     list(range(100, 140)), [30000, 30001, 30010])]
    with torch.no_grad():
        text_emb = clap.encode_text(texts)
        bt = clap.text_encoder.tokenizer(texts, padding="longest", truncation=True, max_length=30)
    models = {}
    for boost in sorted({c[5] for c in MAGIC_CFGS}):
        models[boost] = _caption_model("mlp", stop_boost=boost)
        _refshim.legacy_cache(models[boost].gpt)
    model = models[2.0]
    emb = S.synthetic_clap_embeddings(n_clips, seed=77)
    label_ids = S.label_token_table()
    hard_rows = [[1858, 389] + label_ids[3 * i] + [287, 428, 6597, 13] for i in range(n_clips)]
    hard, hard_len = _pad(hard_rows)
    out = {}
    for c, (beam, width, alpha, beta, entry, boost) in enumerate(MAGIC_CFGS):
        model = models[boost]
        rows = []
        for i in range(n_clips):
            with torch.no_grad():
                pe, _ = model.clap_to_gpt(emb[i:i + 1].unsqueeze(0),
                                          model.gpt.transformer.wte(torch.tensor([hard_rows[i]])))
                res = G.generate_beam_magic(model, clap, tok, audio_embeds=emb[i:i + 1], embed=pe,
                                            beam_size=beam, entry_length=entry, magic_width=width,
                                            alpha=alpha, beta=beta)
            rows.append([WordTokenizer.parse(t) for t in res])
            print(f"  magic cfg{c} clip {i}: {[len(r) for r in rows[-1]]}", flush=True)
        ids, lens = _pad([r for clip in rows for r in clip])
        out[f"beam_cfg{c}_ids"] = ids.reshape(n_clips, beam, -1)
        out[f"beam_cfg{c}_len"] = lens.reshape(n_clips, beam)
    model = models[2.0]
    search = []
    for i in range(n_clips):
        with torch.no_grad():
            pe, _ = model.clap_to_gpt(emb[i:i + 1].unsqueeze(0),
                                      model.gpt.transformer.wte(torch.tensor([hard_rows[i]])))
            t = G.magic_search(model, tok, emb[i:i + 1], clap, embed=pe, beam_width=15,
                               decoding_len=pe.shape[1] + 10)
        search.append(WordTokenizer.parse(t))
    s_ids, s_len = _pad(search)
    _save("magic.npz", clap_emb=emb.numpy(), hard_ids=hard, hard_len=hard_len,
          bert_layers=np.int64(L), cfgs=np.array(MAGIC_CFGS, dtype=np.float64),
          text_ids=_pad(bt["input_ids"])[0], text_emb=text_emb.numpy(),
          search_ids=s_ids, search_len=s_len, **out)


MISTRAL_CFG = dict(vocab_size=32000, hidden_size=1024, intermediate_size=3072,
                   num_hidden_layers=2, num_attention_heads=8, num_key_value_heads=2,
                   rms_norm_eps=1e-5, rope_theta=10000.0, tie_word_embeddings=False,
                   max_position_embeddings=4096, sliding_window=4096)
MISTRAL_TAGS = {"en": [1, 523, 269, 28767], "zh": [1, 523, 26715, 28767], "fr": [1, 523, 1642, 28767]}


def gen_mistral(n_clips=6):
    """One batch of ``n_clips`` through the reference's Mistral caption path, two languages."""
    _refshim.install_mistral(MISTRAL_CFG)
    from models.caption_model import ClapCaption_Mistralai_prompt
    from zsaac import synthetic as SS
    m = ClapCaption_Mistralai_prompt(10, clip_length=10, prefix_size=1024, num_layers=8,
                                     mapping_type="mlp")
    lm_sd = SS.mistral_state_dict()
    m.LMmodel.base_model.model.load_state_dict(lm_sd)
    D = MISTRAL_CFG["hidden_size"]
    mlp = SS.mlp_mapper_state_dict(31, prefix_length=10, d=D)
    missing, unexpected = m.clap_project.load_state_dict(
        {k.replace("clap_project.", ""): v for k, v in mlp.items()})
    m.eval()
    emb = S.synthetic_clap_embeddings(n_clips, seed=55).unsqueeze(1)     # [B, 1, 1024] (collate)
    g = torch.Generator().manual_seed(56)
    lens = [int(x) for x in torch.randint(5, 12, (n_clips,), generator=g)]
    H = max(lens)
    hard = torch.zeros(n_clips, H, dtype=torch.long)                   # padding_captions: pad 0
    for b, n in enumerate(lens):
        hard[b, :n] = torch.randint(3, 32000, (n,), generator=g)
    out = {}
    with torch.no_grad():
        eh = m.LMmodel.base_model.model.model.embed_tokens(hard)
        for tag in ("en", "fr"):
            tk = torch.tensor([MISTRAL_TAGS[tag]]).repeat(n_clips, 1)
            et = m.LMmodel.base_model.model.model.embed_tokens(tk)
            pe, _ = m.clap_to_gpt(emb, eh, et)
            am = torch.ones(pe.shape[:-1]).long()
            ids = m.LMmodel.generate(inputs_embeds=pe, attention_mask=am, do_sample=False,
                                     max_length=60, eos_token_id=2, pad_token_id=2)
            out[f"ids_{tag}"] = ids.numpy()
            print(f"  mistral {tag}: P={pe.shape[1]} out {tuple(ids.shape)} "
                  f"eos rows {int((ids == 2).any(1).sum())}", flush=True)
    _save("mistral.npz", clap_emb=emb[:, 0].numpy(), hard_ids=hard.numpy(),
          hard_len=np.array(lens), tag_en=np.array(MISTRAL_TAGS["en"]),
          tag_fr=np.array(MISTRAL_TAGS["fr"]), **out)


ALL = {"prompt": gen_prompt, "mappers": gen_mappers, "htsat": gen_htsat, "cnn14": gen_cnn14,
       "beam": gen_beam, "c1": gen_c1, "keys": gen_keys,
       "margin": gen_margin, "margin_flat": lambda: gen_margin(name="c2_margin_flat"),
       "gpt2init": lambda: gen_margin(name="c2_gpt2init"), "tolerance": gen_tolerance,
       "variants": gen_variants, "magic": gen_magic, "temperature": gen_temperature,
       "beam_tol": gen_beam_tolerance,
       "mistral": gen_mistral}

if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count() or 8)
    torch.manual_seed(0)
    for name in (sys.argv[1:] or list(ALL)):
        t = time.time()
        print(f"[{name}]", flush=True)
        ALL[name]()
        print(f"[{name}] done in {time.time() - t:.1f}s", flush=True)

