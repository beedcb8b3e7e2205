#!/usr/bin/env python3
"""Greedy token-id agreement of the HIP caption path with the reference's goldens (bf16 perf mode
and f32 parity mode), with the reference's own top-1/top-2 logit margin at every divergence.

The goldens (tests/golden/*.npz, made by tests/golden/make_goldens.py by running the reference
on seeded weights) hold CLAP embeddings, the reference's greedy ids and, for c1_greedy /
c2_margin / c2_margin_flat, the reference's logit margin at every generated step.  Used by
bench.py (``id_agreement`` in the JSON line) and tests/test_gpu_idparity.py (assertions).

    python tools/idparity.py [bf16|f32]
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

# decoder weights each golden was generated with (make_goldens.py GPT2_KW / MARGIN_GPT2_KW)
C1_GPT2_KW = dict(seed=0, std=0.1, emb_std=0.1, stop_boost=2.0)


def golden_gpt2_kw(g) -> dict:
    if "gpt2_kw" in g:
        s, std, es, sb = (float(v) for v in g["gpt2_kw"])
        return dict(seed=int(s), std=std, emb_std=es, stop_boost=sb)
    return dict(C1_GPT2_KW)


def run_greedy(g, dtype, device):
    """The batched pipeline (prompt assembly -> MLP mapper -> prefill -> greedy) on the golden's
    CLAP embeddings; returns (ids list per clip, hard ids list per clip)."""
    import torch
    n = g["clap_emb"].shape[0]
    pipe = _pipeline(g, dtype, device)
    out = pipe.caption_emb(torch.from_numpy(g["clap_emb"]).to(device))
    hard = out.hard_ids.cpu().numpy()
    hl = out.hard_len.cpu().numpy()
    return out.captions(), [hard[b, :hl[b]].tolist() for b in range(n)]


def _pipeline(g, dtype, device):
    import torch
    from zsaac import synthetic as S
    from zsaac.pipeline import CaptionConfig, CaptionPipeline
    csd = S.gpt2_state_dict(**golden_gpt2_kw(g))
    csd.update(S.mlp_mapper_state_dict(1))
    cfg = CaptionConfig(dtype=dtype, batch=g["clap_emb"].shape[0], entry_length=int(g["entry_length"]))
    return CaptionPipeline(csd, None, S.label_table(), S.label_token_table(), cfg, device=device)


def first_step_logits(pipe, emb):
    """Logits of the first generated token after the pipeline's prompt assembly, mapper and
    prefill: ln_f of each row's last prompt position @ wte^T (f32 on the host)."""
    from zsaac import ops
    B, cfg, dec = emb.shape[0], pipe.cfg, pipe.decoder
    ops.prompt_assemble(emb, pipe.labels, cfg.sound_effect_num, pipe.label_tok, pipe.label_len,
                        pipe.hard_ids[:B], pipe.hard_len[:B])
    soft = pipe.mapper(ops.l2norm(emb, out=pipe.prefix[:B]))
    ops.prefill_embed(pipe.hard_ids[:B], pipe.hard_len[:B], soft, pipe.mapper.soft_ld, 10,
                      pipe.gpt.wte, pipe.gpt.wpe, B, pipe.Pmax, pipe.embed[:B * pipe.Pmax], dec.x,
                      dec.plen, dec.last_row)
    dec.prefill(B, pipe.Pmax)
    return (dec.hf[:B].float() @ pipe.gpt.wte.float().t()).cpu()


def bf16_logit_error(g, device) -> float:
    """max |bf16 - f32| of the first-step logits over the golden's clips (the f32 path is
    bit-exact to the reference's ids; its logits are within ~1e-5 of the reference's)."""
    import torch
    emb = torch.from_numpy(g["clap_emb"]).to(device)
    l16 = first_step_logits(_pipeline(g, torch.bfloat16, device), emb)
    l32 = first_step_logits(_pipeline(g, torch.float32, device), emb)
    return float((l16 - l32).abs().max())


def agreement(g, caps, hards=None) -> dict:
    """Per-clip first divergence from the golden ids (None = identical sequence) and the
    reference's margin there."""
    ref_ids, ref_len = g["greedy_ids"], g["greedy_len"]
    margin = g["margin"] if "margin" in g else None
    n = len(caps)
    first, marg, agree_tok, total_tok = [], [], 0, 0
    for b in range(n):
        ref = ref_ids[b, :ref_len[b]].tolist()
        got = caps[b]
        d = next((i for i in range(max(len(ref), len(got)))
                  if i >= len(ref) or i >= len(got) or ref[i] != got[i]), None)
        total_tok += len(ref)
        agree_tok += len(ref) if d is None else min(d, len(ref))
        first.append(d)
        if d is not None and margin is not None and d < len(ref):
            marg.append(float(margin[b, d]))
    div = [d for d in first if d is not None]
    res = {"clips": n, "exact_frac": round(1.0 - len(div) / max(n, 1), 4),
           "token_agree_frac": round(agree_tok / max(total_tok, 1), 4),
           "first_divergence_mean": round(float(np.mean(div)), 2) if div else None,
           "oracle_margin_at_divergence_median": round(float(np.median(marg)), 4) if marg else None,
           "oracle_margin_at_divergence_max": round(float(np.max(marg)), 4) if marg else None,
           "first_divergence": first}
    if hards is not None:
        hl = g["hard_len"]
        res["hard_prompt_exact_frac"] = round(float(np.mean(
            [hards[b] == g["hard_ids"][b, :hl[b]].tolist() for b in range(n)])), 4)
    if margin is not None:
        # clips whose reference margins stay above tau at every step up to the end
        res["min_margin_per_clip"] = [round(float(margin[b, :ref_len[b]].min()), 4)
                                      for b in range(n)]
    return res


# the bf16 id-parity rule (tests/test_gpu_idparity.py, bench.py id_agreement): a bf16 divergence
# from the reference's ids may only start at a step whose reference top-1 / top-2 margin is below
# TAU_MULT x bf16_ref_err -- the reference's OWN bf16-vs-f32 first-step logit error, computed by
# make_goldens.py (gen_tolerance) and stored with the golden: doubled for the growth of the
# rounding error over the decode steps (the stored per-step errors grow <= 1.7x over 67 steps).
# Every token before that step is compared; the compared fraction per golden is stated and
# asserted (MIN_COMPARED_FRAC).
TAU_MULT = 2.0
MIN_COMPARED_FRAC = {"c2_margin_flat": 0.5,
                     "c2_gpt2init": 0.6}     # GPT-2's init scale (the bench's weights)
# the bf16 gates: c1_greedy (std 0.1) and c2_margin (std 0.05) are reported by summary() but not
# gated -- the reference's own bf16 error there is ~1 / 0.23 logit at step 0, so the rule would
# compare < 2 % of their tokens
GOLDENS_BF16 = ("c1_greedy", "c2_margin", "c2_margin_flat", "c2_gpt2init")
GATED_BF16 = ("c2_margin_flat", "c2_gpt2init")


def margin_gate(g, caps) -> dict:
    """Apply the bf16 id-parity rule to generated ids ``caps`` against golden ``g``: the tokens
    compared (every step before the first ambiguous one), and the clips that broke the rule."""
    tau = TAU_MULT * float(g["bf16_ref_err"])
    margin, ref_ids, ref_len = g["margin"], g["greedy_ids"], g["greedy_len"]
    compared, total, exact_needed, bad = 0, int(ref_len.sum()), 0, []
    for b in range(len(caps)):
        L = int(ref_len[b])
        ref = ref_ids[b, :L].tolist()
        amb = next((i for i in range(L) if margin[b, i] < tau), None)
        upto = L if amb is None else amb
        compared += upto
        got = caps[b]
        if amb is None:
            exact_needed += 1
            if got != ref:
                bad.append((b, "exact sequence expected"))
        elif got[:upto] != ref[:upto]:
            d = next(i for i in range(upto) if i >= len(got) or got[i] != ref[i])
            bad.append((b, f"diverged at step {d} before the first ambiguous step {amb}"))
    return {"tau": round(tau, 4), "bf16_ref_err": round(float(g["bf16_ref_err"]), 4),
            "compared_tokens": compared, "total_tokens": total,
            "compared_frac": round(compared / max(1, total), 4),
            "clips_exact_required": exact_needed, "violations": bad}


def load(name):
    path = os.path.join(GOLDEN, name + ".npz")
    return dict(np.load(path)) if os.path.exists(path) else None


def summary(dtype, device, names=GOLDENS_BF16) -> dict:
    import torch
    out = {}
    for name in names:
        g = load(name)
        if g is None:
            continue
        caps, hards = run_greedy(g, dtype, device)
        r = agreement(g, caps, hards)
        r.pop("first_divergence")
        r.pop("min_margin_per_clip", None)
        if dtype != torch.float32:
            r["first_step_logit_max_err_vs_f32"] = round(bf16_logit_error(g, device), 4)
            if "bf16_ref_err" in g:
                gate = margin_gate(g, caps)
                gate["violations"] = len(gate["violations"])
                gate["gated"] = name in GATED_BF16
                r["margin_gate"] = gate
        out[name] = r
    return out


if __name__ == "__main__":
    import json
    import torch
    dt = torch.float32 if (sys.argv[1:] or ["bf16"])[0] == "f32" else torch.bfloat16
    print(json.dumps(summary(dt, torch.device("cuda", 0)), indent=1))
