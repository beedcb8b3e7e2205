"""Greedy token-id parity against the reference goldens, with the reference's own logit margins
(tests/golden/{c1_greedy,c2_margin,c2_margin_flat,c2_gpt2init}.npz, made by running the reference;
tools/idparity.py runs the batched pipeline on their CLAP embeddings).

  * f32 parity mode: every clip's ids BIT-EXACT on all four goldens.
  * bf16 perf mode: every clip's ids equal the reference's up to the first generated step at
    which the reference's top-1 / top-2 logit margin is below tau — a divergence may only start
    where the reference's own choice is within bf16 rounding of a tie; clips whose margins stay
    above tau at every step are bit-exact end to end.  tau is FIXED per golden: 2 x the
    reference's own bf16-vs-f32 first-step logit error, stored with the golden
    (make_goldens.py gen_tolerance); the GPU's bf16 error must not exceed it.  The compared
    fraction of tokens is asserted per golden: c2_gpt2init (GPT-2's init scale, the bench's own
    weights) >= 0.6, c2_margin_flat >= 0.5.  c1_greedy and c2_margin (std 0.1 / 0.05 blocks) are
    too chaotic for a bf16 id gate -- the reference's OWN bf16 run is off by ~1 logit at step 0,
    so their rule would compare < 2 % of the tokens; they are bit-exact in f32 only and are not
    listed as bf16 gates.
"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GOLDENS = ["c1_greedy", "c2_margin", "c2_margin_flat", "c2_gpt2init"]
# every bf16 golden: the error bound and zero violations hold on all four; the compared-fraction
# floor applies where the rule compares most tokens (c1_greedy / c2_margin: reference bf16 error
# ~1 / 0.23 logit at step 0, < 2 % of their tokens compared)
GOLDENS_BF16 = ["c1_greedy", "c2_margin", "c2_margin_flat", "c2_gpt2init"]


@pytest.mark.parametrize("name", GOLDENS)
def test_f32_ids_bit_exact(cuda, name):
    from tools import idparity
    g = idparity.load(name)
    caps, hards = idparity.run_greedy(g, torch.float32, cuda)
    r = idparity.agreement(g, caps, hards)
    assert r["hard_prompt_exact_frac"] == 1.0
    bad = [b for b, d in enumerate(r["first_divergence"]) if d is not None]
    assert not bad, f"{name}: f32 greedy ids differ on clips {bad}"


@pytest.mark.parametrize("name", GOLDENS_BF16)
def test_bf16_ids_exact_above_margin(cuda, name):
    """The bf16 rule with a FIXED tolerance stored with the golden (tools/idparity.py
    margin_gate): tau = 2 x the reference's own bf16-vs-f32 first-step logit error; the GPU's bf16
    first-step error must not exceed that reference error; every token before the first step
    whose reference margin is below tau must equal the reference's; the compared fraction of the
    golden's tokens is printed and asserted (MIN_COMPARED_FRAC)."""
    from tools import idparity
    g = idparity.load(name)
    assert "bf16_ref_err" in g, f"{name}: no stored bf16 tolerance (make_goldens.py tolerance)"
    err = idparity.bf16_logit_error(g, cuda)
    assert err <= float(g["bf16_ref_err"]), (
        f"{name}: bf16 first-step logit error {err:.4f} above the reference's own bf16 error "
        f"{float(g['bf16_ref_err']):.4f}")
    caps, hards = idparity.run_greedy(g, torch.bfloat16, cuda)
    r = idparity.margin_gate(g, caps)
    print(f"{name} bf16: first-step error {err:.4f} (reference bf16 {r['bf16_ref_err']}), tau "
          f"{r['tau']}, compared {r['compared_tokens']} / {r['total_tokens']} tokens "
          f"({r['compared_frac']}), clips required exact {r['clips_exact_required']}")
    assert not r["violations"], f"{name}: {r['violations']}"
    assert r["compared_frac"] >= idparity.MIN_COMPARED_FRAC.get(name, 0.0), r
