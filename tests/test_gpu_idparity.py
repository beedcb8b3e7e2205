"""Greedy token-id parity against the reference goldens, with the reference's own logit margins
(tests/golden/{c1_greedy,c2_margin,c2_margin_flat}.npz, made by running the reference;
tools/idparity.py runs the batched pipeline on their CLAP embeddings).

  * f32 parity mode: every clip's ids BIT-EXACT on all three goldens.
  * bf16 perf mode: every clip's ids equal the reference's up to the first generated step at
    which the reference's top-1 / top-2 logit margin is below TAU — a divergence may only start
    where the reference's own choice is within bf16 rounding of a tie; clips whose margins stay
    above TAU at every step are bit-exact end to end.  TAU = 2 x the largest first-step logit
    error of bf16 against f32 measured on the same golden's clips (at least 0.2 logits; the
    logits' std is ~2.8): the error bound of this network in bf16, doubled for the growth of the
    KV-cache error over the steps.
"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TAU = 0.2
GOLDENS = ["c1_greedy", "c2_margin", "c2_margin_flat"]


@pytest.mark.parametrize("name", GOLDENS)
def test_f32_ids_bit_exact(cuda, name):
    from tools import idparity
    g = idparity.load(name)
    caps, hards = idparity.run_greedy(g, torch.float32, cuda)
    r = idparity.agreement(g, caps, hards)
    assert r["hard_prompt_exact_frac"] == 1.0
    bad = [b for b, d in enumerate(r["first_divergence"]) if d is not None]
    assert not bad, f"{name}: f32 greedy ids differ on clips {bad}"


@pytest.mark.parametrize("name", GOLDENS)
def test_bf16_ids_exact_above_margin(cuda, name):
    from tools import idparity
    g = idparity.load(name)
    assert "margin" in g, f"{name} has no reference margins (regenerate with make_goldens.py)"
    tau = max(TAU, 2.0 * idparity.bf16_logit_error(g, cuda))
    caps, hards = idparity.run_greedy(g, torch.bfloat16, cuda)
    r = idparity.agreement(g, caps, hards)
    margin, ref_len = g["margin"], g["greedy_len"]
    exact_needed, late = 0, []
    for b, d in enumerate(r["first_divergence"]):
        L = int(ref_len[b])
        ambiguous = next((i for i in range(L) if margin[b, i] < tau), None)
        if ambiguous is None:
            exact_needed += 1
            assert d is None, f"{name} clip {b}: margins >= {tau:.3f} everywhere, diverged at {d}"
        elif d is not None:
            assert d >= ambiguous, (f"{name} clip {b}: diverged at step {d} before the first "
                                    f"ambiguous step {ambiguous} (margin {margin[b, d]:.3f})")
            late.append(d - ambiguous)
    r.pop("first_divergence")
    r.pop("min_margin_per_clip", None)
    print(f"{name} bf16: tau {tau:.3f}; {r}; clips with every margin >= tau: {exact_needed}")
