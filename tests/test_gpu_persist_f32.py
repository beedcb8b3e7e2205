"""The f32 parity mode's grid decode (decode_grid.hip namespace f32: zs_gpt2_decode_persist_f32 and
zs_gpt2_decode_phases_f32, G = 192):

  * ids equal the reference goldens BIT-EXACT (c1_greedy: 50 clips x 67 steps with std-0.1
    weights, c2_gpt2init: GPT-2's init scale) through the persistent launch, through the phase
    launches and through the round-4 f32 row-kernel path (ZSAAC_GRID_DECODE_F32=0);
  * the persistent and the phase launches leave bit-identical decode state;
  * ragged batches and short entry lengths behave as the full batch;
  * a give-up in the middle of the launch resumes on the phase launches with the same ids.
"""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _pipe(g, device, persist, batch=None, entry_length=None):
    from tools import idparity
    from zsaac import synthetic as S
    from zsaac.pipeline import CaptionConfig, CaptionPipeline
    csd = S.gpt2_state_dict(**idparity.golden_gpt2_kw(g))
    csd.update(S.mlp_mapper_state_dict(1))
    cfg = CaptionConfig(dtype=torch.float32, batch=batch or g["clap_emb"].shape[0],
                        entry_length=entry_length or int(g["entry_length"]),
                        persist_decode=persist)
    return CaptionPipeline(csd, None, S.label_table(), S.label_token_table(), cfg, device=device)


def _state(p, B):
    d = p.decoder
    st = {k: t[:B].cpu().numpy().copy() for k, t in
          (("pos", d.pos), ("done", d.done), ("out_len", d.out_len), ("next_tok", d.next_tok),
           ("out_ids", d.out_ids))}
    st["step_ctr"] = np.array([d.step_ctr.item()])
    st["finished"] = np.array([d.all_done[0].item(), d.all_done[2].item()])
    return st


@pytest.mark.parametrize("name", ["c1_greedy", "c2_gpt2init"])
def test_f32_grid_decode_bit_exact(cuda, name, monkeypatch):
    from tools import idparity
    g = idparity.load(name)
    emb = torch.from_numpy(g["clap_emb"]).to(cuda)
    B = emb.shape[0]
    res = {}
    for mode in ("persist", "phases", "rows"):
        if mode == "rows":
            monkeypatch.setenv("ZSAAC_GRID_DECODE_F32", "0")
        p = _pipe(g, cuda, mode == "persist")
        assert p.decoder.f32_grid == (mode != "rows")
        assert p.decoder.persist == (mode == "persist")
        out = p.caption_emb(emb)
        res[mode] = (out.captions(), _state(p, B))
        assert p.decoder.gave_up == 0
        r = idparity.agreement(g, res[mode][0])
        bad = [b for b, d in enumerate(r["first_divergence"]) if d is not None]
        assert not bad, f"{name} {mode}: f32 ids differ from the reference on clips {bad}"
    for k in res["persist"][1]:
        assert np.array_equal(res["persist"][1][k], res["phases"][1][k]), k
    for k in ("out_ids", "out_len", "done"):
        assert np.array_equal(res["persist"][1][k], res["rows"][1][k]), k


def test_f32_ragged_and_short(cuda):
    from tools import idparity
    g = idparity.load("c2_gpt2init")
    emb = torch.from_numpy(g["clap_emb"]).to(cuda)
    full = _pipe(g, cuda, True).caption_emb(emb).captions()
    for persist in (True, False):
        p = _pipe(g, cuda, persist, batch=7)
        for c0 in range(0, 21, 7):
            assert p.caption_emb(emb[c0:c0 + 7]).captions() == full[c0:c0 + 7], (persist, c0)
    res = {}
    for persist in (True, False):
        p = _pipe(g, cuda, persist, batch=16, entry_length=2)
        res[persist] = (p.caption_emb(emb[:16]).captions(), _state(p, 16))
    assert res[True][0] == res[False][0]
    for k in ("pos", "done", "out_len", "next_tok", "out_ids", "finished"):
        assert np.array_equal(res[True][1][k], res[False][1][k]), k
    assert all(len(c) <= 2 for c in res[True][0])


def test_f32_give_up_resumes(cuda):
    """dp_abort_step 3: every workgroup of the persistent f32 launch gives up at the start of
    step 3; the host resumes on the f32 phase launches and the ids and state equal an
    uninterrupted run's; then ConcurrentRunner (grid 192) with the knob off."""
    from tools import idparity
    from zsaac._lib import call
    from zsaac.pipeline import ConcurrentRunner
    g = idparity.load("c2_gpt2init")
    emb = torch.from_numpy(g["clap_emb"][:16]).to(cuda)
    p = _pipe(g, cuda, True, batch=16)
    ref = p.caption_emb(emb).captions()
    ref_state = _state(p, 16)
    call("zs_tune_set", b"dp_abort_step", 3)
    try:
        g0 = p.decoder.gave_up
        got = p.caption_emb(emb).captions()
        assert p.decoder.gave_up == g0 + 1, "the forced give-up did not happen"
        assert got == ref
        st = _state(p, 16)
        for k in ("pos", "done", "out_len", "next_tok", "out_ids"):
            assert np.array_equal(st[k], ref_state[k]), k
    finally:
        call("zs_tune_set", b"dp_abort_step", -1)
    runner = ConcurrentRunner(p, 2)
    assert runner.grids == [192]
    runner.warmup_emb(emb[:8])
    outs = runner.run([emb[:8], emb[8:]], inputs="emb")
    assert [c for o in outs for c in o.captions()] == ref
    assert runner.gave_up == 0
