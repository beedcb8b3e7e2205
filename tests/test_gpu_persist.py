"""The persistent greedy decode (zs_gpt2_decode_persist: all steps of generate2 after step 0 for
one bs <= 64 batch in one launch) against the per-step launch chain it replaces and against the
reference goldens.

Both bf16 paths round the same values to bf16 (LN-folded c_attn / c_fc weights, bf16 q/k/v,
attention output and MLP hidden rows, f32 residual stream) but sum in different orders, so ids
agree wherever the reference's own top-1 / top-2 margin is not within bf16 noise:
  * c2_margin_flat (reference margins large at every step): persistent ids == stepwise ids ==
    reference ids on every clip, at the full batch and at ragged batches of 1, 7 and 21 rows;
  * decode state after the launch (pos, done, out_len, step counter, finished flag) equals the
    stepwise path's, including entry_length 1 (no persistent step) and 2 (one step);
  * the margin-gated reference parity of tests/test_gpu_idparity.py runs this path too (bf16 at
    <= 64 rows is persistent by default).
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
    cfg = CaptionConfig(dtype=torch.bfloat16, batch=batch or g["clap_emb"].shape[0],
                        entry_length=entry_length or int(g["entry_length"]),
                        persist_decode=persist)
    p = CaptionPipeline(csd, None, S.label_table(), S.label_token_table(), cfg, device=device)
    assert p.decoder.persist == persist
    return p


def _state(p, B):
    d = p.decoder
    return {k: t[:B].cpu().numpy().copy() for k, t in
            (("pos", d.pos), ("done", d.done), ("out_len", d.out_len), ("next_tok", d.next_tok))}


@pytest.fixture(scope="module")
def flat():
    from tools import idparity
    return idparity.load("c2_margin_flat")


def test_persist_equals_stepwise_and_reference(cuda, flat):
    from tools import idparity
    emb = torch.from_numpy(flat["clap_emb"]).to(cuda)
    B = emb.shape[0]
    outs = {}
    for persist in (True, False):
        p = _pipe(flat, cuda, persist)
        out = p.caption_emb(emb)
        outs[persist] = (out.captions(), _state(p, B), p.decoder.step_ctr.item(),
                         p.decoder.all_done.tolist())
    (cp, sp, kp, ap), (cs, ss, ks, as_) = outs[True], outs[False]
    assert cp == cs
    for k in sp:
        assert np.array_equal(sp[k], ss[k]), k
    assert kp == ks and ap[0] == as_[0] == 1 and ap[2] == as_[2]
    r = idparity.agreement(flat, cp)
    assert r["exact_frac"] == 1.0, r


@pytest.mark.parametrize("B", [1, 7, 21])
def test_persist_ragged_batches(cuda, flat, B):
    emb = torch.from_numpy(flat["clap_emb"]).to(cuda)
    full = _pipe(flat, cuda, True).caption_emb(emb).captions()
    p = _pipe(flat, cuda, True, batch=B)
    for c0 in range(0, emb.shape[0], B):
        got = p.caption_emb(emb[c0:c0 + B]).captions()
        assert got == full[c0:c0 + B], c0


@pytest.mark.parametrize("entry", [1, 2, 5])
def test_persist_short_entry_length(cuda, flat, entry):
    emb = torch.from_numpy(flat["clap_emb"][:16]).to(cuda)
    res = []
    for persist in (True, False):
        p = _pipe(flat, cuda, persist, batch=16, entry_length=entry)
        out = p.caption_emb(emb)
        res.append((out.captions(), _state(p, 16), p.decoder.step_ctr.item()))
    assert res[0][0] == res[1][0]
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[1][1][k]), (entry, k)
    assert res[0][2] <= entry   # the stepwise graph chunks run a few no-op steps past the end


def test_persist_bench_weights_agreement(cuda):
    """The bench's decoder weights (margins mostly within bf16 noise after a few steps): the two
    bf16 paths agree on every clip's first generated ids and on most tokens."""
    from tools import idparity
    g = idparity.load("c1_greedy")
    emb = torch.from_numpy(g["clap_emb"]).to(cuda)
    a = _pipe(g, cuda, True).caption_emb(emb).captions()
    b = _pipe(g, cuda, False).caption_emb(emb).captions()
    lead = [next((i for i, (x, y) in enumerate(zip(u, v)) if x != y), min(len(u), len(v)))
            for u, v in zip(a, b)]
    assert min(lead) >= 1, lead
    assert np.mean(lead) >= 4, lead


def test_persist_temperature(cuda, flat):
    """generate2's temperature (logits / T before the argmax) in the persistent kernel: ids equal
    the stepwise path's (zs_lmhead_topk_t) at T = 0.7 on the large-margin golden."""
    emb = torch.from_numpy(flat["clap_emb"][:16]).to(cuda)
    res = []
    for persist in (True, False):
        p = _pipe(flat, cuda, persist, batch=16)
        p.decoder.temperature = 0.7
        res.append(p.caption_emb(emb).captions())
    assert res[0] == res[1]


@pytest.mark.parametrize("B", [64, 7])
def test_persist_grid_shapes(cuda, flat, B):
    """Every grid shape (col_split, row_split) -- row_split 2: twice the workgroups, each a column
    slice for half of the rows; col_split 2: half the workgroups, each two column slices -- gives
    the ids and decode state of the default grid, and the reference's ids."""
    from tools import idparity
    emb = torch.from_numpy(flat["clap_emb"]).to(cuda)
    emb = torch.cat([emb, emb])[:B]           # 64: the golden's 32 clips twice (a full batch)
    from zsaac._lib import call
    res = {}
    # fuse 1: the MLP as phases D' + R (mlp.c_proj partial sums, zs_tune_set dp_fuse)
    for cs, rs, fuse in ((1, 1, 0), (1, 2, 0), (2, 1, 0), (2, 2, 0), (1, 1, 1), (2, 1, 1)):
        p = _pipe(flat, cuda, True, batch=B)
        p.decoder.persist_row_split, p.decoder.persist_col_split = rs, cs
        call("zs_tune_set", b"dp_fuse", fuse)
        try:
            out = p.caption_emb(emb)
        finally:
            call("zs_tune_set", b"dp_fuse", 0)
        res[cs, rs, fuse] = (out.captions(), _state(p, B), p.decoder.step_ctr.item())
    base = res[1, 1, 0]
    for shape, r in res.items():
        assert r[0] == base[0], shape
        for k in base[1]:
            assert np.array_equal(r[1][k], base[1][k]), (shape, k)
        assert r[2] == base[2], shape
    if B == 64:
        assert base[0][:32] == base[0][32:]
        assert idparity.agreement(flat, base[0][:32])["exact_frac"] == 1.0


def test_persist_give_up_resumes_stepwise(cuda, flat):
    """A persistent launch whose grid barrier gives up (forced: zs_tune_set dp_spin < 0 gives up
    at the first unmet poll) reports all_done[1] = -1 with its starting decode state intact; the
    host resumes the batch on the per-step path and the ids equal a normal run's -- through
    Gpt2Decoder.greedy (synchronous) and through ConcurrentRunner (two batches in flight)."""
    from zsaac._lib import call
    from zsaac.pipeline import ConcurrentRunner
    emb = torch.from_numpy(flat["clap_emb"][:16]).to(cuda)
    p = _pipe(flat, cuda, True, batch=16)
    ref = p.caption_emb(emb).captions()
    call("zs_tune_set", b"dp_spin", -1)
    try:
        g0 = p.decoder.gave_up
        got = p.caption_emb(emb).captions()
        assert p.decoder.gave_up == g0 + 1, "the forced give-up did not happen"
        assert got == ref
        runner = ConcurrentRunner(p, 2)
        runner.warmup_emb(emb[:8])
        outs = runner.run([emb[:8], emb[8:]], inputs="emb")
        assert [c for o in outs for c in o.captions()] == ref
        assert sum(q.decoder.gave_up for q in runner.pipes) >= 2
    finally:
        call("zs_tune_set", b"dp_spin", 0)
    assert p.caption_emb(emb).captions() == ref


def test_concurrent_runner_bf16_persist(cuda, flat):
    """The headline's arrangement: bf16 batches through ConcurrentRunner (10 pipelines, persistent
    grids of every shape -- 96 / 48 / 24 workgroups, chosen per batch by choose_persist_shape --
    several in flight, ragged batches included): every batch's ids equal the single-stream
    persistent run's and the reference's (c2_margin_flat, exact on every clip)."""
    from tools import idparity
    from zsaac.pipeline import ConcurrentRunner, persist_shapes
    emb = torch.from_numpy(flat["clap_emb"]).to(cuda)
    ref = [flat["greedy_ids"][b, :flat["greedy_len"][b]].tolist() for b in range(emb.shape[0])]
    p = _pipe(flat, cuda, True)
    single = p.caption_emb(emb).captions()
    assert single == ref
    runner = ConcurrentRunner(p, 10, shapes=persist_shapes("12,11,21"))
    assert runner.n_inflight == 10
    runner.warmup_emb(emb)
    used = set()
    for sizes in ([32] * 6 + [7, 3], [32, 21]):
        batches, want = [], []
        for i, n in enumerate(sizes):
            rows = [(5 * i + j) % 32 for j in range(n)]
            batches.append(emb[rows])
            want.append([ref[r] for r in rows])
        outs = runner.run(batches, inputs="emb")
        for i, o in enumerate(outs):
            assert o.captions() == want[i], (sizes, i, runner.shape[i])
            assert int(o.lengths.shape[0]) == sizes[i]
        used |= set(runner.shape[:len(sizes)])
        assert all(s >= 2 for s in runner.decode_steps[:len(sizes)])
    assert {(1, 2), (1, 1), (2, 1)} <= used, used
    assert sum(q.decoder.gave_up for q in runner.pipes) == 0
