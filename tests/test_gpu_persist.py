"""The grid decode of one bs <= 64 greedy batch (decode_grid.hip): the persistent launch
(zs_gpt2_decode_persist) at every grid size and the phase launches (zs_gpt2_decode_phases, the
per-step path and the give-up fallback) run one canonical arithmetic, so

  * ids AND decode state (pos, done, out_len, next_tok, step counter, finished flag) are
    bit-identical across grids 48 / 96 / 192 and the phase launches at grids 48 / 96 / 192, on the
    bench-scale goldens c1_greedy (std-0.1 weights) and c2_gpt2init (GPT-2's init scale) as well as
    c2_margin_flat -- whatever grid a concurrent schedule picks, a caption does not change;
  * on c2_margin_flat (reference margins large at every step) the ids equal the reference's;
  * ragged batches (1, 7, 21 rows), entry_length 1 / 2 / 5 and temperature behave as the full
    batch / the phase launches;
  * a give-up (forced at the first barrier, or in the middle of the launch at a chosen step)
    resumes from the last committed step on the phase launches with ids equal to an
    uninterrupted run's, synchronously and under ConcurrentRunner.
"""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GRIDS = (48, 96, 192)


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
    assert p.decoder.persist == persist and p.decoder.grid_decode
    return p


def _state(p, B):
    d = p.decoder
    st = {k: t[:B].cpu().numpy().copy() for k, t in
          (("pos", d.pos), ("done", d.done), ("out_len", d.out_len), ("next_tok", d.next_tok),
           ("out_ids", d.out_ids))}
    st["step_ctr"] = np.array([d.step_ctr.item()])
    st["finished"] = np.array([d.all_done[0].item(), d.all_done[2].item()])
    return st


def _run_all(g, device, emb, batch=None, entry_length=None):
    """{(mode, grid): (captions, state)} for the persistent launch and the phase launches."""
    res = {}
    B = emb.shape[0]
    for mode in ("persist", "phases"):
        p = _pipe(g, device, mode == "persist", batch=batch, entry_length=entry_length)
        for grid in GRIDS:
            if mode == "persist":
                p.decoder.persist_grid = grid
            else:
                p.decoder.phase_grid = grid
                p.decoder.graphs.clear()      # the captured chunk holds the old grid
            out = p.caption_emb(emb)
            res[mode, grid] = (out.captions(), _state(p, B))
            assert p.decoder.gave_up == 0
    return res


def _assert_identical(res):
    base = res["persist", 48]
    for key, (caps, st) in res.items():
        assert caps == base[0], key
        for k in base[1]:
            assert np.array_equal(st[k], base[1][k]), (key, k)


@pytest.mark.parametrize("name", ["c1_greedy", "c2_gpt2init", "c2_margin_flat"])
def test_grids_and_phases_bit_identical(cuda, name):
    from tools import idparity
    g = idparity.load(name)
    emb = torch.from_numpy(g["clap_emb"]).to(cuda)
    emb = emb[:64]
    res = _run_all(g, cuda, emb)
    _assert_identical(res)
    caps = res["persist", 48][0]
    if name == "c2_margin_flat":
        assert idparity.agreement(g, caps)["exact_frac"] == 1.0
    if "bf16_ref_err" in g:       # the stored-tolerance rule holds on the grid decode's ids
        assert idparity.margin_gate(g, caps)["violations"] == []


def test_full_batch_of_64(cuda):
    """A full 64-row batch (every row block of every tile live): the golden's 32 clips twice."""
    from tools import idparity
    g = idparity.load("c2_margin_flat")
    e = torch.from_numpy(g["clap_emb"]).to(cuda)
    emb = torch.cat([e, e])[:64]
    res = _run_all(g, cuda, emb, batch=64)
    _assert_identical(res)
    caps = res["persist", 192][0]
    assert caps[:32] == caps[32:]
    assert idparity.agreement(g, caps[:32])["exact_frac"] == 1.0


@pytest.mark.parametrize("B", [1, 7, 21])
def test_ragged_batches(cuda, B):
    from tools import idparity
    g = idparity.load("c2_gpt2init")
    emb = torch.from_numpy(g["clap_emb"]).to(cuda)
    full = _pipe(g, cuda, True).caption_emb(emb).captions()
    for persist in (True, False):
        p = _pipe(g, cuda, persist, batch=B)
        for c0 in range(0, emb.shape[0], B):
            got = p.caption_emb(emb[c0:c0 + B]).captions()
            assert got == full[c0:c0 + B], (persist, c0)


@pytest.mark.parametrize("entry", [1, 2, 5])
def test_short_entry_length(cuda, entry):
    from tools import idparity
    g = idparity.load("c2_margin_flat")
    emb = torch.from_numpy(g["clap_emb"][:16]).to(cuda)
    res = {}
    for persist in (True, False):
        p = _pipe(g, cuda, persist, batch=16, entry_length=entry)
        out = p.caption_emb(emb)
        res[persist] = (out.captions(), _state(p, 16))
    assert res[True][0] == res[False][0]
    for k in ("pos", "done", "out_len", "next_tok", "out_ids", "finished"):
        assert np.array_equal(res[True][1][k], res[False][1][k]), (entry, k)
    assert res[True][1]["step_ctr"][0] <= entry


def test_temperature(cuda):
    """generate2's temperature (logits / T before the argmax): persistent == phase launches at
    T = 0.7."""
    from tools import idparity
    g = idparity.load("c1_greedy")
    emb = torch.from_numpy(g["clap_emb"][:16]).to(cuda)
    res = {}
    for persist in (True, False):
        p = _pipe(g, cuda, persist, batch=16)
        p.decoder.temperature = 0.7
        res[persist] = p.caption_emb(emb).captions()
    assert res[True] == res[False]


@pytest.mark.parametrize("how", ["first_poll", "step_3"])
def test_give_up_resumes_on_phases(cuda, how):
    """A persistent launch that gives up (forced: zs_tune_set dp_spin -1 gives up at the first
    unmet poll; dp_abort_step 3: every workgroup gives up at the start of step 3, after steps
    1-2 were committed) reports all_done[1] = -1; the host resumes from the committed state on
    the phase launches and the ids equal an uninterrupted run's -- synchronously and through
    ConcurrentRunner (two batches in flight)."""
    from tools import idparity
    from zsaac._lib import call
    from zsaac.pipeline import ConcurrentRunner
    g = idparity.load("c2_gpt2init")
    emb = torch.from_numpy(g["clap_emb"][:16]).to(cuda)
    p = _pipe(g, cuda, True, batch=16)
    ref = p.caption_emb(emb).captions()
    ref_state = _state(p, 16)
    knob = (b"dp_spin", -1) if how == "first_poll" else (b"dp_abort_step", 3)
    call("zs_tune_set", *knob)
    try:
        g0 = p.decoder.gave_up
        got = p.caption_emb(emb).captions()
        assert p.decoder.gave_up == g0 + 1, "the forced give-up did not happen"
        assert got == ref
        st = _state(p, 16)
        for k in ("pos", "done", "out_len", "next_tok", "out_ids"):
            assert np.array_equal(st[k], ref_state[k]), k
        runner = ConcurrentRunner(p, 2, grids=[48], budget=512)
        runner.warmup_emb(emb[:8])
        outs = runner.run([emb[:8], emb[8:]], inputs="emb")
        assert [c for o in outs for c in o.captions()] == ref
        assert runner.gave_up == 2
    finally:
        call("zs_tune_set", knob[0], 0 if how == "first_poll" else -1)
    assert p.caption_emb(emb).captions() == ref


def test_concurrent_runner_mixed_grids(cuda):
    """The headline's arrangement: bf16 batches through ConcurrentRunner with grids 192 / 96 / 48
    chosen per batch by choose_persist_grid (several in flight, ragged batches included): every
    batch's ids equal the single-stream run's and the reference's (c2_margin_flat, exact on every
    clip), and no launch gave up."""
    from tools import idparity
    from zsaac.pipeline import ConcurrentRunner
    g = idparity.load("c2_margin_flat")
    emb = torch.from_numpy(g["clap_emb"]).to(cuda)
    ref = [g["greedy_ids"][b, :g["greedy_len"][b]].tolist() for b in range(emb.shape[0])]
    p = _pipe(g, cuda, True)
    assert p.caption_emb(emb).captions() == ref
    runner = ConcurrentRunner(p, 8, grids=[192, 96, 48], budget=384)
    assert runner.n_inflight == 8
    runner.warmup_emb(emb)
    used = set()
    for sizes in ([32] * 6 + [7, 3], [32, 21], [32, 32, 32]):
        batches, want = [], []
        for i, n in enumerate(sizes):
            rows = [(5 * i + j) % 32 for j in range(n)]
            batches.append(emb[rows])
            want.append([ref[r] for r in rows])
        outs = runner.run(batches, inputs="emb")
        for i, o in enumerate(outs):
            assert o.captions() == want[i], (sizes, i, runner.grid[i])
            assert int(o.lengths.shape[0]) == sizes[i]
        used |= set(runner.grid[:len(sizes)])
        assert all(s >= 2 for s in runner.decode_steps[:len(sizes)])
    assert {192, 96, 48} <= used, used
    assert runner.gave_up == 0


@pytest.mark.parametrize("staged", [0, 1, 2, 4], ids=["pipelined", "begin_first", "begin_group2", "begin_group4"])
def test_concurrent_headline_schedule_ids_equal_single_stream(cuda, staged):
    """The headline's schedule at the headline's size on the bench's own weights (c2_gpt2init,
    GPT-2's init scale, small margins): 1045 embeddings in 17 eval batches of <= 64 (the last 21)
    through ConcurrentRunner -- pipelined: its default grids and budget, ten batches in flight,
    grids chosen per batch; begin_first: a pipeline per batch, every begin first, ten grids of 48
    at a time within the staged budget; begin_group4 (the bench's schedule): begin_first with one
    begin (mapper, get_prefix_tokens, prefill at 256 rows) per 4 consecutive batches and a
    sub-decoder per batch -- give, batch for batch, the ids of a single-stream run of the same
    batches (each its own begin, persistent grid 48, one batch at a time), and no launch gave
    up."""
    from tools import idparity
    from zsaac.pipeline import ConcurrentRunner, persist_budget
    g = idparity.load("c2_gpt2init")
    base = torch.from_numpy(g["clap_emb"]).to(cuda)
    n = 1045
    i = torch.arange(n, device=cuda, dtype=torch.float32)[:, None]
    emb = base[torch.arange(n, device=cuda) % base.shape[0]] * (1.0 + 0.05 * torch.sin(0.37 * i))
    batches = [emb[a:a + 64] for a in range(0, n, 64)]
    p = _pipe(g, cuda, True, batch=64)
    p.decoder.persist_grid = 48
    single = [p.caption_emb(b).captions() for b in batches]
    if staged:
        cus = torch.cuda.get_device_properties(cuda).multi_processor_count
        runner = ConcurrentRunner(p, len(batches) if staged == 1 else 10, begin_first=True,
                                  budget=persist_budget(cus, staged=True),
                                  begin_group=0 if staged == 1 else staged, n_batches=len(batches))
        assert runner.begin_group == (0 if staged == 1 else staged)
    else:
        runner = ConcurrentRunner(p, 10)
    runner.warmup_emb(batches[0])
    fails = []
    for rep in range(3):
        outs = runner.run(batches, inputs="emb")
        for k, o in enumerate(outs):
            caps = o.captions()
            if caps != single[k]:
                r = next(r for r in range(len(caps)) if caps[r] != single[k][r])
                s = next((t for t, (x, y) in enumerate(zip(caps[r], single[k][r])) if x != y),
                         min(len(caps[r]), len(single[k][r])))
                fails.append({"rep": rep, "batch": k, "row": r, "step": s,
                              "grid": runner.grid[k], "pipe": dict((b, i) for i, b in runner.assign)[k],
                              "gave_up": runner.gave_up})
    assert not fails, f"concurrent ids differ from the single-stream run: {fails}"
    assert sum(len(c) for c in single) == n
    assert runner.gave_up == 0


def test_begin_groups_ragged_batches(cuda):
    """Begin groups over eval batches of uneven sizes (44 / 64 / 30 / 64 clips, 12 batches: the
    staged, grouped path): each batch's sub-decoder decodes exactly that batch's clips -- ids and
    prompt lengths equal a single-stream run of the same batches."""
    from tools import idparity
    from zsaac.pipeline import ConcurrentRunner, persist_budget
    g = idparity.load("c2_gpt2init")
    base = torch.from_numpy(g["clap_emb"]).to(cuda)
    sizes = [44, 64, 30, 64] * 3
    n = sum(sizes)
    i = torch.arange(n, device=cuda, dtype=torch.float32)[:, None]
    emb = base[torch.arange(n, device=cuda) % base.shape[0]] * (1.0 + 0.03 * torch.cos(0.29 * i))
    offs = [sum(sizes[:k]) for k in range(len(sizes))]
    batches = [emb[o:o + z] for o, z in zip(offs, sizes)]
    p = _pipe(g, cuda, True, batch=64)
    p.decoder.persist_grid = 48
    single = [(p.caption_emb(b).captions(), p.result().plen.tolist()) for b in batches]
    cus = torch.cuda.get_device_properties(cuda).multi_processor_count
    runner = ConcurrentRunner(p, 10, begin_first=True, budget=persist_budget(cus, staged=True),
                              begin_group=4, n_batches=len(batches))
    runner.warmup_emb(batches[1])
    outs = runner.run(batches, inputs="emb")
    assert runner.bdec is not None, "the grouped path did not run"
    for k, o in enumerate(outs):
        assert o.ids.shape[0] == sizes[k]
        assert o.captions() == single[k][0], f"batch {k} ({sizes[k]} clips): ids differ"
        assert o.plen.tolist() == single[k][1]
    assert runner.gave_up == 0


def test_prompts_beside_grids_deterministic(cuda):
    """The sound-effect prompt (prompt_kernel, gpt2.hip) computed on ten streams while ten
    persistent decode grids run on ten others equals the prompt computed alone, for all 1045
    clips, over 10 rounds (tools/prompt_stress.py grid mode; round 5's 512-thread LDS version
    chose different labels for ~0.03 % of clips there, this test's predecessor of the fix)."""
    import subprocess
    import json as _json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prompt_stress.py"), "10", "grid"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    res = _json.loads(r.stdout.strip().splitlines()[-1])
    assert res["differences"] == 0, res["first"]
