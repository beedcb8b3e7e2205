"""CPU: the oracle (oracle/) against the golden fixtures produced by running the reference
(tests/golden/make_goldens.py).  This pins the checker itself before it is trusted."""
import numpy as np
import pytest
import torch

from zsaac import synthetic as S

GPT2_KW = dict(seed=0, std=0.1, emb_std=0.1, stop_boost=2.0)


@pytest.fixture(scope="module")
def csd():
    sd = S.gpt2_state_dict(**GPT2_KW)
    sd.update(S.mlp_mapper_state_dict(1))
    sd.update(S.transformer_mapper_state_dict(2))
    return sd


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


def test_mappers(golden, csd):
    from oracle import caption as C
    g = golden("mappers.npz")
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        assert _rel(C.mlp_mapper(x, csd), g["mlp_out"]) < 1e-6
        assert _rel(C.transformer_mapper(x, csd), g["tmapper_out"]) < 1e-6
        pe = C.clap_to_gpt(x[:1], torch.from_numpy(g["tm_hard_ids"]), csd, "transformer")
    assert _rel(pe[0], g["tm_prefix_embed"]) < 1e-6


def test_htsat_and_proj(golden):
    from oracle import audio as A
    g = golden("htsat.npz")
    sd = dict(S.htsat_state_dict(3))
    sd.update(S.audio_proj_state_dict(5, audio_width=768))
    with torch.no_grad():
        e = A.htsat_embedding(torch.from_numpy(g["logmel"]), sd)
        p = A.audio_project(e, sd)
    assert _rel(e, g["embedding768"]) < 1e-5
    assert _rel(p, g["clap_emb"]) < 1e-5


def test_cnn14_and_proj(golden):
    from oracle import audio as A
    g = golden("cnn14.npz")
    sd = dict(S.cnn14_state_dict(4))
    sd.update(S.audio_proj_state_dict(5, audio_width=2048))
    with torch.no_grad():
        e = A.cnn14_embedding(torch.from_numpy(g["logmel"]), sd)
        p = A.audio_project(e, sd)
    assert _rel(e, g["embedding2048"]) < 1e-5
    assert _rel(p, g["clap_emb"]) < 1e-5


def test_c1_prompt_ids_all_clips(golden):
    """ClapTestDataset_withHardPrompt.__getitem__ + collate (reference) == oracle prompt ids."""
    from oracle import caption as C
    g = golden("c1_greedy.npz")
    table, lt = S.label_table(), S.label_token_table()
    emb = torch.from_numpy(g["clap_emb"])
    for i in range(emb.shape[0]):
        idx = C.sound_effect_choice(emb[i:i + 1], table, int(g["sound_effect_num"]))[0].tolist()
        assert C.prompt_ids(idx, lt) == g["hard_ids"][i, :g["hard_len"][i]].tolist()


@pytest.mark.parametrize("clip", [0, 3, 18])
def test_c1_greedy_kv_oracle(golden, csd, clip):
    """generate2 token ids (reference, full recompute) == oracle KV-cache greedy, incl. stops."""
    from oracle import caption as C
    g = golden("c1_greedy.npz")
    n = int(g["hard_len"][clip])
    hard = torch.from_numpy(g["hard_ids"][clip:clip + 1, :n])
    pre = torch.nn.functional.normalize(torch.from_numpy(g["clap_emb"][clip:clip + 1]), dim=-1)[None]
    with torch.no_grad():
        pe = C.clap_to_gpt(pre, hard, csd)
    if clip < g["prefix_embed"].shape[0]:
        assert _rel(pe[0], g["prefix_embed"][clip, :n + 10]) < 1e-6
    toks = C.generate2(pe, csd, use_cache=True)
    assert toks == g["greedy_ids"][clip, :g["greedy_len"][clip]].tolist()
    assert C.prefix_tokens(pe, csd) == g["prefix_tokens"][clip, :n + 10].tolist()


def test_full_recompute_equals_kv_cache(golden, csd):
    """The oracle's reference-semantics full recompute and its KV-cache variant agree."""
    from oracle import caption as C
    g = golden("c1_greedy.npz")
    pe = torch.from_numpy(g["prefix_embed"][1, :int(g["hard_len"][1]) + 10])[None]
    assert C.generate2(pe, csd, entry_length=6) == C.generate2(pe, csd, entry_length=6, use_cache=True)


@pytest.mark.parametrize("beam", [5, 3])
def test_beam_kv_oracle(golden, csd, beam):
    from oracle import caption as C
    g = golden("beam.npz")
    c = 0
    n = int(g["hard_len"][c])
    hard = torch.from_numpy(g["hard_ids"][c:c + 1, :n])
    with torch.no_grad():
        pe = C.clap_to_gpt(torch.from_numpy(g["clap_emb"][c:c + 1])[None], hard, csd)
    outs, _ = C.generate_beam(pe, csd, beam_size=beam, use_cache=True)
    ref = [g[f"beam{beam}_ids"][c, i, :g[f"beam{beam}_len"][c, i]].tolist() for i in range(beam)]
    assert outs == ref


@pytest.mark.parametrize("tag,T", [("t07", 0.7), ("t16", 1.6)])
def test_beam_temperature_oracle(golden, csd, tag, T):
    """generate_beam with temperature != 1 (logits / T before softmax().log(),
    gpt2_prefix_eval.py:121-122): the oracle against the reference's own output."""
    from oracle import caption as C
    g = golden("temperature.npz")
    c = 1
    n = int(g["hard_len"][c])
    hard = torch.from_numpy(g["hard_ids"][c:c + 1, :n])
    with torch.no_grad():
        pe = C.clap_to_gpt(torch.from_numpy(g["clap_emb"][c:c + 1])[None], hard, csd)
    outs, _ = C.generate_beam(pe, csd, beam_size=3, entry_length=int(g["entry_length"]),
                              use_cache=True, temperature=T)
    ref = [g[f"beam3_{tag}_ids"][c, i, :g[f"beam3_{tag}_len"][c, i]].tolist() for i in range(3)]
    assert outs == ref
    ids = C.generate2(pe, csd, entry_length=int(g["entry_length"]), use_cache=True, temperature=0.7)
    assert ids == g["greedy_t07_ids"][c, :g["greedy_t07_len"][c]].tolist()


@pytest.mark.parametrize("name,clip", [("c2_gpt2init", 0), ("c2_gpt2init", 5), ("c2_margin_flat", 2)])
def test_margin_golden_greedy_kv_oracle(golden, name, clip):
    """The margin goldens (incl. c2_gpt2init, GPT-2's init scale): the oracle's KV-cache greedy
    reproduces the reference's ids, and the stored bf16 tolerance is a positive logit error below
    the reference's median step margin (tools/idparity.py margin_gate)."""
    from oracle import caption as C
    from tools import idparity
    g = golden(name + ".npz")
    sd = S.gpt2_state_dict(**idparity.golden_gpt2_kw(g))
    sd.update(S.mlp_mapper_state_dict(1))
    n = int(g["hard_len"][clip])
    hard = torch.from_numpy(g["hard_ids"][clip:clip + 1, :n])
    pre = torch.nn.functional.normalize(torch.from_numpy(g["clap_emb"][clip:clip + 1]), dim=-1)[None]
    with torch.no_grad():
        pe = C.clap_to_gpt(pre, hard, sd)
    toks = C.generate2(pe, sd, entry_length=int(g["entry_length"]), use_cache=True)
    assert toks == g["greedy_ids"][clip, :g["greedy_len"][clip]].tolist()
    err = float(g["bf16_ref_err"])
    m = g["margin"][g["margin"] > 0]
    assert 0 < err < float(np.median(m)), (err, float(np.median(m)))
