"""CPU: host-side logic — prompt text/ids, tokenizer table, synthetic weights, weight packing
layouts, beam output ordering, the drop-in module surface."""
import numpy as np
import pytest
import torch

from zsaac import synthetic as S


def test_prompt_strings_match_reference(golden):
    from zsaac.tokenizer import compose_prompt_text, synthetic_label_names
    g = golden("prompt.npz")
    names = synthetic_label_names()
    sets = [[], [names[0]], [names[5], names[77]], [names[1], names[2], names[3], names[526]]]
    for s, ref in zip(sets, g["strings"]):
        assert compose_prompt_text(s) == str(ref)


def test_padding_captions_semantics(golden):
    """utils.py:190-208: right-pad with 0, float mask of valid positions."""
    g = golden("prompt.npz")
    assert g["pad_ids"].tolist() == [[5, 6, 7, 0, 0], [1, 0, 0, 0, 0], [9, 8, 7, 6, 5]]
    assert g["pad_mask"].tolist() == [[1, 1, 1, 0, 0], [1, 0, 0, 0, 0], [1, 1, 1, 1, 1]]


def test_table_tokenizer_equals_piece_concatenation():
    from oracle import caption as C
    from zsaac.tokenizer import TableTokenizer, compose_prompt_text, synthetic_label_names
    names, lt = synthetic_label_names(), S.label_token_table()
    tok = TableTokenizer.for_labels(names, lt)
    rng = np.random.default_rng(0)
    for k in range(0, 5):
        idx = rng.choice(527, size=k, replace=False).tolist()
        assert tok.encode(compose_prompt_text([names[i] for i in idx])) == C.prompt_ids(idx, lt)


def test_synthetic_is_deterministic():
    a = S.mlp_mapper_state_dict(1)
    b = S.mlp_mapper_state_dict(1)
    assert all(torch.equal(a[k], b[k]) for k in a)
    c = S.gpt2_state_dict(seed=0, std=0.1)
    assert len(c) == 149 and c["gpt.lm_head.weight"] is c["gpt.transformer.wte.weight"]
    n = sum(v.numel() for k, v in c.items() if k != "gpt.lm_head.weight")
    assert n == 124439808                     # GPT-2 small, tied head
    assert sum(v.numel() for v in a.values()) == 33434880   # MLP mapper
    t = S.transformer_mapper_state_dict(2)
    assert sum(v.numel() for v in t.values()) == 45677568   # TransformerMapper


def test_gpt2_weight_packing_layout():
    from zsaac.decoder import Gpt2Weights
    sd = S.gpt2_state_dict(seed=0, std=0.1)
    w = Gpt2Weights(sd, "cpu", torch.float32)
    ly = w.layers[3]
    # HF Conv1D [in, out] -> kernel layout [out, in] (y = x @ W + b == x @ W_packed^T + b)
    assert torch.equal(ly["attn_w"], sd["gpt.transformer.h.3.attn.c_attn.weight"].t())
    assert ly["fc_w"].shape == (3072, 768) and ly["mproj_w"].shape == (768, 3072)
    x = torch.randn(2, 768)
    ref = x @ sd["gpt.transformer.h.3.mlp.c_fc.weight"] + sd["gpt.transformer.h.3.mlp.c_fc.bias"]
    assert torch.allclose(x @ ly["fc_w"].t() + ly["fc_b"], ref, atol=1e-5)
    assert torch.allclose(w.wte_norm.norm(dim=1), torch.ones(w.V), atol=1e-5)


def test_gpt2_bf16_ln_affine_fold():
    """bf16 packing folds ln_1 / ln_2 (weight, bias) into c_attn / c_fc: normalise-only LN ->
    folded GEMM equals LN -> GEMM (f32 check of the fold; bf16 rounding of W' only)."""
    from zsaac.decoder import Gpt2Weights
    sd = S.gpt2_state_dict(seed=0, std=0.1)
    w = Gpt2Weights(sd, "cpu", torch.bfloat16)
    assert w.folded
    h = "gpt.transformer.h.5."
    ly = w.layers[5]
    assert ly["ln2_gemm"] == (None, None) and torch.equal(ly["ln2"][0], torch.ones(768))
    x = torch.randn(4, 768) * 3 + 1
    xh = torch.nn.functional.layer_norm(x, (768,), eps=1e-5)
    ref = torch.nn.functional.layer_norm(x, (768,), sd[h + "ln_2.weight"], sd[h + "ln_2.bias"], 1e-5)
    ref = ref @ sd[h + "mlp.c_fc.weight"] + sd[h + "mlp.c_fc.bias"]
    got = xh @ ly["fc_w"].float().t() + ly["fc_b"]
    assert (got - ref).abs().max() < 0.02 * ref.abs().max()


def test_cnn14_packing_and_bn_fold():
    from zsaac.encoder import Cnn14Weights
    sd = S.cnn14_state_dict(4)
    w = Cnn14Weights(sd, "cpu", torch.float32)
    ci, co, wp, sc, sh = w.convs[2]           # block 2 conv1: 64 -> 128
    assert (ci, co) == (64, 128) and wp.shape == (128, 9 * 64)
    x = torch.randn(1, 64, 5, 6)
    ref = torch.nn.functional.conv2d(x, sd["audio_encoder.audio_enc.conv_block2.conv1.weight"], padding=1)
    xn = torch.nn.functional.pad(x, (1, 1, 1, 1)).permute(0, 2, 3, 1)   # NHWC padded
    got = torch.zeros(5, 6, 128)
    for h in range(5):
        for q in range(6):
            patch = xn[0, h:h + 3, q:q + 3, :].reshape(-1)                 # (ky, kx, ci)
            got[h, q] = wp @ patch
    assert torch.allclose(got.permute(2, 0, 1), ref[0], atol=1e-4)
    first = w.convs[0]
    assert first[2].shape == (64, 32)         # 9 taps zero-padded to one 32-deep k-tile


def test_beam_output_ordering():
    """CaptionBatch.beams: order by scores/seq_len descending, truncate to seq_len
    (gpt2_prefix_eval.py:153-158)."""
    from zsaac.pipeline import CaptionBatch
    ids = torch.tensor([[[1, 2, 3, 0], [4, 5, 0, 0], [6, 7, 8, 9]]], dtype=torch.int32)
    ln = torch.tensor([[3.0, 2.0, 4.0]])
    sc = torch.tensor([[-3.0, -1.0, -8.0]])      # averages -1.0, -0.5, -2.0
    cb = CaptionBatch(ids, ln, sc, None, None, None, None, None)
    assert cb.beams() == [[[4, 5], [1, 2, 3], [6, 7, 8, 9]]]
    assert cb.captions() == [[4, 5]]


def test_shard_range_covers_all():
    from zsaac.dist import shard_range
    for n in (1, 7, 1045):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
