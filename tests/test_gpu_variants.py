"""The other caption-model classes of models/caption_model.py on the HIP kernels, against
goldens from the reference (tests/golden/variants.npz): ClapCaptionModel with the sound-effect
MLP tokens, ClapCaptionCrossattention, ClapCaptionCrossattention_v2 (eval) and
ClapCaptionPrefix.  f32 parity mode: clap_to_gpt outputs within 1e-5 (relative to the largest
element) and generate2 ids bit-exact; bf16 perf mode: clap_to_gpt within 3e-2."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GPT2_KW = dict(seed=0, std=0.1, emb_std=0.1, stop_boost=2.0)


def _model(name, cuda):
    import models.caption_model as CM
    from zsaac import synthetic as S
    table = S.label_table().to(cuda)
    sd = S.gpt2_state_dict(**GPT2_KW)
    sd.update(S.mlp_mapper_state_dict(1))
    kw = dict(prefix_size=1024, mapping_type="mlp")
    if name == "se_mlp":
        m = CM.ClapCaptionModel(10, sound_effect_embeddings=table, sound_effect_num=3, **kw)
        sd.update(S.sound_effect_mlp_state_dict(11))
    elif name == "prefix":
        m = CM.ClapCaptionPrefix(10, **kw)
    else:
        cls = CM.ClapCaptionCrossattention if name == "xattn" else CM.ClapCaptionCrossattention_v2
        m = cls(10, sound_effect_embeddings=table, sound_effect_num=3, **kw)
        sd.update(S.sound_effect_mha_state_dict(12))
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected and all("attn.bias" in k or "masked_bias" in k for k in missing)
    return m.to(cuda).eval()


@pytest.mark.parametrize("name", ["se_mlp", "xattn", "xattn_v2", "prefix"])
def test_caption_variant(cuda, golden, name):
    import gpt2_prefix_eval as G
    from zsaac.tokenizer import IdTokenizer
    g = golden("variants.npz")
    m = _model(name, cuda)
    prefix = torch.from_numpy(g["prefix"]).to(cuda)
    tokens = torch.from_numpy(g["tokens"]).to(cuda)
    with torch.no_grad():
        cat, _ = m.clap_to_gpt(prefix, m.gpt.transformer.wte(tokens))
    ref = g[f"{name}_cat"]
    got = cat.float().cpu().numpy()
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max(), name
    ids = g[f"{name}_ids"]
    for i in range(prefix.shape[0]):
        with torch.no_grad():
            pe, _ = m.clap_to_gpt(prefix[i:i + 1])
            out = G.generate2(m, IdTokenizer(), embed=pe, entry_length=int(g["entry_length"]))
        assert [int(t) for t in out.split()] == ids[i, :g[f"{name}_len"][i]].tolist(), (name, i)
    # bf16 perf mode of the same module
    m.set_dtype(torch.bfloat16)
    with torch.no_grad():
        cat16, _ = m.clap_to_gpt(prefix, m.gpt.transformer.wte(tokens))
    assert np.abs(cat16.float().cpu().numpy() - ref).max() <= 3e-2 * np.abs(ref).max(), name
