"""GPU: the reference-shaped drop-in API (models.caption_model, models.mapper,
gpt2_prefix_eval, retrieval.models.ase_model) driven exactly like predict_prompt.py:129-144 /
embeddings_generator.py:63, checked against the reference goldens (f32 parity mode)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GPT2_KW = dict(seed=0, std=0.1, emb_std=0.1, stop_boost=2.0)


class _PrefixTok:
    def encode(self, s):
        return [13]

    def decode(self, ids):
        if isinstance(ids, int):
            ids = [ids]
        return "".join(f"{int(i)}|" for i in ids)


@pytest.fixture(scope="module")
def model(cuda):
    from models.caption_model import ClapCaption_prompt
    from zsaac import synthetic as S
    m = ClapCaption_prompt(10, clip_length=10, prefix_size=1024, num_layers=8, mapping_type="mlp")
    sd = S.gpt2_state_dict(**GPT2_KW)
    sd.update(S.mlp_mapper_state_dict(1))
    m.load_state_dict(sd)
    return m.to(cuda).eval()


def test_predict_loop_greedy(cuda, golden, model):
    import gpt2_prefix_eval as G
    from zsaac.tokenizer import IdTokenizer
    g = golden("c1_greedy.npz")
    embeddings = torch.nn.functional.normalize(model.gpt.get_input_embeddings().weight.data, 2, 1)
    for clip in (0, 3):
        n = int(g["hard_len"][clip])
        prefix = torch.nn.functional.normalize(torch.from_numpy(g["clap_emb"][clip:clip + 1]), dim=-1)
        prefix = prefix[None].to(cuda)                             # [1,1,1024] as collate() builds
        hard = torch.from_numpy(g["hard_ids"][clip:clip + 1, :n]).to(cuda)
        emb_h = model.gpt.transformer.wte(hard)                    # predict_prompt.py:133
        with torch.no_grad():
            pe, _ = model.clap_to_gpt(prefix, emb_h)               # :136
            ps = G.get_prefix_tokens(pe, embeddings, _PrefixTok())   # :137
        assert [int(t) for t in ps[0].split("|") if t] == g["prefix_tokens"][clip, :n + 10].tolist()
        if clip < g["prefix_embed"].shape[0]:
            assert float((pe[0].cpu() - torch.from_numpy(g["prefix_embed"][clip, :n + 10])).abs().max()) < 1e-5
        out = G.generate2(model, IdTokenizer(), embed=pe)          # :144
        assert [int(t) for t in out.split()] == g["greedy_ids"][clip, :g["greedy_len"][clip]].tolist()


def test_generate_beam_dropin(cuda, golden, model):
    import gpt2_prefix_eval as G
    from zsaac.tokenizer import IdTokenizer
    g = golden("beam.npz")
    c = 1
    n = int(g["hard_len"][c])
    hard = torch.from_numpy(g["hard_ids"][c:c + 1, :n]).to(cuda)
    with torch.no_grad():
        pe, _ = model.clap_to_gpt(torch.from_numpy(g["clap_emb"][c:c + 1])[None].to(cuda),
                                  model.gpt.transformer.wte(hard))
    texts = G.generate_beam(model, IdTokenizer(), beam_size=3, embed=pe)
    ref = [g["beam3_ids"][c, i, :g["beam3_len"][c, i]].tolist() for i in range(3)]
    assert [[int(t) for t in s.split()] for s in texts] == ref


@pytest.mark.parametrize("tag,T", [("t07", 0.7), ("t16", 1.6)])
def test_generate_temperature_dropin(cuda, golden, model, tag, T):
    """generate_beam / generate2 with temperature != 1 (the LM head divides the logits before the
    top-k and the softmax statistics) against the reference's own outputs (temperature.npz)."""
    import gpt2_prefix_eval as G
    from zsaac.tokenizer import IdTokenizer
    g = golden("temperature.npz")
    E = int(g["entry_length"])
    for c in range(g["clap_emb"].shape[0]):
        n = int(g["hard_len"][c])
        hard = torch.from_numpy(g["hard_ids"][c:c + 1, :n]).to(cuda)
        with torch.no_grad():
            pe, _ = model.clap_to_gpt(torch.from_numpy(g["clap_emb"][c:c + 1])[None].to(cuda),
                                      model.gpt.transformer.wte(hard))
        texts = G.generate_beam(model, IdTokenizer(), beam_size=3, embed=pe, entry_length=E,
                                temperature=T)
        ref = [g[f"beam3_{tag}_ids"][c, i, :g[f"beam3_{tag}_len"][c, i]].tolist() for i in range(3)]
        assert [[int(t) for t in s.split()] for s in texts] == ref, (tag, c)
        if tag == "t07":
            out = G.generate2(model, IdTokenizer(), embed=pe, entry_length=E, temperature=0.7)
            assert [int(t) for t in out.split()] == g["greedy_t07_ids"][c, :g["greedy_t07_len"][c]].tolist()


def test_gpt_full_logits(cuda, golden, model):
    from oracle import caption as OC
    from zsaac import synthetic as S
    g = golden("c1_greedy.npz")
    pe = torch.from_numpy(g["prefix_embed"][0, :int(g["hard_len"][0]) + 10])[None]
    got = model.gpt(inputs_embeds=pe.to(cuda), output_hidden_states=True).logits.cpu()
    sd = S.gpt2_state_dict(**GPT2_KW)
    with torch.no_grad():
        ref = OC.gpt2_logits(pe, sd)[0]
    assert float((got - ref).abs().max() / ref.abs().max()) < 1e-4


def test_ase_encode_audio(cuda):
    from oracle import audio as A, frontend as OF
    from retrieval.models.ase_model import ASE
    from zsaac import synthetic as S
    cfg = {"audio_args": {"sr": 32000, "n_fft": 1024, "hop_length": 320, "f_min": 50, "f_max": 14000,
                          "n_mels": 64, "max_length": 10, "mono": True},
           "audio_encoder_args": {"type": "transformer", "pretrained": False, "freeze": False},
           "training": {"spec_augmentation": True}, "embed_size": 1024}
    ase = ASE(cfg)
    sd = ase.state_dict()
    sd.update(S.htsat_state_dict(3))
    sd.update(S.audio_proj_state_dict(5))
    ase.load_state_dict(sd)
    ase = ase.to(cuda).eval()
    wav = S.synthetic_waveforms(2)
    got = ase.encode_audio(wav.to(cuda)).cpu()
    with torch.no_grad():
        ref = A.audio_project(A.htsat_embedding(OF.logmel(wav), sd), sd)
    assert float((got - ref).abs().max()) < 2e-3


def test_extract_embeddings_ragged(cuda):
    """Extract_embeddings semantics (embeddings_generator.py:53-59): a 25 s clip is cropped to
    its first 10 s, a 4 s clip zero-padded, an empty clip skipped; embeddings equal the encoder on
    the cropped / padded waveforms and the oracle within the bf16 bound; records as the
    reference's data.pkl."""
    from oracle import audio as A, frontend as OF
    from zsaac import synthetic as S
    from zsaac.extract import EmbeddingExtractor
    asd = S.htsat_state_dict(3)
    asd.update(S.audio_proj_state_dict(5))
    g = torch.Generator(device="cpu").manual_seed(25)
    clips = [(torch.randn(800000, generator=g) * 0.1).clamp(-1, 1), torch.zeros(0),
             (torch.randn(128000, generator=g) * 0.1).clamp(-1, 1)]
    ex = EmbeddingExtractor(asd, "htsat", torch.bfloat16, batch=4, device=cuda)
    recs = ex.extract(clips, ["a", "empty", "c"], [["cap a"], ["x"], ["cap c"]])
    assert [r["audio_id"] for r in recs] == ["a", "c"]
    fitted = torch.stack([clips[0][:320000], torch.nn.functional.pad(clips[2], [0, 192000])])
    direct = ex.enc.encode(fitted.to(cuda)).cpu()
    got = torch.cat([r["audio_embedding"] for r in recs])
    assert torch.equal(got, direct)
    with torch.no_grad():
        ref = A.audio_project(A.htsat_embedding(OF.logmel(fitted), asd), asd)
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    assert float(cos.min()) > 0.995, cos
