"""GPU: CLAP-guided ("magic") decoding and the CLAP text tower on the HIP kernels against the
reference goldens (tests/golden/magic.npz from gpt2_prefix_eval.py:341-689 and ASE.encode_text;
see tests/test_magic_oracle.py for the oracle pinned to the same fixtures).

f32 parity mode: token ids bit-exact (every beam, in order) for all three (beam, width, alpha,
beta, entry_length, stop boost) configurations and magic_search; text embeddings within 1e-4.
bf16 perf mode: text embeddings cosine >= 0.99 and the decode runs end to end (ids reported)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bert_tokenizer():
    from transformers import BertTokenizer
    from zsaac import synthetic as S
    return BertTokenizer(vocab={t: i for i, t in enumerate(S.bert_vocab())}, do_lower_case=True)


def _texts():
    from zsaac.tokenizer import WordTokenizer
    return [WordTokenizer().decode(t) for t in ([5, 123, 13], [7], [1000, 2005, 3, 11, 764, 49999, 50000],
                                                list(range(100, 140)), [30000, 30001, 30010])]


@pytest.fixture(scope="module")
def gold(golden):
    return golden("magic.npz")


def _clap(cuda, layers, dtype):
    from retrieval.models.ase_model import ASE
    from zsaac import synthetic as S
    cfg = {"audio_args": {"sr": 32000, "n_fft": 1024, "hop_length": 320, "f_min": 50,
                          "f_max": 14000, "n_mels": 64, "max_length": 10, "mono": True},
           "audio_encoder_args": {"type": "transformer", "model": "Cnn14", "pretrained": False,
                                  "freeze": False},
           "embed_size": 1024, "temp": 0.07,
           "text_encoder_args": {"type": "bert-base-uncased", "freeze": False,
                                 "vocab": {t: i for i, t in enumerate(S.bert_vocab())},
                                 "vocab_size": len(S.bert_vocab()), "num_layers": layers}}
    clap = ASE(cfg)
    sd = S.bert_state_dict(layers=layers)
    missing, unexpected = clap.load_state_dict(sd, strict=False)
    assert not unexpected and all(m.startswith("audio") for m in missing)
    clap.zs_dtype = dtype
    return clap.to(cuda).eval()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_encode_text_vs_reference(cuda, gold, dtype):
    clap = _clap(cuda, int(gold["bert_layers"]), dtype)
    got = clap.encode_text(_texts()).cpu()
    ref = torch.from_numpy(gold["text_emb"])
    if dtype == torch.float32:
        assert float((got - ref).abs().max()) < 1e-4
    else:
        cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
        assert float(cos.min()) > 0.99, cos


def _engine(cuda, gold, dtype, stop_boost, beam, width, steps, C):
    from zsaac import synthetic as S
    from zsaac.decoder import Gpt2Weights
    from zsaac.magic import MagicDecoder
    csd = S.gpt2_state_dict(seed=0, std=0.1, emb_std=0.1, stop_boost=stop_boost)
    w = Gpt2Weights(csd, cuda, dtype)
    clap = _clap(cuda, int(gold["bert_layers"]), dtype)
    H = gold["hard_ids"].shape[1]
    return MagicDecoder(w, clap.text_engine(), C, H + 10, beam=beam, width=width,
                        max_steps=steps), clap, csd


def _inputs(cuda, gold, csd):
    from oracle import caption as OC
    from zsaac import synthetic as S
    sd = dict(csd)
    sd.update(S.mlp_mapper_state_dict(1))
    emb = torch.from_numpy(gold["clap_emb"])
    soft = OC.mlp_mapper(emb, sd).view(-1, 10, 768)           # clap_to_gpt's projection rows
    hard = torch.from_numpy(gold["hard_ids"]).clamp(min=0).to(torch.int32)
    hl = torch.from_numpy(gold["hard_len"]).to(torch.int32)
    return hard.to(cuda), hl.to(cuda), soft.contiguous().to(cuda), emb.to(cuda)


@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_generate_beam_magic_f32_bit_exact(cuda, gold, cfg):
    from zsaac.tokenizer import WordTokenizer
    beam, width, alpha, beta, entry, boost = gold["cfgs"][cfg]
    beam, width, entry = int(beam), int(width), int(entry)
    C = gold["clap_emb"].shape[0]
    eng, clap, csd = _engine(cuda, gold, torch.float32, float(boost), beam, width, entry, C)
    hard, hl, soft, emb = _inputs(cuda, gold, csd)
    res = eng.beam_magic(hard, hl, soft, 10, emb, WordTokenizer(), clap.text_encoder.tokenizer,
                         beam, width, entry, alpha, beta, float(clap.temp))
    ids, ln = gold[f"beam_cfg{cfg}_ids"], gold[f"beam_cfg{cfg}_len"]
    for k, (toks, _) in enumerate(res):
        for b in range(beam):
            assert toks[b] == ids[k, b, :ln[k, b]].tolist(), (cfg, k, b)


def test_magic_search_f32_bit_exact(cuda, gold):
    from zsaac.tokenizer import WordTokenizer
    C = gold["clap_emb"].shape[0]
    eng, clap, csd = _engine(cuda, gold, torch.float32, 2.0, 1, 15, 12, C)
    hard, hl, soft, emb = _inputs(cuda, gold, csd)
    P = hl.cpu() + 10
    # the goldens ran magic_search(decoding_len = P + 10) per clip: 10 steps each
    outs = []
    for k in range(C):
        r = eng.search(hard[k:k + 1], hl[k:k + 1], soft[k:k + 1], 10, emb[k:k + 1], WordTokenizer(),
                       clap.text_encoder.tokenizer, width=15, decoding_len=int(P[k]) + 10,
                       alpha=0.1, beta=0.2, temp=float(clap.temp))
        outs.append(r[0])
    for k in range(C):
        assert outs[k] == gold["search_ids"][k, :gold["search_len"][k]].tolist(), k


def test_dropin_generate_beam_magic(cuda, gold):
    """gpt2_prefix_eval.generate_beam_magic / magic_search called like predict_prompt.py:140."""
    import gpt2_prefix_eval as G
    from models.caption_model import ClapCaption_prompt
    from zsaac import synthetic as S
    from zsaac.tokenizer import WordTokenizer
    m = ClapCaption_prompt(10, clip_length=10, prefix_size=1024, num_layers=8, mapping_type="mlp")
    sd = S.gpt2_state_dict(seed=0, std=0.1, emb_std=0.1, stop_boost=2.0)
    sd.update(S.mlp_mapper_state_dict(1))
    m.load_state_dict(sd)
    m = m.to(cuda).eval()
    clap = _clap(cuda, int(gold["bert_layers"]), torch.float32)
    k = 1
    n = int(gold["hard_len"][k])
    emb = torch.from_numpy(gold["clap_emb"][k:k + 1]).to(cuda)
    hard = torch.from_numpy(gold["hard_ids"][k:k + 1, :n]).to(cuda)
    with torch.no_grad():
        pe, _ = m.clap_to_gpt(emb[None], m.gpt.transformer.wte(hard))
    beam, width, alpha, beta, entry, _ = gold["cfgs"][0]
    texts = G.generate_beam_magic(m, clap, WordTokenizer(), audio_embeds=emb[None], embed=pe,
                                  beam_size=int(beam), magic_width=int(width), alpha=alpha,
                                  beta=beta, entry_length=int(entry))
    ref = gold["beam_cfg0_ids"][k]
    assert [WordTokenizer.parse(t) for t in texts] == [ref[b, :gold["beam_cfg0_len"][k, b]].tolist()
                                                        for b in range(int(beam))]
    out = G.magic_search(m, WordTokenizer(), emb, clap, embed=pe, beam_width=15,
                         decoding_len=pe.shape[1] + 10)
    assert WordTokenizer.parse(out) == gold["search_ids"][k, :gold["search_len"][k]].tolist()


def test_generate_beam_magic_bf16_runs(cuda, gold):
    """bf16 perf mode end to end: the same clips decode, every beam has entry_length tokens or
    ends on '.', and the first chosen token matches the f32 reference on most clips."""
    from zsaac.tokenizer import WordTokenizer
    beam, width, alpha, beta, entry, boost = gold["cfgs"][0]
    beam, width, entry = int(beam), int(width), int(entry)
    C = gold["clap_emb"].shape[0]
    eng, clap, csd = _engine(cuda, gold, torch.bfloat16, float(boost), beam, width, entry, C)
    hard, hl, soft, emb = _inputs(cuda, gold, csd)
    res = eng.beam_magic(hard, hl, soft, 10, emb, WordTokenizer(), clap.text_encoder.tokenizer,
                         beam, width, entry, alpha, beta, float(clap.temp))
    ids = gold["beam_cfg0_ids"]
    first = 0
    for k, (toks, sc) in enumerate(res):
        assert len(toks) == beam and all(np.isfinite(sc))
        for t in toks:
            assert len(t) == entry or t[-1] == 13
        first += toks[0][0] == ids[k, 0, 0]
    print(f"bf16 magic: first token equal on {first}/{C} clips")
    assert first >= C - 1


def test_row_topk_kernel(cuda):
    from zsaac import ops
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(7, 50257, generator=g) * 3
    xd = x.to(cuda)
    for mode in (0, 1):
        v = torch.empty(7, 25, device=cuda)
        i = torch.empty(7, 25, device=cuda, dtype=torch.int32)
        ops.row_topk(xd, 25, v, i, mode=mode)
        rv, ri = torch.topk(x, 25, dim=-1)
        assert torch.equal(i.cpu().long(), ri)
        ref = (x.log_softmax(-1) if mode == 0 else x.softmax(-1)).gather(1, ri)
        assert float((v.cpu() - ref).abs().max()) < 1e-5
