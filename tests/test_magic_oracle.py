"""oracle/magic.py pinned to the reference's CLAP-guided decoding goldens (tests/golden/magic.npz,
made by tests/golden/make_goldens.py from gpt2_prefix_eval.py:341-689 and the ASE text tower)."""
import os

import numpy as np
import pytest
import torch

from oracle import caption as OC
from oracle import magic as OM
from zsaac import synthetic as S
from zsaac.tokenizer import WordTokenizer

G = os.path.join(os.path.dirname(__file__), "golden", "magic.npz")


def bert_tokenizer():
    from transformers import BertTokenizer
    return BertTokenizer(vocab={t: i for i, t in enumerate(S.bert_vocab())}, do_lower_case=True)


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(G))


@pytest.fixture(scope="module")
def sds(gold):
    csd = S.gpt2_state_dict(seed=0, std=0.1, emb_std=0.1, stop_boost=2.0)
    csd.update(S.mlp_mapper_state_dict(1))
    return csd, S.bert_state_dict(layers=int(gold["bert_layers"]))


def _embed(gold, csd, i):
    h = gold["hard_ids"][i, :gold["hard_len"][i]]
    emb = torch.from_numpy(gold["clap_emb"][i:i + 1])
    return OC.clap_to_gpt(emb.unsqueeze(0), torch.from_numpy(h)[None], csd), emb


def test_encode_text_vs_reference(gold, sds):
    tok = bert_tokenizer()
    texts = [WordTokenizer().decode(t) for t in ([5, 123, 13], [7], [1000, 2005, 3, 11, 764, 49999, 50000],
                                                 list(range(100, 140)), [30000, 30001, 30010])]
    got = OM.text_encoder(tok, sds[1], int(gold["bert_layers"]))(texts)
    ids = tok(texts, padding="longest", truncation=True, max_length=30)["input_ids"]
    for i, r in enumerate(ids):
        assert r == [t for t in gold["text_ids"][i] if t >= 0]
    assert (got - torch.from_numpy(gold["text_emb"])).abs().max() < 1e-5


@pytest.mark.parametrize("cfg,clip", [(1, 0), (2, 2)])
def test_generate_beam_magic_vs_reference(gold, sds, cfg, clip):
    bsd = sds[1]
    beam, width, alpha, beta, entry, boost = gold["cfgs"][cfg]
    csd = S.gpt2_state_dict(seed=0, std=0.1, emb_std=0.1, stop_boost=float(boost))
    csd.update(S.mlp_mapper_state_dict(1))
    enc = OM.text_encoder(bert_tokenizer(), bsd, int(gold["bert_layers"]))
    pe, emb = _embed(gold, csd, clip)
    outs, _ = OM.generate_beam_magic(pe, csd, WordTokenizer().decode, enc, emb, float(bsd["temp"]),
                                     beam_size=int(beam), entry_length=int(entry),
                                     magic_width=int(width), alpha=alpha, beta=beta)
    ref = gold[f"beam_cfg{cfg}_ids"][clip]
    for b, o in enumerate(outs):
        assert o == [t for t in ref[b][:gold[f"beam_cfg{cfg}_len"][clip, b]]]


def test_magic_search_vs_reference(gold, sds):
    csd, bsd = sds
    enc = OM.text_encoder(bert_tokenizer(), bsd, int(gold["bert_layers"]))
    pe, emb = _embed(gold, csd, 1)
    ids = OM.magic_search(pe, csd, WordTokenizer().decode, enc, emb, float(bsd["temp"]),
                          beam_width=15, decoding_len=pe.shape[1] + 10)
    assert ids == gold["search_ids"][1, :gold["search_len"][1]].tolist()
