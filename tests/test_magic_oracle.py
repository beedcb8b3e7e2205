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


def test_tokenize_pieces_equals_full_tokenization():
    """The magic decoder's candidate-text tokenisation (prefix up to the head's last space + cached
    rests, zsaac.bert.tokenize_pieces) gives exactly the ids / lengths of the reference's
    ``tokenizer(texts, padding='longest', truncation=True, max_length=30)`` call on the full
    texts, including word-continuing pieces ('q<id>'), punctuation, empty heads and truncation."""
    import random
    import torch
    from transformers import BertTokenizer
    from zsaac import synthetic as S
    from zsaac.bert import tokenize, tokenize_pieces
    from zsaac.magic import MagicDecoder
    from zsaac.tokenizer import WordTokenizer
    tok = BertTokenizer(vocab={t: i for i, t in enumerate(S.bert_vocab())}, do_lower_case=True)
    wt = WordTokenizer()
    rnd = random.Random(0)
    C, b, W = 3, 2, 7
    for s in (0, 1, 4, 19, 40):
        tok_h = torch.tensor([[rnd.choice([rnd.randrange(50000), 13, 11, 764, 5 * rnd.randrange(9000)])
                               for _ in range(s)] for _ in range(C * b)], dtype=torch.int32)
        cand = torch.tensor([rnd.choice([rnd.randrange(50000), 13, 11, 764, 5 * rnd.randrange(9000)])
                             for _ in range(C * b * W)], dtype=torch.int32)
        pieces = MagicDecoder._texts(None, wt, cand, tok_h, C, b, W, s)
        full = [wt.decode(tok_h[j // W, :s].tolist() + [int(cand[j])]) for j in range(C * b * W)]
        assert [p + r for p, r in pieces] == full
        for L in (30, 8):
            i1, l1 = tokenize(tok, full, L, "cpu")
            i2, l2 = tokenize_pieces(tok, pieces, L, "cpu")
            assert torch.equal(i1, i2) and torch.equal(l1, l2), (s, L)
