"""Real-data harness host pieces, on CPU: GPT-2 BPE against transformers'
own GPT2Tokenizer loaded from the same files, the allow-list unpickler on the reference's data
formats, params.json -> configuration, label-table checks and the output.txt format
(predict_prompt.py:172-181)."""
import json
import os
import pickle

import numpy as np
import pytest
import torch

from zsaac import bpe, predict, safeload
from zsaac import synthetic as S
from zsaac.tokenizer import TEMPLATE_IDS, compose_prompt_text, synthetic_label_names


@pytest.fixture(scope="module")
def vocab_dir(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("gpt2tok"))
    v, m = S.gpt2_vocab(synthetic_label_names())
    bpe.write_vocab(d, v, m)
    return d


TEXTS = ["There are sndaa, sndab, sndzz in this audio.", "There are something in this audio.",
         "a dog barks . a man's car isn't here!", "  spaces   and\ttabs\n", "numbers 123 4.5",
         "unicode: café naïve — 日本", "There are Sndaa in this audio .", "'s 've 're 'll 'd 'm 't"]


def test_bpe_matches_transformers(vocab_dir):
    from transformers import GPT2Tokenizer
    ref = GPT2Tokenizer(os.path.join(vocab_dir, "vocab.json"), os.path.join(vocab_dir, "merges.txt"))
    ours = bpe.GPT2BPE.from_dir(vocab_dir)
    for t in TEXTS:
        assert ours.encode(t) == ref.encode(t), t
    rng = np.random.default_rng(0)
    for _ in range(20):
        ids = rng.integers(0, 50257, size=int(rng.integers(1, 30))).tolist()
        for clean in (False, True):
            assert ours.decode(ids, clean_up_tokenization_spaces=clean) == \
                ref.decode(ids, clean_up_tokenization_spaces=clean)


def test_bpe_template_ids(vocab_dir):
    tok = bpe.GPT2BPE.from_dir(vocab_dir)
    predict.check_template(tok)
    assert tok.encode(".") == [13] and tok.encode(" .") == [764]
    names = synthetic_label_names()[:3]
    whole = tok.encode(compose_prompt_text([n.lower() for n in names]))
    pieces = (TEMPLATE_IDS["There"] + TEMPLATE_IDS[" are"] + tok.encode(" " + names[0]) +
              [11] + tok.encode(" " + names[1]) + [11] + tok.encode(" " + names[2]) +
              TEMPLATE_IDS[" in"] + TEMPLATE_IDS[" this"] + TEMPLATE_IDS[" audio"] + [13])
    assert whole == pieces
    # generate2 output ends with the stop id 764 (" ."): cleaned up like transformers 4.24
    assert tok.decode(tok.encode(" sndaa") + [764]) == " sndaa."


def test_label_table_rejects_merging_labels(vocab_dir, tmp_path):
    tok = bpe.GPT2BPE.from_dir(vocab_dir)
    assert len(predict.label_token_table(tok, synthetic_label_names()[:10])) == 10
    # with a ")," merge (GPT-2 has one), "x)" + "," pre-tokenizes to the one piece "),", whose
    # ids differ from the per-label ids + ","
    v, m = S.gpt2_vocab(synthetic_label_names())
    filler = next(k for k in v if k.startswith("<"))
    v[")" + ","] = v.pop(filler)
    bpe.write_vocab(str(tmp_path), v, m + [(")", ",")])
    tok2 = bpe.GPT2BPE.from_dir(str(tmp_path))
    assert len(predict.label_token_table(tok2, ["bell x"])) == 1
    with pytest.raises(ValueError):
        predict.label_token_table(tok2, ["bell (x)"])


def test_safe_pickle(tmp_path):
    data = [{"audio_embedding": torch.randn(1, 1024), "caption": [{"caption": "A dog"}],
             "audio_id": "a.wav", "text_embedding": np.ones((1, 4), np.float32)}]
    p = tmp_path / "d.pkl"
    with open(p, "wb") as f:
        pickle.dump(data, f)
    got = safeload.load_pickle(str(p))
    assert torch.equal(got[0]["audio_embedding"], data[0]["audio_embedding"])
    assert got[0]["audio_id"] == "a.wav" and np.array_equal(got[0]["text_embedding"], np.ones((1, 4)))
    with open(tmp_path / "two.pkl", "wb") as f:
        pickle.dump([1], f)
        pickle.dump({"caption": "x"}, f)
    assert list(safeload.iter_pickles(str(tmp_path / "two.pkl"))) == [[1], {"caption": "x"}]

    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    with open(tmp_path / "e.pkl", "wb") as f:
        pickle.dump(Evil(), f)
    with pytest.raises(pickle.UnpicklingError):
        safeload.load_pickle(str(tmp_path / "e.pkl"))


def test_params_to_config():
    p = {"mapping_type": "transformer", "prefix_length": 10, "prefix_length_clip": 10,
         "num_layers": 8, "is_rn": True, "normalize_prefix": True, "sound_effect_num": 2}
    cfg = predict.config_from_params(p, True, torch.float32, 16)
    assert (cfg.mapping_type, cfg.beam, cfg.sound_effect_num, cfg.normalize_prefix,
            cfg.mapper_layers, cfg.batch) == ("transformer", 3, 2, True, 8, 16)
    with pytest.raises(NotImplementedError):
        predict.config_from_params(dict(p, is_rn=False), False, torch.float32, 16)


def test_output_format(tmp_path):
    k2p = {"b.wav": ["a dog barks."], "a.wav": ["rain."]}
    k2x = {"b.wav": ["There are x"], "a.wav": ["There are y"]}
    predict.write_outputs(str(tmp_path), k2p, k2x, {})
    out = json.load(open(tmp_path / "output.txt"))
    assert out == {"predictions": [{"filename": "b.wav", "caption": "a dog barks.", "prefix": "There are x"},
                                   {"filename": "a.wav", "caption": "rain.", "prefix": "There are y"}]}
    assert predict.post_processing([{"caption": "A Dog"}, {"caption": "b."}]) == ["a dog.", "b."]


def test_magic_settings_follow_reference_params():
    """predict_prompt.py applies its module-level {'beta': 0.2, 'alpha': 0.1} after params.json
    (lines 19-22, 196-197): a params.json alpha / beta never reaches generate_beam_magic, its
    magic_width does (line 140)."""
    from zsaac.predict import magic_settings
    assert magic_settings({"alpha": 0.5, "beta": 0.9, "magic_width": 30}) == (30, 0.1, 0.2)
    assert magic_settings({}) == (25, 0.1, 0.2)
