"""The real-data harness end to end on the GPU (zsaac.predict = predict_prompt.py): a test_dir with
params.json, best.pth, an AudioSet-format label pickle, a test-data pickle and a GPT-2-format BPE
vocabulary (all synthetic, same file formats as the reference), run through ``predict.main``;
output.txt's captions and prefix strings equal the oracle's reference semantics (whole-string BPE
of the composed prompt, clap_to_gpt, generate2 / generate_beam(3), get_prefix_tokens, decode,
lower-case) in f32 parity mode."""
import json
import os
import pickle

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_CLIPS = 10


def _make_test_dir(root, golden, mapping="mlp"):
    from zsaac import bpe
    from zsaac import synthetic as S
    from zsaac.tokenizer import synthetic_label_names
    sd = S.gpt2_state_dict(seed=0, std=0.1, emb_std=0.1, stop_boost=2.0)
    sd.update(S.mlp_mapper_state_dict(1) if mapping == "mlp" else S.transformer_mapper_state_dict(2))
    torch.save(sd, os.path.join(root, "best.pth"))
    names = synthetic_label_names()
    table = S.label_table()
    labels = [{"label_id": f"/m/{i:05d}", "label": names[i].capitalize(),
               "label_embedding": table[i:i + 1].clone()} for i in range(len(names))]
    with open(os.path.join(root, "audioset_label.pkl"), "wb") as f:
        pickle.dump(labels, f)
    g = golden("c1_greedy.npz")
    clips = [{"audio_embedding": torch.from_numpy(g["clap_emb"][i:i + 1].copy()),
              "caption": [{"caption": f"Reference caption {i}"}], "audio_id": f"clip_{i:03d}.wav",
              "text_embedding": torch.zeros(1, 1024)} for i in range(N_CLIPS)]
    with open(os.path.join(root, "test.pkl"), "wb") as f:
        pickle.dump(clips, f)
    params = {"mapping_type": mapping, "prefix_length": 10, "prefix_length_clip": 10,
              "num_layers": 8, "is_rn": True, "only_prefix": False, "normalize_prefix": True,
              "use_sound_effect": True, "sound_effect": os.path.join(root, "audioset_label.pkl"),
              "sound_effect_num": 3, "device": "cuda"}
    with open(os.path.join(root, "params.json"), "w") as f:
        json.dump(params, f)
    v, m = S.gpt2_vocab(names)
    bpe.write_vocab(os.path.join(root, "tokenizer"), v, m)
    return sd, names, table, clips


@pytest.mark.parametrize("isbeam", [False, True])
def test_predict_harness_matches_oracle(cuda, golden, tmp_path, isbeam):
    from oracle import caption as OC
    from zsaac import bpe, predict
    from zsaac.tokenizer import compose_prompt_text
    root = str(tmp_path)
    sd, names, table, clips = _make_test_dir(root, golden)
    argv = ["--test_dir", root, "--test_data", os.path.join(root, "test.pkl"), "--dtype", "f32",
            "--batch", "4"] + (["--isbeam"] if isbeam else [])
    assert predict.main(argv) == 0
    out = json.load(open(os.path.join(root, "output.txt")))["predictions"]
    assert [p["filename"] for p in out] == [c["audio_id"] for c in clips]
    tok = bpe.GPT2BPE.from_dir(os.path.join(root, "tokenizer"))
    n_check = 4 if isbeam else N_CLIPS
    for c, p in zip(clips[:n_check], out[:n_check]):
        emb = c["audio_embedding"].float()
        idx = OC.sound_effect_choice(emb, table, 3)[0].tolist()
        hard = torch.tensor([tok.encode(compose_prompt_text([names[i].lower() for i in idx]))])
        pe = OC.clap_to_gpt(torch.nn.functional.normalize(emb, dim=-1)[None], hard, sd)
        if isbeam:
            ref = OC.generate_beam(pe, sd, beam_size=3)[0][0]
        else:
            ref = OC.generate2(pe, sd, entry_length=67, use_cache=True)
        assert p["caption"] == tok.decode(ref).lower(), c["audio_id"]
        assert p["prefix"] == tok.decode(OC.prefix_tokens(pe, sd)), c["audio_id"]


def test_predict_harness_magic(cuda, golden, tmp_path):
    """--magic: the harness output equals the oracle's generate_beam_magic(beam 3, width 25) best
    beam (f32), with the CLAP checkpoint and BERT vocabulary read from files like the reference."""
    from oracle import caption as OC
    from oracle import magic as OM
    from transformers import BertTokenizer
    from zsaac import bpe, predict
    from zsaac import synthetic as S
    from zsaac.tokenizer import compose_prompt_text
    root = str(tmp_path)
    sd, names, table, clips = _make_test_dir(root, golden)
    bsd = S.bert_state_dict(layers=2)
    torch.save({"model": dict(bsd)}, os.path.join(root, "clap.pt"))
    vocab = S.bert_vocab()
    with open(os.path.join(root, "vocab.txt"), "w") as f:
        f.write("\n".join(vocab) + "\n")
    argv = ["--test_dir", root, "--test_data", os.path.join(root, "test.pkl"), "--dtype", "f32",
            "--batch", "4", "--magic", "--clap", os.path.join(root, "clap.pt"),
            "--bert_vocab", os.path.join(root, "vocab.txt")]
    assert predict.main(argv) == 0
    out = json.load(open(os.path.join(root, "output.txt")))["predictions"]
    tok = bpe.GPT2BPE.from_dir(os.path.join(root, "tokenizer"))
    btok = BertTokenizer(vocab={t: i for i, t in enumerate(vocab)}, do_lower_case=True)
    enc = OM.text_encoder(btok, bsd, 2)
    for c, p in zip(clips[:2], out[:2]):
        emb = c["audio_embedding"].float()
        idx = OC.sound_effect_choice(emb, table, 3)[0].tolist()
        hard = torch.tensor([tok.encode(compose_prompt_text([names[i].lower() for i in idx]))])
        pref = torch.nn.functional.normalize(emb, dim=-1)
        pe = OC.clap_to_gpt(pref[None], hard, sd)
        outs, _ = OM.generate_beam_magic(pe, sd, tok.decode, enc, pref, float(bsd["temp"]),
                                         beam_size=3, entry_length=20, magic_width=25)
        assert p["caption"] == tok.decode(outs[0]).lower(), c["audio_id"]
