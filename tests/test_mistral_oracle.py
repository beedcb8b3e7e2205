"""oracle/mistral.py pinned to the reference's C5 Mistral caption path goldens
(tests/golden/mistral.npz: ClapCaption_Mistralai_prompt.clap_to_gpt + MistralForCausalLM.generate
as predict_mistralai_multilingual.py:97-111 run them)."""
import numpy as np
import torch

from oracle import mistral as OM
from zsaac import synthetic as S


def _strip(row, eos=2):
    row = [int(t) for t in row]
    if eos in row:
        row = row[:row.index(eos) + 1]
    return row


def test_mistral_generate_vs_reference(golden):
    g = golden("mistral.npz")
    sd = S.mistral_state_dict()
    mlp = S.mlp_mapper_state_dict(31, prefix_length=10, d=1024)
    emb = torch.from_numpy(g["clap_emb"])[:, None]
    hard = torch.from_numpy(g["hard_ids"])
    for tag in ("en", "fr"):
        pe, _ = OM.clap_to_gpt(emb, hard, torch.from_numpy(g[f"tag_{tag}"]), sd, mlp)
        got = OM.generate(pe, sd, 8, 2, 1e-5)
        ref = g[f"ids_{tag}"]
        for b in range(ref.shape[0]):
            assert got[b] == _strip(ref[b]), (tag, b)
