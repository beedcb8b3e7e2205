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


def test_fp8_pack_tiles_layout():
    """zs_fp8_gemm_rows' weight layout (include/zsaac.h): block (split s, tile t, group w, k block j),
    lane l = W[128 t + 16 w + (l & 15)][1024 s + 64 j + 16 (l >> 4) .. +16], rows past N zero."""
    import torch
    from zsaac.mistral import fp8_pack_tiles
    N, K = 200, 2048
    q = torch.randint(0, 255, (N, K), dtype=torch.uint8, generator=torch.Generator().manual_seed(0))
    p = fp8_pack_tiles(q)
    NT = 2
    assert p.numel() == NT * 128 * K
    blk = p.view(K // 1024, NT, 8, 16, 64, 16)
    for n, k in [(0, 0), (17, 1000), (127, 1023), (128, 1024), (199, 2047), (250, 77)]:
        s, kk = divmod(k, 1024)
        j, r = divmod(kk, 64)
        g, b = divmod(r, 16)
        t, nn = divmod(n, 128)
        w, fr = divmod(nn, 16)
        assert int(blk[s, t, w, j, 16 * g + fr, b]) == (int(q[n, k]) if n < N else 0)
