"""Host-side weight packing of the grid decode (CPU): the MFMA fragment orders the kernels read
(decode_grid.hip ldw): bf16 [N/16][K/32][64][8] and f32 [N/16][K/16][64][4], rows past N zero."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))


def test_pack_f32_fragments_layout():
    from zsaac import ops
    g = torch.Generator().manual_seed(0)
    N, K = 40, 64
    W = torch.randn(N, K, generator=g)
    P = ops.pack_f32_fragments(W)
    assert P.shape == (3, K // 16, 64, 4)
    for j in range(3):
        for s in range(K // 16):
            for lane in (0, 5, 17, 38, 63):
                row, k0 = 16 * j + lane % 16, 16 * s + 4 * (lane // 16)
                want = W[row, k0:k0 + 4] if row < N else torch.zeros(4)
                assert torch.equal(P[j, s, lane], want), (j, s, lane)


def test_pack_b_fragments_layout():
    from zsaac import ops
    g = torch.Generator().manual_seed(1)
    N, K = 24, 64
    W = torch.randn(N, K, generator=g).bfloat16()
    P = ops.pack_b_fragments(W)
    assert P.shape == (2, K // 32, 64, 8)
    for j in range(2):
        for s in range(K // 32):
            for lane in (0, 9, 31, 50, 63):
                row, k0 = 16 * j + lane % 16, 32 * s + 8 * (lane // 16)
                want = W[row, k0:k0 + 8] if row < N else torch.zeros(8, dtype=torch.bfloat16)
                assert torch.equal(P[j, s, lane], want), (j, s, lane)


def test_pack_f32_folds_layernorm_affine():
    """Gpt2Weights._pack_f32 (the f32 grid decode's tables): c_attn / c_fc carry the LayerNorm
    weight folded into W (f32) and beta into the bias (b + W beta, summed in f64), ln_f folds into
    the tied head plus a per-token bias; the projections are packed unchanged.  Checked through the
    algebra LN(x) W^T + b == ((x - mean) rstd) W'^T + b' on random rows (float64)."""
    from zsaac import decoder as dec
    from zsaac import ops
    g = torch.Generator().manual_seed(2)
    D, N, V = 32, 48, 40
    w = object.__new__(dec.Gpt2Weights)
    r = lambda *s: torch.randn(*s, generator=g)
    w.layers = [{"attn_w": r(N, D), "attn_b": r(N), "ln1": (1 + 0.1 * r(D), 0.1 * r(D)),
                 "proj_w": r(D, D), "proj_b": r(D),
                 "fc_w": r(N, D), "fc_b": r(N), "ln2": (1 + 0.1 * r(D), 0.1 * r(D)),
                 "mproj_w": r(D, N), "mproj_b": r(D)} for _ in range(2)]
    w.wte = r(V, D)
    w.lnf = (1 + 0.1 * r(D), 0.1 * r(D))
    w.V = V
    w._pack_f32()

    def unpack(P, n, k):
        return P.view(P.shape[0], k // 16, 4, 16, 4).permute(0, 3, 1, 2, 4).reshape(-1, k)[:n]

    x = r(5, D).double()
    mean = x.mean(1, keepdim=True)
    xn = (x - mean) / torch.sqrt(((x - mean) ** 2).mean(1, keepdim=True) + 1e-5)
    for ly, pk in zip(w.layers, w._packed):
        for wk, bk, lk in (("attn_w", "attn_b", "ln1"), ("fc_w", "fc_b", "ln2")):
            W, b, (gam, beta) = ly[wk].double(), ly[bk].double(), ly[lk]
            Wp = unpack(pk[wk], W.shape[0], D).double()
            assert torch.equal(unpack(pk[wk], W.shape[0], D), ly[wk] * gam[None, :])
            ref = (xn * gam.double() + beta.double()) @ W.t() + b
            got = xn @ Wp.t() + pk[bk].double()
            assert torch.allclose(got, ref, rtol=1e-5, atol=1e-5)
        assert torch.equal(unpack(pk["proj_w"], D, D), ly["proj_w"])
        assert torch.equal(unpack(pk["mproj_w"], D, N), ly["mproj_w"])
    gam, beta = w.lnf
    logits = (xn * gam.double() + beta.double()) @ w.wte.double().t()
    got = xn @ unpack(w._wte_packed, V, D).double().t() + w._lm_bias[:V].double()
    assert torch.allclose(got, logits, rtol=1e-5, atol=1e-5)
    assert w._lm_bias.numel() == 16 * ((V + 15) // 16)
