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
