#!/usr/bin/env python3
"""Numerics check of the grid decode against the per-step bf16 kernels: from the same state after
step 0, ONE decode step through the grid decode's phase launches and one through the per-step
kernel chain (zs_gemm_ln / zs_gemm / zs_decode_attention / zs_lmhead_topk); per layer the new K and
V rows, the final residual x (grid decode: its bf16 copy) and the ids.  Differences should be
bf16-rounding sized (~1e-2 relative at most), never structural.

    python tools/dg_check.py [golden=c2_margin]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402


def main():
    from tools import idparity
    from tests.test_gpu_persist import _pipe
    name = sys.argv[1] if len(sys.argv) > 1 else "c2_margin"
    g = idparity.load(name)
    dev = torch.device("cuda", 0)
    emb = torch.from_numpy(g["clap_emb"]).to(dev)
    B = emb.shape[0]
    p = _pipe(g, dev, False, entry_length=3)
    d = p.decoder
    p.begin_emb(emb)          # prefill + step 0 (+ host state); nothing decoded past step 0 yet
    torch.cuda.synchronize()
    state = [t.clone() for t in d._state()]
    kv = [t.clone() for t in d.kc + d.vc]
    pos = d.pos[:B].long().clone()
    R = B

    def restore():
        for t, v in zip(d._state(), state):
            t.copy_(v)
        for t, v in zip(d.kc + d.vc, kv):
            t.copy_(v)
    # grid decode, one step (phase launches)
    restore()
    d._greedy_step_body(R)
    torch.cuda.synchronize()
    base = d.persist_ws.data_ptr()
    ws = d.persist_ws[(-base) % 256:]
    xb = ws[4096 + 2 * 98304: 4096 + 3 * 98304].view(torch.bfloat16).view(4, 24, 64, 8)
    # fragment order -> [64][768]: (rb, s, lane, e) -> row 16 rb + lane % 16, col 32 s + 8 (lane // 16) + e
    x_grid = xb.view(4, 24, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(64, 768)[:B].float()
    k_grid = [d.kc[l][torch.arange(B), :, pos].float().clone() for l in range(12)]
    v_grid = [d.vc[l][torch.arange(B), :, pos].float().clone() for l in range(12)]
    ids_grid = d.next_tok[:B].clone()
    # the per-step kernels
    restore()
    d.grid_decode = False
    d._greedy_step_body(R)
    torch.cuda.synchronize()
    x_old = d.x[:B].float().clone()
    k_old = [d.kc[l][torch.arange(B), :, pos].float().clone() for l in range(12)]
    v_old = [d.vc[l][torch.arange(B), :, pos].float().clone() for l in range(12)]
    ids_old = d.next_tok[:B].clone()
    d.grid_decode = True

    def rel(a, b):
        return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))
    for l in range(12):
        print(f"layer {l:2d}: K rel {rel(k_grid[l], k_old[l]):.2e}  V rel {rel(v_grid[l], v_old[l]):.2e}",
              flush=True)
    print(f"final x rel {rel(x_grid, x_old):.2e} (x_old max {float(x_old.abs().max()):.3g})")
    print(f"ids equal {int((ids_grid == ids_old).sum())}/{B}")
    # per-row worst
    e = (x_grid - x_old).abs().amax(-1) / x_old.abs().amax(-1)
    print("worst rows", [round(float(v), 4) for v in e.topk(5).values])


if __name__ == "__main__":
    main()
