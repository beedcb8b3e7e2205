#!/usr/bin/env python3
"""Correctness screen for forced GEMM tiles (zs_tune_set fast_tile) against a torch fp32 matmul
at ragged and decode shapes:  python3 tools/tile_check.py 105,106,107,108"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402
from zsaac import ops  # noqa: E402
from zsaac._lib import call  # noqa: E402


def main(tiles):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    bad = 0
    for M, N, K in ((8192, 3072, 768), (1000, 2304, 768), (333, 768, 3072), (4096, 770, 64)):
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        bias = torch.randn(N, device=dev)
        ref = a.float() @ w.float().t() + bias
        for t in tiles:
            call("zs_tune_set", b"fast_tile", t)
            out = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
            ops.gemm(a, w, out, bias=bias, split_k=1)
            torch.cuda.synchronize()
            err = ((out.float() - ref).abs() / (ref.abs() + 1.0)).max().item()
            ok = err < 2e-2
            bad += not ok
            print(f"M{M} N{N} K{K} tile {t}: max rel err {err:.3e} {'ok' if ok else 'FAIL'}", flush=True)
    call("zs_tune_set", b"fast_tile", 0)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main([int(t) for t in sys.argv[1].split(",")])
