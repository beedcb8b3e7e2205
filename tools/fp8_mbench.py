#!/usr/bin/env python3
"""Microbenchmark of the weight-only fp8 row GEMM (csrc/mistral.hip) at the Mistral-7B decode
shapes, M = 32, cold weights (launches rotate over > 512 MiB of weight copies); fp8_tile = 0 is
the default dispatch (persistent stream kernel for the long streams), 2 the one-shot kernel only,
1 64-column one-shot tiles.  (Round-2 ablations, before the transposed product / straight-line load
phase: no activation loads -47..-56 % time, no MFMA 0 %, no weight loads -44..-55 %, plain vs
non-temporal weight loads 0 %.)

    python tools/fp8_mbench.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from zsaac._lib import call, lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    M = 32
    for name, N, K in (("gate|up", 28672, 4096), ("down", 4096, 14336), ("qkv", 6144, 4096),
                       ("o", 4096, 4096)):
        ncopy = max(2, -(-(512 << 20) // (N * K)))
        ws = [torch.randint(0, 120, (N, K), dtype=torch.uint8, device=dev) for _ in range(ncopy)]
        sc = torch.full((N,), 1e-3, device=dev)
        a = torch.randn(M, K, device=dev).bfloat16()
        ns = call("zs_fp8_splits", K)
        out = torch.empty(2 * ns * M * N, device=dev)
        act = torch.empty(M, N // 2 + 8, device=dev, dtype=torch.bfloat16)
        res = []
        st = lambda: torch.cuda.current_stream().cuda_stream
        variants = [("fp8_tile=0", 0, None), ("fp8_tile=2", 2, None)]
        variants += [(f"run ks={k} kh={h}", None, (k, h)) for k in (1, 2, 4) for h in (1, 2)
                     if ns % k == 0]
        if name == "gate|up":
            variants.append(("run glu", None, (-ns, 1)))
        for label, tile, ks in variants:
            if ks is None:
                lib().zs_tune_set(b"fp8_tile", tile)

                def launch(i):
                    call("zs_fp8_gemm_rows", a.data_ptr(), K, ws[i % ncopy].data_ptr(),
                         sc.data_ptr(), M, N, K, out.data_ptr(), M * N, N, st())
            else:
                def launch(i, ks=ks[0], kh=ks[1]):
                    call("zs_fp8_gemm_run", a.data_ptr(), K, ws[i % ncopy].data_ptr(),
                         sc.data_ptr(), M, N, K, abs(ks), kh, out.data_ptr(), M * N, N,
                         act.data_ptr() if ks < 0 else None, N // 2 + 8, None, 0, 0.0, st())
            t = bench._graph_time(launch, 2 * ncopy)
            lib().zs_tune_set(b"fp8_tile", 0)
            res.append(f"{label}: {t * 1e6:6.1f}us {N * K / t / 1e9:5.0f}GB/s")
        print(f"{name:8s} N={N} K={K}: " + " | ".join(res), flush=True)
        del ws


if __name__ == "__main__":
    main()
