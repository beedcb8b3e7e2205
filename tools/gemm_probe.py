#!/usr/bin/env python3
"""One GEMM shape launched eagerly N times (for rocprofv3 --pmc / --kernel-trace passes).

    python tools/gemm_probe.py M N K [reps] [fast=1] [out=bf16|f32]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402

from zsaac import ops  # noqa: E402
from zsaac._lib import call  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 50
    fast = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    odt = torch.float32 if (len(sys.argv) > 6 and sys.argv[6] == "f32") else torch.bfloat16
    dev = torch.device("cuda", 0)
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
    b = torch.randn(N, device=dev)
    out = torch.empty(M, N, device=dev, dtype=odt)
    call("zs_tune_set", b"gemm_fast", fast)
    call("zs_tune_set", b"gemm_dbg", int(os.environ.get("ZS_GEMM_DBG", "0")))
    call("zs_tune_set", b"fast_tile", int(os.environ.get("ZS_FAST_TILE", "0")))
    for _ in range(reps):
        ops.gemm(a, w, out, bias=b, split_k=1)
    torch.cuda.synchronize()
    ref = a.float() @ w.float().t() + b
    err = float((out.float() - ref).abs().max() / ref.abs().max())
    print(f"M{M} N{N} K{K} fast={fast} rel_err={err:.2e}")


if __name__ == "__main__":
    main()
