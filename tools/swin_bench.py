#!/usr/bin/env python3
"""Microbenchmark of the fused Swin block (zs_swin_block) at a 64-clip eval batch, per stage,
with the zs_tune_set("swin_dbg", v) ablations (1 = GELU -> identity, 2 = no bias/mask lookups,
4 = skip the MLP).

    python tools/swin_bench.py [dbg values, comma-separated; default 0] [C values; default all]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402

from zsaac import ops  # noqa: E402
from zsaac._lib import call  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_swin import _block_sd, _kernel_blk  # noqa: E402


def main():
    dbgs = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0").split(",")]
    cs = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "96,192,384").split(",")]
    dev = torch.device("cuda", 0)
    B = 64
    for C, res in ((96, 64), (192, 32), (384, 16)):
        if C not in cs:
            continue
        heads = C // 24
        blk = _kernel_blk(_block_sd(C, heads, 1, dev), C, dev)
        x = torch.randn(B * res * res, C, device=dev)
        for dbg in dbgs:
            call("zs_tune_set", b"swin_dbg", dbg)
            for shift in ((4,) if len(cs) == 1 else (0, 4)):
                for _ in range(3):
                    ops.swin_block(x, B, res, res, C, heads, shift, blk)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                n = 20
                e0.record()
                for _ in range(n):
                    ops.swin_block(x, B, res, res, C, heads, shift, blk)
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / n
                M = B * res * res
                fl = 2 * M * (C * 3 * C + C * C + 8 * C * C) + 4 * M * 64 * 24 * heads // heads * heads
                print(f"C={C} shift={shift} dbg={dbg}: {us:8.1f} us/block  "
                      f"{fl / us / 1e6:7.1f} TFLOP/s  {M * C * 8 / us / 1e3:7.1f} GB/s(x rw)")
        call("zs_tune_set", b"swin_dbg", 0)


if __name__ == "__main__":
    main()
