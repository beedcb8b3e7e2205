#!/usr/bin/env python3
"""Microbenchmark of zs_mistral_add_rmsnorm at the Mistral decode shape (M = 32, D = 4096) for the
o-projection (4 slabs) and down-projection (14 slabs) consumers."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from zsaac import ops  # noqa: E402
from zsaac._lib import call  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    M, D = 32, 4096
    x = torch.randn(M, D, device=dev)
    h = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    for ns in (1, 4, 14):
        y = torch.randn(ns, M, D, device=dev)

        def launch(i):
            call("zs_mistral_add_rmsnorm", x.data_ptr(), y.data_ptr(), ns, M * D, M, D, 1e-5, None,
                 h.data_ptr(), ops.dt(h), torch.cuda.current_stream().cuda_stream)
        t = bench._graph_time(launch, 20)
        print(f"add_rmsnorm M={M} D={D} slabs={ns}: {t * 1e6:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
