#!/usr/bin/env python3
"""HBM traffic of the Mistral fp8 stream kernel (fp8_gemm_stream_kernel, gate|up at M = 32, cold
weights) from rocprofv3 PMC counters, against its algorithmic bytes:

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pf8 -o run --output-format csv -- python3 tools/pmc_fp8.py run
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pw8 -o run --output-format csv -- python3 tools/pmc_fp8.py run
    python3 tools/pmc_fp8.py parse gpurun_out/pf8 gpurun_out/pw8 profiles/r2_pmc_fp8.json

Corrections as tools/pmc_traffic.py (MI355X_MICROARCH.md §HBM): read = 2 * 1024 * FETCH_SIZE
(16-B/lane streaming reads on gfx950), write = 1024 * WRITE_SIZE (16-B/lane slab stores)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

M, N, K = 32, 28672, 4096


def run():
    import torch
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    ncopy = max(2, -(-(512 << 20) // (N * K)))            # rotate over > 512 MiB: cold weights
    ws = [torch.randint(0, 120, (N * K,), dtype=torch.uint8, device=dev) for _ in range(ncopy)]
    sc = torch.full((N,), 1e-3, device=dev)
    a = torch.randn(M, K, device=dev).bfloat16()
    ns = call("zs_fp8_splits", K)
    out = torch.empty(ns * M * N, device=dev)
    for i in range(2 * ncopy):
        call("zs_fp8_gemm_rows", a.data_ptr(), K, ws[i % ncopy].data_ptr(), sc.data_ptr(), M, N, K,
             out.data_ptr(), M * N, N, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    print(json.dumps({"launches": 2 * ncopy, "shape": [M, N, K]}))


def parse(dfetch, dwrite, out):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import _per_dispatch
    kname = "fp8_gemm_stream_kernel"
    fetch_kib, n_f = _per_dispatch(dfetch, "FETCH_SIZE", kname)
    write_kib, n_w = _per_dispatch(dwrite, "WRITE_SIZE", kname)
    rd, wr = 2 * 1024 * fetch_kib, 1024 * write_kib
    ns = K // 1024
    algo_rd = N * K + N * 4 + M * K * 2
    algo_wr = ns * M * N * 4
    res = {"kernel": f"{kname} (zs_fp8_gemm_rows) gate|up [{M}x{K}]x[{K}x{N}] fp8 (cold weights)",
           "fetch_size_kib_median": fetch_kib, "write_size_kib_median": write_kib,
           "dispatches": [n_f, n_w], "hbm_read_bytes_per_launch": int(rd),
           "hbm_write_bytes_per_launch": int(wr), "hbm_bytes_per_launch": int(rd + wr),
           "algo_read_bytes_per_launch": algo_rd, "algo_write_bytes_per_launch": algo_wr,
           "read_over_algo": round(rd / algo_rd, 3), "write_over_algo": round(wr / algo_wr, 3),
           "corrections": "read = 2*1024*FETCH_SIZE (gfx950 16B/lane streaming reads); "
                          "write = 1024*WRITE_SIZE"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(*sys.argv[2:5])
