#!/usr/bin/env python3
"""HBM traffic of bench.py's roofline kernel from rocprofv3 PMC counters (roofline.traffic).

Two counter passes (FETCH_SIZE and WRITE_SIZE do not fit one gfx950 TCC pass), each with eager
launches of exactly the launches bench.py times (roofline_setup: cold weights), then a parse:

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 tools/pmc_traffic.py run
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 tools/pmc_traffic.py run
    python3 tools/pmc_traffic.py parse gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r2_pmc_traffic.json

The persistent decode kernel (bench.py's roofline since round 3): ``run_persist`` decodes the
bench's first eval batch (64 synthetic clips, 67 greedy steps) three times on one stream, and
``parse_persist`` writes profiles/r3_pmc_persist.json (per-launch bytes, median launch):

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_pf -o run --output-format csv -- python3 tools/pmc_traffic.py run_persist [grid]
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_pw -o run --output-format csv -- python3 tools/pmc_traffic.py run_persist
    python3 tools/pmc_traffic.py parse_persist gpurun_out/pmc_pf gpurun_out/pmc_pw profiles/r3_pmc_persist.json

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE is in KiB and on gfx950 reports half the
bytes of a 16-B/lane coalesced streaming read (the GEMM's LDS-DMA loads are all 16 B per lane),
so read bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE (KiB) is exact for 16-B/lane stores (the
epilogue's bf16 rows are 16-B/lane stores).
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))


def run():
    """The bench's roofline launches: zs_gemm_ln at the bs=64 decode c_fc shape (64 rows, folded
    LN, gelu_new) rotating over cold weight copies, as bench.roofline_gemm_ln times them."""
    import torch
    import bench
    from zsaac import ops

    class A:
        batch, group, dtype, encoder, mapper, beam, entry_length, compact = \
            64, 1, "bf16", "htsat", "mlp", 0, 67, 1
        encoder_batch = 64
    pipe, _, _ = bench.build(A, torch.device("cuda", 0))
    dec, ly = pipe.decoder, pipe.gpt.layers[0]
    x, hid = dec.x[:64], dec.hid[:64]
    copies = bench._cold_copies(ly["fc_w"])
    for i in range(2 * len(copies)):
        ops.gemm_ln(x, *ly["ln2_gemm"], copies[i % len(copies)], hid, bias=ly["fc_b"],
                    act=ops.ACT_GELU_TANH)
    torch.cuda.synchronize()
    N, K = ly["fc_w"].shape
    print(json.dumps({"launches": 2 * len(copies), "shape": [64, N, K]}))


def _per_dispatch(d, counter, kname):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter or kname not in row.get("Kernel_Name", ""):
                    continue
                key = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kname} under {d}")
    v = sorted(vals.values())
    return v[len(v) // 2], len(v)


def parse(dfetch, dwrite, out, M=64, N=3072, K=768, kname="gemm_rows_kernel"):
    fetch_kib, n_f = _per_dispatch(dfetch, "FETCH_SIZE", kname)
    write_kib, n_w = _per_dispatch(dwrite, "WRITE_SIZE", kname)
    rd = 2 * 1024 * fetch_kib
    wr = 1024 * write_kib
    sys.path.insert(0, ROOT)
    res = {"kernel": f"{kname}<48,4,LN,6> (zs_gemm_ln) decode c_fc [{M}x{K}]x[{K}x{N}] (cold weights)",
           "fetch_size_kib_median": fetch_kib, "write_size_kib_median": write_kib,
           "dispatches": [n_f, n_w], "hbm_read_bytes_per_launch": int(rd),
           "hbm_write_bytes_per_launch": int(wr), "hbm_bytes_per_launch": int(rd + wr),
           "corrections": "read = 2*1024*FETCH_SIZE (gfx950 16B/lane streaming reads); "
                          "write = 1024*WRITE_SIZE"}
    # the shape bench.py checks against before quoting the traffic
    res["shape"] = [M, N, K]
    res["algo_bytes_per_launch"] = N * K * 2 + M * K * 4 + N * 4 + M * N * 2
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


def _bench_pipe():
    import torch
    import bench

    class A:
        batch, group, dtype, encoder, mapper, beam, entry_length, compact = \
            64, 1, "bf16", "htsat", "mlp", 0, 67, 1
        encoder_batch = 64
    pipe, _, _ = bench.build(A, torch.device("cuda", 0))
    return bench, pipe


def run_persist(reps=3, grid=None):
    import torch
    bench, pipe = _bench_pipe()
    assert pipe.decoder.persist, "the persistent decode path is off"
    if grid:
        pipe.decoder.persist_grid = int(grid)
    wav = bench.synthetic_clips(64, 0, torch.device("cuda", 0))
    info = []
    for _ in range(reps):
        pipe.begin_wav(wav)
        pipe.decoder.run_to_completion()
        torch.cuda.synchronize()
        info.append(int(pipe.decoder.step_ctr.item()))
    plen = pipe.decoder.plen[:64].tolist()
    algo = bench.persist_launch_bytes(bench.gpt2_step_weight_bytes(pipe), plen, info[-1])
    d = pipe.decoder
    with open(os.path.join(ROOT, "gpurun_out", "pmc_persist_run.json"), "w") as f:
        json.dump({"steps": info, "plen": plen, "algo_bytes_per_launch": algo,
                   "workgroups": d.persist_grid}, f)
    print(json.dumps({"launches": reps, "steps": info, "algo_bytes_per_launch": algo}))


def parse_persist(dfetch, dwrite, out, kname="dg_persist_kernel"):
    fetch_kib, n_f = _per_dispatch(dfetch, "FETCH_SIZE", kname)
    write_kib, n_w = _per_dispatch(dwrite, "WRITE_SIZE", kname)
    rd, wr = 2 * 1024 * fetch_kib, 1024 * write_kib
    with open(os.path.join(ROOT, "gpurun_out", "pmc_persist_run.json")) as f:
        run_info = json.load(f)
    res = {"kernel": f"{kname} (zs_gpt2_decode_persist): one bs-64 eval batch of the bench "
                     f"(64 synthetic clips), decode steps 1..{run_info['steps'][-1] - 1}, one stream, "
                     f"grid of {run_info.get('workgroups', 48)} 256-thread workgroups",
           "fetch_size_kib_median": fetch_kib, "write_size_kib_median": write_kib,
           "dispatches": [n_f, n_w], "hbm_read_bytes_per_launch": int(rd),
           "hbm_write_bytes_per_launch": int(wr), "hbm_bytes_per_launch": int(rd + wr),
           "algo_bytes_per_launch": run_info["algo_bytes_per_launch"],
           "traffic_over_algo": round((rd + wr) / run_info["algo_bytes_per_launch"], 3),
           "corrections": "read = 2*1024*FETCH_SIZE (gfx950 16B/lane streaming reads; FETCH_SIZE "
                          "counts L2 misses incl. Infinity-Cache hits); write = 1024*WRITE_SIZE"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    elif sys.argv[1] == "run_persist":
        run_persist(grid=sys.argv[2] if len(sys.argv) > 2 else None)
    elif sys.argv[1] == "parse_persist":
        parse_persist(*sys.argv[2:5])
    else:
        parse(*sys.argv[2:5])
