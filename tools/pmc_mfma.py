#!/usr/bin/env python3
"""MFMA utilisation of the bs=64 headline path from rocprofv3 PMC counters.

run:    caption 2 eval batches of 64 clips (the bench pipeline, bf16, one stream) under
        rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
parse:  per kernel family: dispatches, device time, MFMA-busy cycles, and
        util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
        (GRBM_GUI_ACTIVE sums the 8 XCDs' busy clocks, MI355X_MICROARCH.md "DVFS give-back";
        SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy SIMD cycles summed over the chip)

    rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d gpurun_out/pmc_mfma -o run -- python3 tools/pmc_mfma.py run
    python3 tools/pmc_mfma.py parse gpurun_out/pmc_mfma profiles/r2_pmc_mfma.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

SIMDS = 256 * 4


def run():
    import torch
    import bench

    class A:
        batch, dtype, encoder, mapper, beam, entry_length, group, compact = \
            64, "bf16", "htsat", "mlp", 0, 67, 1, 1
        encoder_batch = 64
    pipe, _, _ = bench.build(A, torch.device("cuda", 0))
    wav = bench.synthetic_clips(64, 0, torch.device("cuda", 0))
    for _ in range(2):
        pipe.caption_wav(wav)
    torch.cuda.synchronize()
    print("pmc_mfma run done", flush=True)


def family(name):
    name = re.sub(r"\(.*", "", name)
    return re.sub(r"<.*", "", name).strip()


def parse(d, out):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = family(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[family(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    tot_busy = sum(a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for a in agg.values())
    tot_gui = sum(a.get("GRBM_GUI_ACTIVE", 0) for a in agg.values())
    fams = []
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        gui = a.get("GRBM_GUI_ACTIVE", 0)
        fams.append({"kernel": k, "dispatches": len(disp[k]), "device_s": round(dur.get(k, 0), 6),
                     "mfma_busy_cycles": a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0),
                     "sq_busy_cycles": a.get("SQ_BUSY_CYCLES", 0), "grbm_gui_active": gui,
                     "mfma_util": round(a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui / 8 * SIMDS), 4)
                     if gui else None})
    res = {"workload": "bench pipeline, bs=64, 2 eval batches of 64 clips (wav -> greedy), bf16, one stream",
           "util_formula": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)",
           "overall_mfma_util": round(tot_busy / (tot_gui / 8 * SIMDS), 4) if tot_gui else None,
           "families": fams}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("overall_mfma_util",)}))
    for x in fams[:25]:
        print(f"{x['kernel'][:60]:60s} {x['dispatches']:6d} {x['device_s']*1e3:9.2f} ms  util {x['mfma_util']}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2], sys.argv[3])
