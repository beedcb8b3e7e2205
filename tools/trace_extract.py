#!/usr/bin/env python3
"""Shrinks a rocprofv3 --kernel-trace CSV directory to what profiles/ keeps: the per-kernel
stats CSV stays; the (large) trace CSV is replaced by per-dispatch durations of the kernels
named on the command line (JSON), then deleted.

    python3 tools/trace_extract.py gpurun_out/prof_bench out.json decode_persist_kernel [...]
"""
import csv
import glob
import json
import os
import sys


def main(d, out, *names):
    res = {}
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "")
                for n in names:
                    if n in k:
                        t = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
                        res.setdefault(n, []).append([int(row["Start_Timestamp"]), round(t, 3)])
        os.remove(fn)
    summ = {}
    for n, v in res.items():
        v.sort()
        d_us = [x[1] for x in v]
        summ[n] = {"dispatches": len(v), "avg_us": round(sum(d_us) / len(v), 3),
                   "durations_us_in_order": d_us}
    with open(out, "w") as f:
        json.dump(summ, f, indent=0)
    print(json.dumps({n: {k: s[k] for k in ("dispatches", "avg_us")} for n, s in summ.items()}))


if __name__ == "__main__":
    main(*sys.argv[1:])
