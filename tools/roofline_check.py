#!/usr/bin/env python3
"""Trace-side cross-check of bench.py's roofline: the average duration rocprofv3 recorded for
the roofline kernel's dispatches (same kernel template, same grid) in a kernel trace of the bench
command, next to the value bench.py measured with HIP events in that same run.

    python3 tools/roofline_check.py <rocprof dir> <bench stdout log>
"""
import csv
import glob
import json
import os
import statistics
import sys


def main(pdir, bench_log):
    line = [l for l in open(bench_log) if l.startswith("{")][-1]
    b = json.loads(line)
    rl = b["roofline"]
    # the roofline launches: gemm_lean_kernel dispatches with the c_fc grid of their own tile
    # (template args BM, BN) that run back to back — the decode never launches two c_fc in a row,
    # bench.py's roofline graph replays nothing else, so runs of >= 32 consecutive such
    # dispatches are exactly the timed launches (without the concurrent streams' contention)
    mm = int(rl["kernel"].split("[")[1].split("x")[0])
    rows = []
    for fn in glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(fn)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))

    def is_cfc(r):
        name = r["Kernel_Name"]
        if "gemm_lean_kernel<" not in name:
            return None
        targs = [int(v.strip(" >()")) for v in
                 name.split("gemm_lean_kernel<")[1].split(">")[0].split(",")]
        bm, bn = targs[:2]
        threads = 64 * targs[4] * targs[5] if len(targs) >= 6 else 256
        g = -(-3072 // bn) * -(-mm // bm) * threads
        return g if int(r["Grid_Size_X"]) == g else None

    durs, grid, run = [], None, []
    for r in rows + [None]:
        g = is_cfc(r) if r is not None else None
        if g is not None:
            grid = g
            run.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            continue
        if len(run) >= 32:
            durs += run
        run = []
    out = {"kernel": rl["kernel"], "grid_size_x": grid, "dispatches": len(durs),
           "trace_avg_us": round(statistics.mean(durs), 3) if durs else None,
           "trace_median_us": round(statistics.median(durs), 3) if durs else None,
           "bench_hip_event_avg_us": rl["avg_launch_us"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
