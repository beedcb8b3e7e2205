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
    # the roofline launches are the only gemm_fast_kernel<128, 128, 2...> dispatches with the
    # c_fc grid; the decode's own c_fc launches share it (same kernel, same shape)
    tile = "gemm_fast_kernel<128, 128, 2"
    mm = int(rl["kernel"].split("[")[1].split("x")[0])
    ntiles = -(-3072 // 128) * -(-mm // 128)
    grid = min(ntiles, 512) * 256
    durs = []
    for fn in glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if tile in r["Kernel_Name"] and int(r["Grid_Size_X"]) == grid:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {"kernel": rl["kernel"], "grid_size_x": grid, "dispatches": len(durs),
           "trace_avg_us": round(statistics.mean(durs), 3) if durs else None,
           "trace_median_us": round(statistics.median(durs), 3) if durs else None,
           "bench_hip_event_avg_us": rl["avg_launch_us"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
