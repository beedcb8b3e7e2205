#!/usr/bin/env python3
"""Cross-check of bench.py's roofline against a rocprofv3 kernel trace of the same command: the
dg_persist_kernel launches grouped into runs of the caption region (launches less than a gap
threshold after the previous one's end, the widest of 20 / 10 / 5 / 3 / 2 / 1 ms that yields
17-launch runs; the regions are separated by their encode + begins), the average duration of
every 17-launch run, and bench's own
roofline.avg_launch_us (its last run before the single-stream extras is the untimed log pass the
roofline is measured on).

    python3 tools/roofline_check.py <trace dir> <bench json> <out json>
"""
import csv
import glob
import json
import os
import sys


def main(d, bench_json, out):
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                if "dg_persist_kernel" in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                 r["Kernel_Name"].split("(")[0]))
    rows.sort()
    def group(gap_ns):
        runs, cur, end = [], [], 0
        for r in rows:                  # a run: launches closer than gap_ns to the last one's end
            if cur and r[0] > end + gap_ns:
                runs.append(cur)
                cur = []
            cur.append(r)
            end = max(end, r[1]) if len(cur) > 1 else r[1]
        if cur:
            runs.append(cur)
        return runs
    with open(bench_json) as f:
        b = json.loads(f.read().strip().split("\n")[-1])
    n = b["roofline"].get("launches", 17)
    # the widest gap threshold that separates the regions (a region never has an idle gap: its
    # waves overlap; consecutive regions are separated by a sync and the next encode + begin,
    # a few ms once the encoder passes replay graphs)
    for gap_ms in (20, 10, 5, 3, 2, 1):
        runs = group(gap_ms * 1e6)
        full = [[round(sum(e - s for s, e, _ in r) / len(r) / 1e3, 1), len(r)] for r in runs if len(r) == n]
        if full:
            break
    res = {"bench_roofline_avg_launch_us": b["roofline"]["avg_launch_us"],
           "bench_value": b["value"],
           "rocprof_runs_of_%d_launches_avg_us" % n: full,
           "rocprof_log_pass_avg_us": full[-1][0] if full else None,
           "agreement": (round(full[-1][0] / b["roofline"]["avg_launch_us"], 3) if full else None),
           "region_gap_ms": gap_ms,
           "note": "runs = groups of dg_persist_kernel launches with no idle gap; the bench's "
                   "timed repetitions then its untimed log pass (HIP events around each launch) "
                   "are the 17-launch runs, in order"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])
