#!/usr/bin/env python3
"""The decode grids of the LAST n persistent launches of a rocprofv3 kernel trace: start / end
(ms from the first one's start), duration, queue and stream ids, grid size -- to see stragglers.

    python3 tools/tl_grids.py <trace dir> [n=20]
"""
import csv
import glob
import json
import os
import sys


def main(d, n=20):
    n = int(n)
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                if "dg_persist_kernel" in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                                 r.get("Stream_Id", ""), r["Grid_Size_X"], r["Dispatch_Id"]))
    rows.sort()
    last = rows[-n:]
    t0 = last[0][0]
    out = [{"start_ms": round((a - t0) / 1e6, 2), "end_ms": round((b - t0) / 1e6, 2),
            "dur_ms": round((b - a) / 1e6, 2), "queue": q, "stream": s, "grid_threads": g,
            "dispatch": di} for a, b, q, s, g, di in last]
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main(*sys.argv[1:])
