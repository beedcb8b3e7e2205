#!/usr/bin/env python3
"""Concurrency of the non-decode kernels before the first decode grid of the LAST headline
region of a rocprofv3 kernel trace: distinct stream / queue ids, kernel time per queue, and the
time with k kernels running at once.

    python3 tools/tl_concurrency.py <trace dir> [n_launches=17]
"""
import collections
import csv
import glob
import json
import os
import sys


def main(d, n=17):
    n = int(n)
    rows = []
    cols = None
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            rd = csv.DictReader(f)
            cols = rd.fieldnames
            for r in rd:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             r.get("Stream_Id", ""), r.get("Queue_Id", "")))
    rows.sort()
    per = [r for r in rows if "dg_persist_kernel" in r[2]]
    timed = per[-n:]
    prev_end = per[-n - 1][1] if len(per) > n else rows[0][0]
    t0 = min(r[0] for r in rows if r[0] >= prev_end)
    g0 = min(r[0] for r in timed)
    pre = [r for r in rows if r[0] >= t0 and r[1] <= g0 and "dg_persist_kernel" not in r[2]]
    by_q = collections.defaultdict(float)
    by_s = collections.defaultdict(float)
    for r in pre:
        by_q[r[4]] += (r[1] - r[0]) / 1e6
        by_s[r[3]] += (r[1] - r[0]) / 1e6
    ev = sorted([(r[0], 1) for r in pre] + [(r[1], -1) for r in pre])
    hist = collections.defaultdict(float)
    k, last = 0, t0
    for t, dlt in ev:
        hist[k] += (t - last) / 1e6
        k += dlt
        last = t
    hist[0] += (g0 - last) / 1e6
    print(json.dumps({"columns": cols, "pre_grid_ms": round((g0 - t0) / 1e6, 2),
                      "kernels": len(pre), "kernel_ms": round(sum(by_q.values()), 2),
                      "ms_by_queue": {q: round(v, 2) for q, v in sorted(by_q.items())},
                      "ms_by_stream": {q: round(v, 2) for q, v in sorted(by_s.items())},
                      "ms_with_k_running": {k: round(v, 2) for k, v in sorted(hist.items())}}))


if __name__ == "__main__":
    main(*sys.argv[1:])
