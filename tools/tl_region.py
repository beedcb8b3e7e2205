#!/usr/bin/env python3
"""Timeline of the LAST n persistent decode launches of a rocprofv3 kernel trace (one timed
headline region): each launch's [start, end] in ms from the region start (the first non-decode
kernel after the previous region's last launch), and per 10-ms bucket the summed duration of the
non-decode kernels (encode .. step 0) and of the decode launches, in ms of kernel time per ms.

    python3 tools/tl_region.py <trace dir> [n=17]
"""
import csv
import glob
import json
import os
import sys


def main(d, n=17):
    n = int(n)
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    per = [r for r in rows if "dg_persist_kernel" in r[2]]
    timed = per[-n:]
    prev_end = per[-n - 1][1] if len(per) > n else rows[0][0]
    t0 = min(r[0] for r in rows if r[0] >= prev_end)
    t1 = max(r[1] for r in timed)
    ms = lambda t: round((t - t0) / 1e6, 2)
    launches = [[ms(r[0]), ms(r[1]), r[2].split("<")[1].split(">")[0]] for r in timed]
    nb = int((t1 - t0) / 1e7) + 1
    other, dec = [0.0] * nb, [0.0] * nb
    names = {}
    for r in rows:
        if r[1] < t0 or r[0] > t1:
            continue
        tgt = dec if "dg_persist_kernel" in r[2] else other
        if tgt is other:
            k = r[2].split("(")[0][:60]
            names[k] = names.get(k, 0) + (r[1] - r[0]) / 1e6
        for b in range(max(0, int((r[0] - t0) / 1e7)), min(nb, int((r[1] - t0) / 1e7) + 1)):
            lo, hi = max(r[0], t0 + b * 10 ** 7), min(r[1], t0 + (b + 1) * 10 ** 7)
            if hi > lo:
                tgt[b] += (hi - lo) / 1e7
    print(json.dumps({"span_ms": ms(t1), "launches": launches}))
    print(json.dumps({"per_10ms_other": [round(x, 2) for x in other],
                      "per_10ms_decode": [round(x, 2) for x in dec]}))
    print(json.dumps({"other_kernel_ms": dict(sorted(names.items(), key=lambda kv: -kv[1])[:12])}))


if __name__ == "__main__":
    main(*sys.argv[1:])
