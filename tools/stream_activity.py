#!/usr/bin/env python3
"""GPU busy time from a rocprofv3 kernel trace (run on the GPU box):

    python3 tools/stream_activity.py <trace dir> [t0_frac=0.5] [t1_frac=1.0]

Over the window [t0, t1] of the trace (fractions of its span; default: the second half, past
warmups): the union of all kernel intervals (fraction of wall time with >= 1 kernel running), the
time-weighted number of concurrent kernels, and per queue its busy fraction and kernel count."""
import csv
import glob
import os
import sys


def main(d, f0=0.5, f1=1.0):
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r.get("Queue_Id") or r.get("Stream_Id") or ""))
    rows.sort()
    T0, T1 = rows[0][0], max(r[1] for r in rows)
    a, b = T0 + float(f0) * (T1 - T0), T0 + float(f1) * (T1 - T0)
    win = [(max(s, a), min(e, b), q) for s, e, q in rows if e > a and s < b]
    ev = sorted([(s, 1) for s, e, q in win] + [(e, -1) for s, e, q in win])
    busy = conc = 0.0
    cur, last = 0, a
    for t, d_ in ev:
        if cur > 0:
            busy += t - last
        conc += cur * (t - last)
        cur += d_
        last = t
    span = b - a
    byq = {}
    for s, e, q in win:
        x = byq.setdefault(q, [0.0, 0])
        x[0] += e - s
        x[1] += 1
    print(f"window {span / 1e6:.1f} ms: busy {busy / span:.3f}, mean concurrent kernels "
          f"{conc / span:.2f}, kernels {len(win)}")
    for q, (t, n) in sorted(byq.items(), key=lambda kv: -kv[1][0]):
        print(f"  queue {q}: busy {t / span:.3f}  kernels {n}  mean {t / max(1, n) / 1e3:.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])
