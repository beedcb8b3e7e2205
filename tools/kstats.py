#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace run (rocpd SQLite database or
kernel_trace.csv): calls, total, average, share; optionally per-queue dispatch gaps.

    python tools/kstats.py <results.db | kernel_trace.csv> [top=30]
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, start, end, q in c.execute("select name, start, end, queue_id from kernels"):
            yield name, int(start), int(end), q
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id")


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    agg = defaultdict(lambda: [0, 0])
    perq = defaultdict(list)
    for name, s, e, q in rows(path):
        a = agg[name]
        a[0] += 1
        a[1] += e - s
        perq[q].append((s, e))
    tot = sum(v[1] for v in agg.values())
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / tot * 100:5.1f}% n={n:7d} avg={t / n / 1e3:8.2f}us {name[:100]}")
    print(f"total kernel time {tot / 1e6:.2f} ms")
    for q, iv in perq.items():
        iv.sort()
        gaps = [b[0] - a[1] for a, b in zip(iv, iv[1:]) if 0 <= b[0] - a[1] < 20000]
        if gaps:
            gaps.sort()
            print(f"queue {q}: {len(iv)} kernels, busy {sum(e - s for s, e in iv) / 1e6:.2f} ms, "
                  f"median gap {gaps[len(gaps) // 2] / 1e3:.2f} us (gaps < 20 us)")


if __name__ == "__main__":
    main()
