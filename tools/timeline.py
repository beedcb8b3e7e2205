#!/usr/bin/env python3
"""Timeline of the headline's timed region from a rocprofv3 kernel trace (run on the GPU box,
where the trace CSV lives; writes a small JSON summary):

    python3 tools/timeline.py <kernel_trace.csv dir> <out.json> [first_timed=8] [n_timed=17]

The timed region = from the first to the last of the n_timed dg_persist_kernel dispatches
starting at index first_timed (bench.py's order: per-pipeline warmups, warmup batches, then the
timed batches).  Reports: how many persistent grids run at once over the region (time-weighted),
each timed batch's gap on its queue between the previous persistent launch's end and its own
start (encode + prompt + mapper + prefill + step 0 under contention), and the kernel time of the
non-decode kernels inside the region by name."""
import csv
import glob
import json
import os
import sys


def main(d, out, first=8, n=17):
    first, n = int(first), int(n)
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             r.get("Queue_Id") or r.get("Stream_Id") or ""))
    rows.sort()
    per = [r for r in rows if "persist_kernel" in r[2]]
    timed = per[first:first + n] if first >= 0 else per[len(per) - n:]    # first < 0: the last n
    t0 = min(r[0] for r in timed)
    t1 = max(r[1] for r in timed)
    # time-weighted count of concurrent persistent grids
    ev = sorted([(r[0], 1) for r in timed] + [(r[1], -1) for r in timed])
    hist, cur, last = {}, 0, t0
    for t, dlt in ev:
        hist[cur] = hist.get(cur, 0) + (t - last)
        cur += dlt
        last = t
    span = t1 - t0
    conc = {k: round(v / span, 4) for k, v in sorted(hist.items())}
    # per-queue gaps before each timed persistent launch
    byq = {}
    for r in per[:per.index(timed[-1]) + 1]:
        byq.setdefault(r[3], []).append(r)
    gaps = []
    for q, rs in byq.items():
        for a, b in zip(rs, rs[1:]):
            if b in timed:
                gaps.append((b[0] - a[1]) / 1e6)
    other = {}
    for r in rows:
        if r[0] >= t0 and r[1] <= t1 and "persist_kernel" not in r[2]:
            k = r[2].split("(")[0][:80]
            other[k] = other.get(k, 0) + (r[1] - r[0]) / 1e6
    top = dict(sorted(other.items(), key=lambda kv: -kv[1])[:15])
    res = {"timed_span_ms": round(span / 1e6, 3),
           "persistent_launch_ms_mean": round(sum(r[1] - r[0] for r in timed) / n / 1e6, 3),
           "concurrent_persistent_grids_time_fraction": conc,
           "gap_before_launch_ms": {"mean": round(sum(gaps) / max(1, len(gaps)), 3),
                                    "max": round(max(gaps or [0]), 3), "n": len(gaps)},
           "other_kernels_ms_in_region": {k: round(v, 3) for k, v in top.items()},
           "other_kernels_total_ms": round(sum(other.values()), 3),
           # every timed persistent launch: [start, end] ms from the region's start, its queue
           "launches_ms": [[round((r[0] - t0) / 1e6, 2), round((r[1] - t0) / 1e6, 2), r[3]]
                           for r in timed]}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
