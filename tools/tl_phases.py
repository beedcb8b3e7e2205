#!/usr/bin/env python3
"""Timeline of the LAST headline region of a rocprofv3 kernel trace, split by role: per 5-ms
bucket the kernel-time density (ms of kernel time per ms) of the encoder passes (the encoder
twin's stream: the queue that runs swin_block_kernel), of the begins (every other non-decode
kernel) and the number of decode grids in flight; plus when the first / last grid starts and
ends, and the encoder's and begins' total kernel time inside the region.

    python3 tools/tl_phases.py <trace dir> [n_launches=17] [bucket_ms=5]
"""
import csv
import glob
import json
import os
import sys


def main(d, n=17, bucket=5.0):
    n, bucket = int(n), float(bucket)
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                q = r.get("Stream_Id") or r.get("Queue_Id") or ""
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], q))
    rows.sort()
    per = [r for r in rows if "dg_persist_kernel" in r[2]]
    timed = per[-n:]
    prev_end = per[-n - 1][1] if len(per) > n else rows[0][0]
    t0 = min(r[0] for r in rows if r[0] >= prev_end)
    t1 = max(r[1] for r in timed)
    enc_q = {r[3] for r in rows if r[0] >= t0 and "swin_block" in r[2]}
    ms = lambda t: (t - t0) / 1e6
    nb = int(ms(t1) / bucket) + 1
    enc, beg, dec = [0.0] * nb, [0.0] * nb, [0.0] * nb
    tot = {"encoder": 0.0, "begins": 0.0}
    names = {}
    for r in rows:
        if r[1] < t0 or r[0] > t1:
            continue
        if "dg_persist_kernel" in r[2]:
            tgt = dec
        elif r[3] in enc_q:
            tgt, key = enc, "encoder"
        else:
            tgt, key = beg, "begins"
        if tgt is not dec:
            tot[key] += (r[1] - r[0]) / 1e6
            k = key + ": " + r[2].split("(")[0][:50]
            names[k] = names.get(k, 0) + (r[1] - r[0]) / 1e6
        a, b = ms(r[0]), ms(r[1])
        for i in range(max(0, int(a / bucket)), min(nb, int(b / bucket) + 1)):
            lo, hi = max(a, i * bucket), min(b, (i + 1) * bucket)
            if hi > lo:
                tgt[i] += (hi - lo) / bucket
    # per begin: on each pipeline queue, the kernels between two persistent launches (the
    # begin of the batch whose grid follows): wall (first start -> last end) vs kernel-busy time
    begins = []
    by_q = {}
    for r in rows:
        if r[1] < t0 or r[0] > t1 or r[3] in enc_q:
            continue
        by_q.setdefault(r[3], []).append(r)
    for q, rs in by_q.items():
        seg = []
        for r in rs:
            if "dg_persist_kernel" in r[2]:
                if seg:
                    wall = (max(x[1] for x in seg) - min(x[0] for x in seg)) / 1e6
                    busy = sum(x[1] - x[0] for x in seg) / 1e6
                    begins.append({"start": round(ms(seg[0][0]), 2), "wall_ms": round(wall, 2),
                                   "kernel_ms": round(busy, 2), "kernels": len(seg),
                                   "grid_start_after_ms": round((r[0] - max(x[1] for x in seg)) / 1e6, 2)})
                seg = []
            else:
                seg.append(r)
    begins.sort(key=lambda b: b["start"])
    st = sorted(ms(r[0]) for r in timed)
    en = sorted(ms(r[1]) for r in timed)
    out = {"span_ms": round(ms(t1), 2), "first_grid_start": round(st[0], 2),
           "last_grid_start": round(st[-1], 2), "first_grid_end": round(en[0], 2),
           "launch_ms_mean": round(sum(ms(r[1]) - ms(r[0]) for r in timed) / len(timed), 2),
           "kernel_ms": {k: round(v, 2) for k, v in tot.items()},
           "bucket_ms": bucket,
           "encoder_density": [round(x, 2) for x in enc],
           "begins_density": [round(x, 2) for x in beg],
           "grids_in_flight": [round(x, 2) for x in dec],
           "top_kernels_ms": {k: round(v, 2) for k, v in sorted(names.items(), key=lambda kv: -kv[1])[:14]},
           "begins": begins}
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
