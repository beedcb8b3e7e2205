#!/usr/bin/env python3
"""How many streams run kernels at the same time: k dedicated streams (zs_stream_create) each run
one torch.cuda._sleep kernel (a single spinning workgroup); wall time / single time ~ 1 means all
k ran together, ~2 that pairs of streams shared a hardware queue.

    GPU_MAX_HW_QUEUES=16 python tools/hwq_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402


def main():
    from zsaac import ops
    dev = torch.device("cuda", 0)
    streams = ops.dedicated_streams(16, dev)
    cyc = 20_000_000

    def run(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in streams[:k]:
            with torch.cuda.stream(s):
                torch.cuda._sleep(cyc)
        torch.cuda.synchronize()
        return time.perf_counter() - t0
    run(1)
    t1 = run(1)
    out = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "single_ms": round(t1 * 1e3, 2)}
    out["ratio"] = {k: round(run(k) / t1, 2) for k in (2, 4, 5, 6, 8, 10, 12, 16)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
