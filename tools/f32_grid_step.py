#!/usr/bin/env python3
"""The f32 grid decode alone: one bs-64 batch (64 synthetic clips), the persistent f32 launch's
duration per decode step (HIP events around the launch), and the begin (encode .. step 0) time.

    python tools/f32_grid_step.py [reps=3]
"""
import json
import os
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    from zsaac import decoder as zdec
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(dtype="f32", group=1, encoder="htsat", mapper="mlp", batch=64,
                           encoder_batch=64, beam=0, entry_length=67, compact=1)
    pipe, _, _ = bench.build(args, dev, dtype=torch.float32)
    wav = bench.synthetic_clips(64, 0, dev)
    pipe.caption_wav(wav)
    torch.cuda.synchronize()
    res = {"launch_ms": [], "steps": [], "begin_ms": []}
    for _ in range(reps):
        zdec.PERSIST_LOG = []
        t0 = time.perf_counter()
        pipe.decoder.defer_launch = True
        pipe.begin_wav(wav)
        torch.cuda.synchronize()
        res["begin_ms"].append(round((time.perf_counter() - t0) * 1e3, 2))
        pipe.decoder.defer_launch = False
        pipe.decoder.launch_pending()
        pipe.decoder.run_to_completion()
        torch.cuda.synchronize()
        s, e = zdec.PERSIST_LOG[-1][:2]
        res["launch_ms"].append(round(s.elapsed_time(e), 3))
        res["steps"].append(int(pipe.decoder.step_ctr.item()))
    zdec.PERSIST_LOG = None
    res["us_per_step"] = [round(1e3 * m / max(1, n - 1), 1) for m, n in zip(res["launch_ms"], res["steps"])]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
