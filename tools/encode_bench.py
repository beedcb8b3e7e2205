#!/usr/bin/env python3
"""HTSAT encoder (wav -> CLAP embedding) throughput per pass size, alone on the chip, and the
caption phase after it (ConcurrentRunner on precomputed embeddings: prompt .. decode, 1045 clips
in bs-64 batches) -- the two halves of the encode-first headline.

    python tools/encode_bench.py [sizes=64,128,256,512,1045 (0: none)] [reps=3] [phases=g48,mix,g96]
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

os.environ["GPU_MAX_HW_QUEUES"] = "16"


def main():
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,128,256,512,1045").split(",")
             if int(x) > 0]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    phases = (sys.argv[3] if len(sys.argv) > 3 else "g48,mix,g96").split(",")
    from zsaac.pipeline import ConcurrentRunner
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(dtype="bf16", group=1, encoder="htsat", mapper="mlp", batch=64,
                           encoder_batch=0, beam=0, entry_length=67, compact=1)
    pipe, _, _ = bench.build(args, dev)
    n = 1045
    pool = bench.synthetic_clips(n, 0, dev)
    for B in sizes:
        enc = pipe.encoder.twin(max_batch=B)
        def once():
            for c0 in range(0, n, B):
                enc.encode(pool[c0:min(n, c0 + B)])
        once()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            once()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(json.dumps({"encoder_pass_clips": B, "ms_1045_clips": round(dt * 1e3, 2),
                          "clips_per_s": round(n / dt, 1)}), flush=True)
        del enc
        torch.cuda.empty_cache()
    emb = pipe.encode(pool[:64])
    embs = torch.cat([pipe.encoder.encode(pool[c0:c0 + 64]).clone() for c0 in range(0, n, 64)])
    batches = [embs[a:b] for a, b in bench.split_batches(n, 64)]
    for name, grids, budget in (("g48", [48], 512), ("mix", [192, 96, 48], 512), ("g96", [96], 480)):
        if name not in phases:
            continue
        r = ConcurrentRunner(pipe, 10, grids=grids, budget=budget)
        r.warmup_emb(batches[0])
        r.run(batches, inputs="emb")
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.run(batches, inputs="emb")
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        dt = sorted(ts)[len(ts) // 2]
        print(json.dumps({"caption_phase": name, "ms": round(dt * 1e3, 2),
                          "clips_per_s": round(n / dt, 1), "gave_up": r.gave_up,
                          "all_ms": [round(t * 1e3, 1) for t in ts]}), flush=True)


if __name__ == "__main__":
    main()
