#!/usr/bin/env python3
"""Host enqueue cost and GPU time of one bs-64 batch's begin (encode + prompt + mapper + prefill +
step 0), alone on one stream.  Under `rocprofv3 --kernel-trace` the last repetition's kernels
are the ones between the two `hipDeviceSynchronize`s of the final loop pass.

    python tools/begin_profile.py [reps=5] [dtype=bf16|f32]

The persistent decode launch is deferred (not part of the begin) and run after each repetition.
"""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    dt = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    args = SimpleNamespace(dtype=dt, group=1, encoder="htsat", mapper="mlp", batch=64,
                           encoder_batch=0, beam=0, entry_length=67, compact=1)
    pipe, _, _ = bench.build(args, dev)
    wav = bench.synthetic_clips(64, 0, dev)
    pipe.caption_wav(wav)
    torch.cuda.synchronize()
    host, gpu = [], []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        pipe.decoder.defer_launch = True
        pipe.begin_wav(wav)
        pipe.decoder.defer_launch = False
        e1.record()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        host.append((t1 - t0) * 1e3)
        gpu.append(e0.elapsed_time(e1))
        if pipe.decoder._persist_pending:
            pipe.decoder.launch_pending()
        pipe.decoder.run_to_completion()
    # enqueue-only cost of the begin with the GPU already busy (host time alone)
    print(f"begin_wav host enqueue ms: {['%.2f' % h for h in host]}")
    print(f"begin_wav GPU ms:          {['%.2f' % g for g in gpu]}")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
