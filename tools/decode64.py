#!/usr/bin/env python3
"""Single-stream timing of the bs=64 greedy decode step (the C2 headline's decode shape): builds
the bench pipeline at batch 64, captions one batch, then replays one chunk graph back to back.

    python tools/decode64.py [reps=20]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20

    class A:
        batch, dtype, encoder, mapper, beam, entry_length, group, compact = \
            64, "bf16", "htsat", "mlp", 0, 67, 1, 1
        encoder_batch = 64
    pipe, _, _ = bench.build(A, torch.device("cuda", 0))
    g = torch.Generator(device="cuda").manual_seed(1)
    wav = (torch.randn(64, 320000, device="cuda", generator=g) * 0.1).clamp_(-1, 1)
    pipe.caption_wav(wav)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record()
    for _ in range(3):
        pipe.encode(wav)
    ev[1].record()
    for _ in range(3):
        pipe.caption_wav(wav)
    ev[2].record()
    ev[2].synchronize()
    enc = ev[0].elapsed_time(ev[1]) / 3
    tot = ev[1].elapsed_time(ev[2]) / 3
    dec = pipe.decoder
    dec.done.zero_()
    gr = dec._graph(*dec._chunk_plan(None))
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        gr.replay()
    ev[1].record()
    ev[1].synchronize()
    step = ev[0].elapsed_time(ev[1]) * 1e3 / reps / dec.chunk
    print(f"bs64: encode {enc:.2f} ms, whole batch {tot:.2f} ms, decode step {step:.1f} us "
          f"(chunk {dec.chunk})", flush=True)


if __name__ == "__main__":
    main()
