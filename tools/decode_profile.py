#!/usr/bin/env python3
"""Single-stream profile of one greedy decode step at a given compaction bucket (for
rocprofv3 --kernel-trace): builds the G32 bench pipeline, captions one 2048-clip group, then
replays the chosen chunk graph N times back to back.

    python tools/decode_profile.py [Rb=2048] [reps=10]
    python tools/decode_profile.py encode [reps=2]     # the encoder over one 2048-clip group
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    enc = len(sys.argv) > 1 and sys.argv[1] == "encode"
    Rb = int(sys.argv[1]) if len(sys.argv) > 1 and not enc else 2048
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else (2 if enc else 10)

    class A:
        batch, dtype, encoder, mapper, beam, entry_length, group, compact = \
            64, "bf16", "htsat", "mlp", 0, 67, 32, 1
    pipe, _, _ = bench.build(A, torch.device("cuda", 0))
    g = torch.Generator(device="cuda").manual_seed(1)
    wav = (torch.randn(2048, 320000, device="cuda", generator=g) * 0.1).clamp_(-1, 1)
    pipe.caption_wav(wav)
    if enc:
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            pipe.encode(wav)
        e1.record()
        e1.synchronize()
        print(f"encode 2048 clips: {e0.elapsed_time(e1) / reps:.2f} ms")
        return
    dec = pipe.decoder
    dec.done.zero_()                     # every row active: a full-width step
    gr = dec._graph(*dec._chunk_plan(Rb))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        gr.replay()
    e1.record()
    e1.synchronize()
    print(f"Rb={Rb}: {e0.elapsed_time(e1) * 1e3 / reps / dec.chunk:.1f} us/step")


if __name__ == "__main__":
    main()
