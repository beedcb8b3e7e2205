#!/usr/bin/env python3
"""Timing of the bs=64 greedy decode: the persistent launch (zs_gpt2_decode_persist) against the
per-step graph chain, one batch alone and K batches concurrently (each on its own stream and
pipeline twin, the bench's ConcurrentRunner arrangement).  Decode only: every repetition restarts
generate2 from the same prefill (greedy_begin = step 0 from the prefill rows + the remaining
steps), so the numbers are decode steps per second.

    python tools/persist_bench.py [reps=5] [max_concurrent=5]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
os.environ["GPU_MAX_HW_QUEUES"] = "8"

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    kmax = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    from zsaac import ops
    from zsaac.pipeline import ConcurrentRunner

    class A:
        batch, dtype, encoder, mapper, beam, entry_length, group, compact = \
            64, "bf16", "htsat", "mlp", 0, 67, 1, 1
        encoder_batch = 64
    dev = torch.device("cuda", 0)
    pipe, _, _ = bench.build(A, dev)
    wav = bench.synthetic_clips(64, 0, dev)
    res = {"grid": ops.decode_persist_grid(),
           "cus": torch.cuda.get_device_properties(dev).multi_processor_count}
    for persist in (True, False):
        dec = pipe.decoder
        dec.persist = persist and dec.persist_ws is not None if hasattr(dec, "persist_ws") else False
        pipe.caption_wav(wav)
        torch.cuda.synchronize()

        def one():
            dec.greedy_begin(64)
            dec.run_to_completion()
        one()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            one()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        steps = int(dec.step_ctr.item())
        res["persist" if persist else "stepwise"] = {
            "decode_ms": round(dt * 1e3, 3), "steps": steps,
            "us_per_step": round(dt * 1e6 / max(1, steps - 1), 1)}
        print(json.dumps(res), flush=True)
    # concurrent persistent decodes
    pipe.decoder.persist = True
    runner = ConcurrentRunner(pipe, kmax)
    for p in runner.pipes:
        p.caption_wav(wav)
    torch.cuda.synchronize()
    conc = {}
    for k in range(1, runner.n_inflight + 1):
        pipes, streams = runner.pipes[:k], runner.streams[:k]
        for p, s in zip(pipes, streams):
            s.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            for p, s in zip(pipes, streams):
                with torch.cuda.stream(s):
                    p.decoder.greedy_begin(64)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        steps = sum(int(p.decoder.step_ctr.item()) - 1 for p in pipes)
        assert all(int(p.decoder.all_done[1].item()) >= 0 for p in pipes), "gave up"
        conc[k] = {"wall_ms_per_round": round(dt * 1e3 / reps, 3),
                   "agg_steps_per_s": round(steps * reps / dt, 1),
                   "equiv_us_per_step": round(dt * 1e6 / (steps * reps), 1)}
        res["concurrent"] = conc
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
