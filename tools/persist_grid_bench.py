#!/usr/bin/env python3
"""The bs=64 persistent greedy decode (zs_gpt2_decode_persist) at each grid shape
(col_split, row_split) -> workgroups per batch = 48 / col_split * row_split:

  * one batch alone: microseconds per decode step, and the generated ids against the
    (1, 1) shape's (exact rows, token agreement);
  * k batches at once on k pipeline twins / dedicated streams (decode only: every repetition
    restarts generate2 from the same prefill), aggregate decode steps per second and the
    CU-microseconds one step costs (k x workgroups x wall / steps).

    python tools/persist_grid_bench.py [reps=4] [shapes=11,21,22,12] [ks=1,2,4,5,8,10]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

# one hardware queue per stream (read at HIP init; after bench, whose import sets its default)
os.environ["GPU_MAX_HW_QUEUES"] = "16"


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    shapes = [(int(s[0]), int(s[1])) for s in (sys.argv[2] if len(sys.argv) > 2 else "11,21,22,12").split(",")]
    ks = [int(k) for k in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4,5,8,10").split(",")]
    from zsaac import ops

    class A:
        batch, dtype, encoder, mapper, beam, entry_length, group, compact = \
            64, "bf16", "htsat", "mlp", 0, 67, 1, 1
        encoder_batch = 64
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    pipe, _, _ = bench.build(A, dev)
    wav = bench.synthetic_clips(64, 0, dev)
    nmax = max(k for k in ks if k * min(ops.decode_persist_grid(rs, cs) for cs, rs in shapes) <= cus)
    pipes = [pipe] + [pipe.twin() for _ in range(nmax - 1)]
    streams = ops.dedicated_streams(nmax, dev)
    for p, s in zip(pipes, streams):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            p.caption_wav(wav)
    torch.cuda.synchronize()

    def decode(ps, ss, cs, rs):
        for p, s in zip(ps, ss):
            p.decoder.persist_col_split, p.decoder.persist_row_split = cs, rs
            with torch.cuda.stream(s):
                p.decoder.greedy_begin(64)

    res = {"cus": cus, "alone": {}, "concurrent": {}}
    ref = None
    for cs, rs in shapes:
        key = f"cs{cs}_rs{rs}"
        g = ops.decode_persist_grid(rs, cs)
        decode(pipes[:1], streams[:1], cs, rs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            decode(pipes[:1], streams[:1], cs, rs)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        dec = pipe.decoder
        assert int(dec.all_done[1].item()) >= 0, "gave up"
        steps = int(dec.step_ctr.item())
        ids = dec.out_ids[:64].clone()
        lens = dec.out_len[:64].clone()
        r = {"workgroups": g, "decode_ms": round(dt * 1e3, 3), "steps": steps,
             "us_per_step": round(dt * 1e6 / max(1, steps - 1), 1)}
        if ref is None:
            ref = (ids, lens)
        else:
            same = [(lens[i] == ref[1][i]).item() and bool((ids[i, :lens[i]] == ref[0][i, :lens[i]]).all())
                    for i in range(64)]
            n = torch.minimum(lens, ref[1])
            agree = sum(int((ids[i, :n[i]] == ref[0][i, :n[i]]).sum()) for i in range(64))
            r["rows_equal_to_cs1_rs1"] = sum(same)
            r["token_agreement"] = round(agree / max(1, int(ref[1].sum())), 4)
        res["alone"][key] = r
        print(json.dumps({key: r}), flush=True)
        conc = {}
        for k in ks:
            if k * g > cus or k > nmax:
                continue
            decode(pipes[:k], streams[:k], cs, rs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                decode(pipes[:k], streams[:k], cs, rs)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            assert all(int(p.decoder.all_done[1].item()) >= 0 for p in pipes[:k]), "gave up"
            st = sum(int(p.decoder.step_ctr.item()) - 1 for p in pipes[:k]) * reps
            conc[k] = {"agg_steps_per_s": round(st / dt, 1),
                       "cu_us_per_step": round(k * g * dt * 1e6 / st, 1)}
        res["concurrent"][key] = conc
        print(json.dumps({key: conc}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
