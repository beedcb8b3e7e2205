#!/usr/bin/env python3
"""The bs=64 greedy grid decode (decode_grid.hip) per grid size (256-thread workgroups):

  * one batch alone: microseconds per decode step of the persistent launch
    (zs_gpt2_decode_persist) and of the phase launches (zs_gpt2_decode_phases, the per-step
    path), and the ids against grid 48's (they must be identical);
  * k batches at once on k pipeline twins / dedicated streams (decode only: every repetition
    restarts generate2 from the same prefill), aggregate decode steps per second and the
    workgroup-microseconds one step costs (k x workgroups x wall / steps; a workgroup is half a
    CU).

    python tools/grid_bench.py [reps=4] [grids=48,96,192] [ks=1,2,4,5,8,10] [exps=0]

exps: zs_tune_set("dg_exp") traffic experiments (bit 0: hand-off loads / stores dropped, bit 1:
attention reads one cached key): ids are garbage under them, only the rates mean something.
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
    grids = [int(g) for g in (sys.argv[2] if len(sys.argv) > 2 else "48,96,192").split(",")]
    ks = [int(k) for k in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4,5,8,10").split(",")]
    exps = [int(k) for k in (sys.argv[4] if len(sys.argv) > 4 else "0").split(",")]
    from zsaac import ops
    from zsaac._lib import call

    class A:
        batch, dtype, encoder, mapper, beam, entry_length, group, compact = \
            64, "bf16", "htsat", "mlp", 0, 67, 1, 1
        encoder_batch = 64
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    pipe, _, _ = bench.build(A, dev)
    wav = bench.synthetic_clips(64, 0, dev)
    nmax = max(k for k in ks if k * min(grids) <= 2 * cus)
    pipes = [pipe] + [pipe.twin() for _ in range(nmax - 1)]
    streams = ops.dedicated_streams(nmax, dev)
    for p, s in zip(pipes, streams):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            p.caption_wav(wav)
    torch.cuda.synchronize()

    def decode(ps, ss, g):
        for p, s in zip(ps, ss):
            p.decoder.persist_grid = g
            with torch.cuda.stream(s):
                p.decoder.greedy_begin(64)

    res = {"cus": cus, "alone": {}, "concurrent": {}}
    ref = None
    dec = pipe.decoder
    # the phase launches (one batch, eager: 62 launches per step)
    dec.persist = False
    dec.greedy_begin(64)
    dec.run_to_completion()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dec.greedy_begin(64)
    dec.run_to_completion()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = int(dec.step_ctr.item())
    ref = (dec.out_ids[:64].clone(), dec.out_len[:64].clone())
    res["phases"] = {"grid": dec.phase_grid, "us_per_step": round(dt * 1e6 / max(1, steps - 1), 1),
                     "steps": steps, "note": "graph-replayed chunks incl. host polling"}
    print(json.dumps({"phases": res["phases"]}), flush=True)
    dec.persist = True
    for exp, g in [(e, g) for e in exps for g in grids]:
        call("zs_tune_set", b"dg_exp", exp)
        key = f"g{g}" + (f"_exp{exp}" if exp else "")
        decode(pipes[:1], streams[:1], g)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            decode(pipes[:1], streams[:1], g)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        assert int(dec.all_done[1].item()) >= 0, "gave up"
        steps = int(dec.step_ctr.item())
        ids, lens = dec.out_ids[:64].clone(), dec.out_len[:64].clone()
        r = {"workgroups": g, "decode_ms": round(dt * 1e3, 3), "steps": steps,
             "us_per_step": round(dt * 1e6 / max(1, steps - 1), 1),
             "identical_to_phases": bool(torch.equal(ids, ref[0]) and torch.equal(lens, ref[1]))}
        res["alone"][key] = r
        print(json.dumps({key: r}), flush=True)
        conc = {}
        for k in ks:
            if k * g > 2 * cus or k > nmax:
                continue
            decode(pipes[:k], streams[:k], g)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                decode(pipes[:k], streams[:k], g)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            assert all(int(p.decoder.all_done[1].item()) >= 0 for p in pipes[:k]), "gave up"
            st = sum(int(p.decoder.step_ctr.item()) - 1 for p in pipes[:k]) * reps
            conc[k] = {"agg_steps_per_s": round(st / dt, 1),
                       "wg_us_per_step": round(k * g * dt * 1e6 / st, 1)}
        res["concurrent"][key] = conc
        print(json.dumps({key: conc}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
