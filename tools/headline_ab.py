#!/usr/bin/env python3
"""Headline A/B in ONE process: the bench's C2 timed region (1045 clips, bs 64, persistent
decode) repeated for several arms, interleaved, so box-to-box and run-to-run spread cancel.

An arm is "name:inflight:knob=v,knob=v[:grids[:budget[:encode_ahead]]]" (zs_tune_set knobs, reset
(runner options among the knobs: late=0 sizes each grid at its batch's begin instead of at its
launch; spread=1: exclusive one-CU-per-workgroup grids while the CUs allow; prio=0: default stream
priorities instead of high for the pipelines and low for the encoder; extra=k: k pipelines beyond
the grids the budget holds; one=0: begin every idle pipeline in one pass instead of one per pass; eg=0: encoder passes
enqueued kernel by kernel instead of replayed from a hipGraph)
to the baseline values given with --base between arms; grids: the persistent-decode grid sizes the
runner may use, zsaac.pipeline.persist_grids, e.g. "48" or "96-48" ('-'-separated); budget:
workgroup slots of the in-flight grids; encode_ahead: clips per up-front encoder pass, 0 = each
batch encodes its own clips, suffix "f": every begin waits for the whole encode; a 7th field "bf":
begin_first, every pipeline begins at once and the launches follow within the budget); every arm runs on one shared set of streams.

    python tools/headline_ab.py --reps 6 "b512:10::48:512" "base:5::48:256" "l64:5:lean_min128=64"
"""
import argparse
import os
import statistics
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from zsaac import _lib  # noqa: E402
from zsaac.pipeline import ConcurrentRunner, persist_grids  # noqa: E402

# one hardware queue per stream (read at HIP init; after bench, whose import sets its default)
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("AB_HW_QUEUES", "16")


def knobs(spec):
    out = {}
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        out[k.strip()] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--clips", type=int, default=1045)
    ap.add_argument("--base", default="lean_min128=256", help="knob values restored between arms")
    ap.add_argument("arms", nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(dtype="bf16", group=1, encoder="htsat", mapper="mlp", batch=64,
                           encoder_batch=0, beam=0, entry_length=67, compact=1)
    pipe, _, _ = bench.build(args, dev)
    pool = bench.synthetic_clips(a.clips, 0, dev)
    batches = [pool[x:y] for x, y in bench.split_batches(a.clips, 64)]
    base = knobs(a.base)
    arms = []
    from zsaac import ops
    # one set of dedicated streams per priority for every arm (distinct hardware queues): the
    # pipelines' (prio=1 arms: high priority) and the encoder's (prio=1: low priority)
    nmax = max(int(x.split(":")[1]) for x in a.arms) + 4
    sets = {1: (ops.dedicated_streams(nmax, dev, priority=-1),
                ops.dedicated_streams(1, dev, priority=1)[0])}
    if any("prio=0" in x for x in a.arms):
        sets[0] = (ops.dedicated_streams(nmax, dev), ops.dedicated_streams(1, dev)[0])
    for spec in a.arms:
        name, inflight, kn, *sh = spec.split(":")
        kn = knobs(kn)
        streams, enc_stream = sets[kn.pop("prio", 1)]
        r = ConcurrentRunner(pipe, int(inflight), streams=streams, enc_stream=enc_stream,
                             extra_pipes=kn.pop("extra", 0),
                             grids=persist_grids(sh[0].replace("-", ",")) if sh and sh[0] else None,
                             budget=int(sh[1]) if len(sh) > 1 and sh[1] else None,
                             encode_ahead=int(sh[2].rstrip("f")) if len(sh) > 2 and sh[2] else 0,
                             encode_first=len(sh) > 2 and sh[2].endswith("f"),
                             begin_first=len(sh) > 3 and sh[3] == "bf")
        for size in sorted({b.shape[0] for b in batches}, reverse=True):
            r.warmup(next(b for b in batches if b.shape[0] == size))
        r.late_grid = bool(kn.pop("late", 1))      # runner options, not zs_tune_set knobs
        r.spread = bool(kn.pop("spread", 0))
        r.one_begin = bool(kn.pop("one", 1))
        r.enc_graph = bool(kn.pop("eg", 1))
        arms.append((name, r, kn))
    res = {n: [] for n, _, _ in arms}
    for rep in range(a.reps + 1):
        for name, r, kn in arms:
            for k, v in {**base, **kn}.items():
                _lib.call("zs_tune_set", k.encode(), v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.run(batches)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if r.gave_up:
                print(f"{name}: {r.gave_up} persistent launches gave up", flush=True)
            if rep:                     # rep 0 warms every arm's kernels up
                res[name].append(a.clips / dt)
        if rep:
            print(f"rep {rep}: " + "  ".join(f"{n} {res[n][-1]:.0f}" for n in res), flush=True)
            for name, r, _ in arms:
                if getattr(r, "trace", None):
                    print(name, "host trace (ms):", r.trace, flush=True)
    for n, v in res.items():
        print(f"{n:12s} median {statistics.median(v):8.1f} clips/s  min {min(v):8.1f}  max {max(v):8.1f}")


if __name__ == "__main__":
    main()
