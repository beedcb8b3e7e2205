#!/usr/bin/env python3
"""One rank's strong-scaling shard (131 of the 1045 Clotho-eval clips, zsaac.dist.shard_range)
timed alone under several batchings and persistent-grid shape lists: which choice a rank should
make when it has only a few batches (bench.py strong_scaling_proxy reports the default's).

    python tools/shard_probe.py [reps=5] [arms=parts:shapes;...]

parts: split_batches parts (0 = consecutive bs-64 batches); shapes: ZSAAC_PERSIST_SHAPES.
Prints one JSON line per arm (median seconds, batch sizes, grid shapes taken)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

os.environ["GPU_MAX_HW_QUEUES"] = "16"

DEFAULT_ARMS = "0:12,11,21;3:12,11,21;3:11;3:12,11;4:11;5:11;5:21;3:21"


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    arms = [a.split(":") for a in (sys.argv[2] if len(sys.argv) > 2 else DEFAULT_ARMS).split(";")]
    from zsaac import dist as zd
    args = bench.parse([])
    dev = torch.device("cuda", 0)
    pipe, _, _ = bench.build(args, dev)
    lo, hi = zd.shard_range(bench.CLOTHO_EVAL_CLIPS, 0, 8)
    n = hi - lo
    for parts, shapes in arms:
        os.environ["ZSAAC_PERSIST_SHAPES"] = shapes
        dt, outs, runner, _ = bench.run_captions(args, 1, 0, dev, pipe, n, lo, [n], args.inflight,
                                                 3, parts=int(parts), reps=reps)
        print(json.dumps({"parts": int(parts), "shapes": shapes, "seconds": round(dt, 4),
                          "batches": [int(o.ids.shape[0]) for o in outs],
                          "grid_shapes": [f"cs{c}rs{r}" for c, r in getattr(runner, "shape", [])]}),
              flush=True)
        del outs, runner
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
