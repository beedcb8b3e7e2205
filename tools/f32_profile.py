#!/usr/bin/env python3
"""The bench's f32 parity-mode line alone (1045 clips, bs 64) -- run it under rocprofv3
--kernel-trace --stats to see where the f32 mode's time goes; or sweep configurations:

    python tools/f32_profile.py [clips=1045] [inflight=4] [budget=0] [extra=0] [grid=1] [ahead=256] [runs=1]

grid 0: the round-4 f32 row-kernel decode (ZSAAC_GRID_DECODE_F32=0) instead of the f32 grid decode;
budget / extra: the runner's persistent budget (0 = default) and extra pipelines.
"""
import json
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

os.environ["GPU_MAX_HW_QUEUES"] = "16"


def main():
    v = [int(x) for x in sys.argv[1:]] + [None] * 7
    n, k = v[0] or 1045, v[1] or 4
    budget, extra = v[2] or 0, v[3] or 0
    grid = 1 if v[4] is None else v[4]
    ahead = 256 if v[5] is None else v[5]
    os.environ["ZSAAC_GRID_DECODE_F32"] = str(grid)
    args = SimpleNamespace(dtype="f32", group=1, encoder="htsat", mapper="mlp", batch=64,
                           encoder_batch=0, beam=0, entry_length=67, compact=1,
                           persist_budget=budget, encode_ahead=ahead, extra_pipes=extra)
    runs = v[6] or 1
    for _ in range(runs - 1):       # earlier runs in the same process (process-state A/B)
        r0 = bench.sub_run(args, torch.device("cuda", 0), torch.float32, 1, k, n, 1)
        print(json.dumps({"earlier_run_value": r0["value"]}), flush=True)
    bench.ALL_PERSIST_LOGS.clear()
    res = bench.sub_run(args, torch.device("cuda", 0), torch.float32, 1, k, n, 1)
    logs = bench.ALL_PERSIST_LOGS
    launch_ms = [e0.elapsed_time(e1) for e0, e1, _ in logs]
    print(json.dumps({"inflight": k, "budget": budget, "extra": extra, "grid_decode_f32": grid,
                      "encode_ahead": ahead, "value": res["value"], "ms_per_step": res["ms_per_step"],
                      "persist_launch_ms_mean": round(sum(launch_ms) / max(1, len(launch_ms)), 2),
                      "persist_launches": len(launch_ms),
                      "runner": {kk: res["config"].get(kk) for kk in ("persist_grids", "persist_gave_up", "batches_in_flight")}}),
          flush=True)


if __name__ == "__main__":
    main()
